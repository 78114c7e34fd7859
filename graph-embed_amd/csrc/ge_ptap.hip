// ge_ptap.hip -- Galerkin restriction A_c = P_T * A * P_T^T on gfx950.
//
// Reference call sites: P_T.Mult(A).Mult(P_T.Transpose()) at
// examples/embed.cpp:96-98 and examples/embedder.cpp:213-216 (linalgcpp, not
// vendored).  A_c[a][b] = sum of A[i][j] over i in aggregate a, j in b.
//
// Pinned summation order (identical to oracle/ge_oracle.cpp orc_ptap): B = P_T A
// adds, for each (a, j), the members of a in P_T row order; C = B P adds, for
// each (a, b), B's columns j ascending.  For the unit weights of every benchmark
// graph all sums are exact integers, so the pin matters only for fractional
// weights.
//
// Aggregation SpGEMM by sort + segmented serial sums (integer keys and a stream
// of fp64 weights; HBM-bound, no GEMM shape):
//   1. expand: one thread per emitted entry (P_T position c, CSR entry (i, j, w)
//      of member i = pt_ix[c]), entries numbered in (c, CSR) order; a thread
//      finds its position by binary search over the row-length prefix sums, so
//      a hub row's entries spread over many lanes and every store coalesces.
//   2. one stable radix sort by the composite key (a, b = agg(j), j): equal keys
//      keep emission (= P_T member) order.  When the three fields need more than
//      64 bits (graphs beyond ~2^21 vertices per level with many aggregates) the
//      sort is split LSD-style: stable by j, then stable by (a, b) -- the same
//      final order.
//   3. one thread per (a, b) run walks it once: the inner sum restarts at each
//      new j (B[a][j], members in order), the outer sum adds the B values in j
//      order (C[a][b]).  Row lengths are counted on the device and scanned into
//      indptr; the host receives the finished CSR (one synchronisation for the
//      number of coarse entries, one for the result).
// A row range [a0, a1) restricts steps 1-3 to those coarse rows (one rank's
// share in ge_ptap_dist); agg(j) always uses the whole P_T.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "ge_internal.hpp"
#include "ge_prim.hpp"

namespace ge {
namespace {

using u64 = unsigned long long;

inline unsigned grid_for(long long L) { return (unsigned)((L + 255) / 256); }

// bits needed for the values 0 .. x-1
int bits_below(long long x) {
  int b = 0;
  while (b < 63 && (1ll << b) < x) ++b;
  return b;
}

// heads[c] = number of aggregates a >= 1 whose first position is c; the
// inclusive scan of heads is the aggregate of position c (empty aggregates
// included).
__global__ void agg_heads_kernel(int m, int n, const int* __restrict__ pt_ip,
                                 int* __restrict__ heads) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (a < m && pt_ip[a] < n) atomicAdd(&heads[pt_ip[a]], 1);
}

__global__ void agg_vertex_kernel(int n, const int* __restrict__ pt_ix,
                                  const int* __restrict__ agg_pos, int* __restrict__ agg_vtx) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n) agg_vtx[pt_ix[c]] = agg_pos[c];
}

__global__ void row_len_kernel(int P, int c0, const int* __restrict__ pt_ix,
                               const int* __restrict__ ip, long long* __restrict__ len) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < P) {
    const int i = pt_ix[c0 + c];
    len[c] = ip[i + 1] - ip[i];
  }
}

// Entry t of the (c, CSR)-ordered stream: position c = last q with off[q] <= t.
// Composite key (a - a0, b, j) with b and j in the low bits; LSD (split) mode
// writes the j key and the (a - a0, b) key separately.
template <bool SPLIT>
__global__ void expand_kernel(long long L, int P, int c0, int a0, int bn, int bb,
                              const long long* __restrict__ off, const int* __restrict__ pt_ix,
                              const int* __restrict__ agg_pos, const int* __restrict__ agg_vtx,
                              const int* __restrict__ ip, const int* __restrict__ ix,
                              const double* __restrict__ dx, u64* __restrict__ key,
                              u64* __restrict__ key_hi, double* __restrict__ val) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L) return;
  int lo = 0, hi = P - 1;
  while (lo < hi) {  // largest q with off[q] <= t (rows of length 0 are skipped over)
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  const int c = c0 + lo;
  const int i = pt_ix[c];
  const int e = ip[i] + (int)(t - off[lo]);
  const u64 j = (unsigned)ix[e];
  const u64 ab = ((u64)(unsigned)(agg_pos[c] - a0) << bb) | (unsigned)agg_vtx[j];
  if (SPLIT) {
    key[t] = j;
    key_hi[t] = ab;
  } else {
    key[t] = (ab << bn) | j;
  }
  val[t] = dx[e];
}

// LSD second pass: the (a, b) keys in the order of the j sort.
__global__ void gather_keys_kernel(long long L, const unsigned* __restrict__ perm,
                                   const u64* __restrict__ key_hi, u64* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L) out[t] = key_hi[perm[t]];
}

__global__ void iota_kernel(long long L, unsigned* __restrict__ v) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L) v[t] = (unsigned)t;
}

// LSD mode: entry t of the final order is entry rp[t] of the j-sorted stream,
// i.e. emitted entry pp[rp[t]]; its key becomes (run number, j).
__global__ void compose_kernel(long long L, int bn, const int* __restrict__ flag,
                               const int* __restrict__ runid, const unsigned* __restrict__ rp,
                               const unsigned* __restrict__ pp, const u64* __restrict__ ab,
                               const u64* __restrict__ jsorted, const double* __restrict__ vsrc,
                               u64* __restrict__ key, double* __restrict__ val,
                               u64* __restrict__ ab_run) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L) return;
  const unsigned q = rp[t];
  const int run = runid[t] - 1;
  key[t] = ((u64)(unsigned)run << bn) | jsorted[q];
  val[t] = vsrc[pp[q]];
  if (flag[t]) ab_run[run] = ab[t];
}

// head of an (a, b) run: the key above the j bits changes
__global__ void run_heads_kernel(long long L, int bn, const u64* __restrict__ key,
                                 int* __restrict__ flag) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L) flag[t] = (t == 0 || (key[t] >> bn) != (key[t - 1] >> bn)) ? 1 : 0;
}

__global__ void run_starts_kernel(long long L, const int* __restrict__ flag,
                                  const int* __restrict__ runid, long long* __restrict__ start) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L && flag[t]) start[runid[t] - 1] = t;
}

// One thread per (a, b) run (the pinned order): B[a][j] restarts at each new j
// and adds members in P_T order; C[a][b] adds the B values in ascending j.
// Multiplications by P's 1.0 entries are exact and left out.
__global__ void run_sum_kernel(long long L, const int* __restrict__ nruns_p, int bn, int bb,
                               const long long* __restrict__ start, const u64* __restrict__ key,
                               const double* __restrict__ val, const u64* __restrict__ ab_run,
                               int* __restrict__ out_col,
                               double* __restrict__ out_val, int* __restrict__ row_cnt) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long runs = *nruns_p;
  if (r >= runs) return;
  const long long b0 = start[r];
  const long long b1 = (r + 1 < runs) ? start[r + 1] : L;
  const u64 jmask = (bn >= 64) ? ~0ull : ((1ull << bn) - 1);
  double outer = 0.0, inner = 0.0;
  u64 kprev = key[b0];
  for (long long t = b0; t < b1; ++t) {
    const u64 k = key[t];
    if ((k & jmask) != (kprev & jmask)) {
      outer += inner;
      inner = 0.0;
      kprev = k;
    }
    inner += val[t];
  }
  outer += inner;
  const u64 ab = ab_run ? ab_run[r] : key[b0] >> bn;
  out_col[r] = (int)(ab & ((1ull << bb) - 1));
  out_val[r] = outer;
  atomicAdd(&row_cnt[(int)(ab >> bb)], 1);
}

template <class K, class V>
void sort_pairs(hipStream_t st, K*& k, K*& k2, V*& v, V*& v2, long long L, int end_bit) {
  prim_sort_pairs(st, k, k2, v, v2, (size_t)L, end_bit);
  std::swap(k, k2);
  std::swap(v, v2);
}

template <class T>
void exclusive_scan(hipStream_t st, const T* in, T* out, long long count) {
  prim_exclusive_sum(st, in, out, (size_t)count);
}

template <class T>
void inclusive_scan(hipStream_t st, const T* in, T* out, long long count) {
  prim_inclusive_sum(st, in, out, (size_t)count);
}

}  // namespace

void ptap_device(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix, const double* d_dx,
                 int nnz, int m, const int* h_pt_ip, const int* d_pt_ip, const int* d_pt_ix,
                 int a0, int a1, ge_csr* out) {
  hipStream_t st = ctx->stream;
  const int R = a1 - a0;
  out->rows = R;
  out->cols = m;
  out->indptr.assign(R + 1, 0);
  out->indices.clear();
  out->data.clear();
  const int c0 = h_pt_ip[a0], c1 = h_pt_ip[a1];
  const int P = c1 - c0;
  if (n == 0 || R == 0 || P == 0 || nnz == 0) return;

  // aggregate of every P_T position and of every fine vertex
  DevBuf<int> heads(n), agg_pos(n), agg_vtx(n);
  GE_HIP(hipMemsetAsync(heads.p, 0, sizeof(int) * n, st));
  if (m > 1)
    hipLaunchKernelGGL(agg_heads_kernel, dim3(grid_for(m - 1)), dim3(256), 0, st, m, n, d_pt_ip,
                       heads.p);
  inclusive_scan(st, heads.p, agg_pos.p, n);
  hipLaunchKernelGGL(agg_vertex_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, d_pt_ix,
                     agg_pos.p, agg_vtx.p);

  // emitted entries: prefix sums of the members' row lengths
  DevBuf<long long> len(P + 1), off(P + 1);
  GE_HIP(hipMemsetAsync(len.p + P, 0, sizeof(long long), st));
  hipLaunchKernelGGL(row_len_kernel, dim3(grid_for(P)), dim3(256), 0, st, P, c0, d_pt_ix, d_ip,
                     len.p);
  exclusive_scan(st, len.p, off.p, P + 1);
  long long L = nnz;  // every fine row appears once in P_T
  if (a0 != 0 || a1 != m) {
    GE_HIP(hipMemcpyAsync(&L, off.p + P, sizeof(long long), hipMemcpyDeviceToHost, st));
    GE_HIP(hipStreamSynchronize(st));
  }
  if (L == 0) return;
  GE_REQUIRE(L < (1ll << 31), "P^T A P: more than 2^31 entries in one call (shard the rows)");

  const int bn = bits_below(n), bb = bits_below(m), ba = bits_below(R);
  const bool split = ba + bb + bn > 64 || std::getenv("GE_PTAP_SPLIT_SORT") != nullptr;
  DevBuf<u64> k(L), k2(L);
  DevBuf<double> v(L), v2(L);
  u64 *kp = k.p, *kq = k2.p;
  double *vp = v.p, *vq = v2.p;
  DevBuf<u64> ab_run;  // split mode: (a, b) of each run
  if (!split) {
    hipLaunchKernelGGL(expand_kernel<false>, dim3(grid_for(L)), dim3(256), 0, st, L, P, c0, a0,
                       bn, bb, off.p, d_pt_ix, agg_pos.p, agg_vtx.p, d_ip, d_ix, d_dx, kp,
                       nullptr, vp);
    GE_HIP(hipGetLastError());
    sort_pairs(st, kp, kq, vp, vq, L, std::max(1, ba + bb + bn));
  } else {
    // LSD: stable by j, then stable by (a, b).  The (a, b) pairs are then replaced
    // by their dense run number (< L < 2^31), so (run, j) fits 64 bits again.
    DevBuf<u64> khi(L);
    DevBuf<unsigned> perm(L), perm2(L), rank(L), rank2(L);
    hipLaunchKernelGGL(expand_kernel<true>, dim3(grid_for(L)), dim3(256), 0, st, L, P, c0, a0, bn,
                       bb, off.p, d_pt_ix, agg_pos.p, agg_vtx.p, d_ip, d_ix, d_dx, kp, khi.p, vp);
    hipLaunchKernelGGL(iota_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, perm.p);
    hipLaunchKernelGGL(iota_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, rank.p);
    GE_HIP(hipGetLastError());
    unsigned *pp = perm.p, *pq = perm2.p, *rp = rank.p, *rq = rank2.p;
    sort_pairs(st, kp, kq, pp, pq, L, std::max(1, bn));  // kp[q]: j of entry pp[q], j ascending
    u64 *hs = kq, *ht = khi.p;              // (kq is free now)
    hipLaunchKernelGGL(gather_keys_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, pp, khi.p, hs);
    // khi is read by the gather before the sort below reuses it as scratch (same stream)
    sort_pairs(st, hs, ht, rp, rq, L, std::max(1, ba + bb));  // hs[t]: (a, b) of stream entry rp[t]
    DevBuf<int> flag(L), runid(L);
    hipLaunchKernelGGL(run_heads_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, 0, hs, flag.p);
    inclusive_scan(st, flag.p, runid.p, L);
    ab_run.alloc(L);
    hipLaunchKernelGGL(compose_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, bn, flag.p,
                       runid.p, rp, pp, hs, kp, vp, ht, vq, ab_run.p);
    GE_HIP(hipGetLastError());
    std::swap(kp, ht);  // composed keys (ht was the (a, b) sort's scratch)
    std::swap(vp, vq);
  }

  // (a, b) runs and their serial sums
  DevBuf<int> flag(L), runid(L), row_cnt(R + 1);
  DevBuf<long long> start(L);
  hipLaunchKernelGGL(run_heads_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, bn, kp, flag.p);
  inclusive_scan(st, flag.p, runid.p, L);
  GE_HIP(hipMemsetAsync(row_cnt.p, 0, sizeof(int) * (R + 1), st));
  hipLaunchKernelGGL(run_starts_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, flag.p, runid.p,
                     start.p);
  DevBuf<int> ocol(L);
  DevBuf<double> oval(L);
  hipLaunchKernelGGL(run_sum_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, runid.p + (L - 1),
                     bn, bb, start.p, kp, vp, ab_run.p, ocol.p, oval.p, row_cnt.p);
  GE_HIP(hipGetLastError());
  DevBuf<int> indptr(R + 1);
  exclusive_scan(st, row_cnt.p, indptr.p, R + 1);
  int nc = 0;
  GE_HIP(hipMemcpyAsync(&nc, runid.p + (L - 1), sizeof(int), hipMemcpyDeviceToHost, st));
  GE_HIP(hipStreamSynchronize(st));
  out->indices.resize(nc);
  out->data.resize(nc);
  GE_HIP(hipMemcpyAsync(out->indptr.data(), indptr.p, sizeof(int) * (R + 1),
                        hipMemcpyDeviceToHost, st));
  GE_HIP(hipMemcpyAsync(out->indices.data(), ocol.p, sizeof(int) * nc, hipMemcpyDeviceToHost,
                        st));
  GE_HIP(hipMemcpyAsync(out->data.data(), oval.p, sizeof(double) * nc, hipMemcpyDeviceToHost,
                        st));
  GE_HIP(hipStreamSynchronize(st));
}

}  // namespace ge
