// ge_ptap.hip -- Galerkin restriction A_c = P_T * A * P_T^T on gfx950.
//
// Reference call sites: P_T.Mult(A).Mult(P_T.Transpose()) at
// examples/embed.cpp:96-98 and examples/embedder.cpp:213-216 (linalgcpp, not
// vendored).  A_c[a][b] = sum of A[i][j] over i in aggregate a, j in b.
//
// Aggregation SpGEMM by sort + run-length reduce (no GEMM shape: integer keys
// and a stream of fp64 weights, HBM-bound):
//   1. expand: for every P_T position c (aggregate a = row of c, member
//      i = pt_ix[c]) and every CSR entry (i, j, w): key1 = (a << 32) | j, val w.
//      Entries are emitted in (c, CSR) order.
//   2. stable radix sort by key1; sum each run in emission order  -> B = P_T A
//   3. key2 = (a << 32) | agg(j) for every B entry; stable sort; sum each run in
//      ascending-j order -> C = B P, rows and columns ascending.
// Pinned summation order (identical to oracle/ge_oracle.cpp orc_ptap): B[a][j]
// adds members in P_T row order, C[a][b] adds B's columns ascending.  For the
// unit weights of every benchmark graph all sums are exact integers.

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <vector>

#include "ge_internal.hpp"

namespace ge {
namespace {

__global__ void row_len_kernel(int N, const int* __restrict__ pt_ix, const int* __restrict__ ip,
                               long long* __restrict__ len) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < N) {
    const int i = pt_ix[c];
    len[c] = ip[i + 1] - ip[i];
  }
}

__global__ void agg_of_pos_kernel(int m, const int* __restrict__ pt_ip, int* __restrict__ agg_pos,
                                  const int* __restrict__ pt_ix, int* __restrict__ agg_vtx) {
  const int a = blockIdx.x;
  for (int c = pt_ip[a] + threadIdx.x; c < pt_ip[a + 1]; c += blockDim.x) {
    agg_pos[c] = a;
    agg_vtx[pt_ix[c]] = a;
  }
}

// One thread per P_T position; writes its member's CSR row at off[c].
__global__ void expand_kernel(int N, const int* __restrict__ pt_ix, const int* __restrict__ agg_pos,
                              const int* __restrict__ ip, const int* __restrict__ ix,
                              const double* __restrict__ dx, const long long* __restrict__ off,
                              unsigned long long* __restrict__ key, double* __restrict__ val) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  const int i = pt_ix[c];
  const unsigned long long hi = (unsigned long long)(unsigned)agg_pos[c] << 32;
  long long o = off[c];
  for (int e = ip[i]; e < ip[i + 1]; ++e, ++o) {
    key[o] = hi | (unsigned)ix[e];
    val[o] = dx[e];
  }
}

__global__ void head_flags_kernel(long long L, const unsigned long long* __restrict__ key,
                                  int* __restrict__ flag) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L) flag[t] = (t == 0 || key[t] != key[t - 1]) ? 1 : 0;
}

__global__ void scatter_heads_kernel(long long L, const int* __restrict__ flag,
                                     const int* __restrict__ runid, long long* __restrict__ start) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L && flag[t]) start[runid[t] - 1] = t;
}

// Serial left-to-right sum of each run (the pinned order).  mul = 1.0 models
// the multiplication by P's 1.0 entries.
__global__ void run_sum_kernel(long long runs, long long L, const long long* __restrict__ start,
                               const unsigned long long* __restrict__ key,
                               const double* __restrict__ val, double mul,
                               unsigned long long* __restrict__ okey, double* __restrict__ oval) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= runs) return;
  const long long b = start[r];
  const long long e = (r + 1 < runs) ? start[r + 1] : L;
  double s = 0.0;
  for (long long t = b; t < e; ++t) s += val[t] * mul;
  okey[r] = key[b];
  oval[r] = s;
}

__global__ void rekey_kernel(long long L, const unsigned long long* __restrict__ key,
                             const int* __restrict__ agg_vtx, unsigned long long* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L) {
    const unsigned long long k = key[t];
    out[t] = (k & 0xFFFFFFFF00000000ull) | (unsigned)agg_vtx[(unsigned)(k & 0xFFFFFFFFull)];
  }
}

inline unsigned grid_for(long long L) { return (unsigned)((L + 255) / 256); }

// stable sort pairs by the low `bits` bits of the key
void sort_pairs(hipStream_t st, DevBuf<unsigned long long>& k, DevBuf<double>& v,
                DevBuf<unsigned long long>& k2, DevBuf<double>& v2, long long L, int end_bit) {
  size_t tmp = 0;
  GE_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, k.p, k2.p, v.p, v2.p, (int)L, 0,
                                            end_bit, st));
  DevBuf<unsigned char> scratch(tmp);
  GE_HIP(hipcub::DeviceRadixSort::SortPairs(scratch.p, tmp, k.p, k2.p, v.p, v2.p, (int)L, 0,
                                            end_bit, st));
  std::swap(k.p, k2.p);
  std::swap(v.p, v2.p);
}

// Reduce equal-key runs of (k, v)[0..L) into (k2, v2); returns the run count.
long long reduce_runs(hipStream_t st, const DevBuf<unsigned long long>& k,
                      const DevBuf<double>& v, DevBuf<unsigned long long>& k2,
                      DevBuf<double>& v2, long long L) {
  DevBuf<int> flag(L), runid(L);
  hipLaunchKernelGGL(head_flags_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, k.p, flag.p);
  size_t tmp = 0;
  GE_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tmp, flag.p, runid.p, (int)L, st));
  DevBuf<unsigned char> scratch(tmp);
  GE_HIP(hipcub::DeviceScan::InclusiveSum(scratch.p, tmp, flag.p, runid.p, (int)L, st));
  int runs = 0;
  GE_HIP(hipMemcpyAsync(&runs, runid.p + (L - 1), sizeof(int), hipMemcpyDeviceToHost, st));
  GE_HIP(hipStreamSynchronize(st));
  DevBuf<long long> start(runs);
  hipLaunchKernelGGL(scatter_heads_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, flag.p,
                     runid.p, start.p);
  hipLaunchKernelGGL(run_sum_kernel, dim3(grid_for(runs)), dim3(256), 0, st, (long long)runs, L,
                     start.p, k.p, v.p, 1.0, k2.p, v2.p);
  GE_HIP(hipGetLastError());
  return runs;
}

int bits_for(long long x) {
  int b = 1;
  while ((1ll << b) <= x) ++b;
  return b;
}

}  // namespace

void ptap_device(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix, const double* d_dx,
                 int nnz, int m, const int* d_pt_ip, const int* d_pt_ix, ge_csr* out) {
  hipStream_t st = ctx->stream;
  out->rows = out->cols = m;
  out->indptr.assign(m + 1, 0);
  out->indices.clear();
  out->data.clear();
  if (n == 0 || m == 0 || nnz == 0) return;
  const int N = n;  // one P_T entry per fine vertex
  DevBuf<long long> len(N), off(N);
  DevBuf<int> agg_pos(N), agg_vtx(n);
  hipLaunchKernelGGL(row_len_kernel, dim3(grid_for(N)), dim3(256), 0, st, N, d_pt_ix, d_ip, len.p);
  hipLaunchKernelGGL(agg_of_pos_kernel, dim3(m), dim3(64), 0, st, m, d_pt_ip, agg_pos.p, d_pt_ix,
                     agg_vtx.p);
  size_t tmp = 0;
  GE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, len.p, off.p, N, st));
  {
    DevBuf<unsigned char> scratch(tmp);
    GE_HIP(hipcub::DeviceScan::ExclusiveSum(scratch.p, tmp, len.p, off.p, N, st));
  }
  const long long L = nnz;
  DevBuf<unsigned long long> k(L), k2(L);
  DevBuf<double> v(L), v2(L);
  hipLaunchKernelGGL(expand_kernel, dim3(grid_for(N)), dim3(256), 0, st, N, d_pt_ix, agg_pos.p,
                     d_ip, d_ix, d_dx, off.p, k.p, v.p);
  GE_HIP(hipGetLastError());
  const int key_bits = 32 + bits_for(m);
  sort_pairs(st, k, v, k2, v2, L, key_bits);  // result in k, v
  long long nb = reduce_runs(st, k, v, k2, v2, L);  // B in k2, v2
  std::swap(k.p, k2.p);
  std::swap(v.p, v2.p);  // B in k, v
  hipLaunchKernelGGL(rekey_kernel, dim3(grid_for(nb)), dim3(256), 0, st, nb, k.p, agg_vtx.p, k2.p);
  std::swap(k.p, k2.p);  // rekeyed B in k
  sort_pairs(st, k, v, k2, v2, nb, key_bits);
  long long nc = reduce_runs(st, k, v, k2, v2, nb);  // C in k2, v2
  std::vector<unsigned long long> hk(nc);
  out->data.resize(nc);
  GE_HIP(hipMemcpyAsync(hk.data(), k2.p, sizeof(unsigned long long) * nc, hipMemcpyDeviceToHost, st));
  GE_HIP(hipMemcpyAsync(out->data.data(), v2.p, sizeof(double) * nc, hipMemcpyDeviceToHost, st));
  GE_HIP(hipStreamSynchronize(st));
  out->indices.resize(nc);
  for (long long t = 0; t < nc; ++t) {
    const int a = (int)(hk[t] >> 32);
    out->indices[t] = (int)(hk[t] & 0xFFFFFFFFull);
    out->indptr[a + 1]++;
  }
  for (int a = 0; a < m; ++a) out->indptr[a + 1] += out->indptr[a];
}

}  // namespace ge
