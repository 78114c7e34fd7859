// ge_graph.hip -- synthetic inputs on the device: the Graph500 R-MAT generator
// and the largest connected component (examples/embedder.cpp:35-93), both with
// the results of the host versions in ge_host.cpp (ge_rmat_csr /
// ge_largest_component) bit for bit.
//
//   R-MAT: one thread per draw evaluates the counter-based stream
//   (splitmix64(splitmix64(seed) + 64 e + l), definition in tests/graphs.py) and
//   emits both directions as 64-bit keys row * n + col; a radix sort and a
//   flagged compaction symmetrise and deduplicate; the row histogram scanned
//   gives indptr.  Columns come out ascending, rows sorted, weights 1.0.
//
//   LCC: connected components by hooking (a vertex's root takes the smaller
//   root label across each edge, atomicMin) and pointer jumping until no label
//   changes.  The final label is the smallest vertex id of the component, so
//   "the largest component, ties to the one found first" of the host's DFS
//   (which starts from ascending vertex ids) is the largest size with the
//   smallest label.  Vertices are renumbered by an exclusive scan of membership
//   (ascending original id), which keeps every row's columns ascending.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "ge_internal.hpp"
#include "ge_prim.hpp"

namespace ge {
namespace {

using u64 = unsigned long long;
constexpr u64 kNoKey = ~0ull;

inline unsigned grid_for(long long L) { return (unsigned)((L + 255) / 256); }

u64 splitmix64_host(u64 x) {
  u64 z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill_kernel(long long n, double v, double* __restrict__ p) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) p[t] = v;
}

void fill_ones(double* p, long long n, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, 1.0, p);
}

__device__ __forceinline__ u64 splitmix64_dev(u64 x) {
  u64 z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void rmat_keys_kernel(long long draws, int scale, long long n, u64 base,
                                 u64* __restrict__ keys) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= draws) return;
  const double a = 0.57, b = 0.19, c = 0.19;
  const double ab = a + b, abc = a + b + c;
  long long s = 0, d = 0;
  for (int l = 0; l < scale; ++l) {
    const u64 h = splitmix64_dev(base + (u64)e * 64ull + (u64)l);
    const double u = (double)(h >> 11) * 0x1.0p-53;
    const int q = u < a ? 0 : (u < ab ? 1 : (u < abc ? 2 : 3));
    s = (s << 1) | (q >> 1);
    d = (d << 1) | (q & 1);
  }
  const bool ok = s < n && d < n && s != d;
  keys[2 * e] = ok ? (u64)s * (u64)n + (u64)d : kNoKey;
  keys[2 * e + 1] = ok ? (u64)d * (u64)n + (u64)s : kNoKey;
}

__global__ void unique_flags_kernel(long long L, const u64* __restrict__ k, int* __restrict__ f) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L) f[t] = (k[t] != kNoKey && (t == 0 || k[t] != k[t - 1])) ? 1 : 0;
}

__global__ void emit_csr_kernel(long long L, long long n, const u64* __restrict__ k,
                                const int* __restrict__ f, const int* __restrict__ pos,
                                int* __restrict__ cols, int* __restrict__ rowcnt) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L || !f[t]) return;
  const u64 key = k[t];
  cols[pos[t]] = (int)(key % (u64)n);
  atomicAdd(&rowcnt[(int)(key / (u64)n)], 1);
}

// One block per row, grid-stride over rows: a dispatch covers at most 2^32 work
// items, so a block per row of a 1e8-row matrix would silently drop rows.
constexpr int kRowBlocks = 1 << 20;

__global__ void row_of_entry_kernel(int n, const int* __restrict__ ip, int* __restrict__ row) {
  for (int i = blockIdx.x; i < n; i += gridDim.x)
    for (int e = ip[i] + threadIdx.x; e < ip[i + 1]; e += blockDim.x) row[e] = i;
}

__global__ void iota_kernel(int n, int* __restrict__ v) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) v[t] = t;
}

// hook: across every edge the larger root label points at the smaller one
__global__ void hook_kernel(long long nnz, const int* __restrict__ row, const int* __restrict__ ix,
                            int* __restrict__ lab, int* __restrict__ changed) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const int li = lab[row[e]], lj = lab[ix[e]];
  if (li == lj) return;
  const int hi = li > lj ? li : lj, lo = li > lj ? lj : li;
  if (atomicMin(&lab[hi], lo) > lo) *changed = 1;
}

__global__ void jump_kernel(int n, int* __restrict__ lab) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  int l = lab[v];
  while (lab[l] != l) l = lab[l];
  lab[v] = l;
}

__global__ void comp_size_kernel(int n, const int* __restrict__ lab, int* __restrict__ size) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) atomicAdd(&size[lab[v]], 1);
}

// the largest component, ties to the smallest label: max of (size, -label)
__global__ void best_comp_kernel(int n, const int* __restrict__ size, u64* __restrict__ best) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n && size[v] > 0)
    atomicMax(best, ((u64)(unsigned)size[v] << 32) | (unsigned)(0x7FFFFFFF - v));
}

__global__ void member_kernel(int n, const int* __restrict__ lab, const u64* __restrict__ best,
                              int* __restrict__ keep) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const int b = 0x7FFFFFFF - (int)(*best & 0xFFFFFFFFull);
  keep[v] = lab[v] == b ? 1 : 0;
}

__global__ void lcc_rows_kernel(int n, const int* __restrict__ ip, const int* __restrict__ keep,
                                const int* __restrict__ newid, int* __restrict__ len) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n && keep[v]) len[newid[v]] = ip[v + 1] - ip[v];
}

__global__ void lcc_copy_kernel(int n, const int* __restrict__ ip, const int* __restrict__ ix,
                                const double* __restrict__ dx, const int* __restrict__ keep,
                                const int* __restrict__ newid, const int* __restrict__ nip,
                                int* __restrict__ nix, double* __restrict__ ndx) {
  for (int v = blockIdx.x; v < n; v += gridDim.x) {  // grid-stride (row_of_entry_kernel)
    if (!keep[v]) continue;
    const int o = nip[newid[v]] - ip[v];
    for (int e = ip[v] + threadIdx.x; e < ip[v + 1]; e += blockDim.x) {
      nix[o + e] = newid[ix[e]];  // a component is closed: every neighbour is kept
      ndx[o + e] = dx[e];
    }
  }
}

// Library calls (rocPRIM sort / scan) on at most this many items each: the C5
// generator has 1.6e9 directed draws, which is past what one call is trusted with.
constexpr long long kChunk = 1ll << 28;

// carry[c + 1] = carry[c] + the total of chunk c (its local exclusive scan's last
// value + its last input), before the chunk is shifted
__global__ void chunk_total_kernel(const int* __restrict__ out_last, const int* __restrict__ in_last,
                                   int* __restrict__ carry, int c) {
  carry[c + 1] = carry[c] + *out_last + *in_last;
}

__global__ void add_carry_kernel(long long len, int* __restrict__ out,
                                 const int* __restrict__ carry) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < len) out[t] += *carry;
}

template <class T>
void exclusive_scan(hipStream_t st, const T* in, T* out, long long count) {
  if (count <= kChunk) {
    prim_exclusive_sum(st, in, out, (size_t)count);
    return;
  }
  // chunks of kChunk, each shifted by the running total of the ones before
  static_assert(sizeof(T) == sizeof(int), "chunked scan of int counts");
  const int nc = (int)((count + kChunk - 1) / kChunk);
  DevBuf<int> carry(nc + 1);
  GE_HIP(hipMemsetAsync(carry.p, 0, sizeof(int) * (nc + 1), st));
  for (int c = 0; c < nc; ++c) {
    const long long c0 = c * kChunk, len = std::min(kChunk, count - c0);
    prim_exclusive_sum(st, in + c0, out + c0, (size_t)len);
    hipLaunchKernelGGL(chunk_total_kernel, dim3(1), dim3(1), 0, st,
                       (const int*)(out + c0 + len - 1), (const int*)(in + c0 + len - 1), carry.p, c);
    hipLaunchKernelGGL(add_carry_kernel, dim3(grid_for(len)), dim3(256), 0, st, len,
                       (int*)(out + c0), carry.p + c);
  }
}

// Valid keys per row (duplicates included), to cut the keys into row ranges of at
// most kChunk for the sort.
__global__ void key_rows_kernel(long long L, long long n, const u64* __restrict__ k,
                                int* __restrict__ rowcnt) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L && k[t] != kNoKey) atomicAdd(&rowcnt[(int)(k[t] / (u64)n)], 1);
}

// scatter each valid key into its row range's segment (order inside a segment is
// free: the segment is sorted next)
__global__ void scatter_keys_kernel(long long L, long long n, int nb, const int* __restrict__ bound,
                                    const long long* __restrict__ boff, int* __restrict__ fill,
                                    const u64* __restrict__ k, u64* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L || k[t] == kNoKey) return;
  const int r = (int)(k[t] / (u64)n);
  int b = 0;
  while (b + 1 < nb && bound[b + 1] <= r) ++b;
  out[boff[b] + atomicAdd(&fill[b], 1)] = k[t];
}

template <class T>
T read_back(const T* d, hipStream_t st) {
  T h{};
  GE_HIP(hipMemcpyAsync(&h, d, sizeof(T), hipMemcpyDeviceToHost, st));
  GE_HIP(hipStreamSynchronize(st));
  return h;
}

// Device CSR (indptr n+1, indices, data).
struct DCsr {
  int n = 0;
  long long nnz = 0;
  DevBuf<int> ip, ix;
  DevBuf<double> dx;
};

void rmat_device(ge_ctx* ctx, int n, long long draws, u64 seed, DCsr& out) {
  hipStream_t st = ctx->stream;
  int scale = 1;
  while ((1ll << scale) < n) ++scale;
  long long L = 2 * draws;
  GE_REQUIRE(L < (1ll << 31), "device R-MAT: more than 2^31 directed entries per call");
  DevBuf<u64> k(std::max(L, 1ll)), k2(std::max(L, 1ll));
  if (draws > 0)
    hipLaunchKernelGGL(rmat_keys_kernel, dim3(grid_for(draws)), dim3(256), 0, st, draws, scale,
                       (long long)n, splitmix64_host(seed), k.p);
  GE_HIP(hipGetLastError());
  if (L <= kChunk) {
    const size_t tmp = prim_sort_keys_bytes(st, k.p, k2.p, (size_t)L, 64);
    DevBuf<unsigned char> scratch(tmp);
    // all 64 bits: the kNoKey sentinel sorts last
    prim_sort_keys(st, scratch.p, tmp, k.p, k2.p, (size_t)L, 64);
  } else {
    // Large inputs: cut the valid keys into row ranges of at most kChunk keys
    // (row = key / n, so ranges of rows are ranges of keys), scatter each into its
    // segment and sort the segments one by one -- the concatenation is sorted; the
    // invalid keys are dropped here instead of sorting last.
    DevBuf<int> rc(n);
    GE_HIP(hipMemsetAsync(rc.p, 0, sizeof(int) * n, st));
    hipLaunchKernelGGL(key_rows_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, (long long)n, k.p,
                       rc.p);
    std::vector<int> h_rc(n);
    rc.download(h_rc.data(), n, st);
    GE_HIP(hipStreamSynchronize(st));
    std::vector<int> bound{0};
    std::vector<long long> boff{0};
    long long acc = 0, tot = 0;
    for (int r = 0; r < n; ++r) {
      GE_REQUIRE(h_rc[r] <= kChunk, "device R-MAT: one row exceeds a sort chunk");
      if (acc + h_rc[r] > kChunk) {
        bound.push_back(r);
        boff.push_back(tot);
        acc = 0;
      }
      acc += h_rc[r];
      tot += h_rc[r];
    }
    const int nb = (int)bound.size();
    DevBuf<int> d_bound(nb), d_fill(nb);
    DevBuf<long long> d_boff(nb);
    d_bound.upload(bound.data(), nb, st);
    d_boff.upload(boff.data(), nb, st);
    GE_HIP(hipMemsetAsync(d_fill.p, 0, sizeof(int) * nb, st));
    hipLaunchKernelGGL(scatter_keys_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, (long long)n,
                       nb, d_bound.p, d_boff.p, d_fill.p, k.p, k2.p);
    GE_HIP(hipGetLastError());
    const size_t tmp = prim_sort_keys_bytes(st, k2.p, k.p, (size_t)kChunk, 64);
    DevBuf<unsigned char> scratch(tmp);
    for (int b = 0; b < nb; ++b) {
      const long long b0 = boff[b], b1 = b + 1 < nb ? boff[b + 1] : tot;
      if (b1 > b0)
        prim_sort_keys(st, scratch.p, tmp, k2.p + b0, k.p + b0, (size_t)(b1 - b0), 64);
    }
    std::swap(k.p, k2.p);  // the sorted keys are in k2 from here on, as in the small path
    L = tot;
  }
  DevBuf<int> f(std::max(L, 1ll)), pos(std::max(L, 1ll));
  hipLaunchKernelGGL(unique_flags_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, k2.p, f.p);
  exclusive_scan(st, f.p, pos.p, L);
  const long long nnz = L ? (long long)read_back(pos.p + (L - 1), st) + read_back(f.p + (L - 1), st) : 0;
  out.n = n;
  out.nnz = nnz;
  out.ix.alloc(std::max(nnz, 1ll));
  out.dx.alloc(std::max(nnz, 1ll));
  out.ip.alloc(n + 1);
  DevBuf<int> cnt(n + 1);
  GE_HIP(hipMemsetAsync(cnt.p, 0, sizeof(int) * (n + 1), st));
  hipLaunchKernelGGL(emit_csr_kernel, dim3(grid_for(L)), dim3(256), 0, st, L, (long long)n, k2.p,
                     f.p, pos.p, out.ix.p, cnt.p);
  exclusive_scan(st, cnt.p, out.ip.p, n + 1);
  fill_ones(out.dx.p, nnz, st);  // unit weights
  GE_HIP(hipGetLastError());
}

void lcc_device(ge_ctx* ctx, const DCsr& A, DCsr& out) {
  hipStream_t st = ctx->stream;
  const int n = A.n;
  out.n = 0;
  out.nnz = 0;
  out.ip.alloc(1);
  GE_HIP(hipMemsetAsync(out.ip.p, 0, sizeof(int), st));
  if (n == 0) return;
  DevBuf<int> lab(n), row(std::max(A.nnz, 1ll)), changed(1);
  hipLaunchKernelGGL(iota_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, lab.p);
  hipLaunchKernelGGL(row_of_entry_kernel, dim3(std::min(n, kRowBlocks)), dim3(64), 0, st, n,
                     A.ip.p, row.p);
  for (int it = 0;; ++it) {
    GE_REQUIRE(it <= n + 1, "components: no convergence");
    GE_HIP(hipMemsetAsync(changed.p, 0, sizeof(int), st));
    if (A.nnz)
      hipLaunchKernelGGL(hook_kernel, dim3(grid_for(A.nnz)), dim3(256), 0, st, A.nnz, row.p,
                         A.ix.p, lab.p, changed.p);
    hipLaunchKernelGGL(jump_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, lab.p);
    GE_HIP(hipGetLastError());
    if (!read_back(changed.p, st)) break;
  }
  DevBuf<int> size(n), keep(n), newid(n + 1), len(n + 1);
  DevBuf<u64> best(1);
  GE_HIP(hipMemsetAsync(size.p, 0, sizeof(int) * n, st));
  GE_HIP(hipMemsetAsync(best.p, 0, sizeof(u64), st));
  hipLaunchKernelGGL(comp_size_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, lab.p, size.p);
  hipLaunchKernelGGL(best_comp_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, size.p, best.p);
  hipLaunchKernelGGL(member_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, lab.p, best.p, keep.p);
  exclusive_scan(st, keep.p, newid.p, n);
  const int k = read_back(newid.p + (n - 1), st) + read_back(keep.p + (n - 1), st);
  GE_HIP(hipMemsetAsync(len.p, 0, sizeof(int) * (n + 1), st));
  hipLaunchKernelGGL(lcc_rows_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, A.ip.p, keep.p,
                     newid.p, len.p);
  out.n = k;
  out.ip.alloc(k + 1);
  exclusive_scan(st, len.p, out.ip.p, k + 1);
  out.nnz = read_back(out.ip.p + k, st);
  out.ix.alloc(std::max(out.nnz, 1ll));
  out.dx.alloc(std::max(out.nnz, 1ll));
  hipLaunchKernelGGL(lcc_copy_kernel, dim3(std::min(n, kRowBlocks)), dim3(64), 0, st, n, A.ip.p,
                     A.ix.p, A.dx.p,
                     keep.p, newid.p, out.ip.p, out.ix.p, out.dx.p);
  GE_HIP(hipGetLastError());
}

void to_host(const DCsr& d, hipStream_t st, ge_csr* h) {
  h->rows = h->cols = d.n;
  h->indptr.resize(d.n + 1);
  h->indices.resize(d.nnz);
  h->data.resize(d.nnz);
  d.ip.download(h->indptr.data(), d.n + 1, st);
  d.ix.download(h->indices.data(), d.nnz, st);
  d.dx.download(h->data.data(), d.nnz, st);
  GE_HIP(hipStreamSynchronize(st));
}

}  // namespace
}  // namespace ge

extern "C" {

int ge_rmat_csr_device(ge_ctx* ctx, int n, long long draws, unsigned long long seed, int lcc,
                       ge_csr** out) {
  return ge::guarded([&] {
    GE_REQUIRE(ctx && out && n > 1 && draws >= 0, "bad R-MAT arguments");
    ge::DeviceGuard g(ctx);
    ge::DCsr A;
    ge::rmat_device(ctx, n, draws, seed, A);
    auto* h = new ge_csr();
    try {
      if (lcc) {
        ge::DCsr B;
        ge::lcc_device(ctx, A, B);
        ge::to_host(B, ctx->stream, h);
      } else {
        ge::to_host(A, ctx->stream, h);
      }
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int ge_largest_component_device(ge_ctx* ctx, int n, const int* ip, const int* ix,
                                const double* dx, ge_csr** out) {
  return ge::guarded([&] {
    GE_REQUIRE(ctx && out && n >= 0 && (n == 0 || (ip && ix && dx)), "bad arguments");
    ge::DeviceGuard g(ctx);
    hipStream_t st = ctx->stream;
    ge::DCsr A;
    A.n = n;
    A.nnz = n ? ip[n] : 0;
    A.ip.alloc(n + 1);
    A.ix.alloc(std::max(A.nnz, 1ll));
    A.dx.alloc(std::max(A.nnz, 1ll));
    A.ip.upload(ip, n + 1, st);
    A.ix.upload(ix, A.nnz, st);
    A.dx.upload(dx, A.nnz, st);
    ge::DCsr B;
    ge::lcc_device(ctx, A, B);
    auto* h = new ge_csr();
    ge::to_host(B, st, h);
    *out = h;
  });
}

}  // extern "C"
