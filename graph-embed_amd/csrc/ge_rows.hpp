// ge_rows.hpp -- degree-classed CSR row kernels with an in-order edge sum.
//
// The reference adds a row's edge terms to its force one after the other in
// stored order (include/forceatlas.hpp:169-203, :415-467), so a row's sum is a
// serial chain; but each TERM depends only on the two endpoints.  Rows are
// therefore split by degree:
//   light  (deg <= kMedDeg)    one thread per row, terms added as computed;
//   medium (deg <= kHeavyDeg)  one wave per row: 64 terms at a time into LDS,
//                              then every lane adds them in order (same chain,
//                              broadcast reads);
//   heavy                      one block per row: three waves evaluate the next
//                              chunk while the first adds the current one.
// A term computed alone is 0 + t, equal to t up to the sign of zero; the
// accumulator starts at +0 and a round-to-nearest sum is -0 only when both
// operands are, so it is never -0 and adding the stored term later gives the
// reference's bits.
//
// One launch covers all three classes: blocks [0, nheavy) take heavy rows
// (scheduled first: longest chains), then 4 medium rows per block, then 256
// light rows per block.  `rows` lists heavy, then medium, then light rows.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <vector>

namespace ge {

constexpr int kRowT = 256;
constexpr int kMedDeg = 32;
constexpr int kHeavyDeg = 2048;

struct RowClasses {
  const int* rows = nullptr;
  int nheavy = 0, nmed = 0, nlight = 0;
  int grid() const { return nheavy + (nmed + 3) / 4 + (nlight + kRowT - 1) / kRowT; }
};

// Host: order `ids` (row ids with their degrees) into heavy, medium, light.
// GE_ROWS_MED / GE_ROWS_HEAVY override the class bounds (tuning only).
inline void classify_rows(const std::vector<int>& ids, const std::vector<int>& deg,
                          std::vector<int>& out, int& nheavy, int& nmed, int& nlight) {
  // few rows (a small level): latency, not throughput -- rows of more than 4
  // entries take a wave (n = 536: attraction 26 -> 13 us per iteration)
  int med = ids.size() <= 65536 ? 4 : kMedDeg, heavy = kHeavyDeg;
  if (const char* e = std::getenv("GE_ROWS_MED")) med = std::atoi(e);
  if (const char* e = std::getenv("GE_ROWS_HEAVY")) heavy = std::atoi(e);
  out.clear();
  for (size_t q = 0; q < ids.size(); ++q)
    if (deg[q] > heavy) out.push_back(ids[q]);
  nheavy = (int)out.size();
  for (size_t q = 0; q < ids.size(); ++q)
    if (deg[q] > med && deg[q] <= heavy) out.push_back(ids[q]);
  nmed = (int)out.size() - nheavy;
  for (size_t q = 0; q < ids.size(); ++q)
    if (deg[q] <= med && deg[q] <= heavy) out.push_back(ids[q]);
  nlight = (int)out.size() - nheavy - nmed;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int G>
__device__ __forceinline__ void group_sync() {
  if (G == 64)
    wave_lds_sync();
  else
    __syncthreads();
}

// acc += term(e0) + term(e0+1) + ... in order; G threads (g = 0..G-1) share buf
// (G*U*D doubles, 16-byte aligned).  The terms are evaluated by all G threads;
// the ordered adds are done by the group's first wave only (for G = 64: the
// whole group), whose lanes all end with the same acc -- the other waves'
// acc is not updated.  Two terms (2D doubles) are read with D 16-byte loads.
template <int D, int G, int U, class Term>
__device__ __forceinline__ void ordered_edge_sum(int e0, int e1, int g, double* buf, Term&& term,
                                                 double (&acc)[D]) {
  const bool summer = G == 64 || g < 64;
  for (int b = e0; b < e1; b += G * U) {
    group_sync<G>();  // the previous chunk has been read
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = b + g + G * u;
      if (e < e1) {
        double t[D];
#pragma unroll
        for (int k = 0; k < D; ++k) t[k] = 0.0;
        term(e, t);
#pragma unroll
        for (int k = 0; k < D; ++k) buf[(g + G * u) * D + k] = t[k];
      }
    }
    group_sync<G>();
    if (summer) {
      const int cnt = min(G * U, e1 - b);
      int l = 0;
#pragma unroll 2
      for (; l + 1 < cnt; l += 2) {
        const double2* p = reinterpret_cast<const double2*>(buf + l * D);  // l even: aligned
        double v[2 * D];
#pragma unroll
        for (int q = 0; q < D; ++q) {
          const double2 w = p[q];
          v[2 * q] = w.x;
          v[2 * q + 1] = w.y;
        }
#pragma unroll
        for (int k = 0; k < D; ++k) acc[k] = acc[k] + v[k];
#pragma unroll
        for (int k = 0; k < D; ++k) acc[k] = acc[k] + v[D + k];
      }
      if (l < cnt)
#pragma unroll
        for (int k = 0; k < D; ++k) acc[k] = acc[k] + buf[l * D + k];
    }
  }
}

// Heavy rows (one 256-thread block per row): waves 1-3 evaluate the next chunk
// of kSplitChunk terms while wave 0 adds the current chunk in order, so the
// serial add chain -- the floor for a hub row -- overlaps the gathers.  buf
// holds two chunks.  Only wave 0's acc is the row's sum.
constexpr int kSplitU = 4;
constexpr int kSplitChunk = 192 * kSplitU;  // 3 computing waves x 64 lanes x U

template <int D, class Term>
__device__ __forceinline__ void ordered_edge_sum_split(int e0, int e1, int tid, double* buf,
                                                       Term&& term, double (&acc)[D]) {
  const bool summer = tid < 64;
  const int w = tid - 64;  // computing lane 0..191
  // branch-free over the U terms of a lane (indices clamped into the row, the
  // surplus terms dropped by the summer's count), so the compiler can issue
  // all U gathers before the arithmetic
  auto compute = [&](int b, double* dst) {
    double t[kSplitU][D];
#pragma unroll
    for (int u = 0; u < kSplitU; ++u) {
      const int e = min(b + w + 192 * u, e1 - 1);
#pragma unroll
      for (int k = 0; k < D; ++k) t[u][k] = 0.0;
      term(e, t[u]);
    }
#pragma unroll
    for (int u = 0; u < kSplitU; ++u)
#pragma unroll
      for (int k = 0; k < D; ++k) dst[(w + 192 * u) * D + k] = t[u][k];
  };
  if (!summer && e0 < e1) compute(e0, buf);
  __syncthreads();
  int c = 0;
  for (int b = e0; b < e1; b += kSplitChunk, ++c) {
    double* cur = buf + (c & 1) * kSplitChunk * D;
    if (summer) {
      // blocks of 8 terms: all 4D 16-byte loads of a block are issued before its
      // adds, and unrolling lets the next block's loads overlap this block's
      // add chain (the LDS latency would otherwise sit on the critical path)
      const int cnt = min(kSplitChunk, e1 - b);
      int l = 0;
#pragma unroll 2
      for (; l + 8 <= cnt; l += 8) {
        const double2* p = reinterpret_cast<const double2*>(cur + l * D);  // l % 8 == 0
        double v[8 * D];
#pragma unroll
        for (int q = 0; q < 4 * D; ++q) {
          const double2 x = p[q];
          v[2 * q] = x.x;
          v[2 * q + 1] = x.y;
        }
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
          for (int k = 0; k < D; ++k) acc[k] = acc[k] + v[t * D + k];
      }
      for (; l < cnt; ++l)
#pragma unroll
        for (int k = 0; k < D; ++k) acc[k] = acc[k] + cur[l * D + k];
    } else if (b + kSplitChunk < e1) {
      compute(b + kSplitChunk, buf + ((c + 1) & 1) * kSplitChunk * D);
    }
    __syncthreads();
  }
}

// P: a row policy with
//   struct State (holds acc[D] and the edge range e0, e1)
//   load(row, State&), term(const State&, e, t[D]), finish(State&, bool writer).
template <int D, class P>
__global__ void __launch_bounds__(kRowT) classed_rows_kernel(RowClasses L, P p) {
  __shared__ __attribute__((aligned(16))) double buf[2 * kSplitChunk * D];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  typename P::State st;
  if (b < L.nheavy) {
    p.load(L.rows[b], st);
    ordered_edge_sum_split<D>(st.e0, st.e1, tid, buf,
                              [&](int e, double (&t)[D]) { p.term(st, e, t); }, st.acc);
    p.finish(st, tid == 0);
    return;
  }
  const int mblocks = (L.nmed + 3) / 4;
  if (b < L.nheavy + mblocks) {
    const int q = (b - L.nheavy) * 4 + (tid >> 6);
    if (q >= L.nmed) return;  // wave-uniform; no block barrier on this path
    const int lane = tid & 63;
    p.load(L.rows[L.nheavy + q], st);
    ordered_edge_sum<D, 64, 1>(
        st.e0, st.e1, lane, buf + (tid >> 6) * 64 * D,
        [&](int e, double (&t)[D]) { p.term(st, e, t); }, st.acc);
    p.finish(st, lane == 0);
    return;
  }
  const int q = (b - L.nheavy - mblocks) * kRowT + tid;
  if (q >= L.nlight) return;
  p.load(L.rows[L.nheavy + L.nmed + q], st);
  for (int e = st.e0; e < st.e1; ++e) {
    double t[D];
#pragma unroll
    for (int k = 0; k < D; ++k) t[k] = 0.0;
    p.term(st, e, t);
#pragma unroll
    for (int k = 0; k < D; ++k) st.acc[k] = st.acc[k] + t[k];
  }
  p.finish(st, true);
}

}  // namespace ge
