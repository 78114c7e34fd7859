// ge_fa.hip -- single-level ForceAtlas on gfx950.
//
// Reference: partition::forceAtlas, include/forceatlas.hpp:89-305.
//
// One iteration = two kernels on the context stream:
//   fa_repulse_*        O(n^2) all-pairs repulsion for rows [rb,re)       (:151-167)
//                       -> Frep (per-row partial force, fp64)
//   fa_attract_update_* CSR attraction continuing each row's sum (:169-203),
//                       gravity (:205-211), swing (:214-217), speed clamp and
//                       position update (:246-261) -> X_next rows, Fprev rows
// The global swing/traction sums of :219-244 are dead (overwritten with 1.0 at
// :228, :242) and are not computed.
//
// STRICT mode (default) keeps the reference's serial op order per row: the
// j loop is ascending over all vertices, the CSR walk is in stored order, every
// multiply/add/div/sqrt rounds separately (-ffp-contract=off, IEEE div/sqrt).
// Each thread owns R rows and streams the coordinates of all j through LDS
// tiles, so a row's sum is exactly the reference's sum.  Two exact rewrites:
//   * -(x_j - x_i) is computed as (x_i - x_j).  They differ only in the sign of
//     a zero, and a zero contribution never changes a running force sum: the
//     sum starts at +0.0 and IEEE round-to-nearest never produces -0.0 from a
//     sum unless both addends are -0.0.  For the same reason the j == i term
//     (direction 0/eps = 0) is accumulated instead of branched around.
//   * 0.0 + t*t (the first term of distance(), :72-75) is t*t.
//
// FAST mode re-associates: 2-D tiles over (row block, j block) partial sums,
// FMA, one reciprocal square root per pair.  Checked against strict within
// 1e-5 relative after the iteration counts the reference runs (tests).
//
// Small graphs (n <= 1024, e.g. the coarsest level, 1e5 iterations) run all
// iterations inside one workgroup with coordinates resident in LDS.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <cstdlib>
#include <cmath>
#include <memory>
#include <vector>

#include "ge_internal.hpp"
#include "ge_pair.hpp"
#include "ge_rows.hpp"

namespace ge {
namespace {

constexpr double kEps = kFaEps;
FaConst make_const(const ge_fa_params& p) { return make_fa_const(p); }

// deg[i] + 1 with deg the serial row sum of include/forceatlas.hpp:127-140.
__global__ void degp1_kernel(int n, const int* __restrict__ ip, const double* __restrict__ dx,
                             int use_weights, double* __restrict__ dp1) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double d;
  if (use_weights) {
    // same serial adds; the loads of 16 entries are issued before their adds,
    // so a hub row waits on one memory latency per 16 entries, not per entry
    d = 0.0;
    const int e1 = ip[i + 1];
    int e = ip[i];
    for (; e + 16 <= e1; e += 16) {
      double w[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) w[u] = dx[e + u];
#pragma unroll
      for (int u = 0; u < 16; ++u) d += w[u];
    }
    for (; e < e1; ++e) d += dx[e];
  } else {
    d = 1.0 * (ip[i + 1] - ip[i]);
  }
  dp1[i] = d + 1;
}

// ---------------------------------------------------------------------------
// STRICT repulsion.  A persistent grid of one 512-thread block per CU; block b
// owns the contiguous rows [rb + b*per, rb + (b+1)*per) and walks them in
// chunks of 512*R rows (thread t, slot r -> row c0 + t + 512 r).  Each wave
// skips the slots it has no rows in (wave-uniform), so the work per SIMD is
// balanced to one 64-row slot.  The j range is streamed through an LDS tile of
// 256 records {x_0..x_{D-1}, deg+1}; every row's sum runs over j ascending.
// Independent work per lane for latency hiding comes from R rows and U
// consecutive partners: the U*R pair terms are evaluated together and then
// added to each row's sum in j order (R*U = 8; few rows per CU, as on a row
// shard of N GPUs, take small R and large U).

constexpr int kRepThreads = 512;
constexpr int kTileJ = 256;
constexpr int kRepRU = 8;  // row slots x partners in flight per lane

template <int D>
struct Rec {
  static constexpr int W = (D + 1 <= 4) ? 4 : 8;  // doubles per LDS record
};

// One LDS tile of partners for the first NR row slots of a wave (NR is the
// wave's slot count, dispatched at run time): no per-slot branches, so each
// partner record is read once for all NR rows and the NR x U independent pair
// chains interleave.  With U > 1 the U terms of a row are added in j order
// after they are all evaluated.
template <int D, bool REPEL_ONE, int R, int U, int NR>
__device__ __forceinline__ void rep_tile(const double* tile, int cnt, const double (&xi)[R][D],
                                         const double (&di)[R], double repel,
                                         double (&acc)[R][D]) {
  constexpr int W = Rec<D>::W;
  int jj = 0;
  if constexpr (U > 1) {
    for (; jj + U <= cnt; jj += U) {
      double t[U][NR][D];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double* xj = &tile[(jj + u) * W];
        const double dj = tile[(jj + u) * W + D];
#pragma unroll
        for (int r = 0; r < NR; ++r) rep_term<D, true, REPEL_ONE>(xi[r], xj, di[r], dj, repel, t[u][r]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
          for (int k = 0; k < D; ++k) acc[r][k] = acc[r][k] + t[u][r][k];
    }
  }
  for (; jj < cnt; ++jj) {
    const double* xj = &tile[jj * W];
    const double dj = tile[jj * W + D];
#pragma unroll
    for (int r = 0; r < NR; ++r) rep_pair<D, true, REPEL_ONE>(xi[r], xj, di[r], dj, repel, acc[r]);
  }
}

template <int D, bool REPEL_ONE, int R, int U, int NR>
__device__ __forceinline__ void rep_tile_dispatch(int nr, const double* tile, int cnt,
                                                  const double (&xi)[R][D], const double (&di)[R],
                                                  double repel, double (&acc)[R][D]) {
  if constexpr (NR >= 1) {
    if (nr == NR) rep_tile<D, REPEL_ONE, R, U, NR>(tile, cnt, xi, di, repel, acc);
    else rep_tile_dispatch<D, REPEL_ONE, R, U, NR - 1>(nr, tile, cnt, xi, di, repel, acc);
  }
}

template <int D, bool REPEL_ONE, int R>
__global__ void __launch_bounds__(kRepThreads)
fa_repulse_strict(int n, int rb, int re, int per_block, const double* __restrict__ X,
                  const double* __restrict__ dp1, double repel, double* __restrict__ Frep) {
  constexpr int W = Rec<D>::W;
  constexpr int U = kRepRU / R;
  __shared__ __attribute__((aligned(16))) double tile[kTileJ * W];
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int bbeg = rb + blockIdx.x * per_block;
  const int bend = min(re, bbeg + per_block);
  const bool repel_ok = REPEL_ONE || weight_ok(repel);

  for (int c0 = bbeg; c0 < bend; c0 += kRepThreads * R) {
    // slots with at least one row in this wave: r < nr (wave-uniform)
    const int first = c0 + wave * 64;
    const int nr = first >= bend ? 0 : min(R, (bend - first + kRepThreads - 1) / kRepThreads);
    double xi[R][D], di[R], acc[R][D];
    bool rows_ok = repel_ok;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = c0 + tid + r * kRepThreads;
      const bool ok = i < bend;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        xi[r][k] = ok ? X[(size_t)i * D + k] : 0.0;
        acc[r][k] = 0.0;
      }
      di[r] = ok ? dp1[i] : 1.0;
      rows_ok = rows_ok && vertex_ok<D>(xi[r], di[r]);
    }
    for (int j0 = 0; j0 < n; j0 += kTileJ) {
      const int cnt = min(kTileJ, n - j0);
      __syncthreads();
      bool ok = rows_ok;
      if (tid < cnt) {
        const int j = j0 + tid;
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const double v = X[(size_t)j * D + k];
          tile[tid * W + k] = v;
          ok = ok && coord_ok(v);
        }
        const double w = dp1[j];
        tile[tid * W + D] = w;
        ok = ok && weight_ok(w);
      }
      // block-uniform: every coordinate of this tile and of the block's rows is
      // in the exact shared-reciprocal domain (ge_math.hpp)
      if (__syncthreads_and(ok)) {
        rep_tile_dispatch<D, REPEL_ONE, R, U, R>(nr, tile, cnt, xi, di, repel, acc);
      } else {
        for (int jj = 0; jj < cnt; ++jj) {
          const double* xj = &tile[jj * W];
          const double dj = tile[jj * W + D];
#pragma unroll
          for (int r = 0; r < R; ++r)
            if (r < nr)
              rep_pair_fb<D, REPEL_ONE>(xi[r], xj, di[r], dj, repel,
                                        j0 + jj == c0 + tid + r * kRepThreads, acc[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = c0 + tid + r * kRepThreads;
      if (i < bend) {
#pragma unroll
        for (int k = 0; k < D; ++k) Frep[(size_t)(i - rb) * D + k] = acc[r][k];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// FAST repulsion: (row block) x (j block) tiles; each block writes a partial
// sum for its rows into Fpart[jb][row]; fa_reduce_parts sums the partials.
// Pair term in closed form: F_i += c_ij * (x_i - x_j) / dis^3, dis from one
// rsqrt + one Newton step, FMA everywhere.

constexpr int kFastJBlocks = 16;  // j-range split

constexpr int kFastThreads = 256;

template <int D, int R>
__global__ void __launch_bounds__(kFastThreads)
fa_repulse_fast(int n, int rb, int re, const double* __restrict__ X,
                const double* __restrict__ dp1, double repel, int jblocks,
                double* __restrict__ Fpart) {
  constexpr int W = Rec<D>::W;
  __shared__ __attribute__((aligned(16))) double tile[kTileJ * W];
  const int tid = threadIdx.x;
  const int rows_here = re - rb;
  const int base = rb + blockIdx.x * (kFastThreads * R);
  const int jb = blockIdx.y;
  const int jchunk = (n + jblocks - 1) / jblocks;
  const int jbeg = jb * jchunk;
  const int jend = min(n, jbeg + jchunk);
  const double inv_eps = 1.0 / kEps;

  double xi[R][D], di[R], acc[R][D];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = base + tid + r * kFastThreads;
    const bool ok = i < re;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      xi[r][k] = ok ? X[(size_t)i * D + k] : 0.0;
      acc[r][k] = 0.0;
    }
    di[r] = (ok ? dp1[i] : 1.0) * repel;
  }
  for (int j0 = jbeg; j0 < jend; j0 += kTileJ) {
    const int cnt = min(kTileJ, jend - j0);
    __syncthreads();
    if (tid < cnt) {
      const int j = j0 + tid;
#pragma unroll
      for (int k = 0; k < D; ++k) tile[tid * W + k] = X[(size_t)j * D + k];
      tile[tid * W + D] = dp1[j];
    }
    __syncthreads();
    for (int jj = 0; jj < cnt; ++jj) {
      double xj[D];
#pragma unroll
      for (int k = 0; k < D; ++k) xj[k] = tile[jj * W + k];
      const double dj = tile[jj * W + D];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        double e[D];
#pragma unroll
        for (int k = 0; k < D; ++k) e[k] = xi[r][k] - xj[k];
        double s = e[0] * e[0];
#pragma unroll
        for (int k = 1; k < D; ++k) s = fma(e[k], e[k], s);
        // y = 1/max(sqrt(s), eps): hardware estimate + two Newton steps.
        // s == 0 gives inf -> NaN after Newton -> fmin picks 1/eps.
        double y = __builtin_amdgcn_rsq(s);
        const double hs = 0.5 * s;
        y = y * fma(-hs * y, y, 1.5);
        y = y * fma(-hs * y, y, 1.5);
        y = fmin(y, inv_eps);
        const double w = di[r] * dj * (y * y * y);
#pragma unroll
        for (int k = 0; k < D; ++k) acc[r][k] = fma(e[k], w, acc[r][k]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = base + tid + r * kFastThreads;
    if (i < re) {
#pragma unroll
      for (int k = 0; k < D; ++k)
        Fpart[((size_t)jb * rows_here + (i - rb)) * D + k] = acc[r][k];
    }
  }
}

template <int D>
__global__ void fa_reduce_parts(int rows, int jblocks, const double* __restrict__ Fpart,
                                double* __restrict__ Frep) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * D) return;
  double s = 0.0;
  for (int b = 0; b < jblocks; ++b) s += Fpart[(size_t)b * rows * D + t];
  Frep[t] = s;
}

// ---------------------------------------------------------------------------
// Attraction + gravity + swing + update per row (serial CSR order).

// Coherent (agent-scope) accesses of the persistent coarsest-level kernel: its
// coordinates cross XCDs between iterations, and the per-XCD L2s are not kept
// coherent for plain loads and stores.
__device__ __forceinline__ double coh_ld(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void coh_st(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int D, bool COH = false>
__device__ __forceinline__ void finish_row(int i, int li, const double (&xi)[D], double (&acc)[D],
                                           const double (&fprev)[D], double dip1, const FaConst& c,
                                           double* __restrict__ Fprev,
                                           double* __restrict__ Xnext, bool write = true) {
  double m2 = xi[0] * xi[0];
#pragma unroll
  for (int k = 1; k < D; ++k) m2 = m2 + xi[k] * xi[k];
  const double mag = sqrt(m2);  // not clamped (:205)
  double unit[D], F[D];
  neg_over<D>(xi, mag, unit);
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const double g = unit[k] * c.gravity * dip1;
    F[k] = acc[k] + g;
  }
  double s = 0.0, f2 = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const double t = fprev[k] - F[k];
    s = (k == 0) ? t * t : s + t * t;
    f2 = (k == 0) ? F[k] * F[k] : f2 + F[k] * F[k];
  }
  const double swing = sqrt(s);  // not clamped in single-level (:216)
  const double totalF = sqrt(f2);
  double speed = c.ks_gS / (1 + c.gS * sqrt(swing));
  const double cap = c.ksmax / totalF;
  if (speed > cap) speed = cap;
  if (!write) return;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    if (COH) coh_st(&Xnext[(size_t)i * D + k], F[k] * speed + xi[k]);
    else Xnext[(size_t)i * D + k] = F[k] * speed + xi[k];
    Fprev[(size_t)li * D + k] = F[k];
  }
}

// Row policy for classed_rows_kernel (ge_rows.hpp): attraction (:169-203) added
// to the repulsion sum in CSR order, then gravity, swing and update.
template <int D>
struct FaRows {
  int rb;
  const int *ip, *ix;
  const double *dx, *X, *dp1, *Frep;
  double *Fprev, *Xnext;
  FaConst c;
  struct State {
    int i, e0, e1;
    double xi[D], acc[D], fprev[D], dip1;
    bool row_ok;
  };
  __device__ __forceinline__ void load(int i, State& s) const {
    s.i = i;
    s.e0 = ip[i];
    s.e1 = ip[i + 1];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      s.xi[k] = X[(size_t)i * D + k];
      s.acc[k] = Frep[(size_t)(i - rb) * D + k];
      s.fprev[k] = Fprev[(size_t)(i - rb) * D + k];  // loaded early: off the row's critical path
    }
    s.dip1 = dp1[i];
    s.row_ok = all_coord_ok<D>(s.xi);
  }
  __device__ __forceinline__ void term(const State& s, int e, double (&t)[D]) const {
    // the neighbour's coordinates into registers first: all of a tile thread's
    // gathers issue before any domain test (C5: 37.9 -> 31.2 ms per pass)
    double xv[D];
    const double* src = X;
    const size_t j = (size_t)ix[e] * D;
#pragma unroll
    for (int k = 0; k < D; ++k) xv[k] = src[j + k];
    const double* xj = xv;
    const double a = c.use_weights ? dx[e] : 1.0;
    if (s.row_ok && all_coord_ok<D>(xj))
      attr_edge<D, true>(s.xi, xj, a, s.dip1, c, t);
    else
      attr_edge<D, false>(s.xi, xj, a, s.dip1, c, t);
  }
  __device__ __forceinline__ void finish(State& s, bool writer) const {
    finish_row<D>(s.i, s.i - rb, s.xi, s.acc, s.fprev, s.dip1, c, Fprev, Xnext, writer);
  }
};

// ---------------------------------------------------------------------------
// Small graphs (the coarsest level's 1e5 iterations, src/embed.cpp:586): one
// 1024-thread workgroup runs every iteration, coordinates in LDS.  Row i is
// owned by a group of G lanes: the G lanes evaluate the terms of G consecutive
// partners (or CSR entries) at once, and the group's first lane adds them in
// order -- the reference's serial sum, with G times the parallelism of one
// lane per row (n = 127 gives 16 waves instead of 2).

constexpr int kSmallMax = 512;  // one row group per thread group below
constexpr int kSmallDefault = 64;
constexpr int kSmallNnz = 6144;
// CSR entries staged in LDS (the 4-D double-buffered term tile leaves less room)
constexpr int small_nnz_cap(int D) { return D == 4 ? 4096 : kSmallNnz; }

// The G lanes of a group hold U terms each (term u of lane g is partner
// g + G*u of the chunk); the group's first lane adds the first cnt in order.
template <int D, int G, int U>
__device__ __forceinline__ void group_add(const double (&t)[U][D], int tid, int g, int cnt,
                                          bool leader, double* __restrict__ tb,
                                          double (&acc)[D]) {
  if (G == 1) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < cnt)
#pragma unroll
        for (int k = 0; k < D; ++k) acc[k] = acc[k] + t[u][k];
    return;
  }
  const int base = tid - g;  // the group's first lane
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int k = 0; k < D; ++k) tb[(base * U + g + G * u) * D + k] = t[u][k];
  wave_lds_sync();
  if (leader) {
    constexpr int B = (G * U < 8) ? G * U : 8;  // terms read ahead of the ordered adds
#pragma unroll
    for (int l0 = 0; l0 < G * U; l0 += B) {
      double v[B][D];
#pragma unroll
      for (int l = 0; l < B; ++l)
#pragma unroll
        for (int k = 0; k < D; ++k) v[l][k] = tb[(base * U + l0 + l) * D + k];
#pragma unroll
      for (int l = 0; l < B; ++l)
        if (l0 + l < cnt)
#pragma unroll
          for (int k = 0; k < D; ++k) acc[k] = acc[k] + v[l][k];
    }
  }
  wave_lds_sync();
}

// a += p[0] + ... + p[cnt-1] in order for a chunk of G slots (p 16-byte
// aligned; slots >= cnt are added as +0.0, which leaves a unchanged: a running
// sum is never -0).  Branch-free, so the reads of a batch issue together.
template <int G>
__device__ __forceinline__ double group_chain(double a, const double* p, int cnt) {
  constexpr int B = G < 16 ? G : 16;  // terms per batch of reads
#pragma unroll
  for (int b0 = 0; b0 < G; b0 += B) {
    double v[B];
#pragma unroll
    for (int l = 0; l < B; l += 2) {
      const double2 x = *reinterpret_cast<const double2*>(p + b0 + l);
      v[l] = x.x;
      v[l + 1] = x.y;
    }
    if (cnt >= G) {  // full chunk (group-uniform): no masking
#pragma unroll
      for (int l = 0; l < B; ++l) a = a + v[l];
    } else {
#pragma unroll
      for (int l = 0; l < B; ++l) a = a + ((b0 + l < cnt) ? v[l] : 0.0);
    }
  }
  return a;
}

// Software-pipelined ordered group sum for the domain-only kernels: the terms
// of chunk c+1 are evaluated while the sums of chunk c are formed.  Lane k (< D)
// of a group carries dimension k's running sum (one dependent add per term);
// the group's terms sit dimension-major in its region of the chunk buffer
// (groups smaller than D: every lane adds every dimension).  All lanes of a
// group end with the full acc.  term(q, t) writes the term of
// chunk-local item q.  tb holds two chunk buffers of T*D doubles (16-byte
// aligned); G >= 2.
template <int D, int G, int T, class Term>
__device__ __forceinline__ void pipelined_group_sum(int nitems, int tid, int g, double* tb,
                                                    Term&& term, double (&acc)[D]) {
  static_assert(G <= 64, "a group lives in one wave");
  if (nitems <= 0) return;
  if constexpr (G == 1) {  // (callers take other paths for G == 1)
    for (int q = 0; q < nitems; ++q) {
      double t[D];
      term(q, t);
#pragma unroll
      for (int k = 0; k < D; ++k) acc[k] = acc[k] + t[k];
    }
    return;
  }
  const int base = tid - g;
  // G >= D: lane k carries dimension k; smaller groups: every lane all of them
  constexpr bool kLaneDim = G >= D;
  const int kd = g < D ? g : D - 1;
  double a = lane_dim_value<D>(acc, kd);
  double t[D];
  term(g, t);  // chunk 0
#pragma unroll
  for (int k = 0; k < D; ++k) tb[base * D + k * G + g] = t[k];
  for (int c0 = 0; c0 < nitems; c0 += G) {
    const int cur = (c0 / G) & 1;
    wave_lds_sync();
    const bool more = c0 + G < nitems;
    // next chunk, independent of the adds below; evaluated unconditionally (the
    // terms clamp their item) so the compiler can interleave it with the chain
    term(c0 + G + g, t);
    const double* reg = tb + cur * T * D + base * D;
    const int cnt = min(G, nitems - c0);
    if constexpr (kLaneDim) {
      a = group_chain<G>(a, reg + kd * G, cnt);
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k) acc[k] = group_chain<G>(acc[k], reg + k * G, cnt);
    }
    wave_lds_sync();
    if (more)
#pragma unroll
      for (int k = 0; k < D; ++k) tb[(cur ^ 1) * T * D + base * D + k * G + g] = t[k];
  }
  if constexpr (kLaneDim)
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = __shfl(a, (base & 63) + k);
}

// STAGED: the CSR indices and weights (nnz <= kSmallNnz) are copied to LDS once.
// DOMAIN_ONLY: the branch-free in-domain bodies only.  Such a kernel stops at
// the first iteration whose rows leave the exact-division domain (or at
// stop_at, a test hook) and records it in *it_state; the general kernel (both bodies) resumes from *it_state.
// State crossing between the two: coordinates in Xg, previous forces in Fp.
// Splitting keeps the fast kernel within 128 VGPRs, so it runs 1024 threads;
// it has the linear attraction only and is skipped for linlog / delta != 1.
template <int D, int G, int T, bool STAGED, bool DOMAIN_ONLY>
__global__ void __launch_bounds__(T)
fa_small_strict(int n, const int* __restrict__ ip, const int* __restrict__ ixg,
                const double* __restrict__ dxg, const double* __restrict__ dp1g,
                double* __restrict__ Xg, double* __restrict__ Fp, int* __restrict__ it_state,
                int iterations, int stop_at, FaConst c) {
  constexpr int W = Rec<D>::W;
  constexpr int U = 1;
  __shared__ __attribute__((aligned(16))) double sx[kSmallMax * W];
  __shared__ __attribute__((aligned(16))) double tb[(G > 1 ? T * U * (DOMAIN_ONLY ? 2 : 1) : 1) * D];
  __shared__ int s_ix[STAGED ? small_nnz_cap(D) : 1];
  __shared__ double s_dx[STAGED ? small_nnz_cap(D) : 1];
  const int it0 = DOMAIN_ONLY ? 0 : *it_state;
  if (it0 >= iterations) return;
  if (STAGED) {
    for (int e = threadIdx.x; e < ip[n]; e += T) {
      s_ix[e] = ixg[e];
      s_dx[e] = dxg[e];
    }
  }
  const int* __restrict__ ix = STAGED ? s_ix : ixg;
  const double* __restrict__ dx = STAGED ? s_dx : dxg;
  const int tid = threadIdx.x;
  const int g = tid % G;
  const int i = tid / G;
  const bool active = i < n;
  const bool leader = active && g == 0;
  for (int q = tid; q < n; q += T) {
#pragma unroll
    for (int k = 0; k < D; ++k) sx[q * W + k] = Xg[(size_t)q * D + k];
    sx[q * W + D] = dp1g[q];
  }
  const int e0 = active ? ip[i] : 0;
  const int e1 = active ? ip[i + 1] : 0;
  double fprev[D], F[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    fprev[k] = leader ? Fp[(size_t)i * D + k] : 0.0;
    F[k] = 0.0;
  }
  int it = it0;
  for (; it < iterations; ++it) {
    __syncthreads();
    double xi[D], acc[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      xi[k] = active ? sx[i * W + k] : 0.0;
      acc[k] = 0.0;
    }
    const double dip1 = active ? sx[i * W + D] : 1.0;
    const bool row_ok = all_coord_ok<D>(xi);
    const bool rep_ok = row_ok && weight_ok(dip1) && weight_ok(c.repel);
    // every row in the shared-reciprocal domain: branch-free pair and edge
    // bodies the compiler can interleave
    const bool dom = __syncthreads_and(!active || rep_ok);
    if (DOMAIN_ONLY && (!dom || it == stop_at)) break;  // block-uniform: hand over
    if (DOMAIN_ONLY && G > 1) {
      // :151-167, j ascending; then :169-203, CSR order
      pipelined_group_sum<D, G, T>(n, tid, g, tb, [&](int q, double (&t)[D]) {
        const int jj = min(q, n - 1);
        rep_term<D, true, false>(xi, &sx[jj * W], dip1, sx[jj * W + D], c.repel, t);
        if (q >= n)
#pragma unroll
          for (int k = 0; k < D; ++k) t[k] = 0.0;
      }, acc);
      pipelined_group_sum<D, G, T>(e1 - e0, tid, g, tb, [&](int q, double (&t)[D]) {
        const int ee = min(e0 + q, e1 - 1);
#pragma unroll
        for (int k = 0; k < D; ++k) t[k] = 0.0;
        if (e1 > e0)
          attr_edge<D, true, true>(xi, &sx[ix[ee] * W], c.use_weights ? dx[ee] : 1.0, dip1, c,
                                   t);
        if (e0 + q >= e1)
#pragma unroll
          for (int k = 0; k < D; ++k) t[k] = 0.0;
      }, acc);
    } else if (DOMAIN_ONLY || dom) {
      for (int j0 = 0; j0 < n; j0 += G * U) {  // :151-167, j ascending
        double t[U][D];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = j0 + g + G * u;
          const int jj = min(j, n - 1);
          rep_term<D, true, false>(xi, &sx[jj * W], dip1, sx[jj * W + D], c.repel, t[u]);
          if (j >= n)
#pragma unroll
            for (int k = 0; k < D; ++k) t[u][k] = 0.0;
        }
        group_add<D, G, U>(t, tid, g, min(G * U, n - j0), leader, tb, acc);
      }
      for (int b = e0; b < e1; b += G * U) {  // :169-203, CSR order
        double t[U][D];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = b + g + G * u;
          const int ee = min(e, e1 - 1);
#pragma unroll
          for (int k = 0; k < D; ++k) t[u][k] = 0.0;
          attr_edge<D, true, DOMAIN_ONLY>(xi, &sx[ix[ee] * W], c.use_weights ? dx[ee] : 1.0,
                                          dip1, c, t[u]);
          if (e >= e1)
#pragma unroll
            for (int k = 0; k < D; ++k) t[u][k] = 0.0;
        }
        group_add<D, G, U>(t, tid, g, min(G * U, e1 - b), leader, tb, acc);
      }
    } else if (!DOMAIN_ONLY) {
      for (int j0 = 0; j0 < n; j0 += G * U) {  // :151-167, j ascending
        double t[U][D];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = j0 + g + G * u;
#pragma unroll
          for (int k = 0; k < D; ++k) t[u][k] = 0.0;
          if (active && j < n) {
            const double* xj = &sx[j * W];
            if (rep_ok && vertex_ok<D>(xj, sx[j * W + D]))
              rep_pair<D, true, false>(xi, xj, dip1, sx[j * W + D], c.repel, t[u]);
            else
              rep_pair_fb<D, false>(xi, xj, dip1, sx[j * W + D], c.repel, j == i, t[u]);
          }
        }
        group_add<D, G, U>(t, tid, g, min(G * U, n - j0), leader, tb, acc);
      }
      for (int b = e0; b < e1; b += G * U) {  // :169-203, CSR order
        double t[U][D];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = b + g + G * u;
#pragma unroll
          for (int k = 0; k < D; ++k) t[u][k] = 0.0;
          if (e < e1) {
            const double* xj = &sx[ix[e] * W];
            const double a = c.use_weights ? dx[e] : 1.0;
            if (row_ok && all_coord_ok<D>(xj))
              attr_edge<D, true>(xi, xj, a, dip1, c, t[u]);
            else
              attr_edge<D, false>(xi, xj, a, dip1, c, t[u]);
          }
        }
        group_add<D, G, U>(t, tid, g, min(G * U, e1 - b), leader, tb, acc);
      }
    }
    if (leader) {  // gravity :205-211 (mag not clamped)
      double m2 = xi[0] * xi[0];
#pragma unroll
      for (int k = 1; k < D; ++k) m2 = m2 + xi[k] * xi[k];
      const double mag = sqrt(m2);
      double unit[D];
      neg_over<D>(xi, mag, unit);
#pragma unroll
      for (int k = 0; k < D; ++k) F[k] = acc[k] + unit[k] * c.gravity * dip1;
    }
    __syncthreads();
    if (leader) {  // swing + update :214-269
      double s2 = 0.0, f2 = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const double t = fprev[k] - F[k];
        s2 = (k == 0) ? t * t : s2 + t * t;
        f2 = (k == 0) ? F[k] * F[k] : f2 + F[k] * F[k];
      }
      const double swing = sqrt(s2);
      const double totalF = sqrt(f2);
      double speed = c.ks_gS / (1 + c.gS * sqrt(swing));
      const double cap = c.ksmax / totalF;
      if (speed > cap) speed = cap;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        sx[i * W + k] = F[k] * speed + sx[i * W + k];
        fprev[k] = F[k];
      }
    }
  }
  __syncthreads();
  for (int q = tid; q < n; q += T)
#pragma unroll
    for (int k = 0; k < D; ++k) Xg[(size_t)q * D + k] = sx[q * W + k];
  if (leader)
#pragma unroll
    for (int k = 0; k < D; ++k) Fp[(size_t)i * D + k] = fprev[k];
  if (DOMAIN_ONLY && tid == 0) *it_state = it;
}

// lanes per row for n rows in a T-thread workgroup
inline int small_group(int n, int T) {
  if (const char* e = std::getenv("GE_SMALL_G")) {  // tuning override
    const int g = std::atoi(e);
    if ((g == 1 || g == 2 || g == 4 || g == 8 || g == 16) && n * g <= T) return g;
  }
  int G = 1;
  while (G < 16 && n * G * 2 <= T) G *= 2;
  return G;
}

constexpr int kSmallFastT = 1024;  // domain-only kernel
constexpr int kSmallGenT = 512;    // general kernel

// Fp: n*D scratch, it_state: one int (device).
template <int D>
void launch_small(hipStream_t s, int n, int nnz, const int* ip, const int* ix, const double* dx,
                  const double* dp1, double* X, double* Fp, int* it_state, int iterations,
                  const FaConst& c) {
  GE_HIP(hipMemsetAsync(Fp, 0, sizeof(double) * (size_t)n * D, s));
  GE_HIP(hipMemsetAsync(it_state, 0, sizeof(int), s));
  const bool staged = nnz <= small_nnz_cap(D);
  int stop_at = iterations;  // test hook: hand over to the general kernel there
  if (const char* e = std::getenv("GE_SMALL_HANDOVER")) stop_at = std::atoi(e);
  auto go = [&](auto GG, auto TT, auto ST, auto DO) {
    hipLaunchKernelGGL((fa_small_strict<D, decltype(GG)::value, decltype(TT)::value,
                                        decltype(ST)::value, decltype(DO)::value>),
                       dim3(1), dim3(decltype(TT)::value), 0, s, n, ip, ix, dx, dp1, X, Fp,
                       it_state, iterations, stop_at, c);
  };
  using F = std::false_type;
  using Tt = std::true_type;
  auto by_group = [&](int G, auto TT, auto DO) {
    auto by_stage = [&](auto GG) {
      if (staged) go(GG, TT, Tt(), DO);
      else go(GG, TT, F(), DO);
    };
    switch (G) {
      case 16: by_stage(std::integral_constant<int, 16>()); break;
      case 8: by_stage(std::integral_constant<int, 8>()); break;
      case 4: by_stage(std::integral_constant<int, 4>()); break;
      case 2: by_stage(std::integral_constant<int, 2>()); break;
      default: by_stage(std::integral_constant<int, 1>()); break;
    }
  };
  // the domain-only kernel has the linear attraction only (linlog == 0, delta == 1)
  if (!std::getenv("GE_SMALL_GENERAL_ONLY") && !c.linlog && c.delta == 1.0)
    by_group(small_group(n, kSmallFastT), std::integral_constant<int, kSmallFastT>(), Tt());
  by_group(small_group(n, kSmallGenT), std::integral_constant<int, kSmallGenT>(), F());
}

// ---------------------------------------------------------------------------
// STRICT repulsion for small n (n <= grouped_cap, e.g. the coarsest levels of
// configs[3]): too few rows to fill the chip one lane per row, so G lanes share
// a row -- they evaluate G consecutive partners at once and the group adds the
// terms in j order (pipelined_group_sum).  Every block stages all n records in
// LDS; the exact-division domain is checked once per block.

// Records [first, first + cnt) of X / dp1 into rec (Rec<D>::W doubles each) by
// the T threads of the block: SU records per thread per round with all their
// loads issued before the stores (a plain strided loop waits for one record at
// a time).  Returns whether every staged value lies in the exact-division domain.
template <int D, int T, int SU, bool COH = false>
__device__ __forceinline__ bool stage_records(const double* __restrict__ X,
                                              const double* __restrict__ dp1, int first, int cnt,
                                              double* rec) {
  constexpr int W = Rec<D>::W;
  bool ok = true;
  for (int q0 = 0; q0 < cnt; q0 += T * SU) {
    double v[SU][D + 1];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int q = min(q0 + (int)threadIdx.x + T * u, cnt - 1);  // clamped into the range
#pragma unroll
      for (int k = 0; k < D; ++k)
        v[u][k] = COH ? coh_ld(&X[(size_t)(first + q) * D + k]) : X[(size_t)(first + q) * D + k];
      v[u][D] = dp1[first + q];
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int q = q0 + (int)threadIdx.x + T * u;
      if (q < cnt) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
          rec[q * W + k] = v[u][k];
          ok = ok && coord_ok(v[u][k]);
        }
        rec[q * W + D] = v[u][D];
        ok = ok && weight_ok(v[u][D]);
      }
    }
  }
  return ok;
}

// Persistent small-level barrier ordering (tuning switch, scripts/build_variant.sh):
// 0 relaxed arrival + agent-scope staging loads; 1 release arrival; 2 release + an
// acquire fence after the poll; 3 acquire fence only and plain (L2-cached) staging
// loads; 4 release + acquire and plain staging loads.  The coordinates are always
// stored with agent-scope stores.
// Measured (n = 919, 20 000 iterations, one box, scripts/coarsest_time.py,
// profiles/r04/coarsest_barrier_variants.log): packed rows 17.9 / 20.6 / 18.8 /
// 20.0 us per iteration for orders 0 / 2 / 3 / 4 -- the release write-back and
// the acquire invalidate each cost more than the whole barrier's ordering is worth
// here, so the shipped order is 0: agent-scope (L2-bypassing) stores and loads of
// the coordinates, every store completed (s_waitcnt 0) before the arrival.
// (Round 5 measured the phases of an iteration with diagnostics builds of this
// kernel -- per-phase clock stamps, chunks or staging skipped -- DESIGN.md 5c,
// profiles/r05/coarsest_phase_diag.log; removed from the source in round 6.)
#ifndef GE_BAR_ORDER
#define GE_BAR_ORDER 0
#endif
constexpr bool kBarCohStage = GE_BAR_ORDER < 3;

constexpr int kGrpT = 256;
constexpr int grouped_cap(int D) { return (D + 1 <= 4) ? 3072 : 1536; }  // <= 96 KiB of records
inline size_t grouped_lds_bytes(int n, int D) {
  return sizeof(double) * ((size_t)n * ((D + 1 <= 4) ? 4 : 8) + 2 * kGrpT * D);
}

template <int D, int G, bool REPEL_ONE>
__global__ void __launch_bounds__(kGrpT)
fa_repulse_grouped(int n, int rb, int re, const double* __restrict__ X,
                   const double* __restrict__ dp1, double repel, double* __restrict__ Frep) {
  constexpr int W = Rec<D>::W;
  // dynamic LDS: n records, then the two term buffers (grouped_lds_bytes)
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* rec = smem;
  double* tb = smem + (size_t)n * W;
  const int tid = threadIdx.x;
  const int g = tid % G;
  const int i = rb + blockIdx.x * (kGrpT / G) + tid / G;
  const bool active = i < re;
  const bool ok =
      stage_records<D, kGrpT, 4>(X, dp1, 0, n, rec) && (REPEL_ONE || weight_ok(repel));
  __syncthreads();
  double xi[D], acc[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    xi[k] = active ? rec[i * W + k] : 0.0;
    acc[k] = 0.0;
  }
  const double di = active ? rec[i * W + D] : 1.0;
  if (__syncthreads_and(ok)) {  // block-uniform: every record in the domain
    if (G > 1) {
      pipelined_group_sum<D, G, kGrpT>(n, tid, g, tb, [&](int q, double (&t)[D]) {
        const int jj = min(q, n - 1);
        rep_term<D, true, REPEL_ONE>(xi, &rec[jj * W], di, rec[jj * W + D], repel, t);
        if (q >= n)
#pragma unroll
          for (int k = 0; k < D; ++k) t[k] = 0.0;
      }, acc);
    } else {
      for (int j = 0; j < n; ++j)
        rep_pair<D, true, REPEL_ONE>(xi, &rec[j * W], di, rec[j * W + D], repel, acc);
    }
  } else {
    const bool row_ok = vertex_ok<D>(xi, di) && (REPEL_ONE || weight_ok(repel));
    for (int j0 = 0; j0 < n; j0 += G) {
      double t[1][D];
#pragma unroll
      for (int k = 0; k < D; ++k) t[0][k] = 0.0;
      const int j = j0 + g;
      if (j < n) {
        const double* xj = &rec[j * W];
        if (row_ok && vertex_ok<D>(xj, rec[j * W + D]))
          rep_pair<D, true, REPEL_ONE>(xi, xj, di, rec[j * W + D], repel, t[0]);
        else
          rep_pair_fb<D, REPEL_ONE>(xi, xj, di, rec[j * W + D], repel, j == i, t[0]);
      }
      group_add<D, G, 1>(t, tid, g, min(G, n - j0), active && g == 0, tb, acc);
    }
  }
  if (active && g == 0)
#pragma unroll
    for (int k = 0; k < D; ++k) Frep[(size_t)(i - rb) * D + k] = acc[k];
}

// One whole iteration of a small level (n <= grouped_cap) in one launch: the
// repulsion group sum, then the CSR row's attraction terms (neighbours from the
// LDS records) continuing the same ordered sum, then gravity, swing and the
// update (:146-269).  Rows [rb, re); Fprev indexed by row - rb.  LINEAR: the
// caller guarantees linlog == 0 and delta == 1 (the in-domain bodies use it).
template <int D, int G, bool REPEL_ONE, bool LINEAR, bool COH>
__device__ __forceinline__ void grouped_iteration(int blk, int n, int rb, int re,
                                                  const int* __restrict__ ip,
                                                  const int* __restrict__ ix,
                                                  const double* __restrict__ dx,
                                                  const double* __restrict__ X,
                                                  const double* __restrict__ dp1, const FaConst& c,
                                                  double* __restrict__ Fprev,
                                                  double* __restrict__ Xnext, double* smem,
                                                  int row0 = -1, int rend = 0x7fffffff) {
  constexpr int W = Rec<D>::W;
  double* rec = smem;
  double* tb = smem + (size_t)n * W;
  const int tid = threadIdx.x;
  const int g = tid % G;
  // rows rb + blk * (kGrpT / G) + [0, kGrpT / G), or from row0 (below rend) when given
  const int i = (row0 >= 0 ? row0 : rb + blk * (kGrpT / G)) + tid / G;
  const bool active = i < min(re, rend);
  const bool ok =
      stage_records<D, kGrpT, 4, COH && kBarCohStage>(X, dp1, 0, n, rec) &&
      (REPEL_ONE || weight_ok(c.repel));
  double xi[D], acc[D], fprev[D];
  const int e0 = active ? ip[i] : 0;
  const int e1 = active ? ip[i + 1] : 0;
#pragma unroll
  for (int k = 0; k < D; ++k) fprev[k] = (active && g == 0) ? Fprev[(size_t)(i - rb) * D + k] : 0.0;
  // the CSR row's first chunk, loaded while the records are being staged
  const int pe = min(e0 + g, e1 - 1);
  const int pix = e1 > e0 ? ix[pe] : 0;
  const double pdx = (e1 > e0 && c.use_weights) ? dx[pe] : 1.0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < D; ++k) {
    xi[k] = active ? rec[i * W + k] : 0.0;
    acc[k] = 0.0;
  }
  const double di = active ? rec[i * W + D] : 1.0;
  if (__syncthreads_and(ok) && G > 1) {  // block-uniform: every record in the domain
    pipelined_group_sum<D, G, kGrpT>(n, tid, g, tb, [&](int q, double (&t)[D]) {
      const int jj = min(q, n - 1);
      rep_term<D, true, REPEL_ONE>(xi, &rec[jj * W], di, rec[jj * W + D], c.repel, t);
      if (q >= n)
#pragma unroll
        for (int k = 0; k < D; ++k) t[k] = 0.0;
    }, acc);
    pipelined_group_sum<D, G, kGrpT>(e1 - e0, tid, g, tb, [&](int q, double (&t)[D]) {
      const int ee = min(e0 + q, e1 - 1);
#pragma unroll
      for (int k = 0; k < D; ++k) t[k] = 0.0;
      const int j = q < G ? pix : ix[ee];  // chunk 0 (q = g) was prefetched
      const double a = q < G ? pdx : (c.use_weights ? dx[ee] : 1.0);
      attr_edge<D, true, LINEAR>(xi, &rec[j * W], a, di, c, t);
      if (e0 + q >= e1)
#pragma unroll
        for (int k = 0; k < D; ++k) t[k] = 0.0;
    }, acc);
  } else {
    const bool row_ok = vertex_ok<D>(xi, di) && (REPEL_ONE || weight_ok(c.repel));
    for (int j0 = 0; j0 < n; j0 += G) {  // :151-167, j ascending
      double t[1][D];
#pragma unroll
      for (int k = 0; k < D; ++k) t[0][k] = 0.0;
      const int j = j0 + g;
      if (active && j < n) {
        const double* xj = &rec[j * W];
        if (row_ok && vertex_ok<D>(xj, rec[j * W + D]))
          rep_pair<D, true, REPEL_ONE>(xi, xj, di, rec[j * W + D], c.repel, t[0]);
        else
          rep_pair_fb<D, REPEL_ONE>(xi, xj, di, rec[j * W + D], c.repel, j == i, t[0]);
      }
      group_add<D, G, 1>(t, tid, g, min(G, n - j0), active && g == 0, tb, acc);
    }
    const bool xi_ok = all_coord_ok<D>(xi);
    for (int b = 0; b < e1 - e0; b += G) {  // :169-203, CSR order
      double t[1][D];
#pragma unroll
      for (int k = 0; k < D; ++k) t[0][k] = 0.0;
      const int e = e0 + b + g;
      if (e < e1) {
        const double* xj = &rec[ix[e] * W];
        const double a = c.use_weights ? dx[e] : 1.0;
        if (xi_ok && all_coord_ok<D>(xj))
          attr_edge<D, true>(xi, xj, a, di, c, t[0]);
        else
          attr_edge<D, false>(xi, xj, a, di, c, t[0]);
      }
      group_add<D, G, 1>(t, tid, g, min(G, e1 - e0 - b), active && g == 0, tb, acc);
    }
  }
  if (active && g == 0)
    finish_row<D, COH>(i, i - rb, xi, acc, fprev, di, c, Fprev, Xnext, true);
}


// Packed rows (the coarsest level's persistent kernel, 4 rows per block as with 64
// lanes per row).  With one wave per row, each chunk of 64 partners costs the
// wave its 64 terms AND 64 ordered adds (one full-wave instruction each for 3
// active lanes), ~13 ns per partner at n ~ 1000.  Here wave 0 only adds: lane
// r * D + k carries row r's dimension k (12 lanes for 4 rows in 3-D), one dependent
// add per term, while waves 1-3 evaluate the next chunk of kPackU x 48 partners
// per row into the other half of a double buffer.  The per-row order of additions
// is the reference's (partners ascending, then the CSR row in stored order), so
// the bits are those of grouped_iteration.  In-domain blocks only: a block whose
// records leave the exact-division domain runs grouped_iteration<G = 64> (the same
// rows) instead.
// R rows per block (4, or 6 when 4 would need more blocks than CUs: C4's coarsest level
// has n = 1 068 = 267 blocks of 4 on 256 CUs, and a CU holding two blocks slows the
// whole grid): 192 / R producer lanes per row, each evaluating kPackC R / 192 partners
// of a chunk.
constexpr int kPackC = 96;  // partners per row per chunk
// Term-buffer line of one (row, dimension): kPackC terms + 2 doubles of padding, so the
// adder lanes' 16-byte reads (one line each, same offset) fall in different LDS banks.
// Unpadded (768-byte lines) all 12 lanes hit one bank: n = 998, the chunk loop took
// 10.2 us per iteration (0.85 us per chunk of 96 partners) against ~0.3 us of adds.
constexpr int kPackS = kPackC + 2;
inline size_t packed_lds_bytes(int n, int D, int R) {
  return sizeof(double) * ((size_t)n * ((D + 1 <= 4) ? 4 : 8) + 2 * (size_t)R * D * kPackS);
}

// group_chain for the packed adder lane: the first nb batches (of 16 terms) of a chunk,
// the reads GE_CHAIN_AHEAD batches ahead of the adds, so the LDS latency hides behind
// the dependent adds (3: n = 998 18.2 us per iteration against 18.4 / 18.8 at 2 / 1).
// No per-lane count: the producers write every slot of a chunk, +0.0 past a row's own
// terms, and adding +0.0 leaves a sum that starts at +0.0 unchanged (it is never -0.0),
// so a lane adds the batches any lane of the block needs (nb, block-uniform) and skips
// the rest.  Round 5 tested a count per lane and per batch (26 cycles per add against
// 12 without, scripts/micro/adder_chain.hip) and added all six batches of every chunk.
#ifndef GE_CHAIN_AHEAD
#define GE_CHAIN_AHEAD 3
#endif
template <int G>
__device__ __forceinline__ double chain_prefetch(double a, const double* p, int nb) {
  constexpr int B = 16, NB = G / B, P = GE_CHAIN_AHEAD, R = P + 1;
  static_assert(G % B == 0, "batches of 16");
  double v[R][B];
#pragma unroll
  for (int b = 0; b < P && b < NB; ++b) {
    if (b >= nb) break;
#pragma unroll
    for (int l = 0; l < B; l += 2) {
      const double2 x = *reinterpret_cast<const double2*>(p + b * B + l);
      v[b][l] = x.x;
      v[b][l + 1] = x.y;
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b >= nb) break;
    if (b + P < NB && b + P < nb) {
#pragma unroll
      for (int l = 0; l < B; l += 2) {
        const double2 x = *reinterpret_cast<const double2*>(p + (b + P) * B + l);
        v[(b + P) % R][l] = x.x;
        v[(b + P) % R][l + 1] = x.y;
      }
    }
#pragma unroll
    for (int l = 0; l < B; ++l) a = a + v[b % R][l];
  }
  return a;
}

template <int D, bool REPEL_ONE, bool LINEAR, bool COH, int R>
__device__ __forceinline__ void packed_iteration(int blk, int n, int rb, int re,
                                                 const int* __restrict__ ip,
                                                 const int* __restrict__ ix,
                                                 const double* __restrict__ dx,
                                                 const double* __restrict__ X,
                                                 const double* __restrict__ dp1, const FaConst& c,
                                                 double* __restrict__ Fprev,
                                                 double* __restrict__ Xnext, double* smem) {
  static_assert(R * D <= 64, "one adder lane per (row, dimension)");
  static_assert(kPackC % 16 == 0 && kPackS % 2 == 0, "chain_prefetch reads 16-byte pairs");
  constexpr int W = Rec<D>::W;
  constexpr int PL = kGrpT - 64;               // producer lanes
  constexpr int CL = PL / R;                   // producer lanes per row
  constexpr int kPackU = kPackC / CL;          // terms per producer lane per chunk
  static_assert(CL * R == PL && kPackU * CL == kPackC, "producer lanes tile the chunk");
  constexpr int BUF = R * D * kPackS;          // one half of the term buffer
  __shared__ int s_e[R][2];
  double* rec = smem;
  double* tb = smem + (size_t)n * W;
  const int tid = threadIdx.x;
  const int r0 = rb + blk * R;
  const bool ok =
      stage_records<D, kGrpT, 4, COH && kBarCohStage>(X, dp1, 0, n, rec) &&
      (REPEL_ONE || weight_ok(c.repel));
  if (tid < R) {
    const int i = r0 + tid;
    s_e[tid][0] = i < re ? ip[i] : 0;
    s_e[tid][1] = i < re ? ip[i + 1] : 0;
  }
  if (!__syncthreads_and(ok)) {  // block-uniform: the general bodies, same rows
    for (int q = 0; q < R; q += kGrpT / 64)  // kGrpT / 64 rows per call
      grouped_iteration<D, 64, REPEL_ONE, LINEAR, COH>(blk, n, rb, re, ip, ix, dx, X, dp1, c,
                                                       Fprev, Xnext, smem, r0 + q, r0 + R);
    return;
  }
  // producer lane: row pr, chunk slots pj + CL * u
  const bool prod = tid >= 64;
  const int p = tid - 64, pr = prod ? p / CL : 0, pj = prod ? p % CL : 0;
  const int ip_row = r0 + pr;
  const bool pact = prod && ip_row < re;
  double xp[D], dp = 1.0;
#pragma unroll
  for (int k = 0; k < D; ++k) xp[k] = pact ? rec[ip_row * W + k] : 0.0;
  if (pact) dp = rec[ip_row * W + D];
  auto rep_chunk = [&](int ch, double* dst) {  // terms of partners ch * C + slot
    double t[kPackU][D];
#pragma unroll
    for (int u = 0; u < kPackU; ++u) {
      const int j = ch * kPackC + pj + CL * u;
      const int jj = min(j, n - 1);
      rep_term<D, true, REPEL_ONE>(xp, &rec[jj * W], dp, rec[jj * W + D], c.repel, t[u]);
      if (j >= n || !pact)
#pragma unroll
        for (int k = 0; k < D; ++k) t[u][k] = 0.0;
    }
#pragma unroll
    for (int u = 0; u < kPackU; ++u)
#pragma unroll
      for (int k = 0; k < D; ++k) dst[(pr * D + k) * kPackS + pj + CL * u] = t[u][k];
  };
  const int pe0 = s_e[pr][0], pe1 = s_e[pr][1];
  auto att_chunk = [&](int ch, double* dst) {  // CSR entries e0 + ch * C + slot
    double t[kPackU][D];
#pragma unroll
    for (int u = 0; u < kPackU; ++u) {
      const int q = ch * kPackC + pj + CL * u;
      const int ee = min(pe0 + q, pe1 - 1);
#pragma unroll
      for (int k = 0; k < D; ++k) t[u][k] = 0.0;
      if (pact && pe0 + q < pe1)
        attr_edge<D, true, LINEAR>(xp, &rec[ix[ee] * W], c.use_weights ? dx[ee] : 1.0, dp, c,
                                   t[u]);
    }
#pragma unroll
    for (int u = 0; u < kPackU; ++u)
#pragma unroll
      for (int k = 0; k < D; ++k) dst[(pr * D + k) * kPackS + pj + CL * u] = t[u][k];
  };
  // adder lane: row ar, dimension ak
  const int ar = tid / D, ak = tid - ar * D;
  const bool adder = tid < R * D;
  double a = 0.0;
  const int nrep = (n + kPackC - 1) / kPackC;
  int maxdeg = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) maxdeg = max(maxdeg, s_e[r][1] - s_e[r][0]);
  const int natt = (maxdeg + kPackC - 1) / kPackC;
  const int ntot = nrep + natt;  // the repulsion chunks, then the attraction chunks
  if (prod && ntot > 0) {
    if (nrep > 0) rep_chunk(0, tb);
    else att_chunk(0, tb);
  }
  __syncthreads();
  for (int ch = 0; ch < ntot; ++ch) {
    const double* cur = tb + (ch & 1) * BUF;
    if (tid < 64) {
      // the largest count of the chunk over the block's rows (uniform)
      const int cmax = ch < nrep ? min(kPackC, n - ch * kPackC)
                                 : min(kPackC, maxdeg - (ch - nrep) * kPackC);
      if (adder) a = chain_prefetch<kPackC>(a, cur + (ar * D + ak) * kPackS, (cmax + 15) >> 4);
    } else if (ch + 1 < ntot) {
      double* nxt = tb + ((ch + 1) & 1) * BUF;
      if (ch + 1 < nrep) rep_chunk(ch + 1, nxt);
      else att_chunk(ch + 1 - nrep, nxt);
    }
    __syncthreads();
  }
  if (tid < 64) {
    // the row's leader lane (r * D) gathers its dimensions, then gravity / update
    double acc[D];
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = __shfl(a, (tid / D) * D + k);
    const int i = r0 + ar;
    if (adder && ak == 0 && i < re) {
      double xi[D], fprev[D];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        xi[k] = rec[i * W + k];
        fprev[k] = Fprev[(size_t)(i - rb) * D + k];
      }
      finish_row<D, COH>(i, i - rb, xi, acc, fprev, rec[i * W + D], c, Fprev, Xnext, true);
    }
  }
}

template <int D, int G, bool REPEL_ONE, bool LINEAR>
__global__ void __launch_bounds__(kGrpT)
fa_grouped_step(int n, int rb, int re, const int* __restrict__ ip, const int* __restrict__ ix,
                const double* __restrict__ dx, const double* __restrict__ X,
                const double* __restrict__ dp1, FaConst c, double* __restrict__ Fprev,
                double* __restrict__ Xnext) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  grouped_iteration<D, G, REPEL_ONE, LINEAR, false>(blockIdx.x, n, rb, re, ip, ix, dx, X, dp1, c,
                                                    Fprev, Xnext, smem);
}

// ---------------------------------------------------------------------------
// The coarsest level's 1e5 iterations (src/embed.cpp:586) as ONE launch: the
// blocks of fa_grouped_step stay resident and run every iteration, separated by
// a grid-wide barrier (the next iteration stages every block's coordinates).
// The coordinates alternate between two buffers (iteration it reads buffer
// it & 1), so one barrier per iteration suffices; each row's previous force
// is read and written by the row's own leader lane only.  Coordinates are stored and staged with
// agent-scope accesses; a block's stores have completed (s_waitcnt 0) before it
// arrives, and the waiters poll the grid counter, so what a block stages after
// the barrier is what every other block stored before it.
//
// bar layout (ints): [1] error flag, then a 128-byte line for the grid counter
// and one per arrival group (kBarGroup blocks).
// Counters only grow (target = arrivals * (iteration + 1)), so nothing is reset
// between barriers.
// A wait longer than ~limit ticks of the 100 MHz wall clock sets the error flag
// and ends the kernel (every block then ends at its own next wait), so a
// non-resident grid cannot hang the device.
constexpr int kBarGroup = 16;
constexpr int kBarLine = 32;  // ints per 128-byte line
inline size_t persist_bar_ints(int nb) {
  return (size_t)kBarLine * (2 + (nb + kBarGroup - 1) / kBarGroup);
}

__device__ __forceinline__ int coh_ldi(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Thread 0 of each block: arrive at barrier number it (0-based) and wait for all.
// Two levels: the last arrival of each group of kBarGroup blocks adds one to the
// grid counter, which the waiters poll (one counter for every block was measured
// slower: n = 998 22.3 against 19.7 us per iteration).
__device__ bool grid_arrive_wait(int* bar, int nb, int it, long long limit) {
  int* cnt = bar + kBarLine;  // its own line, away from the error flag
  const int ngroups = (nb + kBarGroup - 1) / kBarGroup;
  const int grp = blockIdx.x / kBarGroup;
  const int members = min(kBarGroup, nb - grp * kBarGroup);
  int* gc = bar + kBarLine * (2 + grp);
  // Ordering as shipped (GE_BAR_ORDER 0): the arrival and the group's hand-on are
  // RELAXED agent-scope atomics with no acquire fence after the poll.  What orders a
  // block's coordinate stores before another block's staging loads is the hardware,
  // not the HIP memory model: the coordinates are written and read with agent-scope
  // (L2-bypassing) accesses, every store has completed at the memory side
  // (s_waitcnt 0, in fa_grouped_persistent) before the block's thread 0 arrives, and
  // a waiter's staging loads are issued only after its poll has seen the count.  The
  // release / acquire orders 1-4 below follow the model and were measured slower
  // (17.9 against 20.6 us per iteration, profiles/r04/coarsest_barrier_variants.log).
  // A compiler change could break the shipped order silently: the canaries are
  // tests/test_gpu_parity.py test_fa_coarsest_level_production_horizon (1e5
  // iterations against the oracle fixture) and test_fa_coarsest_level_shared_device,
  // which must stay in the suite.
  constexpr bool rel = GE_BAR_ORDER == 1 || GE_BAR_ORDER == 2 || GE_BAR_ORDER == 4;
  constexpr int kRel = rel ? __ATOMIC_RELEASE : __ATOMIC_RELAXED;
  constexpr int kAR = rel ? __ATOMIC_ACQ_REL : __ATOMIC_RELAXED;
  const int old = __hip_atomic_fetch_add(gc, 1, kRel, __HIP_MEMORY_SCOPE_AGENT);
  if (old == members * (it + 1) - 1)  // the group's last arrival
    __hip_atomic_fetch_add(cnt, 1, kAR, __HIP_MEMORY_SCOPE_AGENT);
  const int target = ngroups * (it + 1);
  const long long t0 = wall_clock64();
  while (coh_ldi(cnt) < target) {
    if (coh_ldi(bar + 1) != 0 || wall_clock64() - t0 > limit) {
      __hip_atomic_store(bar + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (GE_BAR_ORDER >= 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

template <int D, int G, bool REPEL_ONE, bool LINEAR, int PACKED = 0>  // PACKED: rows per block
__global__ void __launch_bounds__(kGrpT)
fa_grouped_persistent(int n, const int* __restrict__ ip, const int* __restrict__ ix,
                      const double* __restrict__ dx, double* __restrict__ Xa,
                      double* __restrict__ Xb, const double* __restrict__ dp1, FaConst c,
                      double* __restrict__ Fprev, int* __restrict__ bar, int iterations,
                      long long limit) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int s_ok;
  for (int it = 0; it < iterations; ++it) {
    const double* X = (it & 1) ? Xb : Xa;
    double* Xn = (it & 1) ? Xa : Xb;
    if constexpr (PACKED > 0)
      packed_iteration<D, REPEL_ONE, LINEAR, true, PACKED>(blockIdx.x, n, 0, n, ip, ix, dx, X, dp1, c,
                                                   Fprev, Xn, smem);
    else
      grouped_iteration<D, G, REPEL_ONE, LINEAR, true>(blockIdx.x, n, 0, n, ip, ix, dx, X, dp1,
                                                       c, Fprev, Xn, smem);
    if (it + 1 == iterations) break;
    // this thread's coordinate stores have completed before the block arrives;
    // the signal fences keep the compiler from moving memory accesses across
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __syncthreads();
    if (threadIdx.x == 0) s_ok = grid_arrive_wait(bar, gridDim.x, it, limit) ? 1 : 0;
    __syncthreads();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (!s_ok) return;
  }
}

// Mid-size levels (grouped_cap < n <= kStreamMax): the same fused iteration
// with the records streamed through LDS in tiles of kStreamTile (the in-domain
// test per tile, the attraction's neighbours read from X), so a coarsest level
// of a few thousand to tens of thousands of vertices keeps G lanes per row.
constexpr int kStreamTile = 2048;
constexpr int kStreamMax = 65536;
// GE_STREAM_MAX overrides the bound (tuning / tests)
inline int stream_max() {
  if (const char* e = std::getenv("GE_STREAM_MAX")) return std::atoi(e);
  return kStreamMax;
}
inline size_t stream_lds_bytes(int D) {
  return sizeof(double) * ((size_t)kStreamTile * ((D + 1 <= 4) ? 4 : 8) + 2 * kGrpT * D);
}

template <int D, int G, bool REPEL_ONE, bool LINEAR>
__global__ void __launch_bounds__(kGrpT)
fa_grouped_stream(int n, int rb, int re, const int* __restrict__ ip, const int* __restrict__ ix,
                  const double* __restrict__ dx, const double* __restrict__ X,
                  const double* __restrict__ dp1, FaConst c, double* __restrict__ Fprev,
                  double* __restrict__ Xnext) {
  constexpr int W = Rec<D>::W;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* rec = smem;
  double* tb = smem + (size_t)kStreamTile * W;
  const int tid = threadIdx.x;
  const int g = tid % G;
  const int i = rb + blockIdx.x * (kGrpT / G) + tid / G;
  const bool active = i < re;
  double xi[D], acc[D], fprev[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    xi[k] = active ? X[(size_t)i * D + k] : 0.0;
    fprev[k] = (active && g == 0) ? Fprev[(size_t)(i - rb) * D + k] : 0.0;
    acc[k] = 0.0;
  }
  const double di = active ? dp1[i] : 1.0;
  const bool row_ok = !active || (vertex_ok<D>(xi, di) && (REPEL_ONE || weight_ok(c.repel)));
  const int e0 = active ? ip[i] : 0;
  const int e1 = active ? ip[i + 1] : 0;
  for (int t0 = 0; t0 < n; t0 += kStreamTile) {  // :151-167, j ascending
    const int cnt = min(kStreamTile, n - t0);
    __syncthreads();  // the previous tile has been consumed
    const bool ok = stage_records<D, kGrpT, 8>(X, dp1, t0, cnt, rec) && row_ok;
    if (__syncthreads_and(ok) && G > 1) {  // block-uniform: row and tile in the domain
      pipelined_group_sum<D, G, kGrpT>(cnt, tid, g, tb, [&](int q, double (&t)[D]) {
        const int jj = min(q, cnt - 1);
        rep_term<D, true, REPEL_ONE>(xi, &rec[jj * W], di, rec[jj * W + D], c.repel, t);
        if (q >= cnt)
#pragma unroll
          for (int k = 0; k < D; ++k) t[k] = 0.0;
      }, acc);
    } else {
      const bool rok = active && vertex_ok<D>(xi, di) && (REPEL_ONE || weight_ok(c.repel));
      for (int j0 = 0; j0 < cnt; j0 += G) {
        double t[1][D];
#pragma unroll
        for (int k = 0; k < D; ++k) t[0][k] = 0.0;
        const int j = j0 + g;
        if (active && j < cnt) {
          const double* xj = &rec[j * W];
          if (rok && vertex_ok<D>(xj, rec[j * W + D]))
            rep_pair<D, true, REPEL_ONE>(xi, xj, di, rec[j * W + D], c.repel, t[0]);
          else
            rep_pair_fb<D, REPEL_ONE>(xi, xj, di, rec[j * W + D], c.repel, t0 + j == i, t[0]);
        }
        group_add<D, G, 1>(t, tid, g, min(G, cnt - j0), active && g == 0, tb, acc);
      }
      if (G > 1)  // group_add leaves the sum in the group's first lane only
#pragma unroll
        for (int k = 0; k < D; ++k) acc[k] = __shfl(acc[k], (tid - g) & 63);
    }
  }
  // :169-203, CSR order; neighbours from X (per-edge domain test)
  const bool xi_ok = all_coord_ok<D>(xi);
  if (G > 1) {
    pipelined_group_sum<D, G, kGrpT>(e1 - e0, tid, g, tb, [&](int q, double (&t)[D]) {
      const int ee = min(e0 + q, e1 - 1);
#pragma unroll
      for (int k = 0; k < D; ++k) t[k] = 0.0;
      if (e1 > e0) {
        const double* xj = X + (size_t)ix[ee] * D;
        const double a = c.use_weights ? dx[ee] : 1.0;
        if (xi_ok && all_coord_ok<D>(xj))
          attr_edge<D, true, LINEAR>(xi, xj, a, di, c, t);
        else
          attr_edge<D, false>(xi, xj, a, di, c, t);
      }
      if (e0 + q >= e1)
#pragma unroll
        for (int k = 0; k < D; ++k) t[k] = 0.0;
    }, acc);
  } else {
    for (int e = e0; e < e1; ++e) {
      const double* xj = X + (size_t)ix[e] * D;
      const double a = c.use_weights ? dx[e] : 1.0;
      if (xi_ok && all_coord_ok<D>(xj))
        attr_edge<D, true>(xi, xj, a, di, c, acc);
      else
        attr_edge<D, false>(xi, xj, a, di, c, acc);
    }
  }
  if (active && g == 0)
    finish_row<D>(i, i - rb, xi, acc, fprev, di, c, Fprev, Xnext, true);
}

// ---------------------------------------------------------------------------
// host-side launch helpers

constexpr int kRowsPerThreadFast = 4;

int device_cus() {
  int dev = 0, cus = 0;
  GE_HIP(hipGetDevice(&dev));
  GE_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return cus > 0 ? cus : 256;
}

// Lanes per row of the small-level kernels.
inline int grouped_lanes(int rows) {
  int G = 1;  // lanes per row: aim for >= 128 K lanes, at most one wave per row
  while (G < 64 && (long long)rows * G < 131072) G *= 2;  // n = 4373: G = 32 (175 us, G = 16: 211)
  if (const char* e = std::getenv("GE_GRP_G")) {  // tuning / test override
    const int g = std::atoi(e);
    if (g >= 1 && g <= 64 && (g & (g - 1)) == 0) G = g;
  }
  return G;
}

template <int D>
void launch_repulsion(hipStream_t s, int mode, int n, int rb, int re, const double* X,
                      const double* dp1, double repel, double* Frep, double* Fpart, int cus) {
  const int rows = re - rb;
  if (rows <= 0) return;
  if (mode == GE_MODE_FAST) {
    const int per = kFastThreads * kRowsPerThreadFast;
    const int jb = std::max(1, std::min(kFastJBlocks, (n + kTileJ - 1) / kTileJ));
    dim3 grid((rows + per - 1) / per, jb);
    hipLaunchKernelGGL((fa_repulse_fast<D, kRowsPerThreadFast>), grid, dim3(kFastThreads), 0, s,
                       n, rb, re, X, dp1, repel, jb, Fpart);
    const int tot = rows * D;
    hipLaunchKernelGGL((fa_reduce_parts<D>), dim3((tot + 255) / 256), dim3(256), 0, s, rows, jb,
                       Fpart, Frep);
    return;
  }
  if (n <= grouped_cap(D)) {
    const int G = grouped_lanes(rows);
    auto go = [&](auto GG) {
      constexpr int GC = decltype(GG)::value;
      const int nb = (rows + kGrpT / GC - 1) / (kGrpT / GC);
      const size_t lds = grouped_lds_bytes(n, D);
      if (lds > 65536) {  // above the default dynamic-LDS limit
        GE_HIP(hipFuncSetAttribute(
            reinterpret_cast<const void*>(&fa_repulse_grouped<D, GC, true>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        GE_HIP(hipFuncSetAttribute(
            reinterpret_cast<const void*>(&fa_repulse_grouped<D, GC, false>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      }
      if (repel == 1.0)
        hipLaunchKernelGGL((fa_repulse_grouped<D, GC, true>), dim3(nb), dim3(kGrpT), lds, s, n,
                           rb, re, X, dp1, repel, Frep);
      else
        hipLaunchKernelGGL((fa_repulse_grouped<D, GC, false>), dim3(nb), dim3(kGrpT), lds, s, n,
                           rb, re, X, dp1, repel, Frep);
    };
    switch (G) {
      case 64: go(std::integral_constant<int, 64>()); break;
      case 32: go(std::integral_constant<int, 32>()); break;
      case 16: go(std::integral_constant<int, 16>()); break;
      case 8: go(std::integral_constant<int, 8>()); break;
      case 4: go(std::integral_constant<int, 4>()); break;
      case 2: go(std::integral_constant<int, 2>()); break;
      default: go(std::integral_constant<int, 1>()); break;
    }
    return;
  }
  // one block per CU, rows split evenly (rounded to whole 64-row wave slots)
  int cap = cus;
  if (const char* e = std::getenv("GE_REP_BLOCKS")) cap = std::max(1, std::atoi(e));  // tests
  const int blocks = std::max(1, std::min(cap, (rows + 63) / 64));
  int per = (rows + blocks - 1) / blocks;
  per = (per + 63) / 64 * 64;
  const int nb = (rows + per - 1) / per;
  // Row slots per lane.  Measured at C2 size (scripts/shard_tune.py, rows of
  // an N-GPU shard): with more than 1024 rows per block 8 slots x 1 partner is
  // fastest (500 K rows: 581 against 563 Gpairs/s for R = 1); at 1024 and below
  // 1 slot x 8 partners (250 K rows: R = 1 566, R = 8 551; 125 K rows: R = 1
  // 565 Gpairs/s).
  int R = per > 2 * kRepThreads ? 8 : 1;
  if (const char* e = std::getenv("GE_REP_R")) {  // tuning / test override
    const int r = std::atoi(e);
    if (r == 1 || r == 2 || r == 4 || r == 8) R = r;
  }
  auto go = [&](auto RR) {
    constexpr int RC = decltype(RR)::value;
    if (repel == 1.0)
      hipLaunchKernelGGL((fa_repulse_strict<D, true, RC>), dim3(nb), dim3(kRepThreads), 0, s, n,
                         rb, re, per, X, dp1, repel, Frep);
    else
      hipLaunchKernelGGL((fa_repulse_strict<D, false, RC>), dim3(nb), dim3(kRepThreads), 0, s, n,
                         rb, re, per, X, dp1, repel, Frep);
  };
  switch (R) {
    case 8: go(std::integral_constant<int, 8>()); break;
    case 4: go(std::integral_constant<int, 4>()); break;
    case 2: go(std::integral_constant<int, 2>()); break;
    default: go(std::integral_constant<int, 1>()); break;
  }
}

// Small levels (n <= grouped_cap: fa_grouped_step) and mid-size ones (n <=
// stream_max: fa_grouped_stream): one launch per iteration.
template <int D>
void launch_grouped_step(hipStream_t s, int n, int rb, int re, const int* ip, const int* ix,
                         const double* dx, const double* X, const double* dp1, const FaConst& c,
                         double* Fprev, double* Xnext) {
  const int rows = re - rb;
  if (rows <= 0) return;
  const bool stream = n > grouped_cap(D);
  const size_t lds = stream ? stream_lds_bytes(D) : grouped_lds_bytes(n, D);
  auto go = [&](auto GG) {
    constexpr int GC = decltype(GG)::value;
    const int nb = (rows + kGrpT / GC - 1) / (kGrpT / GC);
    auto one = [&](auto RO, auto LI) {
      constexpr bool R1 = decltype(RO)::value, LIN = decltype(LI)::value;
      const void* fn = stream ? reinterpret_cast<const void*>(&fa_grouped_stream<D, GC, R1, LIN>)
                              : reinterpret_cast<const void*>(&fa_grouped_step<D, GC, R1, LIN>);
      if (lds > 65536)  // above the default dynamic-LDS limit
        GE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      if (stream)
        hipLaunchKernelGGL((fa_grouped_stream<D, GC, R1, LIN>), dim3(nb), dim3(kGrpT), lds, s, n,
                           rb, re, ip, ix, dx, X, dp1, c, Fprev, Xnext);
      else
        hipLaunchKernelGGL((fa_grouped_step<D, GC, R1, LIN>), dim3(nb), dim3(kGrpT), lds, s, n,
                           rb, re, ip, ix, dx, X, dp1, c, Fprev, Xnext);
    };
    const bool lin = !c.linlog && c.delta == 1.0;
    using T = std::true_type;
    using F = std::false_type;
    if (c.repel == 1.0) {
      if (lin) one(T(), T());
      else one(T(), F());
    } else {
      if (lin) one(F(), T());
      else one(F(), F());
    }
  };
  switch (grouped_lanes(rows)) {
    case 64: go(std::integral_constant<int, 64>()); break;
    case 32: go(std::integral_constant<int, 32>()); break;
    case 16: go(std::integral_constant<int, 16>()); break;
    case 8: go(std::integral_constant<int, 8>()); break;
    case 4: go(std::integral_constant<int, 4>()); break;
    case 2: go(std::integral_constant<int, 2>()); break;
    default: go(std::integral_constant<int, 1>()); break;
  }
}

template <int D>
void launch_attract(hipStream_t s, const RowClasses& rc, RowStreams& rs, int rb, const int* ip,
                    const int* ix, const double* dx, const double* X, const double* dp1,
                    const double* Frep, double* Fprev, double* Xnext, const FaConst& c) {
  const FaRows<D> fr{rb, ip, ix, dx, X, dp1, Frep, Fprev, Xnext, c};
  launch_rows<D>(rc, fr, s, rs);
}

}  // namespace
}  // namespace ge

// ---------------------------------------------------------------------------
// plan

struct ge_fa_plan {
  ge_ctx* ctx = nullptr;
  int n = 0, nnz = 0, dim = 0, rb = 0, re = 0;
  const int* ip = nullptr;
  const int* ix = nullptr;
  const double* dx = nullptr;
  ge_fa_params p{};
  ge::FaConst c{};
  ge::DevBuf<double> dp1, frep, fprev, fpart;
  ge::DevBuf<int> rows;  // rb..re in degree classes (ge_rows.hpp)
  ge::RowClasses rc;
  ge::RowStreams rstreams;
  int cus = 256;
  bool profiling = false;
  std::vector<hipEvent_t> events;  // 3 per timed step
  size_t next_event = 0;
  // Symmetric repulsion (ge_sym.hpp) for a whole large level in STRICT mode: the n
  // vertices as one "aggregate" of T = ceil(n / 64) row tiles, every unordered pair
  // evaluated once.  ctl = {queue, prog[T]}, zeroed before every launch.
  bool sym = false;
  int sym_units = 0, sym_blocks = 0;
  long long sym_limit = 0;
  ge::DevBuf<int4> units;
  ge::DevBuf<int> ctl, seg;
  ge::DevBuf<double> hand;
  int* sym_err_h = nullptr;  // pinned, device-mapped: a timed-out hand-over wait
  int* sym_err_d = nullptr;
  ~ge_fa_plan() {
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    if (sym_err_h) (void)hipHostFree(sym_err_h);
  }
};

namespace ge {

static void plan_init(ge_fa_plan* pl) {
  const int rows = pl->re - pl->rb;
  pl->cus = device_cus();
  pl->dp1.alloc(pl->n);
  pl->frep.alloc((size_t)std::max(rows, 1) * pl->dim);
  pl->fprev.alloc((size_t)std::max(rows, 1) * pl->dim);
  if (pl->p.mode == GE_MODE_FAST)
    pl->fpart.alloc((size_t)std::max(rows, 1) * pl->dim * kFastJBlocks);
  hipStream_t s = pl->ctx->stream;
  if (rows > 0) {
    std::vector<int> h_ip(pl->re - pl->rb + 1), ids(rows), deg(rows), order;
    GE_HIP(hipMemcpyAsync(h_ip.data(), pl->ip + pl->rb, sizeof(int) * h_ip.size(),
                          hipMemcpyDeviceToHost, s));
    GE_HIP(hipStreamSynchronize(s));
    for (int q = 0; q < rows; ++q) {
      ids[q] = pl->rb + q;
      deg[q] = h_ip[q + 1] - h_ip[q];
    }
    // single level: a row's sum starts at its repulsion over all n vertices, far
    // above the edge terms, so heavy rows split into binade-sum segments
    classify_rows(ids, deg, order, pl->rc, kSegBinade);
    pl->rows.alloc(order.size());
    pl->rows.upload(order.data(), order.size(), s);
    pl->rc.bind(pl->rows.p);
    pl->rstreams.attach(pl->rc, pl->dim, s);
    GE_HIP(hipStreamSynchronize(s));
  }
  hipLaunchKernelGGL(degp1_kernel, dim3((pl->n + 255) / 256), dim3(256), 0, s, pl->n, pl->ip,
                     pl->dx, pl->p.use_weights, pl->dp1.p);
  GE_HIP(hipGetLastError());
  GE_HIP(hipMemsetAsync(pl->fprev.p, 0, sizeof(double) * pl->fprev.n, s));
  // Symmetric repulsion: STRICT, every row on this plan (a row shard keeps the
  // ordered-pair kernel), and a level past the grouped / streamed kernels.
  // GE_FA_SYM=0 keeps fa_repulse_strict (comparisons), GE_FA_SYM=1 forces it.
  {
    const char* e = std::getenv("GE_FA_SYM");
    const bool force = e && *e == '1', off = e && *e == '0';
    pl->sym = !off && pl->p.mode == GE_MODE_STRICT && pl->rb == 0 && pl->re == pl->n &&
              (force || pl->n > stream_max());
  }
  // (Round 4 also built a degree-ordered gather copy of the coordinates for the
  // neighbour gathers: C2 0.324 against 0.301 ms per pass, C5 31.8 against 30.3 ms;
  // removed in round 5)
}

// The symmetric path's units, progress counters and hand-over buffer (n x d).  Made
// when the plan is created (ge_fa_plan_create, and before any graph capture in
// fa_run_device), so every symmetric plan holds them, one used only for
// ge_fa_plan_attract included; the step's call is a no-op then.
static void sym_prepare(ge_fa_plan* pl) {
  if (!pl->sym || pl->sym_units > 0) return;
  hipStream_t s = pl->ctx->stream;
  {
    const int T = (pl->n + 63) / 64;
    std::vector<int4> h_units(T);
    for (int A = 0; A < T; ++A) h_units[A] = make_int4(0, A, 0, 0);  // earliest start 2A
    pl->sym_units = T;
    pl->units.alloc(T);
    pl->units.upload(h_units.data(), T, s);
    pl->ctl.alloc(1 + T);  // queue, progress counters
    const int h_seg[2] = {0, pl->n};
    pl->seg.alloc(2);
    pl->seg.upload(h_seg, 2, s);
    pl->hand.alloc((size_t)pl->n * pl->dim);
    pl->sym_blocks = pl->cus * sym_blocks_per_cu(pl->dim);
    int dev = 0, khz = 0;
    GE_HIP(hipGetDevice(&dev));
    GE_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    pl->sym_limit = (long long)std::max(khz, 1000) * 5000;  // ~5 s per hand-over wait
    GE_HIP(hipHostMalloc((void**)&pl->sym_err_h, sizeof(int), hipHostMallocMapped));
    *pl->sym_err_h = 0;
    GE_HIP(hipHostGetDevicePointer((void**)&pl->sym_err_d, pl->sym_err_h, 0));
    GE_HIP(hipStreamSynchronize(s));
  }
}


// A symmetric launch whose hand-over wait timed out (seen through the pinned
// error word, without a synchronisation) fails the next step or the run's end.
static void sym_check(ge_fa_plan* pl) {
  if (pl->sym_err_h && __atomic_load_n(pl->sym_err_h, __ATOMIC_ACQUIRE)) {
    *pl->sym_err_h = 0;
    throw Error(GE_ERR_STATE, "forceAtlas: a symmetric sweep's hand-over wait timed out");
  }
}

static void plan_step(ge_fa_plan* pl, const double* xc, double* xn) {
  hipStream_t s = pl->ctx->stream;
  hipEvent_t* ev = nullptr;
  if (pl->profiling) {
    if (pl->next_event + 3 > pl->events.size()) {
      for (int k = 0; k < 3 * 64; ++k) {
        hipEvent_t e;
        GE_HIP(hipEventCreate(&e));
        pl->events.push_back(e);
      }
    }
    ev = &pl->events[pl->next_event];
    pl->next_event += 3;
    GE_HIP(hipEventRecord(ev[0], s));
  }
  dispatch_dim(pl->dim, [&](auto Dc) {
    constexpr int D = decltype(Dc)::value;
    if (pl->p.mode == GE_MODE_STRICT && pl->n <= stream_max() && !std::getenv("GE_GRP_SPLIT")) {
      launch_grouped_step<D>(s, pl->n, pl->rb, pl->re, pl->ip, pl->ix, pl->dx, xc, pl->dp1.p,
                             pl->c, pl->fprev.p, xn);
      if (ev) GE_HIP(hipEventRecord(ev[1], s));
      return;
    }
    if (pl->sym) {
      sym_prepare(pl);
      sym_check(pl);
      GE_HIP(hipMemsetAsync(pl->ctl.p, 0, sizeof(int) * pl->ctl.n, s));
      sym_repulse_launch(D, pl->sym_blocks, s, pl->sym_units, pl->units.p, pl->ctl.p,
                         pl->seg.p, xc, pl->dp1.p, pl->p.repel, pl->frep.p, pl->hand.p,
                         (size_t)pl->n, pl->ctl.p + 1, pl->sym_err_d, pl->sym_limit);
    } else {
      launch_repulsion<D>(s, pl->p.mode, pl->n, pl->rb, pl->re, xc, pl->dp1.p, pl->p.repel,
                          pl->frep.p, pl->fpart.p, pl->cus);
    }
    if (ev) GE_HIP(hipEventRecord(ev[1], s));
    launch_attract<D>(s, pl->rc, pl->rstreams, pl->rb, pl->ip, pl->ix, pl->dx, xc, pl->dp1.p, pl->frep.p,
                      pl->fprev.p, xn, pl->c);
  });
  GE_HIP(hipGetLastError());
  if (ev) GE_HIP(hipEventRecord(ev[2], s));
}

// ge_fa_plan_attract: the row kernels alone on a caller-supplied repulsion sum
// (profiling: the repulsion interval is empty).
static void plan_attract(ge_fa_plan* pl, const double* xc, const double* frep, double* xn) {
  hipStream_t s = pl->ctx->stream;
  hipEvent_t* ev = nullptr;
  if (pl->profiling) {
    if (pl->next_event + 3 > pl->events.size()) {
      for (int k = 0; k < 3 * 64; ++k) {
        hipEvent_t e;
        GE_HIP(hipEventCreate(&e));
        pl->events.push_back(e);
      }
    }
    ev = &pl->events[pl->next_event];
    pl->next_event += 3;
    GE_HIP(hipEventRecord(ev[0], s));
    GE_HIP(hipEventRecord(ev[1], s));
  }
  dispatch_dim(pl->dim, [&](auto Dc) {
    constexpr int D = decltype(Dc)::value;
    launch_attract<D>(s, pl->rc, pl->rstreams, pl->rb, pl->ip, pl->ix, pl->dx, xc, pl->dp1.p, frep,
                      pl->fprev.p, xn, pl->c);
  });
  GE_HIP(hipGetLastError());
  if (ev) GE_HIP(hipEventRecord(ev[2], s));
}

// All iterations of a small level (n <= grouped_cap, every row) in one launch of
// fa_grouped_persistent.  The grid must fit the device at its block occupancy:
// the lanes per row halve from grouped_lanes(n) until it does.  The launch is
// cooperative, so the runtime either makes the whole grid resident or refuses it.  Other work on the device (another rank's persistent kernel on the
// same GPU, another process) can still delay blocks past the barrier's ~2 s
// bound: then the start state (coordinates, previous forces) is restored and the
// caller runs the per-iteration path from it.  Returns false (nothing computed)
// when no G fits, the launch is refused or the barrier timed out;
// GE_PERSIST_REQUIRE=1 (tests) makes each of these an error.  The result is in
// Xa for an even iteration count, in Xb for an odd one.
constexpr int kPersistMin = 128;  // fewer iterations: per-iteration launches
template <int D>
bool launch_persistent(ge_fa_plan* pl, double* Xa, double* Xb, int iterations) {
  const int n = pl->n;
  if (n > grouped_cap(D) || pl->rb != 0 || pl->re != n) return false;
  hipStream_t s = pl->ctx->stream;
  // 64 lanes per row: the packed rows (packed_iteration) unless GE_FA_PACKED=0
  const bool packed_on = !(std::getenv("GE_FA_PACKED") && *std::getenv("GE_FA_PACKED") == '0');
  bool launched = false, fits = false, refused = false;
  DevBuf<int> bar;
  // the start state, restored when the barrier times out: taken only once a fitting
  // configuration is about to launch
  DevBuf<double> x0, f0;
  auto snapshot = [&] {
    if (x0.p) return;
    x0.alloc((size_t)n * D);
    f0.alloc((size_t)n * D);
    GE_HIP(hipMemcpyAsync(x0.p, Xa, sizeof(double) * n * D, hipMemcpyDeviceToDevice, s));
    GE_HIP(hipMemcpyAsync(f0.p, pl->fprev.p, sizeof(double) * n * D, hipMemcpyDeviceToDevice, s));
  };
  auto go = [&](auto GG) {
    constexpr int GC = decltype(GG)::value;
    const int nb = (n + kGrpT / GC - 1) / (kGrpT / GC);
    auto one = [&](auto RO, auto LI) {
      constexpr bool R1 = decltype(RO)::value, LIN = decltype(LI)::value;
      const bool pk = GC == 64 && packed_on;
      // packed rows per block: 4, or 6 where the blocks of 4 would not all be resident
      // at once.  Round 5 took 6 past one block of 4 per CU (C4's n = 1 068: 178 blocks
      // of 6 against 267 of 4); since the adder skips the batches no row needs (round
      // 6), 4 is faster at every size measured, 998-1 380 (16.1-16.6 against 16.9-17.1
      // us per iteration on the C4-sized fixture, profiles/r06/coarse_rows_sweep.log).
      // GE_FA_PACK_ROWS=4|6 overrides (tuning).
      auto kernel_of = [&](int r) {
        return !pk     ? reinterpret_cast<const void*>(&fa_grouped_persistent<D, GC, R1, LIN>)
               : r == 6 ? reinterpret_cast<const void*>(
                              &fa_grouped_persistent<D, GC, R1, LIN, GC == 64 ? 6 : 0>)
                        : reinterpret_cast<const void*>(
                              &fa_grouped_persistent<D, GC, R1, LIN, GC == 64 ? 4 : 0>);
      };
      auto lds_of = [&](int r) {
        return pk ? std::max(grouped_lds_bytes(n, D), packed_lds_bytes(n, D, r))
                  : grouped_lds_bytes(n, D);
      };
      auto occupancy = [&](int r) {
        const void* f = kernel_of(r);
        const size_t l = lds_of(r);
        if (l > 65536)
          GE_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l));
        int o = 0;
        GE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, f, kGrpT, l));
        return o;
      };
      int R = pk ? 4 : 0;
      if (const char* e = std::getenv("GE_FA_PACK_ROWS"); pk && e)
        R = std::atoi(e) == 6 ? 6 : 4;
      else if (pk && (long long)((n + 3) / 4) > (long long)occupancy(4) * pl->cus)
        R = 6;
      const int nbk = pk ? (n + R - 1) / R : nb;
      const size_t lds = lds_of(R);
      const void* fn = kernel_of(R);
      const int occ = occupancy(R);
      if ((long long)nbk > (long long)occ * pl->cus) return;  // the whole grid resident
      fits = true;
      int dev = 0, khz = 0;
      GE_HIP(hipGetDevice(&dev));
      GE_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
      const long long limit = (long long)std::max(khz, 1000) * 2000;  // ~2 s per barrier
      snapshot();
      bar.alloc(persist_bar_ints(nbk));
      GE_HIP(hipMemsetAsync(bar.p, 0, sizeof(int) * bar.n, s));
      int n_ = n, it_ = iterations;
      long long lim_ = limit;
      const int* ip_ = pl->ip;
      const int* ix_ = pl->ix;
      const double* dx_ = pl->dx;
      const double* dp_ = pl->dp1.p;
      FaConst c_ = pl->c;
      double* fp_ = pl->fprev.p;
      int* bar_ = bar.p;
      void* args[] = {&n_, &ip_, &ix_, &dx_, &Xa, &Xb, &dp_, &c_, &fp_, &bar_, &it_, &lim_};
      const hipError_t e = hipLaunchCooperativeKernel(fn, dim3(nbk), dim3(kGrpT), args,
                                                      (unsigned)lds, s);
      if (e == hipErrorCooperativeLaunchTooLarge) {
        (void)hipGetLastError();
        refused = true;
        return;
      }
      GE_HIP(e);
      launched = true;
    };
    const bool lin = !pl->c.linlog && pl->c.delta == 1.0;
    using T = std::true_type;
    using F = std::false_type;
    if (pl->c.repel == 1.0) {
      if (lin) one(T(), T());
      else one(T(), F());
    } else {
      if (lin) one(F(), T());
      else one(F(), F());
    }
  };
  for (int G = grouped_lanes(n); G >= 1 && !fits; G /= 2) {
    switch (G) {
      case 64: go(std::integral_constant<int, 64>()); break;
      case 32: go(std::integral_constant<int, 32>()); break;
      case 16: go(std::integral_constant<int, 16>()); break;
      case 8: go(std::integral_constant<int, 8>()); break;
      case 4: go(std::integral_constant<int, 4>()); break;
      case 2: go(std::integral_constant<int, 2>()); break;
      default: go(std::integral_constant<int, 1>()); break;
    }
  }
  const char* req = std::getenv("GE_PERSIST_REQUIRE");
  const bool require = req && *req == '1';
  if (!launched) {
    if (require)
      throw Error(GE_ERR_STATE, refused ? "forceAtlas: the cooperative launch was refused"
                                        : "forceAtlas: the persistent kernel does not fit");
    return false;
  }
  int err = 0;
  GE_HIP(hipMemcpyAsync(&err, bar.p + 1, sizeof(int), hipMemcpyDeviceToHost, s));
  GE_HIP(hipStreamSynchronize(s));
  if (err) {
    if (require)
      throw Error(GE_ERR_STATE,
                  "forceAtlas: the persistent small-level kernel's grid barrier timed out");
    std::fprintf(stderr, "libge: the persistent coarsest-level kernel's grid barrier timed out "
                         "(device shared?); rerunning per iteration\n");
    GE_HIP(hipMemcpyAsync(Xa, x0.p, sizeof(double) * n * D, hipMemcpyDeviceToDevice, s));
    GE_HIP(hipMemcpyAsync(pl->fprev.p, f0.p, sizeof(double) * n * D, hipMemcpyDeviceToDevice, s));
    GE_HIP(hipStreamSynchronize(s));
    return false;
  }
  return true;
}

void fa_run_device(ge_ctx* ctx, int n, int nnz, const int* d_ip, const int* d_ix,
                   const double* d_dx, int dim, double* d_x, int iterations,
                   const ge_fa_params& p) {
  if (n <= 0 || iterations <= 0) return;
  hipStream_t s = ctx->stream;
  // One workgroup wins only for tiny levels (n = 14: 3.7 against 12 us per
  // iteration); from n ~ 100 the multi-block grouped path does (n = 125: 17 us
  // against 26).  GE_SMALL_MAX moves the bound (tests use it up to kSmallMax).
  int small_max = kSmallDefault;
  if (const char* e = std::getenv("GE_SMALL_MAX")) small_max = std::min(kSmallMax, std::atoi(e));
  if (n <= small_max && p.mode == GE_MODE_STRICT) {
    DevBuf<double> dp1(n), fp((size_t)n * dim);
    DevBuf<int> it_state(1);
    hipLaunchKernelGGL(degp1_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, d_ip, d_dx,
                       p.use_weights, dp1.p);
    FaConst c = make_const(p);
    dispatch_dim(dim, [&](auto Dc) {
      constexpr int D = decltype(Dc)::value;
      launch_small<D>(s, n, nnz, d_ip, d_ix, d_dx, dp1.p, d_x, fp.p, it_state.p, iterations, c);
    });
    GE_HIP(hipGetLastError());
    GE_HIP(hipStreamSynchronize(s));
    return;
  }
  ge_fa_plan pl;
  pl.ctx = ctx;
  pl.n = n;
  pl.nnz = nnz;
  pl.dim = dim;
  pl.rb = 0;
  pl.re = n;
  pl.ip = d_ip;
  pl.ix = d_ix;
  pl.dx = d_dx;
  pl.p = p;
  pl.c = make_const(p);
  plan_init(&pl);
  sym_prepare(&pl);  // before any graph capture below
  DevBuf<double> other((size_t)n * dim);
  double* cur = d_x;
  double* nxt = other.p;
  int it = 0;
  if (p.mode == GE_MODE_STRICT && iterations >= kPersistMin && !std::getenv("GE_NO_PERSIST")) {
    bool done = false;
    dispatch_dim(dim, [&](auto Dc) {
      done = launch_persistent<decltype(Dc)::value>(&pl, d_x, other.p, iterations);
    });
    if (done) {
      if (iterations & 1)
        GE_HIP(hipMemcpyAsync(d_x, other.p, sizeof(double) * n * dim, hipMemcpyDeviceToDevice, s));
      GE_HIP(hipStreamSynchronize(s));
      return;
    }
  }
  // Long runs (the coarsest level's 1e5 iterations) replay a captured graph of
  // kGraphSteps iterations: host launch overhead would otherwise dominate the
  // microsecond-scale kernels of a small level.
  constexpr int kGraphSteps = 32;  // even: the buffers are back in place after a replay
  if (iterations >= 4 * kGraphSteps && !std::getenv("GE_NO_GRAPH")) {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    GE_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < kGraphSteps; ++k) {
      plan_step(&pl, cur, nxt);
      std::swap(cur, nxt);
    }
    GE_HIP(hipStreamEndCapture(s, &graph));
    try {
      GE_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
      for (; it + kGraphSteps <= iterations; it += kGraphSteps) GE_HIP(hipGraphLaunch(exec, s));
    } catch (...) {
      if (exec) (void)hipGraphExecDestroy(exec);
      (void)hipGraphDestroy(graph);
      throw;
    }
    GE_HIP(hipGraphExecDestroy(exec));
    GE_HIP(hipGraphDestroy(graph));
  }
  for (; it < iterations; ++it) {
    plan_step(&pl, cur, nxt);
    std::swap(cur, nxt);
  }
  if (cur != d_x)
    GE_HIP(hipMemcpyAsync(d_x, cur, sizeof(double) * n * dim, hipMemcpyDeviceToDevice, s));
  GE_HIP(hipStreamSynchronize(s));
  sym_check(&pl);
}

}  // namespace ge

extern "C" {

int ge_fa_plan_create(ge_ctx* ctx, int n, int nnz, const int* d_ip, const int* d_ix,
                      const double* d_dx, int dim, const ge_fa_params* p, int rb, int re,
                      ge_fa_plan** out) {
  return ge::guarded([&] {
    GE_REQUIRE(ctx && p && out, "null argument");
    GE_REQUIRE(n > 0 && dim >= 1 && dim <= 4, "bad n or dim (dim must be 1..4)");
    GE_REQUIRE(0 <= rb && rb <= re && re <= n, "bad row range");
    ge::DeviceGuard g(ctx);
    auto* pl = new ge_fa_plan();
    pl->ctx = ctx;
    pl->n = n;
    pl->nnz = nnz;
    pl->dim = dim;
    pl->rb = rb;
    pl->re = re;
    pl->ip = d_ip;
    pl->ix = d_ix;
    pl->dx = d_dx;
    pl->p = *p;
    pl->c = ge::make_const(*p);
    try {
      ge::plan_init(pl);
      // the symmetric path's tables now, not on the first step: that step may run on a
      // caller's stream under graph capture (ge_ctx_set_stream), where sym_prepare's
      // allocations and synchronisation are illegal
      ge::sym_prepare(pl);
    } catch (...) {
      delete pl;
      throw;
    }
    *out = pl;
  });
}

int ge_fa_plan_step(ge_fa_plan* pl, const double* xc, double* xn) {
  return ge::guarded([&] {
    GE_REQUIRE(pl && xc && xn && xc != xn, "bad plan step arguments");
    ge::DeviceGuard g(pl->ctx);
    ge::plan_step(pl, xc, xn);
  });
}

int ge_fa_plan_attract(ge_fa_plan* pl, const double* xc, const double* frep, double* xn) {
  return ge::guarded([&] {
    GE_REQUIRE(pl && xc && xn && frep && xc != xn, "bad plan attract arguments");
    ge::DeviceGuard g(pl->ctx);
    ge::plan_attract(pl, xc, frep, xn);
  });
}

int ge_fa_plan_set_profiling(ge_fa_plan* pl, int enable) {
  return ge::guarded([&] {
    GE_REQUIRE(pl, "null plan");
    pl->profiling = enable != 0;
    pl->next_event = 0;
  });
}

int ge_fa_plan_kernel_ms(ge_fa_plan* pl, double* rep_ms, double* attr_ms, int* launches) {
  return ge::guarded([&] {
    GE_REQUIRE(pl && rep_ms && attr_ms && launches, "null argument");
    ge::DeviceGuard g(pl->ctx);
    GE_HIP(hipStreamSynchronize(pl->ctx->stream));
    ge::sym_check(pl);
    double a = 0.0, b = 0.0;
    int cnt = 0;
    for (size_t k = 0; k + 3 <= pl->next_event; k += 3) {
      float t1 = 0.f, t2 = 0.f;
      GE_HIP(hipEventElapsedTime(&t1, pl->events[k], pl->events[k + 1]));
      GE_HIP(hipEventElapsedTime(&t2, pl->events[k + 1], pl->events[k + 2]));
      a += t1;
      b += t2;
      ++cnt;
    }
    *rep_ms = cnt ? a / cnt : 0.0;
    *attr_ms = cnt ? b / cnt : 0.0;
    *launches = cnt;
  });
}

// Waits for the plan's work; a symmetric launch whose hand-over wait timed out since
// the last step is reported here (GE_ERR_STATE) instead of being lost.  The plan is
// freed either way.
int ge_fa_plan_destroy(ge_fa_plan* pl) {
  return ge::guarded([&] {
    if (!pl) return;
    std::unique_ptr<ge_fa_plan> hold(pl);
    if (pl->sym_err_h) {
      GE_HIP(hipStreamSynchronize(pl->ctx->stream));
      ge::sym_check(pl);
    }
  });
}

}  // extern "C"
