// ge_sym.hpp -- all-pairs repulsion inside an aggregate with every unordered
// pair evaluated once (include/forceatlas.hpp:394-410 multilevel, :151-167),
// bit-exact with the reference's per-row serial sums.
//
// The term of j on i and the term of i on j are exact negatives:
// x_j - x_i = -(x_i - x_j) in RN, the squared distance and dis are shared,
// (deg_i+1)(deg_j+1) is commutative, and a quotient / product of a negated
// operand is the negated result.  Adding -t equals subtracting t.  So one
// evaluation of t(i, j) serves row i (+t) and row j (-t); what has to be kept is
// each row's ORDER of additions: partners ascending.
//
// Schedule.  Members are split into tiles of 64.  A wave owns a row tile A and
// sweeps the columns j >= 64A in ascending order as a systolic array: at step
// s lane l evaluates the pair (row 64A+l, column s-l), so
//   * row l's own sum (lane register) receives its partners j > row in order;
//   * column q's sum travels one lane per step (DPP wave shift), entering lane 0
//     with the value the rows of earlier tiles left in F and collecting the rows
//     of this tile in ascending order before it leaves lane 63 back to F.
// In the diagonal tile, column q's travelling sum (partners < q of the tile,
// after those of earlier tiles) reaches lane q exactly when that lane starts its
// own row, and becomes the row's sum.  Row 64A+l therefore adds, in order:
// partners of tiles < A (sweeps 0..A-1, as a column), partners < itself in tile
// A (travelling), partners > itself (own sweep) -- the reference's order.
//
// Dependencies: the sweep of row tile A may start column tile B only after the
// sweeps 0..A-1 have written it back (prog[B] == A).  Sweeps are taken from a
// queue ordered by their earliest possible start (2A tile-times after the
// aggregate's first sweep): every sweep waits only on sweeps taken before it,
// which are running, so the persistent grid cannot deadlock.  Column sums are
// handed over with agent-scope (L2-bypassing) stores and loads: the waves of
// one aggregate run on different XCDs, whose L2s are not coherent.
#pragma once

#include <hip/hip_runtime.h>

#include "ge_pair.hpp"
#include "ge_rows.hpp"

namespace ge {

constexpr int kSymT = 256;  // threads per block (4 independent waves)

template <int D>
struct SymW {
  static constexpr int v = (D + 1 <= 4) ? 4 : 8;  // record: x[D], deg+1, pad
};

// Wave-wide shift by one lane (DPP wave_shr:1): lane l receives v of lane l-1,
// lane 0 keeps in0 (no source lane: the DPP move leaves the destination alone).
__device__ __forceinline__ double wave_shift_in(double v, double in0) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(in0), __double2loint(v), 0x138, 0xF,
                                             0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(in0), __double2hiint(v), 0x138, 0xF,
                                             0xF, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double agent_ld(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void agent_st(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kSymRing = 128;  // LDS ring of column slots (column q at q & 127)

template <int D>
struct SymI {
  static constexpr int v = D;  // column-sum slot width (3 KB per 128-slot ring at D = 3)
};

// Steps [s0, s1) of a sweep.  DIAG: the steps may meet the diagonal tile
// (s < 127), where a lane takes the travelling sum of its own row over.  The LDS
// reads of step s + 1 (entering column sum, partner record) are issued before
// step s computes: both were staged before the steps began.
template <int D, bool SHARED, bool REPEL_ONE, bool DIAG>
__device__ __forceinline__ void sym_step(int sg, int lane, int ncols, double* out,
                                         const double (&xr)[D], double dr, bool rv, double repel,
                                         const double (&in0)[D], const double (&xq)[D + 1],
                                         double (&racc)[D], double (&flow)[D]) {
  constexpr int IW = SymI<D>::v;
  // column sg enters lane 0 with its stored sum
#pragma unroll
  for (int k = 0; k < D; ++k) flow[k] = wave_shift_in(flow[k], in0[k]);
  if (DIAG && sg - lane == lane) {
#pragma unroll
    for (int k = 0; k < D; ++k) racc[k] = flow[k];
  }
  // Every lane evaluates a term every step (no divergent exec mask): a pair with
  // an inert row or column (deg+1 = 0) and the self pair are +-0, which leave a
  // sum unchanged; below the diagonal (before its own row starts) a lane's racc
  // and the absorbed columns' sums are dead values.
  double t[D];
  rep_term<D, SHARED, REPEL_ONE>(xr, xq, dr, xq[D], repel, t);
  if (!SHARED && DIAG && sg - lane == lane) {  // the `/` form skips the self pair (ge_pair.hpp)
#pragma unroll
    for (int k = 0; k < D; ++k) t[k] = 0.0;
  }
#pragma unroll
  for (int k = 0; k < D; ++k) {
    racc[k] = racc[k] + t[k];
    flow[k] = flow[k] - t[k];
  }
  if (lane == 63) {  // column sg - 63 leaves the wave
    double* o = out + ((sg - 63) & (kSymRing - 1)) * IW;
#pragma unroll
    for (int k = 0; k < D; ++k) o[k] = flow[k];
  }
}

// LDS reads of one step: the entering column sum (broadcast) and the partner record
template <int D>
__device__ __forceinline__ void sym_fetch(int sg, int lane, const double* rec, const double* ini,
                                          double (&i0)[D], double (&xv)[D + 1]) {
  constexpr int WV = SymW<D>::v;
  constexpr int IW = SymI<D>::v;
  const double* ic = ini + (sg & (kSymRing - 1)) * IW;
  // records are stored by component (rec[k][slot]): consecutive lanes read
  // consecutive slots, no bank conflicts
  const int slot = (sg - lane) & (kSymRing - 1);
#pragma unroll
  for (int k = 0; k < D; ++k) i0[k] = ic[k];
#pragma unroll
  for (int k = 0; k <= D; ++k) xv[k] = rec[k * kSymRing + slot];
}

// Steps [s0, s1) of a sweep.  DIAG: the steps may meet the diagonal tile
// (s < 127), where a lane takes the travelling sum of its own row over.  The LDS
// reads of step s + 1 are issued before step s computes (both slots were staged
// before the steps began); two register sets alternate.
template <int D, bool SHARED, bool REPEL_ONE, bool DIAG>
__device__ __forceinline__ void sym_steps(int s0, int s1, int lane, int ncols, const double* rec,
                                          const double* ini, double* out,
                                          const double (&xr)[D], double dr, bool rv, double repel,
                                          double (&racc)[D], double (&flow)[D]) {
  if (s0 >= s1) return;
  double ia[D], xa[D + 1], ib[D], xb[D + 1];
  sym_fetch<D>(s0, lane, rec, ini, ia, xa);
  for (int sg = s0;; sg += 2) {
    sym_fetch<D>(sg + 1, lane, rec, ini, ib, xb);
    sym_step<D, SHARED, REPEL_ONE, DIAG>(sg, lane, ncols, out, xr, dr, rv, repel, ia, xa, racc,
                                         flow);
    if (sg + 1 >= s1) break;
    sym_fetch<D>(sg + 2, lane, rec, ini, ia, xa);
    sym_step<D, SHARED, REPEL_ONE, DIAG>(sg + 1, lane, ncols, out, xr, dr, rv, repel, ib, xb,
                                         racc, flow);
    if (sg + 2 >= s1) break;
  }
}

// Column tile t of the sweep has left lane 63: write its sums back, then let the
// next sweep of the aggregate have it.
template <int D>
__device__ __forceinline__ void sym_handover(int t, int lane, int A, int ncols, size_t cbase,
                                             const double* out, double* F, int* tprog) {
  constexpr int IW = SymI<D>::v;
  wave_lds_sync();
  const int qo = 64 * t + lane;
  if (qo < ncols) {
    const double* o = out + (qo & (kSymRing - 1)) * IW;
#pragma unroll
    for (int k = 0; k < D; ++k) agent_st(F + (cbase + qo) * D + k, o[k]);
  }
  // Ordering (no acquire/release: an agent-scope release would write back the whole
  // L2, ~every 64 steps): the sums are agent-scope stores (they bypass the per-XCD
  // L2), s_waitcnt(0) waits until every one of them has completed at the memory
  // side, and only then is the flag stored.  The signal fences keep the compiler
  // from moving the stores across the wait or the flag store.
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0);  // every lane's sums are stored before the flag
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if (lane == 0) __hip_atomic_store(tprog + t, A + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int D, bool REPEL_ONE, bool DIAG>
__device__ __forceinline__ void sym_steps_any(bool fast, int s0, int s1, int lane, int ncols,
                                              const double* rec, const double* ini, double* out,
                                              const double (&xr)[D], double dr, bool rv,
                                              double repel, double (&racc)[D], double (&flow)[D]) {
  if (fast)
    sym_steps<D, true, REPEL_ONE, DIAG>(s0, s1, lane, ncols, rec, ini, out, xr, dr, rv, repel,
                                        racc, flow);
  else
    sym_steps<D, false, REPEL_ONE, DIAG>(s0, s1, lane, ncols, rec, ini, out, xr, dr, rv, repel,
                                         racc, flow);
}

// A row block of 64 rows against all s members in ascending order, every pair
// evaluated for its row (the plain ordered-pair scheme: no dependencies).  Used
// for aggregates whose sweep chain would outlast the rest of the launch.
template <int D, bool REPEL_ONE>
__device__ __forceinline__ void rows_block(int lane, int base, int s, int A, const double* X,
                                           const double* DP, double repel, bool repel_ok,
                                           double* tile, double* F) {
  constexpr int WV = SymW<D>::v;
  const size_t rb = (size_t)base + 64 * (size_t)A;
  const bool rv = 64 * A + lane < s;
  double xi[D], acc[D], di = 1.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    xi[k] = rv ? X[(rb + lane) * D + k] : 0.0;
    acc[k] = 0.0;
  }
  if (rv) di = DP[rb + lane];
  const bool rows_ok = repel_ok && __all(!rv || vertex_ok<D>(xi, di));
  for (int j0 = 0; j0 < s; j0 += 64) {
    const int cnt = min(64, s - j0);
    wave_lds_sync();  // the previous tile has been read by every lane
    bool ok = true;
    if (lane < cnt) {
      const size_t c = (size_t)base + j0 + lane;
#pragma unroll
      for (int k = 0; k < D; ++k) tile[lane * WV + k] = X[c * D + k];
      tile[lane * WV + D] = DP[c];
      ok = vertex_ok<D>(&tile[lane * WV], tile[lane * WV + D]);
    }
    wave_lds_sync();
    if (rows_ok && __all(ok)) {
      for (int jj = 0; jj < cnt; ++jj)  // the j == i term is +-0 (ge_pair.hpp)
        rep_pair<D, true, REPEL_ONE>(xi, &tile[jj * WV], di, tile[jj * WV + D], repel, acc);
    } else {
      for (int jj = 0; jj < cnt; ++jj)
        rep_pair_fb<D, REPEL_ONE>(xi, &tile[jj * WV], di, tile[jj * WV + D], repel,
                                  j0 + jj == 64 * A + lane, acc);
    }
  }
  if (rv) {
#pragma unroll
    for (int k = 0; k < D; ++k) F[(rb + lane) * D + k] = acc[k];
  }
  wave_lds_sync();
}

// units[q] = {aggregate, row tile A, offset of the aggregate's tiles in prog,
// kind (0: symmetric sweep, 1: row block)} in queue order; prog zeroed before the
// launch; queue = one counter.
// 4 waves per SIMD: <= 128 VGPRs, 40 KB of LDS per block (D = 3)
template <int D, bool REPEL_ONE>
__global__ void __launch_bounds__(kSymT, 4)
faml_sym_repulse(int nunits, const int4* __restrict__ units, int* __restrict__ queue,
                 const int* __restrict__ pt_ip, const double* __restrict__ X,
                 const double* __restrict__ DP, double repel, double* __restrict__ F,
                 int* __restrict__ prog) {
  constexpr int WV = SymW<D>::v;
  constexpr int IW = SymI<D>::v;
  constexpr int NW = kSymT / 64;
  __shared__ __attribute__((aligned(16))) double srec[NW][kSymRing * WV];
  __shared__ __attribute__((aligned(16))) double sini[NW][kSymRing * IW];
  __shared__ __attribute__((aligned(16))) double sout[NW][kSymRing * IW];
  const int lane = threadIdx.x & 63;
  double* rec = srec[threadIdx.x >> 6];
  double* ini = sini[threadIdx.x >> 6];
  double* out = sout[threadIdx.x >> 6];
  const bool repel_ok = REPEL_ONE || weight_ok(repel);
  for (;;) {
    int qi = 0;
    if (lane == 0) qi = atomicAdd(queue, 1);
    qi = __builtin_amdgcn_readfirstlane(qi);
    if (qi >= nunits) break;  // every wave leaves once the queue is drained
    const int4 u = units[qi];
    const int A = u.y;
    const int base = pt_ip[u.x];
    const int s = pt_ip[u.x + 1] - base;
    if (u.w) {
      // a row block spans its aggregate's whole width: the launch's critical path
      // when the aggregate is large, so its wave takes issue priority on the SIMD
      __builtin_amdgcn_s_setprio(3);
      rows_block<D, REPEL_ONE>(lane, base, s, A, X, DP, repel, repel_ok, rec, F);
      __builtin_amdgcn_s_setprio(0);
      continue;
    }
    int* tprog = prog + u.z + A;  // tprog[t]: column tile A + t
    const size_t cbase = (size_t)base + 64 * (size_t)A;
    const bool rv = 64 * A + lane < s;
    double xr[D], racc[D], flow[D], dr = 0.0;  // a row past the aggregate is inert
#pragma unroll
    for (int k = 0; k < D; ++k) {
      xr[k] = rv ? X[(cbase + lane) * D + k] : 0.0;
      racc[k] = 0.0;
      flow[k] = 0.0;
    }
    if (rv) dr = DP[cbase + lane];
    const bool rows_ok = repel_ok && __all(!rv || vertex_ok<D>(xr, dr));
    const int ncols = s - 64 * A;
    const int ntiles = (ncols + 63) >> 6;
    bool ok_prev = true;
    for (int tt = 0; tt < ntiles; ++tt) {
      if (A > 0) {  // the sweeps 0..A-1 have written column tile A + tt back
        while (__hip_atomic_load(tprog + tt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < A)
          __builtin_amdgcn_s_sleep(1);
        // the F loads below are agent-scope (served past the L2) and issued only after
        // the spin has seen the flag (the loop's exit depends on the loaded value); the
        // fence keeps the compiler from hoisting them above the loop
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
      }
      const int qc = 64 * tt + lane;
      const bool cv = qc < ncols;
      double xc[D], ic[D], dc = 0.0;  // a column past the aggregate is inert
#pragma unroll
      for (int k = 0; k < D; ++k) {
        xc[k] = cv ? X[(cbase + qc) * D + k] : 0.0;
        ic[k] = (cv && A > 0) ? agent_ld(F + (cbase + qc) * D + k) : 0.0;
      }
      if (cv) dc = DP[cbase + qc];
      const bool ok_cur = __all(!cv || vertex_ok<D>(xc, dc));
      double* rs = rec + (qc & (kSymRing - 1));
      double* is = ini + (qc & (kSymRing - 1)) * IW;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        rs[k * kSymRing] = xc[k];
        is[k] = ic[k];
      }
      rs[D * kSymRing] = dc;
      wave_lds_sync();
      // the steps of tile tt read tiles tt-1 and tt; the diagonal meets steps < 127
      const bool fast = rows_ok && ok_cur && ok_prev;
      if (tt < 2)
        sym_steps_any<D, REPEL_ONE, true>(fast, 64 * tt, 64 * tt + 64, lane, ncols, rec, ini, out,
                                          xr, dr, rv, repel, racc, flow);
      else
        sym_steps_any<D, REPEL_ONE, false>(fast, 64 * tt, 64 * tt + 64, lane, ncols, rec, ini,
                                           out, xr, dr, rv, repel, racc, flow);
      ok_prev = ok_cur;
      if (tt >= 2) sym_handover<D>(tt - 1, lane, A, ncols, cbase, out, F, tprog);
      wave_lds_sync();  // the slots of tile tt-1 are free for tile tt+1
    }
    {  // drain: the last columns cross the wave; the slots past them hold inert records
      double* rs = rec + ((64 * ntiles + lane) & (kSymRing - 1));
      double* is = ini + ((64 * ntiles + lane) & (kSymRing - 1)) * IW;
#pragma unroll
      for (int k = 0; k <= D; ++k) rs[k * kSymRing] = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) is[k] = 0.0;
      wave_lds_sync();
    }
    const int s0 = 64 * ntiles, s1 = ncols + 63;
    if (ntiles < 2)
      sym_steps_any<D, REPEL_ONE, true>(rows_ok && ok_prev, s0, s1, lane, ncols, rec, ini, out,
                                        xr, dr, rv, repel, racc, flow);
    else
      sym_steps_any<D, REPEL_ONE, false>(rows_ok && ok_prev, s0, s1, lane, ncols, rec, ini, out,
                                         xr, dr, rv, repel, racc, flow);
    if (ntiles >= 2) sym_handover<D>(ntiles - 1, lane, A, ncols, cbase, out, F, tprog);
    if (rv) {
#pragma unroll
      for (int k = 0; k < D; ++k) F[(cbase + lane) * D + k] = racc[k];
    }
    wave_lds_sync();
  }
}

}  // namespace ge
