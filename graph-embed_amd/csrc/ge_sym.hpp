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
//   * column q's sum travels one lane per step (through its slot of the wave's LDS
//     column ring: lane l + 1 reads at step s + 1 what lane l wrote at step s),
//     entering lane 0 with the value the sweeps of earlier tiles handed over and
//     collecting the rows of this tile in ascending order before it leaves lane 63.
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

__device__ __forceinline__ double agent_ld(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void agent_st(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ long long rt_now() { return (long long)__builtin_amdgcn_s_memrealtime(); }

// LDS of one sweep wave (round 5).  Column q of the sweep (q = column - 64 A) keeps
// its running sum in LDS, in its slot of the column ring `col` (D components,
// kColSlots slots each): at step s lane l reads the sum of column s - l, subtracts its
// term and writes it back, and one step later lane l + 1 reads what lane l wrote --
// one wave's DS instructions execute in issue order, and a compiler barrier between
// the steps keeps their order in the code.  Before round 5 the sums travelled in
// registers one lane per step (a DPP wave shift: 6 moves per step at D = 3) with a
// broadcast read of the entering sum and a predicated store of the leaving one; here
// none of them.  The column's entering sum (from the sweeps before) is staged into its
// slot, and its final sum is in the slot once lane 63 has passed it.
// During column tile tt the steps touch tiles tt - 1 and tt; they sit side by side,
// tile tt - 1 at slots 0..63 and tile tt at 64..127, so lane l reads slot 64 - l + j at
// step 64 tt + j, never wrapping: the current tile moves down to 0..63 (one LDS copy
// per lane and component) before the next one is staged above it.  (Round 5 kept
// column q at slot q & 127, which wrapped inside the even tiles: one select per step
// there, 53-54 VALU per step against 50.  A 192-slot ring that moved only the even
// tiles ran as fast but its 6 KB more LDS per block locked the resident classes'
// kernels out of the CUs during the repulsion launch: attraction passes 4.48 against
// 3.54 ms, profiles/r06/ab_colring.log.)
// Records {x[D], deg+1} are component-major in the ring `rec` (D + 1 components,
// kRecSlots slots each): column q at slot q & 127, and slots 0..63 mirrored at
// 128..191, so that within a column tile every lane reads slot ((64 tt - l) & 127) + j
// at step 64 tt + j without wrapping: the per-step addresses are immediate offsets.
constexpr int kColSlots = 128;  // column ring: tile tt - 1 at 0..63, tile tt at 64..127
constexpr int kSymRing = 128;   // record ring period (column q at q & 127)
constexpr int kRecSlots = 192;  // record ring: 128 slots + the first 64 mirrored
constexpr int kColBase = 64;    // the current tile's first slot

// Compiler barrier between two steps: the next step's reads of the column ring
// must stay after this step's writes (different slots for one lane, the same slot
// for the next lane: a cross-lane dependency the compiler cannot see).  Under the
// HIP memory model this hand-off between lanes is a data race; it is correct because
// one wave's DS instructions execute in issue order and the barrier keeps the issue
// order.  A compiler that reordered DS operations across an asm memory clobber, or
// hardware that completed them out of order, would change the bits: the canaries are
// tests/test_gpu_parity.py::test_faml_symmetric_sweeps, ::test_fa_symmetric_repulsion*,
// test_gpu_configs.py::test_c4_level0_oracle_at_embed_horizon (100 iterations at C4
// against the oracle) and the 1e5-iteration coarsest fixture.
__device__ __forceinline__ void step_barrier() { asm volatile("" ::: "memory"); }

// One step of a sweep at any position (runtime step index sg): the diagonal tiles
// (DIAG: a lane takes its own row's sum over from the column that reaches it), the
// drain, and tiles outside the shared-reciprocal domain (SHARED = false).
// coff: kColBase - 64 tt of the step's tile (column q at slot coff + q).
template <int D, bool SHARED, bool REPEL_ONE, bool DIAG>
__device__ __forceinline__ void col_step(int sg, int lane, int coff, const double* rec, double* col,
                                         const double (&xr)[D], double dr, double repel,
                                         double (&racc)[D]) {
  const int q = sg - lane;
  const int p = q & (kSymRing - 1);
  const int pc = coff + q;
  double xq[D + 1], c[D];
#pragma unroll
  for (int k = 0; k <= D; ++k) xq[k] = rec[k * kRecSlots + p];
#pragma unroll
  for (int k = 0; k < D; ++k) c[k] = col[k * kColSlots + pc];
  if (DIAG && q == lane) {  // column q = this lane's row: its sum so far is the row's
#pragma unroll
    for (int k = 0; k < D; ++k) racc[k] = c[k];
  }
  // Every lane evaluates a term every step (no divergent exec mask): a pair with
  // an inert row or column (deg+1 = 0) and the self pair are +-0, which leave a
  // sum unchanged; below the diagonal (before its own row starts) a lane's racc
  // and the absorbed columns' sums are dead values.
  double t[D];
  rep_term<D, SHARED, REPEL_ONE>(xr, xq, dr, xq[D], repel, t);
  if (!SHARED && DIAG && q == lane) {  // the `/` form skips the self pair (ge_pair.hpp)
#pragma unroll
    for (int k = 0; k < D; ++k) t[k] = 0.0;
  }
#pragma unroll
  for (int k = 0; k < D; ++k) {
    racc[k] = racc[k] + t[k];
    col[k * kColSlots + pc] = c[k] - t[k];
  }
  step_barrier();
}

template <int D, bool REPEL_ONE, bool DIAG>
__device__ __forceinline__ void col_steps(bool fast, int s0, int s1, int lane, int coff,
                                          const double* rec, double* col, const double (&xr)[D],
                                          double dr, double repel, double (&racc)[D]) {
  if (fast)
    for (int sg = s0; sg < s1; ++sg)
      col_step<D, true, REPEL_ONE, DIAG>(sg, lane, coff, rec, col, xr, dr, repel, racc);
  else
    for (int sg = s0; sg < s1; ++sg)
      col_step<D, false, REPEL_ONE, DIAG>(sg, lane, coff, rec, col, xr, dr, repel, racc);
}

// The 64 steps of a full column tile tt >= 2 in the shared-reciprocal domain (the
// bulk of every sweep): eight blocks of eight steps, every LDS access an immediate
// offset from a per-block base, the same code in odd and even tiles.  No prefetch of
// the next step's records into a second register set: the other waves of the SIMD
// hide the LDS latency, and the kernel must stay within 120 VGPRs (see
// faml_sym_repulse).
template <int D, bool REPEL_ONE>
__device__ __forceinline__ void tile_steps(int tt, int lane, const double* rec, double* col,
                                           const double (&xr)[D], double dr, double repel,
                                           double (&racc)[D]) {
  const double* rb = rec + ((64 * tt - lane) & (kSymRing - 1));
  double* cb = col + kColBase - lane;
  for (int j0 = 0; j0 < 64; j0 += 8) {
    const double* rj = rb + j0;
    double* cj = cb + j0;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      double* cp = cj + jj;
      double c[D], xq[D + 1];
#pragma unroll
      for (int k = 0; k <= D; ++k) xq[k] = rj[k * kRecSlots + jj];
#pragma unroll
      for (int k = 0; k < D; ++k) c[k] = cp[k * kColSlots];
      double t[D];
      rep_term<D, true, REPEL_ONE>(xr, xq, dr, xq[D], repel, t);
#pragma unroll
      for (int k = 0; k < D; ++k) {
        racc[k] = racc[k] + t[k];
        cp[k * kColSlots] = c[k] - t[k];
      }
      step_barrier();
    }
  }
}

// Hand-over slot of member c, dimension k: component-major H[k * hs + c].
template <int D>
__device__ __forceinline__ double* hand_at(double* H, size_t hs, size_t c, int k) {
  return H + k * hs + c;
}

// Column tile t of the sweep has left lane 63: write its sums back, then let the
// next sweep of the aggregate have it (tprog[t] = done: row tiles < done added).
// The hand-over buffer H is component-major (H[k * hs + c]): each of the D store
// instructions covers 512 contiguous bytes (8 lines) instead of the 24 lines a
// 24-byte-strided record store spans, which the agent-scope stores pay per line.
// `at`: the column ring slot of the tile's first column (0: it has moved down, the
// tile after it is current).
template <int D>
__device__ __forceinline__ void sym_handover(int t, int lane, int done, int ncols, size_t cbase,
                                             const double* col, int at, double* H, size_t hs,
                                             int* tprog) {
  wave_lds_sync();
  const int qo = 64 * t + lane;
  if (qo < ncols) {
    const double* o = col + at + lane;
#pragma unroll
    for (int k = 0; k < D; ++k) agent_st(hand_at<D>(H, hs, cbase + qo, k), o[k * kColSlots]);
  }
  // Ordering (no acquire/release: an agent-scope release would write back the whole
  // L2, ~every 64 steps): the sums are agent-scope stores (they bypass the per-XCD
  // L2), s_waitcnt(0) waits until every one of them has completed at the memory
  // side, and only then is the flag stored.  The signal fences keep the compiler
  // from moving the stores across the wait or the flag store.
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0);  // every lane's sums are stored before the flag
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if (lane == 0) __hip_atomic_store(tprog + t, done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The counter as the wave sees it, made wave-uniform so the wait loop below is a
// scalar loop: a per-lane exit test would make the compiler treat the loop as
// divergent and hold its counters in VGPRs, which costs the plain kernel the
// two registers that keep it at 120 (3 waves/SIMD beside the resident kernels).
__device__ __forceinline__ int seen(const int* flag) {
  return __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Wait until a column tile's progress counter reaches A.  Bounded: a wait longer
// than `limit` ticks of the 100 MHz clock, or one another wave already reported
// in *err, makes the wave give up waiting for the rest of the launch (and report
// in *err as it leaves), so a scheduling bug ends the launch (with wrong sums and
// an error the host reports) instead of hanging the device.  The store is kept out
// of the loop: inside it, at the kernel's register peak, it cost two VGPRs.
// Returns the ticks spent when STAMP.
// system scope: err may be pinned host memory (single-level plans)
__device__ __forceinline__ void report_give_up(bool give_up, int lane, int* err) {
  if (give_up && lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool STAMP>
__device__ __forceinline__ long long handover_wait(const int* flag, int A, int* err,
                                                   long long limit, bool& give_up) {
  if (give_up) return 0;
  if (seen(flag) >= A) return 0;
  const long long t0 = rt_now();
  for (int k = 1;; ++k) {
    __builtin_amdgcn_s_sleep(1);
    if (seen(flag) >= A) break;
    if ((k & 255) == 0 &&
        (rt_now() - t0 > limit ||
         __builtin_amdgcn_readfirstlane(
             __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)))) {
      give_up = true;  // the kernel reports it on its way out (report_give_up)
      break;
    }
  }
  return STAMP ? rt_now() - t0 : 0;
}

// Issue priority of a row block with `rem` column tiles left: one level per
// `quantum` tiles (capped at 3), so on each SIMD the wave with the most work left
// issues first (longest remaining first).  Equal priorities fall back to the oldest
// wave, which let one wave per SIMD run ahead through the queue while the other two
// starved on the units they took at the start and finished last: on an N = 8 share
// of C4 those units ran 15-25 ms against 5 ms, the launch's tail.
__device__ __forceinline__ void rows_prio(int rem, int quantum) {
  const int lv = quantum > 0 ? rem / quantum : 3;
  if (lv >= 3) __builtin_amdgcn_s_setprio(3);
  else if (lv == 2) __builtin_amdgcn_s_setprio(2);
  else if (lv == 1) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

// A row block: the 64 rows of tile A against all s members in ascending order,
// every pair evaluated for its row (the plain ordered-pair scheme: no dependencies),
// sums from +0, the rows' final sums to F.  Used for whole aggregates whose sweep
// chain would outlast the launch (the shares of a multi-GPU run).  tile: 64
// records of SymW<D> doubles in LDS.  quantum: see rows_prio (0: priority 3).
template <int D, bool REPEL_ONE>
__device__ __forceinline__ void rows_block(int lane, int base, int s, int A, const double* X,
                                           const double* DP, double repel, bool repel_ok,
                                           double* tile, double* F, int quantum) {
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
    rows_prio((s - j0) >> 6, quantum);
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
      // two partners per iteration: their terms are independent instruction chains
      // the scheduler can interleave; the adds stay in partner order
      int jj = 0;
      for (; jj + 1 < cnt; jj += 2) {  // the j == i term is +-0 (ge_pair.hpp)
        double t0[D], t1[D];
        rep_term<D, true, REPEL_ONE>(xi, &tile[jj * WV], di, tile[jj * WV + D], repel, t0);
        rep_term<D, true, REPEL_ONE>(xi, &tile[(jj + 1) * WV], di, tile[(jj + 1) * WV + D], repel,
                                     t1);
#pragma unroll
        for (int k = 0; k < D; ++k) acc[k] = (acc[k] + t0[k]) + t1[k];
      }
      if (jj < cnt)
        rep_pair<D, true, REPEL_ONE>(xi, &tile[jj * WV], di, tile[jj * WV + D], repel, acc);
    } else {
      for (int jj = 0; jj < cnt; ++jj)
        rep_pair_fb<D, REPEL_ONE>(xi, &tile[jj * WV], di, tile[jj * WV + D], repel,
                                  j0 + jj == 64 * A + lane, acc);
    }
  }
  wave_lds_sync();
  __builtin_amdgcn_s_setprio(0);
  if (rv) {
#pragma unroll
    for (int k = 0; k < D; ++k) F[(rb + lane) * D + k] = acc[k];
  }
}

// Per-unit timeline of one launch (STAMP builds only, GE_SYM_STAMPS): 8 words per
// unit in queue order -- s_memrealtime (100 MHz, one clock for the whole chip)
// when the wave took the unit, when its first column tile was handed over, when it
// finished, the ticks spent spinning on hand-overs, HW_ID and XCC_ID.
constexpr int kStampWords = 8;


// One symmetric sweep (unit kind 0): row tile A against the columns >= 64A, the
// column sums handed to the next sweep tile by tile.  rec / col: this wave's rings
// (see kSymRing).  STAMP: spin ticks and the first hand-over time.
template <int D, bool REPEL_ONE, bool STAMP>
__device__ __forceinline__ void sweep_unit(int lane, int A, int base, int s, int* tprog,
                                           const double* __restrict__ X,
                                           const double* __restrict__ DP, double repel,
                                           bool repel_ok, double* __restrict__ F,
                                           double* __restrict__ H, size_t hs, int* err,
                                           long long limit, bool& give_up, double* rec,
                                           double* col, long long& spin, long long& t_first,
                                           double (&rout)[D]) {
  const size_t cbase = (size_t)base + 64 * (size_t)A;
  const bool rv = 64 * A + lane < s;
  double xr[D], racc[D], dr = 0.0;  // a row past the aggregate is inert
#pragma unroll
  for (int k = 0; k < D; ++k) {
    xr[k] = rv ? X[(cbase + lane) * D + k] : 0.0;
    racc[k] = 0.0;
  }
  if (rv) dr = DP[cbase + lane];
  const bool rows_ok = repel_ok && __all(!rv || vertex_ok<D>(xr, dr));
  const int ncols = s - 64 * A;
  const int ntiles = (ncols + 63) >> 6;
  bool ok_prev = true;
  for (int tt = 0; tt < ntiles; ++tt) {
    if (A > 0) {  // the sweeps 0..A-1 have written column tile A + tt back
      const long long w = handover_wait<STAMP>(tprog + tt, A, err, limit, give_up);
      if (STAMP) {
        spin += w;
        if (tt == 0) t_first = rt_now();
      }
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
      ic[k] = (cv && A > 0) ? agent_ld(hand_at<D>(H, hs, cbase + qc, k)) : 0.0;
    }
    if (cv) dc = DP[cbase + qc];
    const bool ok_cur = __all(!cv || vertex_ok<D>(xc, dc));
    const int p = qc & (kSymRing - 1);
    if (tt > 0) {  // the tile before moves down to 0..63 (its hand-over has read 0..63)
#pragma unroll
      for (int k = 0; k < D; ++k) col[k * kColSlots + lane] = col[k * kColSlots + kColBase + lane];
    }
    const int cb = kColBase;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      rec[k * kRecSlots + p] = xc[k];
      col[k * kColSlots + cb + lane] = ic[k];  // the column enters with its sum so far
    }
    rec[D * kRecSlots + p] = dc;
    if (!(tt & 1)) {  // slots 0..63 are mirrored at 128..191
#pragma unroll
      for (int k = 0; k < D; ++k) rec[k * kRecSlots + p + kSymRing] = xc[k];
      rec[D * kRecSlots + p + kSymRing] = dc;
    }
    wave_lds_sync();
    // the steps of tile tt read tiles tt-1 and tt; the diagonal meets steps < 127
    const bool fast = rows_ok && ok_cur && ok_prev;
    const int coff = cb - 64 * tt;
    if (tt < 2)
      col_steps<D, REPEL_ONE, true>(fast, 64 * tt, 64 * tt + 64, lane, coff, rec, col, xr, dr,
                                    repel, racc);
    else if (fast)
      tile_steps<D, REPEL_ONE>(tt, lane, rec, col, xr, dr, repel, racc);
    else
      col_steps<D, REPEL_ONE, false>(false, 64 * tt, 64 * tt + 64, lane, coff, rec, col, xr, dr,
                                     repel, racc);
    ok_prev = ok_cur;
    if (tt >= 2) sym_handover<D>(tt - 1, lane, A + 1, ncols, cbase, col, cb - 64, H, hs, tprog);
    wave_lds_sync();  // the slots of tile tt-1 are free for tile tt+1
  }
  {  // drain: the last columns cross the wave; the slots past them hold inert records
    const int p = (64 * ntiles + lane) & (kSymRing - 1);
#pragma unroll
    for (int k = 0; k <= D; ++k) {
      rec[k * kRecSlots + p] = 0.0;
      if (!(ntiles & 1)) rec[k * kRecSlots + p + kSymRing] = 0.0;
    }
    // the drain is tile ntiles: the last tile moves down to 0..63
#pragma unroll
    for (int k = 0; k < D; ++k) col[k * kColSlots + lane] = col[k * kColSlots + kColBase + lane];
    wave_lds_sync();
  }
  const int s0 = 64 * ntiles, s1 = ncols + 63;
  const int cbd = kColBase, coff = cbd - 64 * ntiles;
  if (ntiles < 2)
    col_steps<D, REPEL_ONE, true>(rows_ok && ok_prev, s0, s1, lane, coff, rec, col, xr, dr, repel,
                                  racc);
  else
    col_steps<D, REPEL_ONE, false>(rows_ok && ok_prev, s0, s1, lane, coff, rec, col, xr, dr, repel,
                                   racc);
  if (ntiles >= 2)
    sym_handover<D>(ntiles - 1, lane, A + 1, ncols, cbase, col, cbd - 64, H, hs, tprog);
  // the rows' sums: the caller writes them to F
#pragma unroll
  for (int k = 0; k < D; ++k) rout[k] = racc[k];
}

// Stamp record of one unit (STAMP builds): see kStampWords.
__device__ __forceinline__ void stamp_unit(long long* stamps, int qi, long long t_take,
                                           long long t_first, long long spin) {
  long long* w = stamps + (size_t)qi * kStampWords;
  w[0] = t_take;
  w[1] = t_first;
  w[2] = rt_now();
  w[3] = spin;
  w[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
  w[5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
}

// Unit kinds: a symmetric sweep, or a whole row block (an aggregate whose sweep
// chain would outlast the launch: a share of a multi-GPU run).  Rounds 3-4 also
// built, bit-exact and measured slower (removed in round 5): pair
// sweeps (two row tiles per wave), banded aggregates (pre row blocks, in-band sweeps,
// post row blocks), segmented row blocks and their round-5 tail split.
constexpr int kUnitSweep = 0, kUnitRows = 1;

// units[q] = {aggregate, row tile A, offset of the aggregate's tiles in prog (a row
// block: its priority quantum), kind}
// in queue order; prog (ptiles progress counters) zeroed before the launch; queue =
// one counter.  Every unit waits only on units before it in the queue.
// 4 waves per SIMD: <= 128 VGPRs, 36 KB of LDS per block (D = 3).  (Round 3 timed a
// diagnostics build in which no sweep waited for its hand-overs -- wrong results --
// at 124 against 138 ms; removed from the source in round 6.)
// The kernel stays at <= 120 VGPRs: three of its waves per SIMD (the plan's three
// blocks per CU) then leave 152 of the 512 registers, room for one wave of the
// resident classes' kernels (143 VGPRs) on the other streams.  At 122-128 (with the
// round-4 band kinds compiled in, or the give-up store inside the wait loop) the
// resident kernels were locked out until the repulsion launches ended and ran
// during the attraction passes instead (C4: 4.44 against 3.52 ms per pass, 140.4
// against 137.0-137.3 ms per step; profiles/r04/ab_rows_r03.log).
template <int D, bool REPEL_ONE, bool STAMP = false>
__global__ void __launch_bounds__(kSymT, 4)
faml_sym_repulse(int nunits, const int4* __restrict__ units, int* __restrict__ queue,
                 const int* __restrict__ pt_ip, const double* __restrict__ X,
                 const double* __restrict__ DP, double repel, double* __restrict__ F,
                 double* __restrict__ H, size_t hs, int* __restrict__ prog,
                 int* __restrict__ err, long long limit, long long* __restrict__ stamps) {
  constexpr int NW = kSymT / 64;
  // per wave: the record ring (also the row blocks' tile: 64 records of SymW<D>
  // doubles) and the column ring
  static_assert(kRecSlots * (D + 1) >= 64 * SymW<D>::v, "row-block tile fits the record ring");
  __shared__ __attribute__((aligned(16))) double srec[NW][kRecSlots * (D + 1)];
  __shared__ __attribute__((aligned(16))) double scol[NW][kColSlots * D];
  const int lane = threadIdx.x & 63;
  double* rec = srec[threadIdx.x >> 6];
  double* col = scol[threadIdx.x >> 6];
  const bool repel_ok = REPEL_ONE || weight_ok(repel);
  bool give_up = false;  // a hand-over wait timed out (err is set on exit)
  for (;;) {
    int qi = 0;
    if (lane == 0) qi = atomicAdd(queue, 1);
    qi = __builtin_amdgcn_readfirstlane(qi);
    if (qi >= nunits) break;  // every wave leaves once the queue is drained
    long long t_take = 0, t_first = 0, spin = 0;
    if (STAMP) t_take = t_first = rt_now();
    const int4 u = units[qi];
    const int A = u.y;
    const int base = pt_ip[u.x];
    const int s = pt_ip[u.x + 1] - base;
    const size_t rb = (size_t)base + 64 * (size_t)A;
    if (u.w == kUnitRows) {
      // a row block spans its aggregate's whole width: the launch's critical path
      // when the aggregate is large, so its wave takes issue priority over the
      // sweeps on the SIMD, by the column tiles it has left (u.z: rows_prio's quantum)
      rows_block<D, REPEL_ONE>(lane, base, s, A, X, DP, repel, repel_ok, rec, F, u.z);
    } else {  // a sweep
      double racc[D];
      sweep_unit<D, REPEL_ONE, STAMP>(lane, A, base, s, prog + u.z + A, X, DP, repel,
                                              repel_ok, F, H, hs, err, limit, give_up, rec, col,
                                              spin, t_first, racc);
      if (64 * A + lane < s) {
#pragma unroll
        for (int k = 0; k < D; ++k) F[(rb + lane) * D + k] = racc[k];
      }
    }
    if (STAMP && lane == 0) stamp_unit(stamps, qi, t_take, t_first, spin);
    wave_lds_sync();
  }
  report_give_up(give_up, lane, err);
}

}  // namespace ge
