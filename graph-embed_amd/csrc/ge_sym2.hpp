// ge_sym2.hpp -- the symmetric in-aggregate repulsion of ge_sym.hpp with each
// sweep spread over the four waves of a workgroup (include/forceatlas.hpp:394-410;
// bit-exact with the reference's per-row serial sums, same order as ge_sym.hpp).
//
// Why.  A sweep is a chain: sweep A of an aggregate may take column tile B only
// after sweep A-1 has passed it on, so the sweeps of an aggregate of T row tiles
// finish ~2.5 T tile-times after the first starts (ge_sym.hpp).  When one wave runs
// a whole sweep, a tile-time is 64 steps of ~66 instructions issued by that wave
// while three other waves share its SIMD.  The level-0 work of the R-MAT configs
// sits almost entirely in a hundred hub aggregates of T = 400-660 tiles, so on a
// share of them (multi-GPU) the chains, not the work, set the launch time.
//
// How.  Only the additions are ordered; the pair terms are not.  A workgroup runs
// one sweep in phases of kSym2C steps separated by workgroup barriers:
//   * three PRODUCER waves hold the sweep's 64 rows and compute the terms of the
//     NEXT phase's steps (step s: lane l = row l against column s - l, ge_sym.hpp's
//     systolic schedule), dealt round robin, into one half of a double-buffered
//     term array in LDS; they also stage the column tiles (coordinates, deg+1) two
//     phases before they are first read, in a 4-tile ring;
//   * one ADDER wave walks THIS phase's steps in order over the other half: the
//     entering column sum, the diagonal take-over, racc += t, flow -= t, the DPP
//     shift -- the arithmetic of ge_sym.hpp's sym_step on the same terms -- and the
//     column-tile hand-overs between sweeps (agent scope, per-tile progress).
// The adder issues ~20 instructions per step instead of ~66, so a sweep's chain
// advances several times faster; the barrier is the only synchronisation.
#pragma once

#include <hip/hip_runtime.h>

#include "ge_pair.hpp"
#include "ge_rows.hpp"
#include "ge_sym.hpp"

namespace ge {

constexpr int kSym2T = 256;    // 1 adder + 3 producer waves
constexpr int kSym2P = 3;      // producer waves
constexpr int kSym2C = 8;      // steps per phase
constexpr int kSym2Rec = 256;  // column record ring: 4 tiles (column q at q & 255)

template <int D>
struct Sym2Smem {
  static constexpr int WV = SymW<D>::v;
  double rec[(D + 1) * kSym2Rec];  // column records by component: rec[k][slot]
  double ini[kSymRing * D];          // entering column sums (adder)
  double out[kSymRing * D];          // leaving column sums (adder)
  double term[2 * kSym2C * D * 64];  // [phase parity][step in phase][k][lane]
  int tile_ok[4];
  int unit;
};

// Stage (producer p's share of) every column tile the steps < reach + 1 read: tile
// u by producer u mod 3, tile ntiles is the inert drain tile.  Tile u takes the
// slots of tile u - 4, last read at step 64u - 130.
template <int D>
__device__ __forceinline__ void sym2_stage(Sym2Smem<D>& sm, int p, int lane, int reach,
                                           int ncols, int ntiles, size_t cbase,
                                           const double* __restrict__ X,
                                           const double* __restrict__ DP, int& staged) {
  while (staged < ntiles && 64 * (staged + 1) <= reach) {
    const int u = ++staged;
    if (u % kSym2P != p) continue;
    const int qc = 64 * u + lane;
    const bool cv = u < ntiles && qc < ncols;  // past the aggregate: inert record
    double xc[D], dc = 0.0;
#pragma unroll
    for (int q = 0; q < D; ++q) xc[q] = cv ? X[(cbase + qc) * D + q] : 0.0;
    if (cv) dc = DP[cbase + qc];
    const bool ok = __all(!cv || vertex_ok<D>(xc, dc));
    double* rs = sm.rec + (qc & (kSym2Rec - 1));  // by component: rec[k][slot]
#pragma unroll
    for (int q = 0; q < D; ++q) rs[q * kSym2Rec] = xc[q];
    rs[D * kSym2Rec] = dc;
    if (lane == 0) sm.tile_ok[u & 3] = ok ? 1 : 0;
  }
}

// Producer p: the terms of phase k's steps j = p, p + 3, ... (step s0 + j).
template <int D, bool REPEL_ONE>
__device__ __forceinline__ void sym2_produce(Sym2Smem<D>& sm, int p, int lane, int k, int nsteps,
                                             const double (&xr)[D], double dr, bool rows_ok,
                                             double repel) {
  const int s0 = k * kSym2C;
  double* tb = sm.term + (k & 1) * kSym2C * D * 64;
  for (int j = p; j < kSym2C && s0 + j < nsteps; j += kSym2P) {
    const int sg = s0 + j;
    const int tt = sg >> 6;
    // step sg reads columns sg - 63 .. sg: tile tt, and tile tt - 1 up to step 64 tt + 62
    const bool need_prev = tt > 0 && sg - 63 < 64 * tt;
    const bool fast = rows_ok && sm.tile_ok[tt & 3] && (!need_prev || sm.tile_ok[(tt - 1) & 3]);
    const double* xq = sm.rec + ((sg - lane) & (kSym2Rec - 1));
    double xv[D + 1];
#pragma unroll
    for (int q = 0; q <= D; ++q) xv[q] = xq[q * kSym2Rec];
    double t[D];
    if (fast) {
      rep_term<D, true, REPEL_ONE>(xr, xv, dr, xv[D], repel, t);
    } else {
      rep_term<D, false, REPEL_ONE>(xr, xv, dr, xv[D], repel, t);
      if (sg - lane == lane) {  // the `/` form skips the self pair (ge_pair.hpp)
#pragma unroll
        for (int q = 0; q < D; ++q) t[q] = 0.0;
      }
    }
#pragma unroll
    for (int q = 0; q < D; ++q) tb[(j * D + q) * 64 + lane] = t[q];
  }
}

// The adder's steps of phase k (ge_sym.hpp's sym_step arithmetic): the entering
// sums of a column tile are fetched at its first step, the hand-overs made when a
// tile's columns have left the wave.
template <int D>
__device__ __forceinline__ void sym2_add(Sym2Smem<D>& sm, int lane, int k, int A, int ncols,
                                         int ntiles, int nsteps, size_t cbase,
                                         int* __restrict__ tprog, double* __restrict__ F,
                                         double (&racc)[D], double (&flow)[D]) {
  const int s0 = k * kSym2C, s1 = min(s0 + kSym2C, nsteps);
  const double* tb = sm.term + (k & 1) * kSym2C * D * 64;
  for (int sg = s0; sg < s1; ++sg) {
    if ((sg & 63) == 0) {  // a new column tile enters: its sums from the sweeps before
      const int tt = sg >> 6;
      const int qc = sg + lane;
      double ic[D];
      if (tt < ntiles && A > 0) {
        while (__hip_atomic_load(tprog + tt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < A)
          __builtin_amdgcn_s_sleep(1);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // see ge_sym.hpp
        const bool cv = qc < ncols;
#pragma unroll
        for (int q = 0; q < D; ++q) ic[q] = cv ? agent_ld(F + (cbase + qc) * D + q) : 0.0;
      } else {
#pragma unroll
        for (int q = 0; q < D; ++q) ic[q] = 0.0;  // first sweep, or the drain
      }
      double* is = sm.ini + (qc & (kSymRing - 1)) * D;
#pragma unroll
      for (int q = 0; q < D; ++q) is[q] = ic[q];
      wave_lds_sync();
    }
    const double* ib = sm.ini + (sg & (kSymRing - 1)) * D;
    double t[D], in0[D];
#pragma unroll
    for (int q = 0; q < D; ++q) {
      t[q] = tb[((sg - s0) * D + q) * 64 + lane];
      in0[q] = ib[q];
    }
#pragma unroll
    for (int q = 0; q < D; ++q) flow[q] = wave_shift_in(flow[q], in0[q]);
    if (sg < 127 && sg - lane == lane) {
#pragma unroll
      for (int q = 0; q < D; ++q) racc[q] = flow[q];
    }
#pragma unroll
    for (int q = 0; q < D; ++q) {
      racc[q] = racc[q] + t[q];
      flow[q] = flow[q] - t[q];
    }
    if (lane == 63) {  // column sg - 63 leaves the wave
      double* o = sm.out + ((sg - 63) & (kSymRing - 1)) * D;
#pragma unroll
      for (int q = 0; q < D; ++q) o[q] = flow[q];
    }
    const int tt = sg >> 6;
    // after tile tt's 64 steps tile tt - 1 has left; after the last step, the last tile
    if ((sg & 63) == 63 && tt >= 2 && tt < ntiles)
      sym_handover<D>(tt - 1, lane, A, ncols, cbase, sm.out, F, tprog);
    if (sg == nsteps - 1 && ntiles >= 2)
      sym_handover<D>(ntiles - 1, lane, A, ncols, cbase, sm.out, F, tprog);
    if ((sg & 63) == 63 || sg == nsteps - 1)
      wave_lds_sync();  // the ini / out slots of tile tt - 1 are free for tile tt + 1
  }
}

// units[q] = {aggregate, row tile A, offset of the aggregate's tiles in prog, kind}:
// kind 0 a sweep (the whole workgroup), kind 1 row blocks A .. A+3 (one per wave,
// ge_sym.hpp rows_block); prog zeroed before the launch; queue = one counter.
template <int D, bool REPEL_ONE>
__global__ void __launch_bounds__(kSym2T, 4)
faml_sym2_repulse(int nunits, const int4* __restrict__ units, int* __restrict__ queue,
                  const int* __restrict__ pt_ip, const double* __restrict__ X,
                  const double* __restrict__ DP, double repel, double* __restrict__ F,
                  int* __restrict__ prog) {
  __shared__ __attribute__((aligned(16))) Sym2Smem<D> sm;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const bool repel_ok = REPEL_ONE || weight_ok(repel);
  for (;;) {
    if (threadIdx.x == 0) sm.unit = atomicAdd(queue, 1);
    __syncthreads();
    const int qi = sm.unit;
    if (qi >= nunits) break;  // uniform: every wave leaves once the queue is drained
    const int4 u = units[qi];
    const int base = pt_ip[u.x];
    const int s = pt_ip[u.x + 1] - base;
    const int A = u.y;
    if (u.w) {
      const int Aw = A + wave;
      if (64 * Aw < s)  // scratch: this wave's quarter of the term array
        rows_block<D, REPEL_ONE>(lane, base, s, Aw, X, DP, repel, repel_ok,
                                 sm.term + wave * (2 * kSym2C * D * 64 / 4), F);
      __syncthreads();
      continue;
    }
    const size_t cbase = (size_t)base + 64 * (size_t)A;
    const bool rv = 64 * A + lane < s;
    const int ncols = s - 64 * A;
    const int ntiles = (ncols + 63) >> 6;
    const int nsteps = ncols + 63;
    const int nphases = (nsteps + kSym2C - 1) / kSym2C;
    int* tprog = prog + u.z + A;
    double racc[D], flow[D], xr[D], dr = 0.0;
    bool rows_ok = false;
    int staged = -1;
    const int p = wave - 1;
    if (wave == 0) {
#pragma unroll
      for (int q = 0; q < D; ++q) {
        racc[q] = 0.0;
        flow[q] = 0.0;
      }
    } else {
#pragma unroll
      for (int q = 0; q < D; ++q) xr[q] = rv ? X[(cbase + lane) * D + q] : 0.0;  // inert row
      if (rv) dr = DP[cbase + lane];
      rows_ok = repel_ok && __all(!rv || vertex_ok<D>(xr, dr));
      // the tiles phases 0 and 1 read
      sym2_stage<D>(sm, p, lane, min(2 * kSym2C, nsteps) - 1, ncols, ntiles, cbase, X, DP, staged);
    }
    __syncthreads();
    // phase k: the adder adds phase k's steps while the producers compute phase
    // k + 1's terms and stage the tiles phase k + 2 will read
    for (int k = -1; k < nphases; ++k) {
      if (wave == 0) {
        if (k >= 0) sym2_add<D>(sm, lane, k, A, ncols, ntiles, nsteps, cbase, tprog, F, racc, flow);
      } else if (k + 1 < nphases) {
        sym2_stage<D>(sm, p, lane, min((k + 3) * kSym2C, nsteps) - 1, ncols, ntiles, cbase, X, DP,
                      staged);
        sym2_produce<D, REPEL_ONE>(sm, p, lane, k + 1, nsteps, xr, dr, rows_ok, repel);
      }
      __syncthreads();
    }
    if (wave == 0 && rv) {
#pragma unroll
      for (int q = 0; q < D; ++q) F[(cbase + lane) * D + q] = racc[q];
    }
  }
}

}  // namespace ge
