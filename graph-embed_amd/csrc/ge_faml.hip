// ge_faml.hip -- multilevel ForceAtlas (one level) on gfx950.
//
// Reference: partition::forceAtlasMultilevel, include/forceatlas.hpp:314-574,
// called once per level with iterations = 100 (src/embed.cpp:793).
//
// Aggregates never exchange data during the iterations (the external pull reads
// only the frozen coarse coordinates coords_A, :454, :462), so each aggregate is
// an independent N-body problem.  Layout: a member's state is indexed by its
// P_T storage position c (aggregate a owns positions pt_ip[a]..pt_ip[a+1]);
// pos_of[fine id] = c.
//
// Aggregates are bucketed by size s:
//   s <= 64          packs of aggregates with <= 64 members total, 64-thread block
//   64 < s <= 256    packs with <= 256 members, 256-thread block
//   256 < s <= 4096  one aggregate per 256-thread block
//   (all three: coordinates resident in LDS, all iterations in ONE launch)
//   s > 4096         "streamed": per iteration a force kernel (j tiles through
//                    LDS) and an update kernel, coordinates in HBM.
//
// STRICT op order, as ge_fa.hip: per member the j loop runs over the aggregate's
// members in P_T order (:394-410), then the CSR row in stored order with the
// reference's internal/external test `v_A[j] == a && j != i` (i the LOCAL index,
// :417), gravity with mag clamped to eps (:411-414), swing clamped (:484-486).
// The centring mean (:540-553) is a serial sum in member order (one thread per
// aggregate); the max norm (:555-561) is order-free.
// Random init replays the reference's single-thread mt19937 draw order: the
// host generates draw c*dim+k for position c (include/forceatlas.hpp:356-360).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <numeric>
#include <queue>
#include <string>
#include <vector>

#include "ge_internal.hpp"
#include "ge_pair.hpp"
#include "ge_rows.hpp"
#include "ge_sym.hpp"

namespace ge {
namespace {

constexpr double kEps = kFaEps;
using MlConst = FaConst;

template <int D>
struct W {
  static constexpr int v = (D + 1 <= 4) ? 4 : 8;
};

// Largest aggregate kept resident in LDS (128 KiB of member records).
constexpr int large_cap(int dim) { return dim + 1 <= 4 ? 4096 : 2048; }

// Internal degree + 1 of member at position c in aggregate a (:362-383).
__device__ __forceinline__ double internal_dp1(int v, int a, const int* __restrict__ ip,
                                               const int* __restrict__ ix,
                                               const double* __restrict__ dx,
                                               const int* __restrict__ vA, int use_weights) {
  double s = 0.0;
  for (int e = ip[v]; e < ip[v + 1]; ++e)
    if (vA[ix[e]] == a) s += use_weights ? dx[e] : 1.0;
  return s + 1;
}

// ((t / dis) * 100.0) / mag for the external pull of one CSR entry (:452-465).
template <int D, bool SHARED>
__device__ __forceinline__ void pull_edge(const double* __restrict__ ca,
                                          const double* __restrict__ cb, double mag,
                                          const Recip& rmag, double (&acc)[D]) {
  double t[D];
#pragma unroll
  for (int k = 0; k < D; ++k) t[k] = cb[k] - ca[k];
  double q = t[0] * t[0];
#pragma unroll
  for (int k = 1; k < D; ++k) q = q + t[k] * t[k];
  const double dis = clamp_eps(sqrt(q));
  if (SHARED) {
    const Recip rc = recip_of(dis);
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = acc[k] + div_by(div_by(t[k], dis, rc) * 100.0, mag, rmag);
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = acc[k] + (t[k] / dis) * 100.0 / mag;
  }
}

// Force on one member (:391-474).  xs(l) returns the coordinates of local member
// l of the same aggregate; xi/dip1 the member's own.
template <int D, class XS, class DS>
__device__ __forceinline__ void member_force(int li, int s, int a, int v, const double (&xi)[D],
                                             double dip1, XS xs, DS ds, int pt_base,
                                             const int* __restrict__ ip, const int* __restrict__ ix,
                                             const double* __restrict__ dx,
                                             const int* __restrict__ vA,
                                             const int* __restrict__ pos_of,
                                             const double* __restrict__ cA, const MlConst& c,
                                             double (&F)[D]) {
  double acc[D];
#pragma unroll
  for (int k = 0; k < D; ++k) acc[k] = 0.0;
  const bool row_ok = all_coord_ok<D>(xi);
  const bool rep_ok = row_ok && weight_ok(dip1) && weight_ok(c.repel);
  for (int j = 0; j < s; ++j) {  // :394-410
    const double* xj = xs(j);
    if (rep_ok && vertex_ok<D>(xj, ds(j)))
      rep_pair<D, true, false>(xi, xj, dip1, ds(j), c.repel, acc);
    else
      rep_pair_fb<D, false>(xi, xj, dip1, ds(j), c.repel, j == li, acc);
  }
  double m2 = xi[0] * xi[0];
#pragma unroll
  for (int k = 1; k < D; ++k) m2 = m2 + xi[k] * xi[k];
  double mag = sqrt(m2);
  if (mag < kEps) mag = kEps;
  const Recip rmag = recip_of(mag);
  const double* ca = cA + (size_t)a * D;
  const bool ca_ok = all_coord_ok<D>(ca);
  for (int e = ip[v]; e < ip[v + 1]; ++e) {  // :415-467
    const int j = ix[e];
    const int b = vA[j];
    if (b == a && j != li) {  // sic: global j against local i (:417)
      const double* xj = xs(pos_of[j] - pt_base);
      const double w = c.use_weights ? dx[e] : 1.0;
      if (row_ok && all_coord_ok<D>(xj))
        attr_edge<D, true>(xi, xj, w, dip1, c, acc);
      else
        attr_edge<D, false>(xi, xj, w, dip1, c, acc);
    } else {
      const double* cb = cA + (size_t)b * D;
      if (row_ok && ca_ok && all_coord_ok<D>(cb))
        pull_edge<D, true>(ca, cb, mag, rmag, acc);
      else
        pull_edge<D, false>(ca, cb, mag, rmag, acc);
    }
  }
  double unit[D];
  neg_over<D>(xi, mag, unit);
#pragma unroll
  for (int k = 0; k < D; ++k) F[k] = acc[k] + unit[k] * c.gravity * dip1;  // :469-474
}

// Swing (clamped) + speed + update of one member (:477-530).
template <int D>
__device__ __forceinline__ void member_update(double (&x)[D], const double (&F)[D],
                                              const double (&Fp)[D], const MlConst& c) {
  double s = 0.0, f2 = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const double t = F[k] - Fp[k];
    s = (k == 0) ? t * t : s + t * t;
    f2 = (k == 0) ? F[k] * F[k] : f2 + F[k] * F[k];
  }
  double swing = sqrt(s);
  if (swing < kEps) swing = kEps;
  const double totalF = sqrt(f2);
  double speed = c.ks_gS / (1 + c.gS * sqrt(swing));
  const double cap = c.ksmax / totalF;
  if (speed > cap) speed = cap;
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = F[k] * speed + x[k];
}

// ---------------------------------------------------------------------------
// Resident kernel: one block = one pack of aggregates (order[pack_beg[p]..
// pack_beg[p+1])), members in LDS, all iterations in-kernel.

template <int D, int T, int CAP>
__global__ void __launch_bounds__(T)
faml_resident(const int* __restrict__ order, const int* __restrict__ pack_beg,
              const int* __restrict__ pt_ip, const int* __restrict__ pt_ix,
              const int* __restrict__ pos_of, const int* __restrict__ vA,
              const int* __restrict__ ip, const int* __restrict__ ix,
              const double* __restrict__ dx, const double* __restrict__ cA,
              const double* __restrict__ rA, const double* __restrict__ init,
              double* __restrict__ Fscr, double* __restrict__ Fprev,
              double* __restrict__ Xout, int iterations, MlConst c) {
  constexpr int WV = W<D>::v;
  constexpr int MAXAGG = (CAP < T) ? CAP : T;  // aggregates per pack <= T
  __shared__ __attribute__((aligned(16))) double rec[CAP * WV];
  __shared__ int seg[MAXAGG + 1];
  __shared__ int agg_of_seg[MAXAGG];
  __shared__ double ball[MAXAGG * (D + 1)];

  const int tid = threadIdx.x;
  const int p0 = pack_beg[blockIdx.x], p1 = pack_beg[blockIdx.x + 1];
  const int naggs = p1 - p0;
  if (tid == 0) {
    int off = 0;
    for (int q = 0; q < naggs; ++q) {
      const int a = order[p0 + q];
      seg[q] = off;
      agg_of_seg[q] = a;
      off += pt_ip[a + 1] - pt_ip[a];
    }
    seg[naggs] = off;
  }
  __syncthreads();
  const int S = seg[naggs];

  // member q -> (segment, aggregate, local index, position)
  auto locate = [&](int q, int& g, int& a, int& li, int& pc) {
    int lo = 0, hi = naggs - 1;
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (seg[mid] <= q) lo = mid; else hi = mid - 1;
    }
    g = lo;
    a = agg_of_seg[lo];
    li = q - seg[lo];
    pc = pt_ip[a] + li;
  };

  for (int q = tid; q < S; q += T) {
    int g, a, li, pc;
    locate(q, g, a, li, pc);
#pragma unroll
    for (int k = 0; k < D; ++k) {
      rec[q * WV + k] = init[(size_t)pc * D + k];
      Fprev[(size_t)pc * D + k] = 0.0;
    }
    rec[q * WV + D] = internal_dp1(pt_ix[pc], a, ip, ix, dx, vA, c.use_weights);
  }

  for (int it = 0; it < iterations; ++it) {
    __syncthreads();
    for (int q = tid; q < S; q += T) {
      int g, a, li, pc;
      locate(q, g, a, li, pc);
      const int s0 = seg[g];
      const int s = seg[g + 1] - s0;
      double xi[D], F[D];
#pragma unroll
      for (int k = 0; k < D; ++k) xi[k] = rec[q * WV + k];
      const double dip1 = rec[q * WV + D];
      member_force<D>(li, s, a, pt_ix[pc], xi, dip1,
                      [&](int l) { return &rec[(s0 + l) * WV]; },
                      [&](int l) { return rec[(s0 + l) * WV + D]; }, pt_ip[a], ip, ix, dx, vA,
                      pos_of, cA, c, F);
#pragma unroll
      for (int k = 0; k < D; ++k) Fscr[(size_t)pc * D + k] = F[k];
    }
    __syncthreads();
    for (int q = tid; q < S; q += T) {
      int g, a, li, pc;
      locate(q, g, a, li, pc);
      double x[D], F[D], Fp[D];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        x[k] = rec[q * WV + k];
        F[k] = Fscr[(size_t)pc * D + k];
        Fp[k] = Fprev[(size_t)pc * D + k];
      }
      member_update<D>(x, F, Fp, c);
#pragma unroll
      for (int k = 0; k < D; ++k) {
        rec[q * WV + k] = x[k];
        Fprev[(size_t)pc * D + k] = F[k];
      }
    }
  }
  __syncthreads();
  // centre + max norm per aggregate (:539-564): serial mean in member order
  for (int g = tid; g < naggs; g += T) {
    const int s0 = seg[g], s = seg[g + 1] - seg[g];
    double avg[D];
#pragma unroll
    for (int k = 0; k < D; ++k) avg[k] = 0.0;
    for (int l = 0; l < s; ++l)
#pragma unroll
      for (int k = 0; k < D; ++k) avg[k] = avg[k] + rec[(s0 + l) * WV + k];
#pragma unroll
    for (int k = 0; k < D; ++k) avg[k] = avg[k] / s;
    double big = 0.0;
    for (int l = 0; l < s; ++l) {
      double m2 = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const double t = rec[(s0 + l) * WV + k] - avg[k];
        m2 = (k == 0) ? t * t : m2 + t * t;
      }
      const double len = sqrt(m2);
      if (len > big) big = len;
    }
    if (big < kEps) big = kEps;
#pragma unroll
    for (int k = 0; k < D; ++k) ball[g * (D + 1) + k] = avg[k];
    ball[g * (D + 1) + D] = big;
  }
  __syncthreads();
  for (int q = tid; q < S; q += T) {
    int g, a, li, pc;
    locate(q, g, a, li, pc);
    const double big = ball[g * (D + 1) + D];
    const int v = pt_ix[pc];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const double x = rec[q * WV + k] - ball[g * (D + 1) + k];
      Xout[(size_t)v * D + k] = cA[(size_t)a * D + k] + rA[a] * (x / big);
    }
  }
}

// ---------------------------------------------------------------------------
// Streamed path for aggregates too large to stay resident.  Per iteration:
//   faml_big_repulse  the in-aggregate all-pairs sum, one WAVE per work item
//                     (aggregate a, rows r0 .. r0 + 64R); items are taken from
//                     an atomic queue in descending-work order (list scheduling
//                     over aggregates of very different sizes);
//   FamlRows          (classed_rows_kernel, ge_rows.hpp) the CSR row's terms
//                     added to the repulsion sum in stored order, then gravity
//                     and the swing/speed update.
// `rows` lists the P_T positions of all streamed members.

constexpr int kHT = 256;   // threads per block of the streamed kernels
constexpr int kBigW = 64;  // records per wave tile
constexpr int kBigDefaultR = 1, kBigDefaultU = 1;

template <int D>
__global__ void __launch_bounds__(kHT)
faml_huge_init(int nrows, const int* __restrict__ rows, const double* __restrict__ init,
               double* __restrict__ Xp, double* __restrict__ Fprev) {
  const int q = blockIdx.x * kHT + threadIdx.x;
  if (q >= nrows) return;
  const int c = rows[q];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    Xp[(size_t)c * D + k] = init[(size_t)c * D + k];
    Fprev[(size_t)c * D + k] = 0.0;
  }
}

// internal deg + 1 of the streamed members (:362-383): a property of the graph
// and P_T, computed once per plan (a hub row's serial sum takes tens of ms).
__global__ void __launch_bounds__(kHT)
faml_huge_dp(int nrows, const int* __restrict__ rows, const int* __restrict__ pt_ix,
             const int* __restrict__ vA, const int* __restrict__ ip, const int* __restrict__ ix,
             const double* __restrict__ dx, double* __restrict__ DP, int use_weights) {
  const int q = blockIdx.x * kHT + threadIdx.x;
  if (q >= nrows) return;
  const int c = rows[q];
  const int v = pt_ix[c];
  DP[c] = internal_dp1(v, vA[v], ip, ix, dx, vA, use_weights);
}

// R row slots per lane, U consecutive partners evaluated together (their terms
// are then added in j order).
template <int D, int R, int U, bool REPEL_ONE>
__global__ void __launch_bounds__(kHT)
faml_big_repulse(int nitems, const int2* __restrict__ items, int* __restrict__ queue,
                 const int* __restrict__ pt_ip, const double* __restrict__ Xp,
                 const double* __restrict__ DP, double repel, double* __restrict__ Fscr) {
  constexpr int WV = W<D>::v;
  __shared__ __attribute__((aligned(16))) double tiles[kHT / 64][kBigW * WV];
  const int lane = threadIdx.x & 63;
  double* tile = tiles[threadIdx.x >> 6];
  const bool repel_ok = REPEL_ONE || weight_ok(repel);
  for (;;) {
    int q = 0;
    if (lane == 0) q = atomicAdd(queue, 1);
    q = __builtin_amdgcn_readfirstlane(q);
    if (q >= nitems) break;  // every wave leaves once the queue is drained
    const int2 item = items[q];
    const int base = pt_ip[item.x];
    const int s = pt_ip[item.x + 1] - base;
    const int r0 = item.y;
    const int nr = min(R, (s - r0 + 63) >> 6);  // wave-uniform
    double xi[R][D], di[R], acc[R][D];
    bool rows_ok = repel_ok;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int li = r0 + lane + 64 * r;
      const bool ok = r < nr && li < s;
      const size_t c = (size_t)base + (ok ? li : 0);
#pragma unroll
      for (int k = 0; k < D; ++k) {
        xi[r][k] = ok ? Xp[c * D + k] : 0.0;
        acc[r][k] = 0.0;
      }
      di[r] = ok ? DP[c] : 1.0;
      rows_ok = rows_ok && vertex_ok<D>(xi[r], di[r]);
    }
    for (int j0 = 0; j0 < s; j0 += kBigW) {
      const int cnt = min(kBigW, s - j0);
      bool ok = rows_ok;
      wave_lds_sync();  // the previous tile has been read by every lane
      if (lane < cnt) {
        const size_t c = (size_t)base + j0 + lane;
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const double v = Xp[c * D + k];
          tile[lane * WV + k] = v;
          ok = ok && coord_ok(v);
        }
        const double w = DP[c];
        tile[lane * WV + D] = w;
        ok = ok && weight_ok(w);
      }
      wave_lds_sync();
      if (__all(ok)) {
        int jj = 0;
        if (nr == R) {
          // every row slot of the wave is used: no per-slot branches, so the
          // partner record is read once for all R rows and the independent
          // chains (R rows x U partners) interleave
          if constexpr (U == 1) {
            for (; jj < cnt; ++jj) {
              const double* xj = &tile[jj * WV];
              const double dj = tile[jj * WV + D];
#pragma unroll
              for (int r = 0; r < R; ++r) rep_pair<D, true, REPEL_ONE>(xi[r], xj, di[r], dj, repel, acc[r]);
            }
          } else {
            for (; jj + U <= cnt; jj += U) {
              double t[U][R][D];
#pragma unroll
              for (int u = 0; u < U; ++u)
#pragma unroll
                for (int r = 0; r < R; ++r)
                  rep_term<D, true, REPEL_ONE>(xi[r], &tile[(jj + u) * WV], di[r],
                                               tile[(jj + u) * WV + D], repel, t[u][r]);
#pragma unroll
              for (int u = 0; u < U; ++u)
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                  for (int k = 0; k < D; ++k) acc[r][k] = acc[r][k] + t[u][r][k];
            }
          }
        } else if (U > 1) {
          for (; jj + U <= cnt; jj += U) {
            double t[U][R][D];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
              for (int r = 0; r < R; ++r) {
#pragma unroll
                for (int k = 0; k < D; ++k) t[u][r][k] = 0.0;
                if (r < nr)
                  rep_pair<D, true, REPEL_ONE>(xi[r], &tile[(jj + u) * WV], di[r],
                                               tile[(jj + u) * WV + D], repel, t[u][r]);
              }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
              for (int r = 0; r < R; ++r)
#pragma unroll
                for (int k = 0; k < D; ++k) acc[r][k] = acc[r][k] + t[u][r][k];
          }
        }
        for (; jj < cnt; ++jj) {
          const double* xj = &tile[jj * WV];
          const double dj = tile[jj * WV + D];
#pragma unroll
          for (int r = 0; r < R; ++r)
            if (r < nr) rep_pair<D, true, REPEL_ONE>(xi[r], xj, di[r], dj, repel, acc[r]);
        }
      } else {
        for (int jj = 0; jj < cnt; ++jj) {
          const double* xj = &tile[jj * WV];
          const double dj = tile[jj * WV + D];
#pragma unroll
          for (int r = 0; r < R; ++r)
            if (r < nr)
              rep_pair_fb<D, REPEL_ONE>(xi[r], xj, di[r], dj, repel,
                                        j0 + jj == r0 + lane + 64 * r, acc[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int li = r0 + lane + 64 * r;
      if (r < nr && li < s) {
#pragma unroll
        for (int k = 0; k < D; ++k) Fscr[((size_t)base + li) * D + k] = acc[r][k];
      }
    }
  }
}

// Per streamed member, after faml_big_repulse: the CSR row (:415-467) added to
// the repulsion sum in stored order (degree-classed, ge_rows.hpp), gravity
// (:469-474) and the swing/speed update (:477-530).
// ecode[e] for a streamed member's CSR entry e: the neighbour's P_T position
// when the entry is internal (v_A[j] == a && j != local i, :417), else
// -(v_A[j] + 1).  Static per level, so the per-iteration edge pass does one
// gather per entry instead of three dependent ones.
__global__ void edge_code_kernel(int nrows, const int* __restrict__ rows,
                                 const int* __restrict__ pt_ip, const int* __restrict__ pt_ix,
                                 const int* __restrict__ pos_of, const int* __restrict__ vA,
                                 const int* __restrict__ ip, const int* __restrict__ ix,
                                 int* __restrict__ ecode) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nrows) return;
  const int c = rows[q];
  const int v = pt_ix[c];
  const int a = vA[v];
  const int li = c - pt_ip[a];
  for (int e = ip[v]; e < ip[v + 1]; ++e) {
    const int j = ix[e];
    const int b = vA[j];
    ecode[e] = (b == a && j != li) ? pos_of[j] : -(b + 1);
  }
}

template <int D>
struct FamlRows {
  const int *pt_ip, *pt_ix, *ecode, *ip, *vA;
  const double *dx, *cA, *Xc, *DP, *Fscr;
  double *Xn, *Fprev;
  MlConst c;
  struct State {
    int cpos, a, li, e0, e1;
    double xi[D], acc[D], fprev[D], dip1, mag;
    Recip rmag;
    bool row_ok, ca_ok;
  };
  __device__ __forceinline__ void load(int cpos, State& s) const {
    const int v = pt_ix[cpos];
    s.cpos = cpos;
    s.a = vA[v];
    s.li = cpos - pt_ip[s.a];
    s.e0 = ip[v];
    s.e1 = ip[v + 1];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      s.xi[k] = Xc[(size_t)cpos * D + k];
      s.acc[k] = Fscr[(size_t)cpos * D + k];
      s.fprev[k] = Fprev[(size_t)cpos * D + k];  // loaded early: off the row's critical path
    }
    s.dip1 = DP[cpos];
    s.row_ok = all_coord_ok<D>(s.xi);
    double m2 = s.xi[0] * s.xi[0];
#pragma unroll
    for (int k = 1; k < D; ++k) m2 = m2 + s.xi[k] * s.xi[k];
    s.mag = sqrt(m2);
    if (s.mag < kEps) s.mag = kEps;
    s.rmag = recip_of(s.mag);
    s.ca_ok = all_coord_ok<D>(cA + (size_t)s.a * D);
  }
  __device__ __forceinline__ void term(const State& s, int e, double (&t)[D]) const {
    const int code = ecode[e];
    // the neighbour's (or its aggregate's) coordinates into registers before
    // the branch, so a thread's gathers issue together
    const double* src = code >= 0 ? Xc + (size_t)code * D : cA + (size_t)(-code - 1) * D;
    double xv[D];
#pragma unroll
    for (int k = 0; k < D; ++k) xv[k] = src[k];
    if (code >= 0) {  // internal entry (edge_code_kernel)
      const double* xj = xv;
      const double wt = c.use_weights ? dx[e] : 1.0;
      if (s.row_ok && all_coord_ok<D>(xj))
        attr_edge<D, true>(s.xi, xj, wt, s.dip1, c, t);
      else
        attr_edge<D, false>(s.xi, xj, wt, s.dip1, c, t);
    } else {
      const double* ca = cA + (size_t)s.a * D;
      const double* cb = xv;
      if (s.row_ok && s.ca_ok && all_coord_ok<D>(cb))
        pull_edge<D, true>(ca, cb, s.mag, s.rmag, t);
      else
        pull_edge<D, false>(ca, cb, s.mag, s.rmag, t);
    }
  }
  __device__ __forceinline__ void finish(State& s, bool writer) const {
    double unit[D], F[D], Fp[D], x[D];
    neg_over<D>(s.xi, s.mag, unit);
#pragma unroll
    for (int k = 0; k < D; ++k) {
      F[k] = s.acc[k] + unit[k] * c.gravity * s.dip1;
      Fp[k] = s.fprev[k];
      x[k] = s.xi[k];
    }
    member_update<D>(x, F, Fp, c);
    if (writer) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        Xn[(size_t)s.cpos * D + k] = x[k];
        Fprev[(size_t)s.cpos * D + k] = F[k];
      }
    }
  }
};

// One block per huge aggregate: serial mean by lane 0, max by reduction.
template <int D>
__global__ void __launch_bounds__(kHT)
faml_huge_finish(const int* __restrict__ huge, const int* __restrict__ pt_ip,
                 const int* __restrict__ pt_ix, const double* __restrict__ Xp,
                 const double* __restrict__ cA, const double* __restrict__ rA,
                 double* __restrict__ Xout) {
  __shared__ double avg[D];
  __shared__ double red[kHT];
  const int a = huge[blockIdx.x];
  const int base = pt_ip[a], s = pt_ip[a + 1] - base;
  if (threadIdx.x == 0) {
    double t[D];
#pragma unroll
    for (int k = 0; k < D; ++k) t[k] = 0.0;
    for (int l = 0; l < s; ++l)
#pragma unroll
      for (int k = 0; k < D; ++k) t[k] = t[k] + Xp[(size_t)(base + l) * D + k];
#pragma unroll
    for (int k = 0; k < D; ++k) avg[k] = t[k] / s;
  }
  __syncthreads();
  double big = 0.0;
  for (int l = threadIdx.x; l < s; l += kHT) {
    double m2 = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const double t = Xp[(size_t)(base + l) * D + k] - avg[k];
      m2 = (k == 0) ? t * t : m2 + t * t;
    }
    const double len = sqrt(m2);
    if (len > big) big = len;
  }
  red[threadIdx.x] = big;
  __syncthreads();
  for (int w = kHT / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w && red[threadIdx.x + w] > red[threadIdx.x])
      red[threadIdx.x] = red[threadIdx.x + w];
    __syncthreads();
  }
  double mx = red[0];
  if (mx < kEps) mx = kEps;
  for (int l = threadIdx.x; l < s; l += kHT) {
    const int v = pt_ix[base + l];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const double x = Xp[(size_t)(base + l) * D + k] - avg[k];
      Xout[(size_t)v * D + k] = cA[(size_t)a * D + k] + rA[a] * (x / mx);
    }
  }
}

__global__ void pos_of_kernel(int N, const int* __restrict__ pt_ix, int* __restrict__ pos_of) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < N) pos_of[pt_ix[c]] = c;
}

// Greedy packs over `ids` (already size-sorted) with total members <= cap.
void build_packs(const std::vector<int>& ids, const int* h_pt_ip, int cap, int max_aggs,
                 std::vector<int>& order, std::vector<int>& beg) {
  beg.push_back((int)order.size());
  int tot = 0, cnt = 0;
  for (int a : ids) {
    const int s = h_pt_ip[a + 1] - h_pt_ip[a];
    if (cnt > 0 && (tot + s > cap || cnt >= max_aggs)) {
      beg.push_back((int)order.size());
      tot = 0;
      cnt = 0;
    }
    order.push_back(a);
    tot += s;
    ++cnt;
  }
  if (cnt > 0) beg.push_back((int)order.size());
}

// Streamed repulsion variants: row slots R x partners in flight U.
#define GE_BIG_VARIANTS(X) X(1, 1) X(1, 2) X(1, 4) X(2, 1) X(4, 1)
constexpr int big_code(int R, int U) { return R * 8 + U; }

template <int D>
void launch_big_repulse(int code, int blocks, hipStream_t st, int nitems, const int2* items,
                        int* queue, const int* pt_ip, const double* X, const double* DP,
                        double repel, double* F) {
  switch (code) {
#define GE_BIG_LAUNCH(RR, UU)                                                                 \
  case big_code(RR, UU):                                                                      \
    if (repel == 1.0)                                                                         \
      hipLaunchKernelGGL((faml_big_repulse<D, RR, UU, true>), dim3(blocks), dim3(kHT), 0, st, \
                         nitems, items, queue, pt_ip, X, DP, repel, F);                       \
    else                                                                                      \
      hipLaunchKernelGGL((faml_big_repulse<D, RR, UU, false>), dim3(blocks), dim3(kHT), 0,    \
                         st, nitems, items, queue, pt_ip, X, DP, repel, F);                   \
    break;
    GE_BIG_VARIANTS(GE_BIG_LAUNCH)
#undef GE_BIG_LAUNCH
    default:
      throw Error(GE_ERR_STATE, "unknown streamed repulsion variant");
  }
}

// resident blocks per CU of faml_big_repulse<dim, R, U>
int rep_occupancy(int dim, int code) {
  int nb = 1;
  dispatch_dim(dim, [&](auto Dc) {
    constexpr int D = decltype(Dc)::value;
    const void* k = nullptr;
    switch (code) {
#define GE_BIG_KERNEL(RR, UU) \
  case big_code(RR, UU): k = (const void*)faml_big_repulse<D, RR, UU, false>; break;
      GE_BIG_VARIANTS(GE_BIG_KERNEL)
#undef GE_BIG_KERNEL
      default: k = (const void*)faml_big_repulse<D, 1, 1, false>;
    }
    GE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kHT, 0));
  });
  return std::max(nb, 1);
}

}  // namespace

}  // namespace ge

// ---------------------------------------------------------------------------
// plan: bucketing, pack tables and scratch built once per (graph, P_T) level

struct ge_faml_plan {
  ge_ctx* ctx = nullptr;
  int n = 0, m = 0, dim = 0, iterations = 0;
  const int *ip = nullptr, *ix = nullptr, *pt_ip = nullptr, *pt_ix = nullptr, *vA = nullptr;
  const double* dx = nullptr;
  ge::FaConst c{};
  int ns = 0, nm = 0, nl = 0, nhuge = 0;
  size_t off_m = 0, off_l = 0;
  ge::DevBuf<int> pos, order, beg, rows, erows, queue, huge, ecode;
  ge::RowClasses ecls;
  ge::RowStreams rstreams;
  ge::DevBuf<int2> items;
  int nrows = 0, nitems = 0, R = 1, code = 0, rep_blocks = 0;
  // symmetric repulsion (ge_sym.hpp): sweep units and per-tile progress counters
  bool sym = false;
  ge::DevBuf<int4> units;
  ge::DevBuf<int> prog;
  ge::DevBuf<double> hand;  // column sums handed between sweeps, component-major [dim][n]
  ge::DevBuf<int> sym_err;  // set by a hand-over wait that timed out
  long long sym_limit = 0;  // that wait's bound in ticks of the device wall clock
  int nunits = 0, ntiles = 0, sym_blocks = 0;
  int rows_mode = 0, swept = 0;  // streamed aggregates by schedule (ge_sym.hpp)
  std::vector<int4> h_units;          // host copy of `units` (timeline dumps)
  ge::DevBuf<long long> stamps;       // GE_SYM_STAMPS: per-unit timeline of the last launch
  std::string stamp_path;
  double streamed_pairs = 0.0;
  ge::DevBuf<double> Fscr, Fprev, Xa, Xb, DP;
  // the size classes are independent: streamed path, large, mid and small
  // packs each run on their own stream and join the context stream at the end
  hipStream_t side[3] = {nullptr, nullptr, nullptr};
  hipEvent_t fork = nullptr, join[3] = {nullptr, nullptr, nullptr};
  bool profiling = false;
  std::vector<hipEvent_t> ev;  // 4 per timed run: start, resident end, streamed start/end
  size_t next_ev = 0;
  std::vector<hipEvent_t> rev;  // 2 per profiled repulsion launch
  size_t next_rev = 0;
  std::vector<hipEvent_t> aev;  // 2 per profiled member-row pass (FamlRows)
  size_t next_aev = 0;
  long long streamed_entries = 0;  // CSR entries of the streamed members' rows
  // aggregates split by row tiles across the ranks of `comm`: this
  // rank computes its rows' forces and updates, and the split aggregates' rows are
  // exchanged after every iteration (exchange_rows, stream-ordered)
  ge_comm* comm = nullptr;
  ge::DevBuf<int> irows;  // positions initialised / given deg+1: rows + the other ranks' split rows
  int nirows = 0;
  ge::DevBuf<int> xrows, xcounts, xfirst;
  ge::DevBuf<double> xbuf;
  std::vector<int> h_xcounts, h_xfirst;
  int xwidth = 0;
};

namespace ge {

// aggs: the aggregates this plan runs (strictly increasing ids).
// split: aggregates whose row tiles are dealt over the ranks of pl->comm (the
// same list on every rank; tiles [T r / N, T (r + 1) / N) to rank r).
static void faml_plan_build(ge_faml_plan* pl, const int* h_pt_ip, const std::vector<int>& aggs,
                            const std::vector<int>& split_aggs = std::vector<int>()) {
  const std::vector<int>& split = split_aggs;
  hipStream_t st = pl->ctx->stream;
  const int dim = pl->dim;
  // Work of aggregate a per iteration ~ s^2.  Aggregates whose share would
  // keep one CU busy for more than a quarter of the per-CU average go to the
  // streamed path (many blocks per aggregate, one launch per iteration);
  // the rest stay resident in LDS for all iterations.
  double W = 0.0;
  for (int a : aggs) {
    const double s = h_pt_ip[a + 1] - h_pt_ip[a];
    W += s * s;
  }
  int dev = 0, cus = 256;
  GE_HIP(hipGetDevice(&dev));
  GE_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const double per_cu = W / std::max(cus, 1);
  int res_cap = (int)std::sqrt(per_cu / 4.0);  // largest aggregate kept resident
  res_cap = std::max(256, std::min(res_cap, large_cap(dim)));

  std::vector<int> small, mid, large, big;
  for (int a : aggs) {
    const int s = h_pt_ip[a + 1] - h_pt_ip[a];
    if (s <= 0) continue;
    if (s <= 64) small.push_back(a);
    else if (s <= 256) mid.push_back(a);
    else if (s <= res_cap) large.push_back(a);
    else big.push_back(a);
  }
  auto by_size = [&](int x, int y) {
    const int sx = h_pt_ip[x + 1] - h_pt_ip[x], sy = h_pt_ip[y + 1] - h_pt_ip[y];
    return sx != sy ? sx > sy : x < y;
  };
  std::sort(small.begin(), small.end(), by_size);
  std::sort(mid.begin(), mid.end(), by_size);
  std::sort(large.begin(), large.end(), by_size);
  std::sort(big.begin(), big.end(), by_size);

  std::vector<int> order, beg_s, beg_m, beg_l;
  build_packs(small, h_pt_ip, 64, 64, order, beg_s);
  build_packs(mid, h_pt_ip, 256, 256, order, beg_m);
  build_packs(large, h_pt_ip, large_cap(dim), 1, order, beg_l);
  // streamed members and their repulsion work items (aggregate, first row):
  // R row slots of 64 per wave, taken in descending-work order
  std::vector<int> rows;
  for (int a : big)
    for (int li = 0; li < h_pt_ip[a + 1] - h_pt_ip[a]; ++li) rows.push_back(h_pt_ip[a] + li);
  // split aggregates: this rank's row tiles are streamed rows like the others; every
  // member is initialised and given its internal degree (all are columns)
  const int rank = pl->comm ? pl->comm->rank : 0, nranks = pl->comm ? pl->comm->nranks : 1;
  auto tiles_of = [&](int a, int r, int& t0, int& t1) {
    const long long T = (h_pt_ip[a + 1] - h_pt_ip[a] + 63) / 64;
    t0 = (int)(T * r / nranks);
    t1 = (int)(T * (r + 1) / nranks);
  };
  std::vector<int> irows = rows;
  std::vector<int> xr, xcounts(nranks, 0);
  for (int r = 0; r < nranks; ++r)
    for (int a : split) {
      const int s = h_pt_ip[a + 1] - h_pt_ip[a];
      int t0, t1;
      tiles_of(a, r, t0, t1);
      for (int li = 64 * t0; li < std::min(s, 64 * t1); ++li) {
        const int c = h_pt_ip[a] + li;
        if (r == rank) rows.push_back(c);
        irows.push_back(c);
        xr.push_back(c);
        ++xcounts[r];
      }
    }
  // row slots x partners in flight (GE_FAML_R / GE_FAML_U override; only the
  // compiled variants of GE_BIG_VARIANTS are accepted)
  int R = kBigDefaultR, U = kBigDefaultU;
  if (const char* e = std::getenv("GE_FAML_R")) R = std::atoi(e);
  if (const char* e = std::getenv("GE_FAML_U")) U = std::atoi(e);
  bool known = false;
#define GE_BIG_KNOWN(RR, UU) known = known || (R == RR && U == UU);
  GE_BIG_VARIANTS(GE_BIG_KNOWN)
#undef GE_BIG_KNOWN
  if (!known) {
    R = kBigDefaultR;
    U = kBigDefaultU;
  }
  std::vector<int> erows;
  if (!rows.empty()) {  // degree classes of the streamed members' CSR rows
    std::vector<int> h_ip(pl->n + 1), h_ptix(pl->n);
    GE_HIP(hipMemcpyAsync(h_ip.data(), pl->ip, sizeof(int) * (pl->n + 1), hipMemcpyDeviceToHost, st));
    GE_HIP(hipMemcpyAsync(h_ptix.data(), pl->pt_ix, sizeof(int) * pl->n, hipMemcpyDeviceToHost,
                          st));
    GE_HIP(hipStreamSynchronize(st));
    std::vector<int> deg(rows.size());
    for (size_t q = 0; q < rows.size(); ++q) {
      const int v = h_ptix[rows[q]];
      deg[q] = h_ip[v + 1] - h_ip[v];
      pl->streamed_entries += deg[q];
    }
    // the in-aggregate repulsion is not far above the external pulls (measured
    // at C3: every heavy row left the binade), so heavy rows store their terms
    std::vector<int> hdeg;
    classify_rows(rows, deg, erows, pl->ecls, kSegStore, &hdeg);
    pl->ecode.alloc(std::max(h_ip[pl->n], 1));
    pl->erows.alloc(erows.size());
    pl->erows.upload(erows.data(), erows.size(), st);
    pl->ecls.bind(pl->erows.p);
    pl->rstreams.attach(pl->ecls, pl->dim, st, hdeg);
  }
  // split tiles are one-row-slot items (R = 1): settle R before any item is built,
  // so the whole-aggregate items step by the R the kernel is launched with
  for (int a : split) {
    int t0, t1;
    tiles_of(a, rank, t0, t1);
    if (t1 > t0) R = 1;
  }
  struct Item { int a, r0; double work; };
  std::vector<Item> its;
  for (int a : big) {
    const int s = h_pt_ip[a + 1] - h_pt_ip[a];
    for (int r0 = 0; r0 < s; r0 += 64 * R)
      its.push_back({a, r0, (double)std::min(R, (s - r0 + 63) / 64) * s});
  }
  for (int a : split) {  // this rank's tiles, one item each (R = 1 rows per slot)
    const int s = h_pt_ip[a + 1] - h_pt_ip[a];
    int t0, t1;
    tiles_of(a, rank, t0, t1);
    for (int t = t0; t < t1; ++t) its.push_back({a, 64 * t, (double)s});
  }
  std::stable_sort(its.begin(), its.end(),
                   [](const Item& x, const Item& y) { return x.work > y.work; });
  std::vector<int2> items;
  for (const Item& it : its) items.push_back(make_int2(it.a, it.r0));
  // symmetric sweeps: one unit per (aggregate, row tile), in the order of their
  // earliest start (2A tile-times into the aggregate), larger aggregates first
  {
    const char* e = std::getenv("GE_FAML_SYM");
    pl->sym = !(e && *e == '0');
  }
  if (pl->sym && (!big.empty() || !split.empty())) {
    // The sweeps of an aggregate with T row tiles form a chain of ~2.5 T tile-times
    // (each sweep starts after its predecessor has passed its first two tiles); the
    // launch takes about (sum of T^2 / 2 sweep tiles) / (resident waves).  While the
    // longest chain exceeds that, the largest aggregate runs as plain row blocks
    // (every ordered pair, ~0.8 the step cost of a sweep, no chain).
    std::vector<int> T(big.size());
    const bool any_big = !big.empty();
    for (size_t b = 0; b < big.size(); ++b) T[b] = (h_pt_ip[big[b] + 1] - h_pt_ip[big[b]] + 63) / 64;
    int occ = 1;
    dispatch_dim(dim, [&](auto Dc) {
      constexpr int D = decltype(Dc)::value;
      GE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &occ, (const void*)faml_sym_repulse<D, false>, kSymT, 0));
    });
    // three blocks (waves) per SIMD of the four that fit: fewer units in flight spin
    // less on hand-overs (C4 N = 1: 137.2 against 138.3 ms per launch; N = 8 shares
    // 30.0 against 32.7 ms; scripts/sym_timeline.py, profiles/r03/sym_timeline)
    const int bpc = std::min(std::max(occ, 1), 3);
    pl->sym_blocks = cus * bpc;
    const double waves = (double)pl->sym_blocks * (kSymT / 64);
    // Per streamed aggregate: symmetric sweeps or whole row blocks.  The launch lasts
    // about max(work / waves, the longest row block, the sweeps' start + the longest
    // sweep chain) tile-times, where
    //   sweeps:  work T^2 / 2 + T,  chain chain_k T (each sweep starts ~2 tiles behind
    //            the one before)
    //   rows:    work row_k T^2,    chain row_k T   (every ordered pair, no chain)
    // Whole row blocks are first in the queue, so when they hold more than the waves
    // the sweeps start late (start = their work / waves).  The k largest aggregates
    // run as row blocks, k minimising the prediction; no mix whose row blocks hold
    // more than half the waves (their raised waves delay and slow the sweeps: per-rank
    // shares of C4, N = 4: 20 of 24 aggregates as row blocks 70 ms per iteration, 7 of
    // 25 58 ms).  At N = 1 (C4) the launch is work-bound and every aggregate sweeps;
    // the shares of a multi-GPU run are chain-bound.
    // row_k: a row-block tile (64 x 64 ordered pairs) against a sweep tile (64 x 64
    // unordered), wave time at full load -- 0.6 measured on an N = 8 share of C4
    // (all row blocks: 17.9 us per row tile per wave, against 29.8 us per sweep tile
    // at N = 1; profiles/r04/sym_timeline_rows_n8.json)
    double chain_k = 2.5;
    const double row_k = 0.6;
    if (const char* e = std::getenv("GE_FAML_SYM_CHAIN")) chain_k = std::atof(e);  // 0: all sweeps
    std::vector<char> as_rows(big.size(), 0);
    double best = 0.0;
    if (chain_k > 0.0 && any_big) {
      std::vector<size_t> by_T(big.size());
      std::iota(by_T.begin(), by_T.end(), 0);
      std::stable_sort(by_T.begin(), by_T.end(), [&](size_t x, size_t y) { return T[x] > T[y]; });
      double work = 0.0, row_work = 0.0, row_units = 0.0, pbest = 1e300;
      size_t best_k = 0;
      for (size_t b = 0; b < big.size(); ++b) work += 0.5 * T[b] * (double)T[b] + T[b];
      for (size_t k = 0; k <= by_T.size(); ++k) {  // the k largest as row blocks
        const double start = row_units > waves ? row_work / waves : 0.0;
        const double sweep_chain = k < by_T.size() ? start + chain_k * T[by_T[k]] : 0.0;
        const double row_path = k > 0 ? row_k * T[by_T[0]] : 0.0;
        const double pred = std::max(work / waves, std::max(sweep_chain, row_path));
        const bool mixed_late = 2.0 * row_units > waves && k < by_T.size();
        if (!mixed_late && pred < pbest * 0.999) {
          pbest = pred;
          best_k = k;
        }
        if (k < by_T.size()) {
          const double t = T[by_T[k]];
          work += row_k * t * t - (0.5 * t * t + t);
          row_work += row_k * t * t;
          row_units += t;
        }
      }
      for (size_t k = 0; k < best_k; ++k) as_rows[by_T[k]] = 1;
      best = pbest;
    }
    pl->rows_mode = pl->swept = 0;
    for (size_t b = 0; b < big.size(); ++b) {
      if (as_rows[b]) ++pl->rows_mode;
      else ++pl->swept;
    }
    struct Unit { int a, A, pb, T, kind; double est; };
    std::vector<Unit> us;
    int pb = 0;
    // Queue position of sweep A of an aggregate of T row tiles: 2A Tmax / T, i.e.
    // every aggregate's sweeps spread over the whole queue, so all aggregates reach
    // their last (chain-bound) sweeps together and the launch ends without a tail of
    // the largest aggregate's chain (C4: tail after the queue drained 8.7 -> 3.5 ms,
    // 148.1 -> 143.2 ms per launch; 2A alone, the sweep's earliest start, was the
    // round-2 order).  Every sweep comes after the sweeps it waits on (sweep A - 1
    // before A).
    const double est_k = 2.0;
    const int Tmax = big.empty() ? 1 : *std::max_element(T.begin(), T.end());
    // Big aggregates a little ahead: positions also scaled by 1 - g T / Tmax (g = 0.3),
    // so the largest chains finish before the queue's end and the small aggregates'
    // short chains fill it (C4, one box, 3 rounds interleaved: 136.2-136.4 against
    // 136.9-137.3 ms per step; g = 0.15 136.5-136.7, 0.5 and 0.7 slower;
    // profiles/r04/ab_big_first.log).  Positions stay increasing in A for g < 1, so
    // every unit still waits only on units before it.
    const double big_first = 0.3;
    auto scale_of = [&](int Tb) {
      return ((double)Tmax / Tb) * (1.0 - big_first * Tb / Tmax);
    };
    // row blocks' issue priority: one level per quarter of the longest row block's
    // column tiles (ge_sym.hpp rows_prio; one level per sixth or eighth: no different,
    // profiles/r05/scale_sim_c4_prio_divisor.log)
    int rows_q = 0;
    const int prio_div = 4;
    for (size_t b = 0; b < big.size(); ++b)
      if (as_rows[b]) rows_q = std::max(rows_q, T[b]);
    for (int a : split) rows_q = std::max(rows_q, (h_pt_ip[a + 1] - h_pt_ip[a] + 63) / 64);
    rows_q = (rows_q + prio_div - 1) / prio_div;
    for (size_t b = 0; b < big.size(); ++b) {
      if (as_rows[b]) {
        // row blocks have no dependencies and each spans its aggregate's whole width:
        // first in the queue, longest first (measured on per-rank shares of C4: N = 4
        // 69 ms per iteration against 80 ms when spread among the sweeps).  Round 5
        // tried cutting the last-taken blocks into a head and a tail segment
        // (McNaughton's wrap-around, so the queue's last round is short): bit-exact,
        // no faster (N = 8 shares 26.6-28.0 against 27.0-27.3 ms per launch,
        // profiles/r05/scale_sim_c4_tailsplit.log) -- the share is bound by the row
        // blocks' instruction stream, not by the queue's last round.
        for (int A = 0; A < T[b]; ++A) us.push_back({big[b], A, rows_q, T[b], kUnitRows, -1.0});
        continue;
      }
      const double sc = scale_of(T[b]);
      // (round 6 measured sweep issue priorities by the followers a sweep holds up:
      // 115.8-116.0 against 115.3-115.4 ms per launch, profiles/r06/ab_sym_prio.log)
      for (int A = 0; A < T[b]; ++A) us.push_back({big[b], A, pb, T[b], kUnitSweep, est_k * A * sc});
      pb += T[b];
    }
    for (int a : split) {  // this rank's row tiles of the split aggregates: row blocks
      int t0, t1;
      tiles_of(a, rank, t0, t1);
      const int Ta = (h_pt_ip[a + 1] - h_pt_ip[a] + 63) / 64;
      for (int A = t0; A < t1; ++A) us.push_back({a, A, rows_q, Ta, kUnitRows, -1.0});
    }
    std::stable_sort(us.begin(), us.end(), [](const Unit& x, const Unit& y) {
      return x.est != y.est ? x.est < y.est : x.T > y.T;
    });
    std::vector<int4> h_units;
    for (const Unit& x : us) h_units.push_back(make_int4(x.a, x.A, x.pb, x.kind));
    pl->nunits = (int)h_units.size();
    pl->ntiles = pb;
    pl->units.alloc(h_units.size());
    pl->units.upload(h_units.data(), h_units.size(), st);
    if (const char* e = std::getenv("GE_SYM_STAMPS")) {  // diagnostics: timeline of each launch
      pl->stamp_path = e;
      pl->h_units = h_units;
      pl->stamps.alloc(h_units.size() * kStampWords);
    }
    pl->prog.alloc(std::max(pb, 1));
    if (pb > 0) pl->hand.alloc((size_t)pl->n * dim);
    pl->sym_err.alloc(1);
    GE_HIP(hipMemsetAsync(pl->sym_err.p, 0, sizeof(int), st));
    int khz = 0;
    GE_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    // one hand-over normally waits at most a few tile-times (tens of microseconds)
    pl->sym_limit = (long long)std::max(khz, 1000) * 5000;  // ~5 s
  }
  pl->R = R;
  pl->code = big_code(R, U);
  for (int a : big) {
    const double sa = h_pt_ip[a + 1] - h_pt_ip[a];
    pl->streamed_pairs += sa * (sa - 1);
  }
  for (int a : split) {  // this rank's rows against all members
    int t0, t1;
    tiles_of(a, rank, t0, t1);
    const double sa = h_pt_ip[a + 1] - h_pt_ip[a];
    pl->streamed_pairs += (std::min(sa, 64.0 * t1) - std::min(sa, 64.0 * t0)) * (sa - 1);
  }
  // 4 waves per SIMD: more items per wave for the queue to balance (C3 level
  // 0: 961 ms per call against 1091 ms at the full 8 waves per SIMD)
  const int occ = rep_occupancy(dim, pl->code);
  const int blocks_cu = std::min(4, occ);
  pl->rep_blocks = cus * blocks_cu;
  std::vector<int> begs;
  begs.insert(begs.end(), beg_s.begin(), beg_s.end());
  pl->off_m = begs.size();
  begs.insert(begs.end(), beg_m.begin(), beg_m.end());
  pl->off_l = begs.size();
  begs.insert(begs.end(), beg_l.begin(), beg_l.end());
  pl->ns = (int)beg_s.size() - 1;
  pl->nm = (int)beg_m.size() - 1;
  pl->nl = (int)beg_l.size() - 1;
  pl->nrows = (int)rows.size();
  pl->nirows = (int)irows.size();
  pl->nitems = (int)items.size();
  std::vector<int> huge = big;  // centred and scaled at the end: the split ones on every rank
  huge.insert(huge.end(), split.begin(), split.end());
  pl->nhuge = (int)huge.size();

  const int n = pl->n;
  pl->pos.alloc(std::max(n, 1));
  pl->order.alloc(std::max<size_t>(order.size(), 1));
  pl->beg.alloc(std::max<size_t>(begs.size(), 1));
  pl->rows.alloc(std::max<size_t>(rows.size(), 1));
  pl->items.alloc(std::max<size_t>(items.size(), 1));
  pl->queue.alloc(std::max(pl->iterations, 1));
  pl->huge.alloc(std::max<size_t>(huge.size(), 1));
  pl->irows.alloc(std::max<size_t>(irows.size(), 1));
  pl->irows.upload(irows.data(), irows.size(), st);
  pl->order.upload(order.data(), order.size(), st);
  pl->beg.upload(begs.data(), begs.size(), st);
  pl->rows.upload(rows.data(), rows.size(), st);
  pl->items.upload(items.data(), items.size(), st);
  pl->huge.upload(huge.data(), huge.size(), st);
  if (!split.empty() && nranks > 1) {  // the per-iteration exchange of the split rows
    pl->h_xcounts = xcounts;
    pl->h_xfirst.assign(nranks + 1, 0);
    for (int r = 0; r < nranks; ++r) pl->h_xfirst[r + 1] = pl->h_xfirst[r] + xcounts[r];
    pl->xwidth = std::max(1, *std::max_element(xcounts.begin(), xcounts.end()));
    pl->xrows.alloc(std::max<size_t>(xr.size(), 1));
    pl->xrows.upload(xr.data(), xr.size(), st);
    pl->xcounts.alloc(nranks);
    pl->xcounts.upload(xcounts.data(), nranks, st);
    pl->xfirst.alloc(nranks + 1);
    pl->xfirst.upload(pl->h_xfirst.data(), nranks + 1, st);
    pl->xbuf.alloc((size_t)pl->xwidth * dim * nranks);
  }
  pl->Fscr.alloc((size_t)std::max(n, 1) * dim);
  pl->Fprev.alloc((size_t)std::max(n, 1) * dim);
  if (pl->nirows > 0) {
    pl->Xa.alloc((size_t)n * dim);
    pl->Xb.alloc((size_t)n * dim);
    pl->DP.alloc(n);
  }
  hipLaunchKernelGGL(pos_of_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, pl->pt_ix,
                     pl->pos.p);
  if (pl->nrows > 0) {
    hipLaunchKernelGGL(edge_code_kernel, dim3((pl->nrows + 255) / 256), dim3(256), 0, st,
                       pl->nrows, pl->rows.p, pl->pt_ip, pl->pt_ix, pl->pos.p, pl->vA, pl->ip,
                       pl->ix, pl->ecode.p);
  }
  if (pl->nirows > 0)
    hipLaunchKernelGGL(faml_huge_dp, dim3((pl->nirows + kHT - 1) / kHT), dim3(kHT), 0, st,
                       pl->nirows, pl->irows.p, pl->pt_ix, pl->vA, pl->ip, pl->ix, pl->dx, pl->DP.p,
                       pl->c.use_weights);
  GE_HIP(hipGetLastError());
  for (int k = 0; k < 3; ++k) {
    GE_HIP(hipStreamCreateWithFlags(&pl->side[k], hipStreamNonBlocking));
    GE_HIP(hipEventCreateWithFlags(&pl->join[k], hipEventDisableTiming));
  }
  GE_HIP(hipEventCreateWithFlags(&pl->fork, hipEventDisableTiming));
  GE_HIP(hipStreamSynchronize(st));
}

static void faml_plan_run(ge_faml_plan* pl, const double* cA, const double* rA, const double* init,
                          double* X) {
  hipStream_t st = pl->ctx->stream;
  hipEvent_t* ev = nullptr;
  if (pl->profiling) {
    if (pl->next_ev + 4 > pl->ev.size())
      for (int k = 0; k < 64; ++k) {
        hipEvent_t e;
        GE_HIP(hipEventCreate(&e));
        pl->ev.push_back(e);
      }
    ev = &pl->ev[pl->next_ev];
    pl->next_ev += 4;
  }
  const int iters = pl->iterations;
  const FaConst& c = pl->c;
  dispatch_dim(pl->dim, [&](auto Dc) {
    constexpr int D = decltype(Dc)::value;
    GE_HIP(hipEventRecord(pl->fork, st));
    for (int k = 0; k < 3; ++k) GE_HIP(hipStreamWaitEvent(pl->side[k], pl->fork, 0));
    if (ev) GE_HIP(hipEventRecord(ev[0], st));
    // resident classes: large on side[1], mid on side[2], small on the context stream
    auto launch_resident = [&] {
      if (pl->nl > 0)
        hipLaunchKernelGGL((faml_resident<D, 256, large_cap(D)>), dim3(pl->nl), dim3(256), 0,
                           pl->side[1], pl->order.p, pl->beg.p + pl->off_l, pl->pt_ip, pl->pt_ix,
                           pl->pos.p, pl->vA, pl->ip, pl->ix, pl->dx, cA, rA, init, pl->Fscr.p,
                           pl->Fprev.p, X, iters, c);
      if (pl->nm > 0)
        hipLaunchKernelGGL((faml_resident<D, 256, 256>), dim3(pl->nm), dim3(256), 0, pl->side[2],
                           pl->order.p, pl->beg.p + pl->off_m, pl->pt_ip, pl->pt_ix, pl->pos.p,
                           pl->vA, pl->ip, pl->ix, pl->dx, cA, rA, init, pl->Fscr.p, pl->Fprev.p,
                           X, iters, c);
      if (pl->ns > 0)
        hipLaunchKernelGGL((faml_resident<D, 64, 64>), dim3(pl->ns), dim3(64), 0, st, pl->order.p,
                           pl->beg.p, pl->pt_ip, pl->pt_ix, pl->pos.p, pl->vA, pl->ip, pl->ix,
                           pl->dx, cA, rA, init, pl->Fscr.p, pl->Fprev.p, X, iters, c);
    };
    // streamed path (side[0])
    hipStream_t ss = pl->side[0];
    if (ev) GE_HIP(hipEventRecord(ev[2], ss));
    if (pl->nirows > 0) {
      const int nr = pl->nirows;
      hipLaunchKernelGGL((faml_huge_init<D>), dim3((nr + kHT - 1) / kHT), dim3(kHT), 0, ss,
                         nr, pl->irows.p, init, pl->Xa.p, pl->Fprev.p);
      GE_HIP(hipMemsetAsync(pl->queue.p, 0, sizeof(int) * iters, ss));
      double* cur = pl->Xa.p;
      double* nxt = pl->Xb.p;
      for (int it = 0; it < iters; ++it) {
        hipEvent_t* re = nullptr;
        if (pl->profiling) {
          if (pl->next_rev + 2 > pl->rev.size())
            for (int k = 0; k < 256; ++k) {
              hipEvent_t e;
              GE_HIP(hipEventCreate(&e));
              pl->rev.push_back(e);
            }
          re = &pl->rev[pl->next_rev];
          pl->next_rev += 2;
          GE_HIP(hipEventRecord(re[0], ss));
        }
        const FamlRows<D> fr{pl->pt_ip, pl->pt_ix, pl->ecode.p, pl->ip, pl->vA, pl->dx,
                             cA, cur, pl->DP.p, pl->Fscr.p, nxt, pl->Fprev.p, c};
        if (pl->sym) {
          if (pl->ntiles) GE_HIP(hipMemsetAsync(pl->prog.p, 0, sizeof(int) * pl->ntiles, ss));
          double* H = pl->hand.p;  // hand-overs component-major (ge_sym.hpp sym_handover)
          const size_t hs = (size_t)pl->n;
          int* err = pl->sym_err.p;
          const long long lim = pl->sym_limit;
          if (!pl->stamp_path.empty()) {
            hipLaunchKernelGGL((faml_sym_repulse<D, false, true>), dim3(pl->sym_blocks),
                               dim3(kSymT), 0, ss, pl->nunits, pl->units.p, pl->queue.p + it,
                               pl->pt_ip, cur, pl->DP.p, c.repel, pl->Fscr.p, H, hs, pl->prog.p,
                               err, lim, pl->stamps.p);
          } else {
            sym_repulse_launch(D, pl->sym_blocks, ss, pl->nunits, pl->units.p, pl->queue.p + it,
                               pl->pt_ip, cur, pl->DP.p, c.repel, pl->Fscr.p, H, hs, pl->prog.p,
                               err, lim);
          }
        } else {
          launch_big_repulse<D>(pl->code, pl->rep_blocks, ss, pl->nitems, pl->items.p,
                                pl->queue.p + it, pl->pt_ip, cur, pl->DP.p, c.repel, pl->Fscr.p);
        }
        if (re) GE_HIP(hipEventRecord(re[1], ss));
        hipEvent_t* ae = nullptr;
        if (pl->profiling) {
          if (pl->next_aev + 2 > pl->aev.size())
            for (int k = 0; k < 256; ++k) {
              hipEvent_t e;
              GE_HIP(hipEventCreate(&e));
              pl->aev.push_back(e);
            }
          ae = &pl->aev[pl->next_aev];
          pl->next_aev += 2;
          GE_HIP(hipEventRecord(ae[0], ss));
        }
        if (pl->nrows > 0) launch_rows<D>(pl->ecls, fr, ss, pl->rstreams);
        if (ae) GE_HIP(hipEventRecord(ae[1], ss));
        if (pl->xwidth > 0)  // every rank's rows of the split aggregates, for the next step
          exchange_rows(pl->comm, ss, D, pl->xrows.p, pl->xcounts.p, pl->xfirst.p,
                        pl->h_xcounts.data(), pl->h_xfirst.data(), pl->xwidth, pl->xbuf.p, nxt);
        std::swap(cur, nxt);
      }
      hipLaunchKernelGGL((faml_huge_finish<D>), dim3(pl->nhuge), dim3(kHT), 0, ss, pl->huge.p,
                         pl->pt_ip, pl->pt_ix, cur, cA, rA, X);
    }
    if (ev) GE_HIP(hipEventRecord(ev[3], ss));
    // the resident classes beside the streamed path: queued after it, they cost the
    // repulsion launch ~0.3 ms; run after it, ~1.4 ms per step; queued before it,
    // nothing changes (profiles/r04/ab_launch_order.log)
    launch_resident();
    for (int k = 0; k < 3; ++k) GE_HIP(hipEventRecord(pl->join[k], pl->side[k]));
    for (int k = 1; k < 3; ++k) GE_HIP(hipStreamWaitEvent(st, pl->join[k], 0));
    if (ev) GE_HIP(hipEventRecord(ev[1], st));  // resident classes done
    GE_HIP(hipStreamWaitEvent(st, pl->join[0], 0));
  });
  GE_HIP(hipGetLastError());
  if (pl->sym && pl->nunits > 0) {  // a hand-over wait that timed out fails the call
    int err = 0;
    GE_HIP(hipMemcpyAsync(&err, pl->sym_err.p, sizeof(int), hipMemcpyDeviceToHost, st));
    GE_HIP(hipStreamSynchronize(st));
    if (err) {
      GE_HIP(hipMemsetAsync(pl->sym_err.p, 0, sizeof(int), st));
      throw Error(GE_ERR_STATE,
                  "forceAtlasMultilevel: a symmetric sweep's hand-over wait timed out");
    }
  }
  if (!pl->stamp_path.empty() && pl->nunits > 0) {  // the last launch's timeline
    std::vector<long long> h((size_t)pl->nunits * kStampWords);
    GE_HIP(hipStreamSynchronize(st));
    GE_HIP(hipMemcpy(h.data(), pl->stamps.p, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
    if (FILE* f = std::fopen(pl->stamp_path.c_str(), "wb")) {
      const int hdr[4] = {pl->nunits, kStampWords, pl->sym_blocks, kSymT};
      std::fwrite(hdr, sizeof(int), 4, f);
      std::fwrite(pl->h_units.data(), sizeof(int4), pl->h_units.size(), f);
      std::fwrite(h.data(), sizeof(long long), h.size(), f);
      std::fclose(f);
    }
  }
}

void sym_repulse_launch(int dim, int blocks, hipStream_t s, int nunits, const int4* units,
                        int* queue, const int* seg, const double* X, const double* DP,
                        double repel, double* F, double* H, size_t hs, int* prog, int* err,
                        long long limit) {
  dispatch_dim(dim, [&](auto Dc) {
    constexpr int D = decltype(Dc)::value;
    if (repel == 1.0)
      hipLaunchKernelGGL((faml_sym_repulse<D, true>), dim3(blocks), dim3(kSymT), 0, s, nunits,
                         units, queue, seg, X, DP, repel, F, H, hs, prog, err, limit, nullptr);
    else
      hipLaunchKernelGGL((faml_sym_repulse<D, false>), dim3(blocks), dim3(kSymT), 0, s, nunits,
                         units, queue, seg, X, DP, repel, F, H, hs, prog, err, limit, nullptr);
  });
  GE_HIP(hipGetLastError());
}

// Blocks per CU of a single-level symmetric launch (one aggregate of n / 64 row
// tiles: one convoy of sweeps, each behind the one before).  Two of the four that
// fit: C2 1539.8 ms per iteration against 1631.9 at three and 1806.8 at four
// (profiles/r04/c2_sym_blocks.log) -- fewer sweeps in flight wait less on each other.
int sym_blocks_per_cu(int dim) {
  int occ = 1;
  dispatch_dim(dim, [&](auto Dc) {
    constexpr int D = decltype(Dc)::value;
    GE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &occ, (const void*)faml_sym_repulse<D, false>, kSymT, 0));
  });
  return std::min(std::max(occ, 1), 2);
}

static void faml_plan_free(ge_faml_plan* pl) {
  if (!pl) return;
  for (int k = 0; k < 3; ++k) {
    if (pl->side[k]) {
      (void)hipStreamSynchronize(pl->side[k]);
      (void)hipStreamDestroy(pl->side[k]);
    }
    if (pl->join[k]) (void)hipEventDestroy(pl->join[k]);
  }
  if (pl->fork) (void)hipEventDestroy(pl->fork);
  for (hipEvent_t e : pl->ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : pl->rev) (void)hipEventDestroy(e);
  for (hipEvent_t e : pl->aev) (void)hipEventDestroy(e);
  delete pl;
}

void faml_run_device(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix, const double* d_dx,
                     int m, const int* h_pt_ip, const int* d_pt_ip, const int* d_pt_ix,
                     const int* d_vA, const double* d_cA, const double* d_rA,
                     const double* d_init, double* d_x, int dim, int iterations,
                     const ge_fa_params& p) {
  GE_REQUIRE(h_pt_ip[m] == n, "P_T must have one entry per fine vertex");
  auto* pl = new ge_faml_plan();
  try {
    pl->ctx = ctx;
    pl->n = n;
    pl->m = m;
    pl->dim = dim;
    pl->iterations = iterations;
    pl->ip = d_ip;
    pl->ix = d_ix;
    pl->dx = d_dx;
    pl->pt_ip = d_pt_ip;
    pl->pt_ix = d_pt_ix;
    pl->vA = d_vA;
    pl->c = make_fa_const(p);
    std::vector<int> all(m);
    std::iota(all.begin(), all.end(), 0);
    faml_plan_build(pl, h_pt_ip, all);
    faml_plan_run(pl, d_cA, d_rA, d_init, d_x);
    GE_HIP(hipStreamSynchronize(ctx->stream));
  } catch (...) {
    faml_plan_free(pl);
    throw;
  }
  faml_plan_free(pl);
}

}  // namespace ge

extern "C" {

static int faml_plan_create_impl(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix,
                                 const double* d_dx, int m, const int* h_pt_ip,
                                 const int* d_pt_ip, const int* d_pt_ix, const int* d_vA,
                                 int dim, const ge_fa_params* p, int iterations,
                                 const std::vector<int>& aggs, ge_faml_plan** out,
                                 ge_comm* comm = nullptr,
                                 const std::vector<int>& split = std::vector<int>()) {
  return ge::guarded([&] {
    ge::DeviceGuard g(ctx);
    auto* pl = new ge_faml_plan();
    try {
      pl->ctx = ctx;
      pl->comm = comm;
      pl->n = n;
      pl->m = m;
      pl->dim = dim;
      pl->iterations = iterations;
      pl->ip = d_ip;
      pl->ix = d_ix;
      pl->dx = d_dx;
      pl->pt_ip = d_pt_ip;
      pl->pt_ix = d_pt_ix;
      pl->vA = d_vA;
      pl->c = ge::make_fa_const(*p);
      ge::faml_plan_build(pl, h_pt_ip, aggs, split);
    } catch (...) {
      ge::faml_plan_free(pl);
      throw;
    }
    *out = pl;
  });
}

static void faml_plan_check(ge_ctx* ctx, int n, int m, const int* h_pt_ip, int dim,
                            const ge_fa_params* p, void* out) {
  GE_REQUIRE(ctx && p && out && h_pt_ip, "null argument");
  GE_REQUIRE(dim >= 1 && dim <= 4, "dimension must be 1..4");
  GE_REQUIRE(n > 0 && m > 0 && h_pt_ip[0] == 0 && h_pt_ip[m] == n,
             "P_T must have one entry per fine vertex");
}

int ge_faml_plan_create(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix, const double* d_dx,
                        int m, const int* h_pt_ip, const int* d_pt_ip, const int* d_pt_ix,
                        const int* d_vA, int dim, const ge_fa_params* p, int iterations,
                        int agg_begin, int agg_end, ge_faml_plan** out) {
  std::vector<int> aggs;
  const int rc = ge::guarded([&] {
    faml_plan_check(ctx, n, m, h_pt_ip, dim, p, out);
    GE_REQUIRE(0 <= agg_begin && agg_begin <= agg_end && agg_end <= m, "bad aggregate range");
    aggs.resize(agg_end - agg_begin);
    std::iota(aggs.begin(), aggs.end(), agg_begin);
  });
  if (rc != GE_OK) return rc;
  return faml_plan_create_impl(ctx, n, d_ip, d_ix, d_dx, m, h_pt_ip, d_pt_ip, d_pt_ix, d_vA, dim,
                               p, iterations, aggs, out);
}

int ge_faml_plan_create_subset(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix,
                               const double* d_dx, int m, const int* h_pt_ip,
                               const int* d_pt_ip, const int* d_pt_ix, const int* d_vA, int dim,
                               const ge_fa_params* p, int iterations, const int* h_aggs,
                               int n_aggs, ge_faml_plan** out) {
  std::vector<int> aggs;
  const int rc = ge::guarded([&] {
    faml_plan_check(ctx, n, m, h_pt_ip, dim, p, out);
    GE_REQUIRE(n_aggs >= 0 && (h_aggs || n_aggs == 0), "bad aggregate list");
    for (int q = 0; q < n_aggs; ++q)
      GE_REQUIRE(h_aggs[q] >= 0 && h_aggs[q] < m && (q == 0 || h_aggs[q] > h_aggs[q - 1]),
                 "aggregate ids must be strictly increasing and < m");
    aggs.assign(h_aggs, h_aggs + n_aggs);
  });
  if (rc != GE_OK) return rc;
  return faml_plan_create_impl(ctx, n, d_ip, d_ix, d_dx, m, h_pt_ip, d_pt_ip, d_pt_ix, d_vA, dim,
                               p, iterations, aggs, out);
}

int ge_faml_plan_create_shard(ge_ctx* ctx, ge_comm* comm, int n, const int* d_ip,
                              const int* d_ix, const double* d_dx, int m, const int* h_pt_ip,
                              const int* d_pt_ip, const int* d_pt_ix, const int* d_vA, int dim,
                              const ge_fa_params* p, int iterations, const int* h_aggs,
                              int n_aggs, const int* h_split, int n_split, ge_faml_plan** out) {
  std::vector<int> aggs, split;
  const int rc = ge::guarded([&] {
    faml_plan_check(ctx, n, m, h_pt_ip, dim, p, out);
    GE_REQUIRE(comm && comm->ctx == ctx, "the communicator must belong to the plan's context");
    GE_REQUIRE(n_aggs >= 0 && (h_aggs || n_aggs == 0) && n_split >= 0 && (h_split || n_split == 0),
               "bad aggregate lists");
    std::vector<char> seen(m, 0);
    for (int q = 0; q < n_aggs; ++q) {
      GE_REQUIRE(h_aggs[q] >= 0 && h_aggs[q] < m && (q == 0 || h_aggs[q] > h_aggs[q - 1]),
                 "aggregate ids must be strictly increasing and < m");
      seen[h_aggs[q]] = 1;
    }
    for (int q = 0; q < n_split; ++q) {
      GE_REQUIRE(h_split[q] >= 0 && h_split[q] < m && (q == 0 || h_split[q] > h_split[q - 1]),
                 "split aggregate ids must be strictly increasing and < m");
      GE_REQUIRE(!seen[h_split[q]], "an aggregate is both whole and split");
    }
    aggs.assign(h_aggs, h_aggs + n_aggs);
    split.assign(h_split, h_split + n_split);
  });
  if (rc != GE_OK) return rc;
  return faml_plan_create_impl(ctx, n, d_ip, d_ix, d_dx, m, h_pt_ip, d_pt_ip, d_pt_ix, d_vA, dim,
                               p, iterations, aggs, out, comm, split);
}

int ge_faml_plan_run(ge_faml_plan* pl, const double* d_cA, const double* d_rA,
                     const double* d_init, double* d_coords) {
  return ge::guarded([&] {
    GE_REQUIRE(pl && d_cA && d_rA && d_init && d_coords, "null argument");
    ge::DeviceGuard g(pl->ctx);
    ge::faml_plan_run(pl, d_cA, d_rA, d_init, d_coords);
  });
}

int ge_faml_plan_set_profiling(ge_faml_plan* pl, int enable) {
  return ge::guarded([&] {
    GE_REQUIRE(pl, "null plan");
    pl->profiling = enable != 0;
    pl->next_ev = 0;
    pl->next_rev = 0;
    pl->next_aev = 0;
  });
}

int ge_faml_plan_kernel_ms(ge_faml_plan* pl, double* resident_ms, double* streamed_ms,
                           int* runs) {
  return ge::guarded([&] {
    GE_REQUIRE(pl && resident_ms && streamed_ms && runs, "null argument");
    ge::DeviceGuard g(pl->ctx);
    GE_HIP(hipStreamSynchronize(pl->ctx->stream));
    double a = 0, b = 0;
    int cnt = 0;
    for (size_t k = 0; k + 4 <= pl->next_ev; k += 4) {
      float t1 = 0.f, t2 = 0.f;
      GE_HIP(hipEventElapsedTime(&t1, pl->ev[k], pl->ev[k + 1]));
      GE_HIP(hipEventElapsedTime(&t2, pl->ev[k + 2], pl->ev[k + 3]));
      a += t1;
      b += t2;
      ++cnt;
    }
    *resident_ms = cnt ? a / cnt : 0.0;
    *streamed_ms = cnt ? b / cnt : 0.0;
    *runs = cnt;
  });
}

int ge_faml_plan_repulse_ms(ge_faml_plan* pl, double* ms, int* launches, double* pairs) {
  return ge::guarded([&] {
    GE_REQUIRE(pl && ms && launches && pairs, "null argument");
    *pairs = pl->streamed_pairs;
    ge::DeviceGuard g(pl->ctx);
    GE_HIP(hipStreamSynchronize(pl->ctx->stream));
    double t = 0;
    int cnt = 0;
    for (size_t k = 0; k + 2 <= pl->next_rev; k += 2) {
      float x = 0.f;
      GE_HIP(hipEventElapsedTime(&x, pl->rev[k], pl->rev[k + 1]));
      t += x;
      ++cnt;
    }
    *ms = cnt ? t / cnt : 0.0;
    *launches = cnt;
  });
}

int ge_faml_plan_rows_ms(ge_faml_plan* pl, double* ms, int* passes, long long* rows,
                         long long* entries) {
  return ge::guarded([&] {
    GE_REQUIRE(pl && ms && passes && rows && entries, "null argument");
    *rows = pl->nrows;
    *entries = pl->streamed_entries;
    ge::DeviceGuard g(pl->ctx);
    GE_HIP(hipStreamSynchronize(pl->ctx->stream));
    double t = 0;
    int cnt = 0;
    for (size_t k = 0; k + 2 <= pl->next_aev; k += 2) {
      float x = 0.f;
      GE_HIP(hipEventElapsedTime(&x, pl->aev[k], pl->aev[k + 1]));
      t += x;
      ++cnt;
    }
    *ms = cnt ? t / cnt : 0.0;
    *passes = cnt;
  });
}

int ge_faml_plan_schedule(ge_faml_plan* pl, int* sweeps, int* banded, int* row_blocks,
                          int* units) {
  return ge::guarded([&] {
    GE_REQUIRE(pl && sweeps && banded && row_blocks && units, "null argument");
    *sweeps = pl->swept;
    *banded = 0;  // bands were removed in round 5 (the ABI keeps the field)
    *row_blocks = pl->rows_mode;
    *units = pl->nunits;
  });
}

int ge_faml_plan_destroy(ge_faml_plan* pl) {
  return ge::guarded([&] { ge::faml_plan_free(pl); });
}

}  // extern "C"

