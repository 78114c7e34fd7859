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
#include <numeric>
#include <vector>

#include "ge_internal.hpp"
#include "ge_pair.hpp"

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
      rep_pair<D, false, false>(xi, xj, dip1, ds(j), c.repel, acc);
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
// Streamed path for huge aggregates.  Block b covers members
// [blk_li[b], blk_li[b]+256) of aggregate blk_agg[b].

constexpr int kHT = 256;

template <int D>
__global__ void __launch_bounds__(kHT)
faml_huge_init(const int* __restrict__ blk_agg, const int* __restrict__ blk_li,
               const int* __restrict__ pt_ip, const int* __restrict__ pt_ix,
               const int* __restrict__ vA, const int* __restrict__ ip,
               const int* __restrict__ ix, const double* __restrict__ dx,
               const double* __restrict__ init, double* __restrict__ Xp,
               double* __restrict__ DP, double* __restrict__ Fprev, int use_weights) {
  const int a = blk_agg[blockIdx.x];
  const int li = blk_li[blockIdx.x] + threadIdx.x;
  const int s = pt_ip[a + 1] - pt_ip[a];
  if (li >= s) return;
  const int c = pt_ip[a] + li;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    Xp[(size_t)c * D + k] = init[(size_t)c * D + k];
    Fprev[(size_t)c * D + k] = 0.0;
  }
  DP[c] = internal_dp1(pt_ix[c], a, ip, ix, dx, vA, use_weights);
}

template <int D>
__global__ void __launch_bounds__(kHT)
faml_huge_force(const int* __restrict__ blk_agg, const int* __restrict__ blk_li,
                const int* __restrict__ pt_ip, const int* __restrict__ pt_ix,
                const int* __restrict__ pos_of, const int* __restrict__ vA,
                const int* __restrict__ ip, const int* __restrict__ ix,
                const double* __restrict__ dx, const double* __restrict__ cA,
                const double* __restrict__ Xp, const double* __restrict__ DP,
                double* __restrict__ Fscr, MlConst c) {
  constexpr int WV = W<D>::v;
  __shared__ __attribute__((aligned(16))) double tile[kHT * WV];
  const int a = blk_agg[blockIdx.x];
  const int base = pt_ip[a];
  const int s = pt_ip[a + 1] - base;
  const int li = blk_li[blockIdx.x] + threadIdx.x;
  const bool ok = li < s;
  const int cpos = base + (ok ? li : 0);
  double xi[D], acc[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    xi[k] = Xp[(size_t)cpos * D + k];
    acc[k] = 0.0;
  }
  const double dip1 = DP[cpos];
  const bool row_ok = all_coord_ok<D>(xi);
  const bool rep_ok = row_ok && weight_ok(dip1) && weight_ok(c.repel);
  for (int j0 = 0; j0 < s; j0 += kHT) {
    const int cnt = min(kHT, s - j0);
    __syncthreads();
    if ((int)threadIdx.x < cnt) {
      const int cj = base + j0 + threadIdx.x;
#pragma unroll
      for (int k = 0; k < D; ++k) tile[threadIdx.x * WV + k] = Xp[(size_t)cj * D + k];
      tile[threadIdx.x * WV + D] = DP[cj];
    }
    __syncthreads();
    for (int jj = 0; jj < cnt; ++jj) {
      const double* xj = &tile[jj * WV];
      if (rep_ok && vertex_ok<D>(xj, tile[jj * WV + D]))
        rep_pair<D, true, false>(xi, xj, dip1, tile[jj * WV + D], c.repel, acc);
      else
        rep_pair<D, false, false>(xi, xj, dip1, tile[jj * WV + D], c.repel, acc);
    }
  }
  if (!ok) return;
  // the rest of member_force with the repulsion sum already in acc
  double m2 = xi[0] * xi[0];
#pragma unroll
  for (int k = 1; k < D; ++k) m2 = m2 + xi[k] * xi[k];
  double mag = sqrt(m2);
  if (mag < kEps) mag = kEps;
  const Recip rmag = recip_of(mag);
  const double* ca = cA + (size_t)a * D;
  const bool ca_ok = all_coord_ok<D>(ca);
  const int v = pt_ix[cpos];
  for (int e = ip[v]; e < ip[v + 1]; ++e) {
    const int j = ix[e];
    const int b = vA[j];
    if (b == a && j != li) {
      const double* xj = Xp + (size_t)pos_of[j] * D;
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
  for (int k = 0; k < D; ++k) Fscr[(size_t)cpos * D + k] = acc[k] + unit[k] * c.gravity * dip1;
}

template <int D>
__global__ void __launch_bounds__(kHT)
faml_huge_update(const int* __restrict__ blk_agg, const int* __restrict__ blk_li,
                 const int* __restrict__ pt_ip, const double* __restrict__ Xc,
                 double* __restrict__ Xn, const double* __restrict__ Fscr,
                 double* __restrict__ Fprev, MlConst c) {
  const int a = blk_agg[blockIdx.x];
  const int li = blk_li[blockIdx.x] + threadIdx.x;
  if (li >= pt_ip[a + 1] - pt_ip[a]) return;
  const size_t cpos = (size_t)(pt_ip[a] + li);
  double x[D], F[D], Fp[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    x[k] = Xc[cpos * D + k];
    F[k] = Fscr[cpos * D + k];
    Fp[k] = Fprev[cpos * D + k];
  }
  member_update<D>(x, F, Fp, c);
#pragma unroll
  for (int k = 0; k < D; ++k) {
    Xn[cpos * D + k] = x[k];
    Fprev[cpos * D + k] = F[k];
  }
}

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

}  // namespace

void faml_run_device(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix, const double* d_dx,
                     int m, const int* h_pt_ip, const int* d_pt_ip, const int* d_pt_ix,
                     const int* d_vA, const double* d_cA, const double* d_rA,
                     const double* d_init, double* d_x, int dim, int iterations,
                     const ge_fa_params& p) {
  hipStream_t st = ctx->stream;
  const int N = h_pt_ip[m];
  GE_REQUIRE(N == n, "P_T must have one entry per fine vertex");
  const MlConst c = make_fa_const(p);

  // bucket aggregates by size (largest first inside each bucket)
  std::vector<int> small, mid, large, huge;
  for (int a = 0; a < m; ++a) {
    const int s = h_pt_ip[a + 1] - h_pt_ip[a];
    if (s <= 0) continue;
    if (s <= 64) small.push_back(a);
    else if (s <= 256) mid.push_back(a);
    else if (s <= large_cap(dim)) large.push_back(a);
    else huge.push_back(a);
  }
  auto by_size = [&](int x, int y) {
    const int sx = h_pt_ip[x + 1] - h_pt_ip[x], sy = h_pt_ip[y + 1] - h_pt_ip[y];
    return sx != sy ? sx > sy : x < y;
  };
  std::sort(small.begin(), small.end(), by_size);
  std::sort(mid.begin(), mid.end(), by_size);
  std::sort(large.begin(), large.end(), by_size);

  std::vector<int> order, beg_s, beg_m, beg_l;
  build_packs(small, h_pt_ip, 64, 64, order, beg_s);
  build_packs(mid, h_pt_ip, 256, 256, order, beg_m);
  build_packs(large, h_pt_ip, large_cap(dim), 1, order, beg_l);

  std::vector<int> blk_agg, blk_li;
  for (int a : huge)
    for (int li = 0; li < h_pt_ip[a + 1] - h_pt_ip[a]; li += kHT) {
      blk_agg.push_back(a);
      blk_li.push_back(li);
    }

  DevBuf<int> d_pos(n), d_order(std::max<size_t>(order.size(), 1));
  std::vector<int> begs;  // concatenated pack offsets
  begs.insert(begs.end(), beg_s.begin(), beg_s.end());
  const size_t off_m = begs.size();
  begs.insert(begs.end(), beg_m.begin(), beg_m.end());
  const size_t off_l = begs.size();
  begs.insert(begs.end(), beg_l.begin(), beg_l.end());
  DevBuf<int> d_beg(std::max<size_t>(begs.size(), 1));
  DevBuf<int> d_blk_agg(std::max<size_t>(blk_agg.size(), 1)),
      d_blk_li(std::max<size_t>(blk_li.size(), 1)), d_huge(std::max<size_t>(huge.size(), 1));
  d_order.upload(order.data(), order.size(), st);
  d_beg.upload(begs.data(), begs.size(), st);
  d_blk_agg.upload(blk_agg.data(), blk_agg.size(), st);
  d_blk_li.upload(blk_li.data(), blk_li.size(), st);
  d_huge.upload(huge.data(), huge.size(), st);
  DevBuf<double> Fscr((size_t)n * dim), Fprev((size_t)n * dim);

  hipLaunchKernelGGL(pos_of_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, d_pt_ix, d_pos.p);

  dispatch_dim(dim, [&](auto Dc) {
    constexpr int D = decltype(Dc)::value;
    const int ns = (int)beg_s.size() - 1, nm = (int)beg_m.size() - 1, nl = (int)beg_l.size() - 1;
    if (ns > 0)
      hipLaunchKernelGGL((faml_resident<D, 64, 64>), dim3(ns), dim3(64), 0, st, d_order.p,
                         d_beg.p, d_pt_ip, d_pt_ix, d_pos.p, d_vA, d_ip, d_ix, d_dx, d_cA, d_rA,
                         d_init, Fscr.p, Fprev.p, d_x, iterations, c);
    if (nm > 0)
      hipLaunchKernelGGL((faml_resident<D, 256, 256>), dim3(nm), dim3(256), 0, st, d_order.p,
                         d_beg.p + off_m, d_pt_ip, d_pt_ix, d_pos.p, d_vA, d_ip, d_ix, d_dx,
                         d_cA, d_rA, d_init, Fscr.p, Fprev.p, d_x, iterations, c);
    if (nl > 0)
      hipLaunchKernelGGL((faml_resident<D, 256, large_cap(D)>), dim3(nl), dim3(256), 0, st, d_order.p,
                         d_beg.p + off_l, d_pt_ip, d_pt_ix, d_pos.p, d_vA, d_ip, d_ix, d_dx,
                         d_cA, d_rA, d_init, Fscr.p, Fprev.p, d_x, iterations, c);
    GE_HIP(hipGetLastError());
    if (!huge.empty()) {
      DevBuf<double> Xa((size_t)n * dim), Xb((size_t)n * dim), DP(n);
      const int nb = (int)blk_agg.size();
      hipLaunchKernelGGL((faml_huge_init<D>), dim3(nb), dim3(kHT), 0, st, d_blk_agg.p,
                         d_blk_li.p, d_pt_ip, d_pt_ix, d_vA, d_ip, d_ix, d_dx, d_init, Xa.p,
                         DP.p, Fprev.p, c.use_weights);
      double* cur = Xa.p;
      double* nxt = Xb.p;
      for (int it = 0; it < iterations; ++it) {
        hipLaunchKernelGGL((faml_huge_force<D>), dim3(nb), dim3(kHT), 0, st, d_blk_agg.p,
                           d_blk_li.p, d_pt_ip, d_pt_ix, d_pos.p, d_vA, d_ip, d_ix, d_dx, d_cA,
                           cur, DP.p, Fscr.p, c);
        hipLaunchKernelGGL((faml_huge_update<D>), dim3(nb), dim3(kHT), 0, st, d_blk_agg.p,
                           d_blk_li.p, d_pt_ip, cur, nxt, Fscr.p, Fprev.p, c);
        std::swap(cur, nxt);
      }
      hipLaunchKernelGGL((faml_huge_finish<D>), dim3((int)huge.size()), dim3(kHT), 0, st,
                         d_huge.p, d_pt_ip, d_pt_ix, cur, d_cA, d_rA, d_x);
      GE_HIP(hipGetLastError());
      GE_HIP(hipStreamSynchronize(st));  // Xa/Xb/DP freed at scope exit
    }
  });
  GE_HIP(hipStreamSynchronize(st));
}

}  // namespace ge
