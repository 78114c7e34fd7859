// ge_radius.hip -- the radius ("kinetic ball growing") step between levels of
// embedMultilevel, src/embed.cpp:615-777, on the device.
//
// The reference keeps, per coarse group b, a list of events (time = -d_ij / 2,
// i, j) over the group's intra-group edges (all pairs in the base case,
// :616-679), and repeatedly pops the largest tuple -- the nearest pair, ties to
// the larger i, then j -- re-sorting after every pop (:636-678, :713-755):
//   only i live  -> r_i = d, every event touching i shifts;
//   only j live  -> r_j = d, every event touching j shifts;
//   both live    -> r_i = r_j = d, every event touching i or j shifts once;
//   both dead    -> nothing.
// A shift is time' = -(2 * (-time) - (-t_pop)).  "Live" is r <= 0.
//
// Parallel rounds with the same result.  A pop writes r only at its live
// endpoints and shifts only events touching them, and shifts only ever move an
// event later (2 d_e - d >= d_e when d <= d_e).  So an event that is the largest
// live event at each of its live endpoints pops exactly as it would in the
// serial order: every event popped before it in that order touches neither of
// its live endpoints, and nothing can overtake it.  Each round pops all such
// events at once (they are disjoint on live endpoints; at least the global
// largest qualifies, so every round makes progress), then applies the shifts --
// an event shifted from both ends in one round takes them in pop order (the
// larger popped tuple first), since the shift does not commute.  Events whose
// endpoints are both dead can never change anything and are dropped.
//
// Exactness conditions, checked: every event distance is > 0 (then an assigned
// r is > 0, a vertex is assigned at most once, and the serial loop's
// `count < m` bound can only cut it off once every vertex is assigned).  A zero
// distance (coincident coarse coordinates) makes the call return false and the
// caller runs the host version (ge_host.cpp), which replays the serial loop.
//
// The rescale (:757-777) runs one wave per coarse group: the max of
// dist(c_b, x_a) + r_a (exact in any order), then the members' update.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "ge_internal.hpp"

namespace ge {
namespace {

using u64 = unsigned long long;

inline unsigned grid_for(long long L) { return (unsigned)((L + 255) / 256); }

// times are < 0 here: a larger time has the smaller magnitude, so the
// complemented bit pattern orders like the time itself
__device__ __forceinline__ u64 time_ord(double t) { return ~(u64)__double_as_longlong(t); }

template <int D>
__device__ __forceinline__ double dist_dev(const double* __restrict__ from,
                                           const double* __restrict__ to) {
  double acc = 0.0;  // serial sum over k (include/forceatlas.hpp:70-78)
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const double t = to[k] - from[k];
    acc = acc + t * t;
  }
  return sqrt(acc);
}

// base case: all pairs i < j of the coarsest level (:619-625)
template <int D>
__global__ void gen_all_pairs(int m, const double* __restrict__ X, int* __restrict__ ei,
                              int* __restrict__ ej, double* __restrict__ et,
                              int* __restrict__ zero) {
  const int i = blockIdx.x;
  const long long base = (long long)i * m - (long long)i * (i + 1) / 2;
  for (int j = i + 1 + threadIdx.x; j < m; j += blockDim.x) {
    const long long e = base + (j - i - 1);
    const double d = dist_dev<D>(X + (size_t)i * D, X + (size_t)j * D);
    ei[e] = i;
    ej[e] = j;
    et[e] = -d / 2;
    if (!(d > 0.0)) atomicOr(zero, 1);
  }
}

__global__ void group_of_kernel(int mc, const int* __restrict__ pip, const int* __restrict__ pix,
                                const double* __restrict__ rAc, int* __restrict__ grp,
                                double* __restrict__ r) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= mc) return;
  for (int c = pip[b]; c < pip[b + 1]; ++c) grp[pix[c]] = b;
  if (pip[b + 1] - pip[b] == 1) r[pix[pip[b]]] = rAc[b];  // :707-711
}

// intra-group edges a < j of A_c (:697-704); event order is irrelevant (the
// tuples are distinct, so the pop order is total)
template <int D>
__global__ void gen_group_edges(int m, const int* __restrict__ aci, const int* __restrict__ acj,
                                const int* __restrict__ grp, const double* __restrict__ X,
                                int* __restrict__ count, int* __restrict__ ei,
                                int* __restrict__ ej, double* __restrict__ et,
                                int* __restrict__ zero) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= m) return;
  for (int kk = aci[a]; kk < aci[a + 1]; ++kk) {
    const int j = acj[kk];
    if (a < j && grp[j] == grp[a]) {
      const double d = dist_dev<D>(X + (size_t)a * D, X + (size_t)j * D);
      const int e = atomicAdd(count, 1);
      ei[e] = a;
      ej[e] = j;
      et[e] = -d / 2;
      if (!(d > 0.0)) atomicOr(zero, 1);
    }
  }
}

__global__ void iota_kernel(int n, int* __restrict__ v) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) v[t] = t;
}

__global__ void best_time_kernel(int nl, const int* __restrict__ live, const int* __restrict__ ei,
                                 const int* __restrict__ ej, const double* __restrict__ et,
                                 const double* __restrict__ r, u64* __restrict__ best_t) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nl) return;
  const int e = live[q];
  const int i = ei[e], j = ej[e];
  const u64 o = time_ord(et[e]);
  if (r[i] <= 0.0) atomicMax(&best_t[i], o);
  if (r[j] <= 0.0) atomicMax(&best_t[j], o);
}

__global__ void best_pair_kernel(int nl, const int* __restrict__ live, const int* __restrict__ ei,
                                 const int* __restrict__ ej, const double* __restrict__ et,
                                 const double* __restrict__ r, const u64* __restrict__ best_t,
                                 u64* __restrict__ best_ij) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nl) return;
  const int e = live[q];
  const int i = ei[e], j = ej[e];
  const u64 o = time_ord(et[e]);
  const u64 ij = ((u64)(unsigned)i << 32) | (unsigned)j;
  if (r[i] <= 0.0 && best_t[i] == o) atomicMax(&best_ij[i], ij);
  if (r[j] <= 0.0 && best_t[j] == o) atomicMax(&best_ij[j], ij);
}

// Pops every event that is the largest at each of its live endpoints.
__global__ void pop_kernel(int nl, int round, const int* __restrict__ live,
                           const int* __restrict__ ei, const int* __restrict__ ej,
                           const double* __restrict__ et, const u64* __restrict__ best_t,
                           const u64* __restrict__ best_ij, double* __restrict__ r,
                           int* __restrict__ asg_round, double* __restrict__ asg_t,
                           u64* __restrict__ asg_ij, int* __restrict__ popped) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nl) return;
  const int e = live[q];
  const int i = ei[e], j = ej[e];
  const double t = et[e];
  const u64 o = time_ord(t);
  const u64 ij = ((u64)(unsigned)i << 32) | (unsigned)j;
  // liveness as of the round's start: best_t is set exactly for the live endpoints
  // (r[] itself is being written by this kernel's other pops)
  const bool li = best_t[i] != 0, lj = best_t[j] != 0;
  const bool ready = (!li || (best_t[i] == o && best_ij[i] == ij)) &&
                     (!lj || (best_t[j] == o && best_ij[j] == ij));
  if (!ready) return;
  popped[e] = round;
  const double d = -t;
  if (li) {
    r[i] = d;
    asg_round[i] = round;
    asg_t[i] = t;
    asg_ij[i] = ij;
  }
  if (lj) {
    r[j] = d;
    asg_round[j] = round;
    asg_t[j] = t;
    asg_ij[j] = ij;
  }
}

// Shifts of the events touching vertices assigned this round (in pop order),
// then the events that can still act move to the next live list.
__global__ void shift_kernel(int nl, int round, const int* __restrict__ live,
                             const int* __restrict__ ei, const int* __restrict__ ej,
                             double* __restrict__ et, const double* __restrict__ r,
                             const int* __restrict__ asg_round, const double* __restrict__ asg_t,
                             const u64* __restrict__ asg_ij, const int* __restrict__ popped,
                             int* __restrict__ next, int* __restrict__ next_count) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nl) return;
  const int e = live[q];
  if (popped[e] == round) return;
  const int i = ei[e], j = ej[e];
  const bool si = asg_round[i] == round, sj = asg_round[j] == round;
  double t = et[e];
  if (si && sj) {
    // two pops touched this event: the larger popped tuple came first
    const bool i_first = asg_t[i] > asg_t[j] || (asg_t[i] == asg_t[j] && asg_ij[i] > asg_ij[j]);
    const double t1 = i_first ? asg_t[i] : asg_t[j], t2 = i_first ? asg_t[j] : asg_t[i];
    t = -(2 * (-t) - (-t1));
    t = -(2 * (-t) - (-t2));
  } else if (si || sj) {
    t = -(2 * (-t) - (-(si ? asg_t[i] : asg_t[j])));
  }
  et[e] = t;
  if (r[i] <= 0.0 || r[j] <= 0.0) next[atomicAdd(next_count, 1)] = e;
}

// :757-777, one wave per coarse group
template <int D>
__global__ void rescale_kernel(int mc, const int* __restrict__ pip, const int* __restrict__ pix,
                               const double* __restrict__ cAc, const double* __restrict__ rAc,
                               double* __restrict__ X, double* __restrict__ r) {
  const int b = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= mc) return;
  double cb[D];
#pragma unroll
  for (int k = 0; k < D; ++k) cb[k] = cAc[(size_t)b * D + k];
  double alpha = 0.0;
  for (int c = pip[b] + lane; c < pip[b + 1]; c += 64) {
    const int a = pix[c];
    const double dis = dist_dev<D>(cb, X + (size_t)a * D) + r[a];
    if (dis > alpha) alpha = dis;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const double o = __shfl_xor(alpha, off, 64);
    if (o > alpha) alpha = o;
  }
  if (alpha < 0.000001) alpha = 0.000001;
  const double s = rAc[b] / alpha;
  for (int c = pip[b] + lane; c < pip[b + 1]; c += 64) {
    const int a = pix[c];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      double& x = X[(size_t)a * D + k];
      x = cb[k] + s * (x - cb[k]);
    }
    r[a] = s * r[a];
  }
}

template <class F>
void with_dim(int dim, F&& f) {
  switch (dim) {
    case 1: f(std::integral_constant<int, 1>()); break;
    case 2: f(std::integral_constant<int, 2>()); break;
    case 3: f(std::integral_constant<int, 3>()); break;
    case 4: f(std::integral_constant<int, 4>()); break;
    default: throw Error(GE_ERR_ARG, "dimension must be 1..4");
  }
}

}  // namespace

bool radius_step_device(ge_ctx* ctx, int m, double* cA, double* rA, int dim, bool base, int mc,
                        const int* PIc, const int* PJc, const double* cAc, const double* rAc,
                        const int* AcI, const int* AcJ) {
  hipStream_t s = ctx->stream;
  std::fill(rA, rA + m, 0.0);
  if (m == 0) return true;
  DevBuf<double> X((size_t)m * dim), r(m);
  X.upload(cA, (size_t)m * dim, s);
  GE_HIP(hipMemsetAsync(r.p, 0, sizeof(double) * m, s));
  DevBuf<int> zero(1), count(1);
  GE_HIP(hipMemsetAsync(zero.p, 0, sizeof(int), s));
  GE_HIP(hipMemsetAsync(count.p, 0, sizeof(int), s));
  long long E = 0;
  DevBuf<int> ei, ej, dpip, dpix;
  DevBuf<double> et, dcAc, drAc;
  if (base) {
    E = (long long)m * (m - 1) / 2;
    GE_REQUIRE(E < (1ll << 31), "radius step: too many coarsest-level pairs");
    ei.alloc(std::max(E, 1ll));
    ej.alloc(std::max(E, 1ll));
    et.alloc(std::max(E, 1ll));
    with_dim(dim, [&](auto Dc) {
      constexpr int D = decltype(Dc)::value;
      hipLaunchKernelGGL(gen_all_pairs<D>, dim3(m), dim3(256), 0, s, m, X.p, ei.p, ej.p, et.p,
                         zero.p);
    });
  } else {
    const int nnz = AcI[m];
    DevBuf<int> aci(m + 1), acj(std::max(nnz, 1)), grp(m);
    aci.upload(AcI, m + 1, s);
    acj.upload(AcJ, nnz, s);
    dpip.alloc(mc + 1);
    dpix.alloc(std::max(PIc[mc], 1));
    dcAc.alloc(std::max<size_t>((size_t)mc * dim, 1));
    drAc.alloc(std::max(mc, 1));
    dpip.upload(PIc, mc + 1, s);
    dpix.upload(PJc, PIc[mc], s);
    dcAc.upload(cAc, (size_t)mc * dim, s);
    drAc.upload(rAc, mc, s);
    GE_HIP(hipMemsetAsync(grp.p, 0xff, sizeof(int) * m, s));
    if (mc)
      hipLaunchKernelGGL(group_of_kernel, dim3(grid_for(mc)), dim3(256), 0, s, mc, dpip.p, dpix.p,
                         drAc.p, grp.p, r.p);
    // one event per stored entry at most (an asymmetric A_c, e.g. one triangle,
    // emits up to nnz; a symmetric one nnz / 2)
    const long long cap = std::max(nnz, 1);
    ei.alloc(cap);
    ej.alloc(cap);
    et.alloc(cap);
    with_dim(dim, [&](auto Dc) {
      constexpr int D = decltype(Dc)::value;
      hipLaunchKernelGGL(gen_group_edges<D>, dim3(grid_for(m)), dim3(256), 0, s, m, aci.p, acj.p,
                         grp.p, X.p, count.p, ei.p, ej.p, et.p, zero.p);
    });
    int ne = 0;
    GE_HIP(hipMemcpyAsync(&ne, count.p, sizeof(int), hipMemcpyDeviceToHost, s));
    GE_HIP(hipStreamSynchronize(s));
    E = ne;
  }
  GE_HIP(hipGetLastError());
  int has_zero = 0;
  GE_HIP(hipMemcpyAsync(&has_zero, zero.p, sizeof(int), hipMemcpyDeviceToHost, s));
  GE_HIP(hipStreamSynchronize(s));
  if (has_zero) return false;  // coincident coordinates: the host replays the serial loop

  if (E > 0) {
    DevBuf<int> la(E), lb(E), popped(E), asg_round(m), next_count(1);
    DevBuf<u64> best_t(m), best_ij(m), asg_ij(m);
    DevBuf<double> asg_t(m);
    GE_HIP(hipMemsetAsync(popped.p, 0xff, sizeof(int) * E, s));
    GE_HIP(hipMemsetAsync(asg_round.p, 0xff, sizeof(int) * m, s));
    hipLaunchKernelGGL(iota_kernel, dim3(grid_for(E)), dim3(256), 0, s, (int)E, la.p);
    int nl = (int)E;
    int* live = la.p;
    int* next = lb.p;
    for (int round = 0; nl > 0; ++round) {
      GE_REQUIRE(round <= E, "radius step: no progress");
      GE_HIP(hipMemsetAsync(best_t.p, 0, sizeof(u64) * m, s));
      GE_HIP(hipMemsetAsync(best_ij.p, 0, sizeof(u64) * m, s));
      GE_HIP(hipMemsetAsync(next_count.p, 0, sizeof(int), s));
      const dim3 g(grid_for(nl)), b(256);
      hipLaunchKernelGGL(best_time_kernel, g, b, 0, s, nl, live, ei.p, ej.p, et.p, r.p, best_t.p);
      hipLaunchKernelGGL(best_pair_kernel, g, b, 0, s, nl, live, ei.p, ej.p, et.p, r.p, best_t.p,
                         best_ij.p);
      hipLaunchKernelGGL(pop_kernel, g, b, 0, s, nl, round, live, ei.p, ej.p, et.p, best_t.p,
                         best_ij.p, r.p, asg_round.p, asg_t.p, asg_ij.p, popped.p);
      hipLaunchKernelGGL(shift_kernel, g, b, 0, s, nl, round, live, ei.p, ej.p, et.p, r.p,
                         asg_round.p, asg_t.p, asg_ij.p, popped.p, next, next_count.p);
      GE_HIP(hipGetLastError());
      GE_HIP(hipMemcpyAsync(&nl, next_count.p, sizeof(int), hipMemcpyDeviceToHost, s));
      GE_HIP(hipStreamSynchronize(s));
      std::swap(live, next);
    }
  }
  if (!base && mc > 0) {
    with_dim(dim, [&](auto Dc) {
      constexpr int D = decltype(Dc)::value;
      hipLaunchKernelGGL(rescale_kernel<D>, dim3((mc + 3) / 4), dim3(256), 0, s, mc, dpip.p,
                         dpix.p, dcAc.p, drAc.p, X.p, r.p);
    });
    GE_HIP(hipGetLastError());
  }
  X.download(cA, (size_t)m * dim, s);
  r.download(rA, m, s);
  GE_HIP(hipStreamSynchronize(s));
  return true;
}

}  // namespace ge

extern "C" int ge_radius_step_device(ge_ctx* ctx, int m, double* cA, double* rA, int dim,
                                     int base, int mc, const int* PIc, const int* PJc,
                                     const double* cAc, const double* rAc, const int* AcI,
                                     const int* AcJ, int* used_device) {
  return ge::guarded([&] {
    GE_REQUIRE(ctx && m >= 0 && cA && rA && dim >= 1 && dim <= 4, "bad radius-step arguments");
    GE_REQUIRE(base || (PIc && PJc && cAc && rAc && AcI && AcJ), "null argument");
    ge::DeviceGuard g(ctx);
    const bool dev = ge::radius_step_device(ctx, m, cA, rA, dim, base != 0, mc, PIc, PJc, cAc,
                                            rAc, AcI, AcJ);
    if (!dev) ge::radius_step_host(m, cA, rA, dim, base != 0, mc, PIc, PJc, cAc, rAc, AcI, AcJ);
    if (used_device) *used_device = dev ? 1 : 0;
  });
}
