// ge_pair.hpp -- per-pair / per-edge ForceAtlas terms shared by the kernels.
//
// Each function evaluates one term of include/forceatlas.hpp exactly as the
// reference writes it (operand order, one rounding per operation).  With
// SHARED = true the three divisions by one denominator reuse its reciprocal
// (ge_math.hpp): same instructions, same bits, valid when the caller has checked
// coord_ok() for every coordinate involved.
#pragma once

#include <hip/hip_runtime.h>

#include "ge_internal.hpp"
#include "ge_math.hpp"

namespace ge {

constexpr double kFaEps = 0.00001;  // include/forceatlas.hpp:110, :337

struct FaConst {
  double ks_gS;  // ks * globalSpeed, globalSpeed = tolerate * 1.0 / 1.0 (:228, :242, :244)
  double gS;
  double ksmax, repel, attract, gravity, delta;
  int use_weights, linlog, nohubs;
};

inline FaConst make_fa_const(const ge_fa_params& p) {
  FaConst c;
  c.gS = p.tolerate * 1.0 / 1.0;
  c.ks_gS = p.ks * c.gS;
  c.ksmax = p.ksmax;
  c.repel = p.repel;
  c.attract = p.attract;
  c.gravity = p.gravity;
  c.delta = p.delta;
  c.use_weights = p.use_weights;
  c.linlog = p.linlog;
  c.nohubs = p.nohubs;
  return c;
}

__device__ __forceinline__ double clamp_eps(double x) { return x < kFaEps ? kFaEps : x; }

// Attraction magnitude (:176-196).  linlog / delta != 1 use device log / pow
// (ocml), which may differ from glibc in the last ulp: only the default branch
// is bit-exact.
__device__ __forceinline__ double attraction_mag(double dis, double a, double dip1,
                                                 const FaConst& c) {
  double f = dis;
  if (c.linlog) f = log(1 + f);
  if (c.delta == 1.0) {
    f = f * a;
  } else if (c.delta != 0.0) {
    const double sgn = (a < 0) ? -1.0 : 1.0;
    const double mg = (a < 0) ? -a : a;
    f = sgn * pow(mg, c.delta) * f;
  }
  if (c.nohubs) f = f / dip1;
  return c.attract * f;
}

// The clamped distance of a pair and the refined reciprocals of dis and dis^2
// (round 5).  The IEEE quotient n / d the kernels replay (ge_math.hpp div_by) is
// q0 = n y, r = fma(-d, q0, n), q0 + r y rounded once: its result is the correctly
// rounded n / d for any y within a fraction of an ulp of 1 / d (q0 + r y = n / d +
// (d y - 1)(n / d - q0), an error of ~2^-106 relative), and recip_of gets such a y
// from v_rcp_f64 and two Newton steps.  Here the reciprocals come without v_rcp:
//   1 / dis   from the sqrt's own Goldschmidt half-reciprocal h1 ~ 1 / (2 sqrt(s))
//             (one Newton step of v_rsq_f64 already), y0 = 2 h1 (capped at 1e5 ~ 1 /
//             eps: s below eps^2, or s = 0 where h1 is NaN and fmin takes 1e5), then
//             one Newton step: y = y0 + y0 (1 - dis y0);
//   1 / dis^2 from (1 / dis)^2 (within ~2 ulp), then one Newton step.
// Each y is then within 2^-80 of 1 / d before its last rounding, like recip_of's (its
// second Newton step starts from ~2^-44), so the two differ only where 1 / d lies
// within ~2^-80 of a rounding boundary, and a y off by one ulp changes the quotient
// only where n / d lies within ~2^-106 of one: the same bits as `/` except with
// probability ~2^-80 per division (ge_selftest.hip compares every term with the
// rcp path and with `/` on 2^30 draws per test call, tests/test_gpu_parity.py).  Two
// quarter-rate v_rcp_f64 and two FMAs fewer per pair than rcp-based reciprocals.
struct PairDen {
  double dis;
  Recip rdis, rdd;  // {dis, ~1/dis}, {dis * dis, ~1/dis^2}
};
__device__ __forceinline__ PairDen pair_den(double s) {
  const double y = __builtin_amdgcn_rsq(s);
  const double g0 = s * y;
  const double h0 = y * 0.5;
  const double r0 = __builtin_fma(-h0, g0, 0.5);
  const double h1 = __builtin_fma(h0, r0, h0);
  const double g1 = __builtin_fma(g0, r0, g0);
  const double d0 = __builtin_fma(-g1, g1, s);
  const double g2 = __builtin_fma(d0, h1, g1);
  const double d1 = __builtin_fma(-g2, g2, s);
  // sqrt_normal(s), clamped (s == 0: NaN, and fmax takes eps)
  const double dis = fmax(__builtin_fma(d1, h1, g2), kFaEps);
  const double y0 = fmin(h1 + h1, 1e5);
  const double yd = __builtin_fma(y0, __builtin_fma(-dis, y0, 1.0), y0);
  const double dd = dis * dis;
  const double z0 = yd * yd;
  const double ydd = __builtin_fma(z0, __builtin_fma(-dd, z0, 1.0), z0);
  return PairDen{dis, Recip{dis, yd}, Recip{dd, ydd}};
}

// Repulsion of j on i (:152-166): the term added to row i's sum, out[k] =
// (e_k / dis) * val.  e = x_i - x_j equals -(x_j - x_i) up to the sign of zero,
// and a zero term never changes the sum (see ge_fa.hip); the j == i term is
// +-0 for the same reason.
template <int D, bool SHARED, bool REPEL_ONE>
__device__ __forceinline__ void rep_term(const double (&xi)[D], const double* __restrict__ xj,
                                         double dip1, double djp1, double repel,
                                         double (&out)[D]) {
  double e[D];
#pragma unroll
  for (int k = 0; k < D; ++k) e[k] = xi[k] - xj[k];
  double s = e[0] * e[0];
#pragma unroll
  for (int k = 1; k < D; ++k) s = s + e[k] * e[k];
  double cij = dip1 * djp1;
  if (!REPEL_ONE) cij = cij * repel;
  if (SHARED) {
    // In-domain s is 0 or >= 2^-504 (>= 2^-767: sqrt_normal is exact).  For
    // s == 0 (the j == i pair, coincident points) sqrt_normal returns NaN
    // (rsq(0) = inf, 0 * inf), and fmax returns its non-NaN operand, so dis is
    // eps exactly as the reference's clamp of sqrt(0) = 0.
#ifdef GE_PAIR_RCP  // A/B variant builds only (scripts/build_variant.sh): recip_of's reciprocals
    const double dis = fmax(sqrt_normal(s), kFaEps);
    const double val = div_by_nz(cij, recip_of(dis * dis));
    const Recip rdis = recip_of(dis);
#pragma unroll
    for (int k = 0; k < D; ++k) out[k] = div_by_nz(e[k], rdis) * val;
#else
    const PairDen pd = pair_den(s);
    const double val = div_by_nz(cij, pd.rdd);  // cij > 0 in-domain
#pragma unroll
    for (int k = 0; k < D; ++k) out[k] = div_by_nz(e[k], pd.rdis) * val;
#endif
  } else {
    const double dis = clamp_eps(sqrt(s));
    const double val = cij / (dis * dis);
#pragma unroll
    for (int k = 0; k < D; ++k) out[k] = (e[k] / dis) * val;
  }
}

// rep_term<SHARED> with recip_of's reciprocals (the form before round 5): the
// selftest's reference for pair_den.
template <int D, bool REPEL_ONE>
__device__ __forceinline__ void rep_term_rcp(const double (&xi)[D], const double* __restrict__ xj,
                                             double dip1, double djp1, double repel,
                                             double (&out)[D]) {
  double e[D];
#pragma unroll
  for (int k = 0; k < D; ++k) e[k] = xi[k] - xj[k];
  double s = e[0] * e[0];
#pragma unroll
  for (int k = 1; k < D; ++k) s = s + e[k] * e[k];
  double cij = dip1 * djp1;
  if (!REPEL_ONE) cij = cij * repel;
  const double dis = fmax(sqrt_normal(s), kFaEps);
  const double dd = dis * dis;
  const double val = div_by_nz(cij, recip_of(dd));
  const Recip rc = recip_of(dis);
#pragma unroll
  for (int k = 0; k < D; ++k) out[k] = div_by_nz(e[k], rc) * val;
}

// rep_term added to acc.  Every sum that receives terms starts from a +0.0
// accumulator and is never seeded with a term: a term may be -0 (e_k = -0), and
// only the +0 start makes adding it an identity (RN: +0 + -0 = +0).
template <int D, bool SHARED, bool REPEL_ONE>
__device__ __forceinline__ void rep_pair(const double (&xi)[D], const double* __restrict__ xj,
                                         double dip1, double djp1, double repel,
                                         double (&acc)[D]) {
  double t[D];
  rep_term<D, SHARED, REPEL_ONE>(xi, xj, dip1, djp1, repel, t);
#pragma unroll
  for (int k = 0; k < D; ++k) acc[k] = acc[k] + t[k];
}

// The out-of-domain (`/`) form with the self pair skipped as the reference does
// (j != i, :151).  In the shared-reciprocal domain the self term is +-0 and may
// be accumulated, but outside it cij / eps^2 can overflow (cij > ~1.8e298) and
// 0 * inf would put a NaN into the row's sum.
template <int D, bool REPEL_ONE>
__device__ __forceinline__ void rep_pair_fb(const double (&xi)[D], const double* __restrict__ xj,
                                            double dip1, double djp1, double repel, bool self,
                                            double (&acc)[D]) {
  if (!self) rep_pair<D, false, REPEL_ONE>(xi, xj, dip1, djp1, repel, acc);
}

// attraction_mag for linlog == 0 and delta == 1 (the defaults): no log / pow
// code, which keeps register-tight kernels within their budget.
__device__ __forceinline__ double attraction_mag_linear(double dis, double a, double dip1,
                                                        const FaConst& c) {
  double f = dis * a;
  if (c.nohubs) f = f / dip1;
  return c.attract * f;
}

// Attraction along one CSR entry (:169-203): t = x_j - x_i.  LINEAR: the caller
// guarantees linlog == 0 and delta == 1.
template <int D, bool SHARED, bool LINEAR = false>
__device__ __forceinline__ void attr_edge(const double (&xi)[D], const double* __restrict__ xj,
                                          double a, double dip1, const FaConst& c,
                                          double (&acc)[D]) {
  double t[D];
#pragma unroll
  for (int k = 0; k < D; ++k) t[k] = xj[k] - xi[k];
  double s = t[0] * t[0];
#pragma unroll
  for (int k = 1; k < D; ++k) s = s + t[k] * t[k];
  const double dis = clamp_eps(SHARED ? (s == 0.0 ? 0.0 : sqrt_normal(s)) : sqrt(s));
  const double Fa = LINEAR ? attraction_mag_linear(dis, a, dip1, c) : attraction_mag(dis, a, dip1, c);
  if (SHARED) {
    const Recip rc = recip_of(dis);
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = acc[k] + div_by(t[k], dis, rc) * Fa;
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = acc[k] + (t[k] / dis) * Fa;
  }
}

template <int D>
__device__ __forceinline__ bool all_coord_ok(const double* x) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < D; ++k) ok = ok && coord_ok(x[k]);
  return ok;
}

// A vertex whose coordinates and deg+1 lie in the exact shared-reciprocal
// domain of rep_pair<SHARED = true>.
template <int D>
__device__ __forceinline__ bool vertex_ok(const double* x, double dp1) {
  return all_coord_ok<D>(x) && weight_ok(dp1);
}

// -x_k / mag for all k (:208 single level, :471 multilevel).
template <int D>
__device__ __forceinline__ void neg_over(const double (&x)[D], double mag, double (&out)[D]) {
  double nx[D];
#pragma unroll
  for (int k = 0; k < D; ++k) nx[k] = -x[k];
  if (exact_den(mag) && all_coord_ok<D>(x)) {
    const Recip rc = recip_of(mag);
#pragma unroll
    for (int k = 0; k < D; ++k) out[k] = div_by(nx[k], mag, rc);
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) out[k] = nx[k] / mag;
  }
}

template <class F>
void dispatch_dim(int dim, F&& f) {
  switch (dim) {
    case 1: f(std::integral_constant<int, 1>()); break;
    case 2: f(std::integral_constant<int, 2>()); break;
    case 3: f(std::integral_constant<int, 3>()); break;
    case 4: f(std::integral_constant<int, 4>()); break;
    default: throw Error(GE_ERR_ARG, "dimension must be 1..4");
  }
}

}  // namespace ge
