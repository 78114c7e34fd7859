// ge_math.hpp -- exact fp64 helpers for the strict (bit-exact) kernels.
//
// IEEE division on gfx950 is a 10-instruction sequence (LLVM AMDGPU
// lowerFDIV64): the denominator is scaled (v_div_scale), its reciprocal
// estimate (v_rcp_f64) is refined by two Newton steps (4 FMA), the scaled
// numerator is multiplied in, one correction FMA follows, then v_div_fmas and
// v_div_fixup.  Only the numerator-side third of that sequence depends on the
// numerator.  The repulsion term divides three numerators by the same dis
// (include/forceatlas.hpp:162) and gravity three numerators by the same mag
// (:208), so the denominator part is computed once and the numerator part
// replayed per numerator: the same instructions on the same operands, hence the
// same bits as `/`.
//
// Inside the operand domain the kernels admit, the sequence simplifies further:
// per the ISA's V_DIV_SCALE_F64 rules v_div_scale returns its input unchanged
// with VCC = 0 unless (a) num == 0 (then v_div_fixup alone fixes the result to
// +-0), (b) |num| >= 2^768 |den|, (c) den or 1/den is denormal, (d) num/den is
// denormal, or (e) |num| < 2^-969; with VCC = 0, v_div_fmas is a plain FMA.
// Every division here has a numerator bounded by ~100x its denominator (a vector
// component over that vector's clamped norm, or 100 times such a ratio over a
// norm), so (b) never holds; the kernels take this path only when every
// coordinate involved is 0 or has magnitude in [2^-200, 2^200] (coord_ok), which
// bounds numerators below by 2^-252, denominators to [1e-5, 2^202] and every
// nonzero quotient above 2^-650, ruling out (c)-(e).  What remains -- rcp,
// two Newton steps, multiply, one FMA correction, FMA, v_div_fixup -- is the
// compiler's own instruction sequence on the same operands, so the bits are the
// same as `/`.  Outside the domain the kernels use `/`.  ge_selftest_math()
// checks the identity on the device (tests/test_gpu_parity.py).
#pragma once

#include <hip/hip_runtime.h>

namespace ge {

struct Recip {
  double ds;  // the denominator (v_div_scale leaves it unchanged in-domain)
  double y;   // refined reciprocal (Fma3 of lowerFDIV64)
};

// Coordinates for which every difference / norm division may share its
// denominator part.  NaN and inf are excluded (the `/` path keeps their
// propagation exactly).
__device__ __forceinline__ bool coord_ok(double x) {
  const double a = __builtin_fabs(x);
  return a == 0.0 || (a >= 0x1p-200 && a <= 0x1p200);
}

__device__ __forceinline__ bool exact_den(double den) {
  const double a = __builtin_fabs(den);
  return a >= 0x1p-960 && a <= 0x1p960;
}

__device__ __forceinline__ Recip recip_of(double den) {
  const double r = __builtin_amdgcn_rcp(den);
  const double e0 = __builtin_fma(-den, r, 1.0);
  const double r1 = __builtin_fma(r, e0, r);
  const double e1 = __builtin_fma(-den, r1, 1.0);
  return Recip{den, __builtin_fma(r1, e1, r1)};
}

// num / den, bit-identical to the compiler's IEEE division inside the domain
// described above.
__device__ __forceinline__ double div_by(double num, double den, const Recip& rc) {
  const double q = num * rc.y;
  const double rem = __builtin_fma(-rc.ds, q, num);
  const double f = __builtin_fma(rem, rc.y, q);
  return __builtin_amdgcn_div_fixup(f, den, num);
}

// div_by without the final v_div_fixup.  In-domain the fixup is the identity
// on every nonzero quotient (it only re-applies the sign and resolves zero,
// inf, NaN and over/underflow operands), so the bits equal `/` whenever
// num != 0; for num == +-0 the result is a zero whose sign may differ from `/`.
// Only used for terms that are added to a running force sum, which is never
// -0 (ge_fa.hip), so a zero of either sign leaves the sum unchanged.
__device__ __forceinline__ double div_by_nz(double num, const Recip& rc) {
  const double q = num * rc.y;
  const double rem = __builtin_fma(-rc.ds, q, num);
  return __builtin_fma(rem, rc.y, q);
}

// sqrt(s) for s in [2^-767, 2^1000]: the compiler's correctly rounded f64
// sqrt expansion (LLVM AMDGPU lowerFSQRTF64: rsq + Goldschmidt refinement)
// with its rescaling of s < 2^-767 and its zero / +inf select removed -- both
// are identities on that range, so the bits equal sqrt(s).  Callers handle
// s == 0 themselves.
__device__ __forceinline__ double sqrt_normal(double s) {
  const double y = __builtin_amdgcn_rsq(s);
  const double g0 = s * y;
  const double h0 = y * 0.5;
  const double r0 = __builtin_fma(-h0, g0, 0.5);
  const double h1 = __builtin_fma(h0, r0, h0);
  const double g1 = __builtin_fma(g0, r0, g0);
  const double d0 = __builtin_fma(-g1, g1, s);
  const double g2 = __builtin_fma(d0, h1, g1);
  const double d1 = __builtin_fma(-g2, g2, s);
  return __builtin_fma(d1, h1, g2);
}

// deg+1 and repel values for which c_ij / dis^2 may use div_by (c_ij in
// [2^-180, 2^180] over dis^2 in [1e-10, 2^404]: quotient normal, (b)-(e) ruled out).
__device__ __forceinline__ bool weight_ok(double w) { return w >= 0x1p-60 && w <= 0x1p60; }

// out[k] = num[k] / den for k < D with one shared denominator.
template <int D>
__device__ __forceinline__ void div_shared(const double (&num)[D], double den, double (&out)[D]) {
  if (exact_den(den)) {
    const Recip rc = recip_of(den);
#pragma unroll
    for (int k = 0; k < D; ++k) out[k] = div_by(num[k], den, rc);
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) out[k] = num[k] / den;
  }
}

}  // namespace ge
