// ge_selftest.hip -- on-device check of the exact shared-reciprocal division
// (ge_math.hpp): for operands in the domain the strict kernels admit, div_by
// must return the same bits as the compiler's IEEE `/`; and the repulsion term
// with pair_den's rcp-free reciprocals (ge_pair.hpp) the same bits as with
// recip_of's and as the `/` form.

#include <hip/hip_runtime.h>

#include "ge_internal.hpp"
#include "ge_math.hpp"
#include "ge_pair.hpp"

namespace ge {
namespace {

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Random double with exponent uniform in [lo, hi], random mantissa, random sign.
__device__ __forceinline__ double rnd_exp(unsigned long long h, int lo, int hi, bool sign) {
  const int e = lo + (int)((h >> 52) % (unsigned long long)(hi - lo + 1));
  const unsigned long long mant = h & 0xFFFFFFFFFFFFFull;
  const unsigned long long bits = ((unsigned long long)(e + 1023) << 52) | mant;
  double v = __longlong_as_double((long long)bits);
  return (sign && ((h >> 51) & 1)) ? -v : v;
}

__device__ __forceinline__ bool same(double a, double b) {
  return __double_as_longlong(a) == __double_as_longlong(b);
}

__global__ void selftest_kernel(long long samples, unsigned long long seed,
                                unsigned long long* bad) {
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  unsigned long long fails = 0;
  for (long long t = t0; t < samples; t += stride) {
    const unsigned long long h0 = mix(seed ^ (unsigned long long)t);
    const unsigned long long h1 = mix(h0), h2 = mix(h1), h3 = mix(h2);
    // denominator: a clamped norm in [1e-5, 2^202], sometimes exactly eps
    double den = rnd_exp(h1, -17, 202, false);
    if ((h0 & 31) == 0) den = 0.00001;
    if ((h0 & 31) == 1) den = rnd_exp(h1, -17, 2, false);
    // numerator: a component with |num| <= den, 0, +-den, or tiny-but-allowed
    double num;
    const unsigned sel = (unsigned)((h0 >> 8) & 7);
    const double u = (double)(h2 >> 11) * 0x1.0p-53;
    switch (sel) {
      case 0: num = 0.0; break;
      case 1: num = ((h2 >> 3) & 1) ? -den : den; break;
      case 2: num = den * u; break;
      case 3: num = -den * u; break;
      default: {
        int ed = 0;
        (void)frexp(den, &ed);
        num = rnd_exp(h2, -252, ed - 1, true);
        break;
      }
    }
    const Recip rc = recip_of(den);
    const double q = div_by(num, den, rc);
    if (!same(q, num / den)) ++fails;
    // pull form: (num/den * 100) / mag
    const double mag = rnd_exp(h3, -17, 202, false);
    const Recip rm = recip_of(mag);
    const double p = div_by(q * 100.0, mag, rm);
    if (!same(p, (num / den) * 100.0 / mag)) ++fails;
    // gravity form: -x / |x| with x in [2^-200, 2^200]
    const double x = rnd_exp(h3 ^ h2, -200, 200, true);
    const double nx = ((h3 >> 7) & 1) ? x : 0.0;
    const double m = fabs(x) * (1.0 + u);
    const Recip rg = recip_of(m);
    if (!same(div_by(-nx, m, rg), -nx / m)) ++fails;
    // sqrt of a squared distance in [2^-504, 2^406]
    const double sq = rnd_exp(h0 ^ h3, -504, 405, false);
    if (!same(sqrt_normal(sq), sqrt(sq))) ++fails;
    // c_ij / dis^2 with c_ij in [2^-180, 2^180], dis in [1e-5, 2^202]
    const double cij = rnd_exp(h2 ^ h1, -180, 180, false);
    const double dd = den * den;
    if (!same(div_by(cij, dd, recip_of(dd)), cij / dd)) ++fails;
    // a repulsion pair (ge_pair.hpp rep_term): pair_den's reciprocals against
    // recip_of's and against `/`.  Coordinates mostly of the layout's scale, some
    // spread over the whole domain, some pairs at or below the eps clamp, and
    // coincident ones; deg+1 and repel over their domain.
    const unsigned long long h4 = mix(h3), h5 = mix(h4), h6 = mix(h5), h7 = mix(h6);
    double xi[3], xj[3];
    const unsigned shape = (unsigned)(h4 & 7);
    const double scale = shape < 4 ? 1.0 : rnd_exp(h7, -190, 190, false);
    for (int k = 0; k < 3; ++k) {
      const unsigned long long hk = mix(h5 + k);
      xi[k] = ((double)(hk >> 11) * 0x1.0p-53 * 2.0 - 1.0) * scale;
      if (!coord_ok(xi[k])) xi[k] = 0.0;
      const unsigned long long hj = mix(h6 + k);
      double off = ((double)(hj >> 11) * 0x1.0p-53 * 2.0 - 1.0) * scale;
      if (shape == 1) off = off * 1e-5;                 // near the eps clamp
      if (shape == 2) off = rnd_exp(hj, -30, -10, true);  // around eps
      if (shape == 3) off = 0.0;                        // coincident
      xj[k] = xi[k] + off;
      if (!coord_ok(xj[k])) xj[k] = xi[k];
    }
    const double di = (h7 & 1) ? 1.0 + (double)((h7 >> 8) & 1023) : rnd_exp(h7, -60, 59, false);
    const double dj = (h6 & 1) ? 1.0 + (double)((h6 >> 8) & 1023) : rnd_exp(h6, -60, 59, false);
    const double rp = (h5 & 3) ? 1.0 : rnd_exp(h5 ^ h7, -60, 0, false);
    if (!(vertex_ok<3>(xi, di) && vertex_ok<3>(xj, dj) && weight_ok(rp) &&
          weight_ok(di * dj * rp)))
      continue;
    double ta[3], tb[3], tc[3];
    rep_term<3, true, false>(xi, xj, di, dj, rp, ta);
    rep_term_rcp<3, false>(xi, xj, di, dj, rp, tb);
    rep_term<3, false, false>(xi, xj, di, dj, rp, tc);
    for (int k = 0; k < 3; ++k) {
      // +-0 terms may differ in sign from `/` (div_by_nz); they never change a sum
      if (!same(ta[k], tb[k])) ++fails;
      if (!same(ta[k], tc[k]) && !(ta[k] == 0.0 && tc[k] == 0.0)) ++fails;
    }
  }
  if (fails) atomicAdd(bad, fails);
}

}  // namespace
}  // namespace ge

extern "C" int ge_selftest_math(ge_ctx* ctx, long long samples, unsigned long long seed,
                                long long* mismatches) {
  return ge::guarded([&] {
    GE_REQUIRE(ctx && mismatches && samples >= 0, "bad arguments");
    ge::DeviceGuard g(ctx);
    ge::DevBuf<unsigned long long> bad(1);
    GE_HIP(hipMemsetAsync(bad.p, 0, sizeof(unsigned long long), ctx->stream));
    hipLaunchKernelGGL(ge::selftest_kernel, dim3(2048), dim3(256), 0, ctx->stream, samples, seed,
                       bad.p);
    GE_HIP(hipGetLastError());
    unsigned long long h = 0;
    GE_HIP(hipMemcpyAsync(&h, bad.p, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
    GE_HIP(hipStreamSynchronize(ctx->stream));
    *mismatches = (long long)h;
  });
}
