// ge_minimize.cpp -- partition::embedViaMinimization (src/embed.cpp:341-559),
// the reference's alternative single-level embedder: Gauss-Seidel sweeps over
// the vertices; for each vertex with a neighbour other than itself, a bisection
// line search (12 halvings of the step, from t = 1/2) towards each of the 2d
// unit directions on the energy sum_r 1/|x_i - x_r| + w sum_(i,r) |x_i - x_r|^2,
// w = 1e6, then a move to the direction of least energy.
//
// Host C++.  It is off the embed() path, and its work per vertex is a chain of
// serial n-term sums whose order fixes the bits (the line search branches on
// their signs), so the device has no lane parallelism to offer inside one call;
// the 2d directions of a vertex are independent and run on OpenMP threads.
// Every sum keeps the reference's order and operand grouping (-ffp-contract=off).

#include <cmath>
#include <limits>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "ge_internal.hpp"

namespace ge {

namespace {

constexpr double kMinEps = 10e-12;  // src/embed.cpp:345 (sic: 1e-11)
constexpr double kEdgeWeight = 1000000.0;  // :415

struct LineResult {
  double t, J;
};

// Line search from x_i towards direction s (:417-494) and the energy at its end.
LineResult line_search(int i, int n, int dim, const int* I, const int* J, const double* X,
                       const double* xs) {
  const double* xi = X + (size_t)i * dim;
  double t = 0.5;
  double jump = 0.25;
  do {
    double dJ = 0.0;
    for (int r = 0; r < n; ++r) {
      if (i == r) continue;
      const double* xr = X + (size_t)r * dim;
      double term1 = 0.0, term2 = 0.0;
      for (int k = 0; k < dim; ++k) {
        const double u = xs[k] - xi[k];
        const double v = xi[k] - xr[k];
        const double z = u * t + v;
        term1 = term1 + z * z;
        term2 = term2 + z * u;
      }
      if (term1 < kMinEps) term1 = kMinEps;
      dJ += -((1.0 / std::sqrt(term1 * term1 * term1)) * term2);
    }
    for (int kk = I[i]; kk < I[i + 1]; ++kk) {
      const int r = J[kk];
      if (i == r) continue;
      const double* xr = X + (size_t)r * dim;
      double term = 0.0;
      for (int k = 0; k < dim; ++k) {
        const double a = (1 - t) * xi[k] + t * xs[k] - xr[k];
        term += kEdgeWeight * 2.0 * a * (xs[k] - xi[k]);
      }
      dJ += term;
    }
    if (dJ < 0.0) t = t + jump;
    else t = t - jump;
    jump = jump / 2.0;
  } while (jump > 1.e-4);
  double Jl = 0.0;  // :496-523
  for (int r = 0; r < n; ++r) {
    if (i == r) continue;
    const double* xr = X + (size_t)r * dim;
    double term1 = 0.0;
    for (int k = 0; k < dim; ++k) {
      const double u = xs[k] - xi[k];
      const double v = xi[k] - xr[k];
      const double z = u * t + v;
      term1 = term1 + z * z;
    }
    if (term1 < kMinEps) term1 = kMinEps;
    Jl = Jl + 1.0 / std::sqrt(term1);
  }
  for (int kk = I[i]; kk < I[i + 1]; ++kk) {
    const int r = J[kk];
    if (i == r) continue;
    const double* xr = X + (size_t)r * dim;
    double term = 0.0;
    for (int k = 0; k < dim; ++k) {
      const double a = (1 - t) * xi[k] + t * xs[k] - xr[k];
      term += a * a;
    }
    Jl += kEdgeWeight * term;
  }
  return {t, Jl};
}

}  // namespace

void embed_via_minimization(int n, const int* I, const int* J, int dim, double* X,
                            bool init_random, unsigned seed, int iterations) {
  if (init_random) uniform_stream(seed, (size_t)n * dim, X);  // :353-361, i-major
  // directions (:363-379): +e_k, -e_k for k = 0..d-1 (the d = 2, 3 lists are this order)
  const int ndir = 2 * dim;
  std::vector<double> dirs((size_t)ndir * dim, 0.0);
  for (int k = 0; k < dim; ++k) {
    dirs[(size_t)(2 * k) * dim + k] = 1;
    dirs[(size_t)(2 * k + 1) * dim + k] = -1;
  }
  std::vector<LineResult> res(ndir);
  for (int iter = 0; iter < iterations; ++iter) {
    for (int i = 0; i < n; ++i) {
      int count = 0;  // :389-394
      for (int kk = I[i]; kk < I[i + 1]; ++kk)
        if (J[kk] != i) count++;
      if (count == 0) continue;
#pragma omp parallel for schedule(static, 1) if (n > 64)
      for (int s = 0; s < ndir; ++s)
        res[s] = line_search(i, n, dim, I, J, X, dirs.data() + (size_t)s * dim);
      double min_J = std::numeric_limits<double>::infinity();
      double min_t = 0.0f;
      double min_s = -1;
      for (int s = 0; s < ndir; ++s) {  // :524-528, in direction order
        if (res[s].J < min_J) {
          min_J = res[s].J;
          min_t = res[s].t;
          min_s = s;
        }
      }
      if (min_s >= 0) {  // :554-558
        const double* ds = dirs.data() + (size_t)min_s * dim;
        for (int k = 0; k < dim; ++k)
          X[(size_t)i * dim + k] = X[(size_t)i * dim + k] * (1 - min_t) + ds[k] * min_t;
      }
    }
  }
  if (n > 1) {  // :562-583: centre on the mean of vertices 1..n-1, scale by their max norm
    std::vector<double> avg(dim, 0.0);
    for (int i = 1; i < n; ++i)
      for (int k = 0; k < dim; ++k) avg[k] = avg[k] + X[(size_t)i * dim + k];
    for (int k = 0; k < dim; ++k) avg[k] = avg[k] / (n - 1);
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < dim; ++k) X[(size_t)i * dim + k] -= avg[k];
    double max_length = 0.0;
    for (int i = 1; i < n; ++i) {
      double acc = 0.0;  // magnitude (include/forceatlas.hpp:80-87)
      for (int k = 0; k < dim; ++k) acc = acc + X[(size_t)i * dim + k] * X[(size_t)i * dim + k];
      const double len = std::sqrt(acc);
      if (max_length < len) max_length = len;
    }
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < dim; ++k) X[(size_t)i * dim + k] = X[(size_t)i * dim + k] / max_length;
  }
}

}  // namespace ge

extern "C" int ge_embed_via_minimization(int n, const int* indptr, const int* indices, int dim,
                                         double* coords, int init_random, unsigned seed,
                                         int iterations) {
  return ge::guarded([&] {
    GE_REQUIRE(n >= 0 && dim >= 1 && iterations >= 0, "bad arguments");
    GE_REQUIRE(n == 0 || (indptr && indices && coords && indptr[0] == 0), "null argument");
    ge::embed_via_minimization(n, indptr, indices, dim, coords, init_random != 0, seed,
                               iterations);
  });
}
