// Drop-in for include/forceatlas.hpp (LLNL/graph-embed).  Same names, parameter
// order and defaults; the iterations run on the MI355X through libge.so.
//   forceAtlas(A, dim, coords, ...)        include/forceatlas.hpp:89-305
//   forceAtlas(A, dim = 2)                 :307-312 (100000 iterations)
//   forceAtlasMultilevel(A, P, v_A, ...)   :314-574
// Differences: the random init uses mt19937(seed) (partition::setSeed / $GE_SEED)
// instead of std::random_device, and forceAtlasMultilevel draws in the
// reference's single-thread order (the reference races on its generator across
// OpenMP threads, :340-358).  The functions are inline (the reference defines
// them non-inline in this header).
#ifndef FORCEATLAS_HPP
#define FORCEATLAS_HPP

#include <cassert>
#include <cmath>
#include <vector>

#include "ge_dropin.hpp"
#include "matrixutils.hpp"

namespace partition {

inline double abs(double val) { return (val < 0) ? -val : val; }

inline double distance(const std::vector<double>& v1, const std::vector<double>& v2) {
  assert(v1.size() == v2.size());
  double acc = 0.0;
  for (size_t k = 0; k < v1.size(); ++k) {
    const double t = v2[k] - v1[k];
    acc += t * t;
  }
  return std::sqrt(acc);
}

inline double magnitude(const std::vector<double>& v) {
  double acc = 0.0;
  for (double x : v) acc += x * x;
  return std::sqrt(acc);
}

inline void forceAtlas(const SparseMatrix& A, const int dim,
                       std::vector<std::vector<double>>& coords, const int iterations = 100000,
                       const double ks = 0.1, const double ksmax = 1.0, const double repel = 1.0,
                       const double attract = 1.0, const double gravity = 1.0,
                       const bool useWeights = true, const bool linlog = false,
                       const bool nohubs = false, const double delta = 1.0,
                       const double tolerate = 1.0, const bool normalize = false) {
  ge_fa_params p;
  ge_fa_params_default(&p);
  p.ks = ks;
  p.ksmax = ksmax;
  p.repel = repel;
  p.attract = attract;
  p.gravity = gravity;
  p.use_weights = useWeights;
  p.linlog = linlog;
  p.nohubs = nohubs;
  p.delta = delta;
  p.tolerate = tolerate;
  p.normalize = normalize;
  p.seed = detail::seed_ref();
  const int n = A.Rows();
  const bool init = coords.empty();
  std::vector<double> X = detail::flatten(coords, n, dim);
  detail::check(ge_force_atlas(detail::context(), n, A.GetIndptr().data(),
                               A.GetIndices().data(), A.GetData().data(), dim, X.data(),
                               init ? 1 : 0, iterations, &p));
  detail::unflatten(X, n, dim, coords);
}

inline std::vector<std::vector<double>> forceAtlas(const SparseMatrix& A, const int dim = 2) {
  std::vector<std::vector<double>> coords(0);
  forceAtlas(A, dim, coords);
  return coords;
}

inline void forceAtlasMultilevel(const SparseMatrix& A, const SparseMatrix& P,
                                 const std::vector<int>& v_A,
                                 const std::vector<std::vector<double>>& coords_A,
                                 const std::vector<double>& r_A,
                                 std::vector<std::vector<double>>& coords, int dim = 2,
                                 int iterations = 10, double ks = 0.1, double ksmax = 1.0,
                                 bool useWeights = true, bool linlog = false, bool nohubs = false,
                                 double repel = 1.0, double attract = 1.0, double gravity = 1.0,
                                 double delta = 1.0, double tolerate = 1.0) {
  ge_fa_params p;
  ge_fa_params_default(&p);
  p.ks = ks;
  p.ksmax = ksmax;
  p.use_weights = useWeights;
  p.linlog = linlog;
  p.nohubs = nohubs;
  p.repel = repel;
  p.attract = attract;
  p.gravity = gravity;
  p.delta = delta;
  p.tolerate = tolerate;
  p.seed = detail::seed_ref();
  const int n = A.Rows();
  const int m = P.Rows();
  std::vector<double> cA = detail::flatten(coords_A, m, dim);
  std::vector<double> X((size_t)n * dim, 0.0);
  detail::check(ge_force_atlas_ml(detail::context(), n, A.GetIndptr().data(),
                                  A.GetIndices().data(), A.GetData().data(), m,
                                  P.GetIndptr().data(), P.GetIndices().data(), v_A.data(),
                                  cA.data(), r_A.data(), X.data(), dim, iterations, &p));
  detail::unflatten(X, n, dim, coords);
}

}  // namespace partition

#endif  // FORCEATLAS_HPP
