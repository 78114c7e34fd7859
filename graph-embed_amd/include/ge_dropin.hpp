// ge_dropin.hpp -- glue between the reference's C++ API (namespace partition)
// and libge.so's C ABI (include/ge.h).  Header-only: the drop-in headers touch a
// SparseMatrix only through GetIndptr/GetIndices/GetData/Rows/Cols and the
// (I, J, D, rows, cols) constructor, so they build against the real linalgcpp
// or against the subset in graph-embed_amd/compat.
#ifndef GE_DROPIN_HPP
#define GE_DROPIN_HPP

#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "ge.h"

namespace partition {
namespace detail {

// Non-zero status -> exception.  The reference has no error reporting beyond
// assert; an uncaught exception terminates like a failed assert does.
inline void check(int rc) {
  if (rc != 0) throw std::runtime_error(std::string("graph-embed_amd: ") + ge_last_error());
}

// One context (device + stream) per host thread, device from $GE_DEVICE.
struct CtxHolder {
  ge_ctx* c = nullptr;
  ~CtxHolder() {
    if (c) ge_ctx_destroy(c);
  }
};

inline ge_ctx* context() {
  thread_local CtxHolder h;
  if (!h.c) {
    const char* d = std::getenv("GE_DEVICE");
    check(ge_ctx_create(d ? std::atoi(d) : 0, &h.c));
  }
  return h.c;
}

// The reference seeds every generator from std::random_device; the drop-in
// uses one fixed seed per thread ($GE_SEED, default 12345; partition::setSeed).
inline unsigned& seed_ref() {
  thread_local unsigned s = [] {
    const char* e = std::getenv("GE_SEED");
    return e ? (unsigned)std::strtoul(e, nullptr, 10) : 12345u;
  }();
  return s;
}

inline std::vector<double> flatten(const std::vector<std::vector<double>>& c, int n, int dim) {
  std::vector<double> out((size_t)n * dim, 0.0);
  for (int i = 0; i < n && i < (int)c.size(); ++i)
    for (int k = 0; k < dim && k < (int)c[i].size(); ++k) out[(size_t)i * dim + k] = c[i][k];
  return out;
}

inline void unflatten(const std::vector<double>& x, int n, int dim,
                      std::vector<std::vector<double>>& c) {
  c.assign(n, std::vector<double>(dim));
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < dim; ++k) c[i][k] = x[(size_t)i * dim + k];
}

template <class M>
inline std::vector<int> vertex_of(const M& P_T) {  // P_T.Transpose().GetIndices()
  std::vector<int> v(P_T.Cols(), 0);
  const auto& I = P_T.GetIndptr();
  const auto& J = P_T.GetIndices();
  for (int a = 0; a < P_T.Rows(); ++a)
    for (int c = I[a]; c < I[a + 1]; ++c) v[J[c]] = a;
  return v;
}

template <class M>
inline M from_ge_csr(ge_csr* c) {
  int rows = 0, cols = 0;
  long long nnz = 0;
  check(ge_csr_shape(c, &rows, &cols, &nnz));
  std::vector<int> I(rows + 1), J((size_t)nnz);
  std::vector<double> D((size_t)nnz);
  check(ge_csr_copy(c, I.data(), J.data(), D.data()));
  ge_csr_free(c);
  return M(I, J, D, rows, cols);
}

}  // namespace detail

// Extension: fix the seed that replaces std::random_device in this thread.
inline void setSeed(unsigned seed) { detail::seed_ref() = seed; }

}  // namespace partition

#endif  // GE_DROPIN_HPP
