// Drop-in for include/partitioner.hpp (LLNL/graph-embed).
//   interpolationMatrix(numCols, partition)   src/partitioner.cpp:29-65
//   modularity(A, P_T)                        src/partitioner.cpp:69-114
//   partition(A, coarseningFactor, ...)       src/partitioner.cpp:1550-1893 (hierarchy)
// plus the extension galerkin(P_T, A) = P_T A P_T^T on the device (what the
// drivers compute with linalgcpp at examples/embed.cpp:96-98).
// The sibling overloads partition(A, bool...) / partition(A, int numParts, ...)
// and the float variants partitionTest/Base/Base2 stay declared, so overload
// resolution is the reference's (a double selects the hierarchy, an int
// numParts), but they are outside this library's scope and throw.
#ifndef PARTITIONER_HPP
#define PARTITIONER_HPP

#include <stdexcept>
#include <vector>

#include "ge_dropin.hpp"
#include "linalgcpp.hpp"
#include "matrixutils.hpp"

using CooMatrix = linalgcpp::CooMatrix<double>;

namespace partition {

inline SparseMatrix interpolationMatrix(const int numCols,
                                        const std::vector<std::vector<int>>& partition) {
  std::vector<int> offs(1, 0), sets;
  for (const auto& s : partition) {
    sets.insert(sets.end(), s.begin(), s.end());
    offs.push_back((int)sets.size());
  }
  ge_csr* c = nullptr;
  detail::check(ge_interpolation_matrix(numCols, (int)partition.size(), offs.data(),
                                        sets.data(), &c));
  return detail::from_ge_csr<SparseMatrix>(c);
}

inline double modularity(const SparseMatrix& A, const SparseMatrix& P_T) {
  const std::vector<int> agg = detail::vertex_of(P_T);
  double q = 0.0;
  detail::check(ge_modularity(A.Rows(), A.GetIndptr().data(), A.GetIndices().data(),
                              A.GetData().data(), P_T.Rows(), agg.data(), &q));
  return q;
}

[[noreturn]] inline void out_of_scope(const char* what) {
  throw std::logic_error(std::string("graph-embed_amd: ") + what +
                         " is outside this library's scope (SURVEY.md section 2)");
}

inline SparseMatrix partitionTest(const SparseMatrix&, const float = 1.0) {
  out_of_scope("partitionTest");
}
inline SparseMatrix partitionBase(const SparseMatrix&, const float = 1.0) {
  out_of_scope("partitionBase");
}
inline SparseMatrix partitionBase2(const SparseMatrix&, const float = 1.0) {
  out_of_scope("partitionBase2");
}
inline SparseMatrix partition(const SparseMatrix&, const bool = false, const bool = true,
                              const double = 1.0, const int = 2, const bool = false) {
  out_of_scope("single-level partition(A, printing, ...)");
}
inline SparseMatrix partition(const SparseMatrix&, const int, const bool = false,
                              const bool = true, const double = 1.0, const int = 2,
                              const bool = false) {
  out_of_scope("partition(A, numParts, ...)");
}

inline std::vector<SparseMatrix> partition(const SparseMatrix& A, const double coarseningFactor,
                                           const bool printing = false,
                                           const bool positiveMerging = true,
                                           const double stallStopThreshold = 1.0,
                                           const int matchingIterations = 2,
                                           const bool mergeLeaves = false) {
  ge_hier* h = nullptr;
  detail::check(ge_partition(detail::context(), A.Rows(), A.GetIndptr().data(),
                             A.GetIndices().data(), A.GetData().data(), coarseningFactor,
                             printing, positiveMerging, stallStopThreshold, matchingIterations,
                             mergeLeaves, &h));
  int levels = 0;
  detail::check(ge_hier_levels(h, &levels));
  std::vector<SparseMatrix> out;
  for (int l = 0; l < levels; ++l) {
    int rows = 0, cols = 0;
    detail::check(ge_hier_shape(h, l, &rows, &cols));
    std::vector<int> I(rows + 1), J(cols);
    detail::check(ge_hier_copy(h, l, I.data(), J.data()));
    out.emplace_back(I, J, std::vector<double>(cols, 1.0), rows, cols);
  }
  ge_hier_free(h);
  return out;
}

// Extension: P_T * A * P_T^T on the device (rows sorted ascending).
inline SparseMatrix galerkin(const SparseMatrix& P_T, const SparseMatrix& A) {
  ge_csr* c = nullptr;
  detail::check(ge_ptap(detail::context(), A.Rows(), A.GetIndptr().data(), A.GetIndices().data(),
                        A.GetData().data(), P_T.Rows(), P_T.GetIndptr().data(),
                        P_T.GetIndices().data(), &c));
  return detail::from_ge_csr<SparseMatrix>(c);
}

}  // namespace partition

#endif  // PARTITIONER_HPP
