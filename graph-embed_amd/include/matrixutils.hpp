// Drop-in for include/matrixutils.hpp (LLNL/graph-embed): the type aliases the
// hot path uses (include/matrixutils.hpp:17-19) and the three Laplacian helpers
// the reference declares there (:22-40, defined in src/matrixutils.cpp:16-98).
// The helpers are off the embedding path (nothing in the library or its drivers
// calls them); they are kept so user code that names them still compiles and
// gets the reference's matrices.  Header-only, host code.
#ifndef MATRIXUTILS_HPP
#define MATRIXUTILS_HPP

#include <vector>

#include "sparsematrix.hpp"

using SparseMatrix = linalgcpp::SparseMatrix<double>;
using coord = std::vector<double>;
using coordinates = std::vector<coord>;

namespace partition {

// n x n identity (src/matrixutils.cpp:16-29: the diagonal-vector constructor).
inline SparseMatrix identity(int n) { return SparseMatrix(std::vector<double>(n, 1.0)); }

// Graph Laplacian L = D - A of an adjacency matrix (src/matrixutils.cpp:31-70).
// Row i of L is row i of A negated, with the diagonal entry (the serial sum of
// row i's stored values, self-loops included) inserted before the first column
// greater than i -- or appended when there is none.  A stored self-loop is kept
// as its own (negated) entry next to the inserted diagonal, as in the reference.
inline SparseMatrix toLaplacian(const SparseMatrix& A) {
  const std::vector<int>& ip = A.GetIndptr();
  const std::vector<int>& ix = A.GetIndices();
  const std::vector<double>& dx = A.GetData();
  const int rows = A.Rows();
  std::vector<int> lp(rows + 1, 0);
  std::vector<int> lj;
  std::vector<double> lv;
  lj.reserve(ix.size() + rows);
  lv.reserve(ix.size() + rows);
  for (int i = 0; i < rows; ++i) {
    double deg = 0;
    for (int e = ip[i]; e < ip[i + 1]; ++e) deg += dx[e];
    bool placed = false;
    for (int e = ip[i]; e < ip[i + 1]; ++e) {
      if (!placed && ix[e] > i) {
        lj.push_back(i);
        lv.push_back(deg);
        placed = true;
      }
      lj.push_back(ix[e]);
      lv.push_back(-dx[e]);
    }
    if (!placed) {
      lj.push_back(i);
      lv.push_back(deg);
    }
    lp[i + 1] = (int)lj.size();
  }
  return SparseMatrix(lp, lj, lv, rows, A.Cols());
}

// Inverse of toLaplacian (src/matrixutils.cpp:72-98): drops, per row, the first
// stored entry whose column is >= i (the diagonal toLaplacian inserted; a row
// without one loses its slot at the end) and negates the rest.
inline SparseMatrix fromLaplacian(const SparseMatrix& L) {
  const std::vector<int>& ip = L.GetIndptr();
  const std::vector<int>& ix = L.GetIndices();
  const std::vector<double>& dx = L.GetData();
  const int rows = L.Rows();
  std::vector<int> ap(rows + 1, 0);
  for (int i = 1; i <= rows; ++i) ap[i] = ip[i] - i;
  std::vector<int> aj(ap[rows] > 0 ? ap[rows] : 0);
  std::vector<double> av(aj.size());
  int skipped = 0;  // entries of L dropped so far
  for (int i = 0; i < rows; ++i) {
    bool dropped = false;
    for (int k = ap[i]; k < ap[i + 1]; ++k) {
      if (!dropped && ix[k + skipped] >= i) {
        ++skipped;
        dropped = true;
      }
      aj[k] = ix[k + skipped];
      av[k] = -dx[k + skipped];
    }
    if (!dropped) ++skipped;
  }
  return SparseMatrix(ap, aj, av, rows, L.Cols());
}

}  // namespace partition

#endif  // MATRIXUTILS_HPP
