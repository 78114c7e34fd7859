// Drop-in for include/matrixutils.hpp (LLNL/graph-embed): the type aliases the
// hot path uses (include/matrixutils.hpp:17-19).  The Laplacian helpers
// identity/toLaplacian/fromLaplacian (src/matrixutils.cpp) are never called by
// the library or its drivers and are not provided.
#ifndef MATRIXUTILS_HPP
#define MATRIXUTILS_HPP

#include <vector>

#include "sparsematrix.hpp"

using SparseMatrix = linalgcpp::SparseMatrix<double>;
using coord = std::vector<double>;
using coordinates = std::vector<coord>;

#endif  // MATRIXUTILS_HPP
