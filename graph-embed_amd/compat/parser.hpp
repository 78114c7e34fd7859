// compat/parser.hpp -- the graph readers / writer of linalgcpp that the
// reference's drivers call (examples/embed.cpp:80-91, examples/embedder.cpp:
// 167-186, examples/run-tests.cpp): ReadAdjList, ReadCooList, ReadTable,
// ReadCSR, ReadMTX, WriteCooList.  linalgcpp (github.com/gelever/linalgcpp) is
// not vendored and has no pinned version, so the file formats below restate its
// public conventions and are PARITY UNPINNED (no fixture in the reference holds
// one of these files):
//   adjacency list  "i j" per line, 0-based (value 1.0)
//   coordinate list "i j value" per line, 0-based
//   table           one line per row: the row's column indices (value 1.0)
//   CSR             "rows cols nnz", then indptr (rows+1), indices (nnz), data (nnz)
//   Matrix Market   coordinate format, 1-based, real / integer / pattern,
//                   general / symmetric (mirrored off-diagonal entries)
// With symmetric = true the list readers also add (j, i) for every (i, j) with
// i != j.  Duplicate entries are summed; the shape is the largest index + 1.
// Every reader throws std::runtime_error on a missing file or malformed line.
#ifndef GE_COMPAT_PARSER_HPP
#define GE_COMPAT_PARSER_HPP

#include <algorithm>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "sparsematrix.hpp"

namespace linalgcpp {

namespace parser_detail {

inline std::ifstream open_in(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open " + path);
  return f;
}

// (i, j, v) triples (+ mirrored) into a CSR with summed duplicates
template <typename T>
SparseMatrix<T> from_triples(std::vector<int> I, std::vector<int> J, std::vector<T> V,
                             int rows, int cols, bool symmetric) {
  if (symmetric) {
    const size_t m = I.size();
    for (size_t k = 0; k < m; ++k)
      if (I[k] != J[k]) {
        I.push_back(J[k]);
        J.push_back(I[k]);
        V.push_back(V[k]);
      }
  }
  for (size_t k = 0; k < I.size(); ++k) {
    rows = std::max(rows, I[k] + 1);
    cols = std::max(cols, J[k] + 1);
  }
  if (symmetric) rows = cols = std::max(rows, cols);
  CooMatrix<T> coo(rows, cols);
  for (size_t k = 0; k < I.size(); ++k) coo.Add(I[k], J[k], V[k]);
  return coo.ToSparse();
}

inline bool content_line(const std::string& line) {
  return line.find_first_not_of(" \t\r") != std::string::npos;
}

}  // namespace parser_detail

inline SparseMatrix<double> ReadAdjList(const std::string& path, bool symmetric = false) {
  auto f = parser_detail::open_in(path);
  std::vector<int> I, J;
  std::string line;
  while (std::getline(f, line)) {
    if (!parser_detail::content_line(line)) continue;
    std::istringstream s(line);
    int i, j;
    if (!(s >> i >> j) || i < 0 || j < 0) throw std::runtime_error("bad adjacency line: " + line);
    I.push_back(i);
    J.push_back(j);
  }
  std::vector<double> V(I.size(), 1.0);
  return parser_detail::from_triples<double>(I, J, V, 0, 0, symmetric);
}

inline SparseMatrix<double> ReadCooList(const std::string& path, bool symmetric = false) {
  auto f = parser_detail::open_in(path);
  std::vector<int> I, J;
  std::vector<double> V;
  std::string line;
  while (std::getline(f, line)) {
    if (!parser_detail::content_line(line)) continue;
    std::istringstream s(line);
    int i, j;
    double v;
    if (!(s >> i >> j >> v) || i < 0 || j < 0) throw std::runtime_error("bad coordinate line: " + line);
    I.push_back(i);
    J.push_back(j);
    V.push_back(v);
  }
  return parser_detail::from_triples<double>(I, J, V, 0, 0, symmetric);
}

template <typename T = double>
SparseMatrix<T> ReadTable(const std::string& path) {
  auto f = parser_detail::open_in(path);
  std::vector<int> I, J;
  std::string line;
  int row = 0;
  while (std::getline(f, line)) {
    std::istringstream s(line);
    int j;
    while (s >> j) {
      if (j < 0) throw std::runtime_error("bad table entry in: " + line);
      I.push_back(row);
      J.push_back(j);
    }
    ++row;
  }
  std::vector<T> V(I.size(), T(1));
  return parser_detail::from_triples<T>(I, J, V, row, 0, false);
}

inline SparseMatrix<double> ReadCSR(const std::string& path) {
  auto f = parser_detail::open_in(path);
  long long rows, cols, nnz;
  if (!(f >> rows >> cols >> nnz) || rows < 0 || cols < 0 || nnz < 0)
    throw std::runtime_error("bad CSR header in " + path);
  std::vector<int> I(rows + 1), J(nnz);
  std::vector<double> D(nnz);
  for (auto& x : I) f >> x;
  for (auto& x : J) f >> x;
  for (auto& x : D) f >> x;
  if (!f || I[0] != 0 || I[rows] != nnz) throw std::runtime_error("bad CSR body in " + path);
  for (long long r = 0; r < rows; ++r)
    if (I[r] > I[r + 1]) throw std::runtime_error("CSR indptr not monotone in " + path);
  for (int j : J)
    if (j < 0 || j >= cols) throw std::runtime_error("CSR column out of range in " + path);
  return SparseMatrix<double>(I, J, D, (int)rows, (int)cols);
}

inline SparseMatrix<double> ReadMTX(const std::string& path) {
  auto f = parser_detail::open_in(path);
  std::string line;
  if (!std::getline(f, line) || line.rfind("%%MatrixMarket", 0) != 0)
    throw std::runtime_error("not a Matrix Market file: " + path);
  std::string lower = line;
  std::transform(lower.begin(), lower.end(), lower.begin(), ::tolower);
  if (lower.find("coordinate") == std::string::npos)
    throw std::runtime_error("only coordinate Matrix Market files are supported: " + path);
  const bool pattern = lower.find("pattern") != std::string::npos;
  const bool symmetric = lower.find("symmetric") != std::string::npos;
  while (std::getline(f, line) && (line.empty() || line[0] == '%')) {
  }
  long long rows, cols, nnz;
  {
    std::istringstream s(line);
    if (!(s >> rows >> cols >> nnz)) throw std::runtime_error("bad Matrix Market size line");
  }
  std::vector<int> I, J;
  std::vector<double> V;
  while ((long long)I.size() < nnz && std::getline(f, line)) {
    if (!parser_detail::content_line(line) || line[0] == '%') continue;
    std::istringstream s(line);
    long long i, j;
    double v = 1.0;
    if (!(s >> i >> j) || (!pattern && !(s >> v)) || i < 1 || j < 1 || i > rows || j > cols)
      throw std::runtime_error("bad Matrix Market entry: " + line);
    I.push_back((int)(i - 1));
    J.push_back((int)(j - 1));
    V.push_back(v);
  }
  if ((long long)I.size() != nnz) throw std::runtime_error("Matrix Market file ended early");
  return parser_detail::from_triples<double>(I, J, V, (int)rows, (int)cols, symmetric);
}

template <typename T>
void WriteCooList(const SparseMatrix<T>& A, const std::string& path, bool symmetric = false) {
  std::ofstream f(path);
  if (!f) throw std::runtime_error("cannot write " + path);
  const auto& I = A.GetIndptr();
  const auto& J = A.GetIndices();
  const auto& D = A.GetData();
  f.precision(17);
  for (int r = 0; r < A.Rows(); ++r)
    for (int k = I[r]; k < I[r + 1]; ++k)
      if (!symmetric || r <= J[k]) f << r << " " << J[k] << " " << D[k] << "\n";
}

}  // namespace linalgcpp

#endif
