// compat/sparsematrix.hpp -- the subset of linalgcpp's SparseMatrix<T> that
// graph-embed's drivers and the drop-in headers use, for building the drop-in
// tests in an image without linalgcpp (github.com/gelever/linalgcpp, not
// vendored by the reference).  With the real linalgcpp installed, put its
// include directory first and leave this one out.
#ifndef GE_COMPAT_SPARSEMATRIX_HPP
#define GE_COMPAT_SPARSEMATRIX_HPP

#include <algorithm>
#include <cassert>
#include <map>
#include <utility>
#include <vector>

namespace linalgcpp {

template <typename T>
class SparseMatrix {
 public:
  SparseMatrix() : indptr_(1, 0) {}
  SparseMatrix(std::vector<int> I, std::vector<int> J, std::vector<T> D, int rows, int cols)
      : indptr_(std::move(I)), indices_(std::move(J)), data_(std::move(D)), rows_(rows),
        cols_(cols) {
    assert((int)indptr_.size() == rows_ + 1);
  }
  explicit SparseMatrix(std::vector<T> diag) : rows_((int)diag.size()), cols_((int)diag.size()) {
    indptr_.resize(rows_ + 1);
    indices_.resize(rows_);
    for (int i = 0; i <= rows_; ++i) indptr_[i] = i;
    for (int i = 0; i < rows_; ++i) indices_[i] = i;
    data_ = std::move(diag);
  }

  int Rows() const { return rows_; }
  int Cols() const { return cols_; }
  int nnz() const { return (int)indices_.size(); }
  const std::vector<int>& GetIndptr() const { return indptr_; }
  const std::vector<int>& GetIndices() const { return indices_; }
  const std::vector<T>& GetData() const { return data_; }

  SparseMatrix<T> Transpose() const {
    std::vector<int> I(cols_ + 1, 0), J(indices_.size());
    std::vector<T> D(indices_.size());
    for (int j : indices_) I[j + 1]++;
    for (int c = 0; c < cols_; ++c) I[c + 1] += I[c];
    std::vector<int> fill(I.begin(), I.end() - 1);
    for (int r = 0; r < rows_; ++r)
      for (int k = indptr_[r]; k < indptr_[r + 1]; ++k) {
        J[fill[indices_[k]]] = r;
        D[fill[indices_[k]]++] = data_[k];
      }
    return SparseMatrix<T>(I, J, D, cols_, rows_);
  }

  // Row-wise product, columns of each result row ascending.
  SparseMatrix<T> Mult(const SparseMatrix<T>& B) const {
    assert(cols_ == B.rows_);
    std::vector<int> I(rows_ + 1, 0), J;
    std::vector<T> D;
    std::map<int, T> row;
    for (int r = 0; r < rows_; ++r) {
      row.clear();
      for (int k = indptr_[r]; k < indptr_[r + 1]; ++k)
        for (int q = B.indptr_[indices_[k]]; q < B.indptr_[indices_[k] + 1]; ++q)
          row[B.indices_[q]] += data_[k] * B.data_[q];
      for (const auto& kv : row) {
        J.push_back(kv.first);
        D.push_back(kv.second);
      }
      I[r + 1] = (int)J.size();
    }
    return SparseMatrix<T>(I, J, D, rows_, B.cols_);
  }

 private:
  std::vector<int> indptr_, indices_;
  std::vector<T> data_;
  int rows_ = 0, cols_ = 0;
};

template <typename T>
class CooMatrix {
 public:
  CooMatrix(int rows, int cols) : rows_(rows), cols_(cols) {}
  void Add(int i, int j, T v) { entries_[{i, j}] += v; }
  SparseMatrix<T> ToSparse() const {
    std::vector<int> I(rows_ + 1, 0), J;
    std::vector<T> D;
    for (const auto& kv : entries_) {
      I[kv.first.first + 1]++;
      J.push_back(kv.first.second);
      D.push_back(kv.second);
    }
    for (int r = 0; r < rows_; ++r) I[r + 1] += I[r];
    return SparseMatrix<T>(I, J, D, rows_, cols_);
  }

 private:
  int rows_, cols_;
  std::map<std::pair<int, int>, T> entries_;
};

}  // namespace linalgcpp

#endif
