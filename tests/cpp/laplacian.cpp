// Calls the drop-in partition::identity / toLaplacian / fromLaplacian
// (graph-embed_amd/include/matrixutils.hpp) on a CSR read from argv[1]
// (int32 n, nnz, indptr, indices; float64 data) and writes the three results
// to argv[2] in the same format, one after the other.
#include <cstdio>
#include <vector>

#include "matrixutils.hpp"

static SparseMatrix read_csr(const char* path) {
  FILE* f = std::fopen(path, "rb");
  int hdr[2];
  if (!f || std::fread(hdr, sizeof(int), 2, f) != 2) throw 1;
  std::vector<int> ip(hdr[0] + 1), ix(hdr[1]);
  std::vector<double> dx(hdr[1]);
  if (std::fread(ip.data(), sizeof(int), ip.size(), f) != ip.size()) throw 2;
  if (std::fread(ix.data(), sizeof(int), ix.size(), f) != ix.size()) throw 3;
  if (std::fread(dx.data(), sizeof(double), dx.size(), f) != dx.size()) throw 4;
  std::fclose(f);
  return SparseMatrix(ip, ix, dx, hdr[0], hdr[0]);
}

static void write_csr(FILE* f, const SparseMatrix& M) {
  const int hdr[2] = {M.Rows(), (int)M.GetIndices().size()};
  std::fwrite(hdr, sizeof(int), 2, f);
  std::fwrite(M.GetIndptr().data(), sizeof(int), M.GetIndptr().size(), f);
  std::fwrite(M.GetIndices().data(), sizeof(int), M.GetIndices().size(), f);
  std::fwrite(M.GetData().data(), sizeof(double), M.GetData().size(), f);
}

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  const SparseMatrix A = read_csr(argv[1]);
  const SparseMatrix L = partition::toLaplacian(A);
  FILE* f = std::fopen(argv[2], "wb");
  write_csr(f, partition::identity(A.Rows()));
  write_csr(f, L);
  write_csr(f, partition::fromLaplacian(L));
  std::fclose(f);
  return 0;
}
