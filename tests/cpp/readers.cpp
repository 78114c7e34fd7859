// Prints the CSR a linalgcpp reader of compat/parser.hpp builds from a file:
//   readers <adjlist|coolist|table|csr|mtx|writecoo> <path> [symmetric] [out]
// ("writecoo" reads a coordinate list and writes it back with WriteCooList).
#include <cstdio>
#include <cstring>
#include <string>

#include "linalgcpp.hpp"

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::string fmt = argv[1], path = argv[2];
  const bool sym = argc > 3 && std::strcmp(argv[3], "1") == 0;
  linalgcpp::SparseMatrix<double> A;
  try {
    if (fmt == "adjlist") A = linalgcpp::ReadAdjList(path, sym);
    else if (fmt == "coolist" || fmt == "writecoo") A = linalgcpp::ReadCooList(path, sym);
    else if (fmt == "table") A = linalgcpp::ReadTable<double>(path);
    else if (fmt == "csr") A = linalgcpp::ReadCSR(path);
    else if (fmt == "mtx") A = linalgcpp::ReadMTX(path);
    else return 2;
    if (fmt == "writecoo") linalgcpp::WriteCooList(A, argv[4]);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  std::printf("%d %d %d\n", A.Rows(), A.Cols(), A.nnz());
  for (int v : A.GetIndptr()) std::printf("%d ", v);
  std::printf("\n");
  for (int v : A.GetIndices()) std::printf("%d ", v);
  std::printf("\n");
  for (double v : A.GetData()) std::printf("%.17g ", v);
  std::printf("\n");
  return 0;
}
