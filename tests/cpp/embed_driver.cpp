// The reference's config-1 driver flow (examples/embed.cpp:93-102) written
// against the drop-in headers only: partition(A, 0.1), P^T A P per level,
// embed(As, hierarchy, d).  The input CSR comes from a small binary file (the
// reference reads it with linalgcpp parsers, examples/embed.cpp:80-91); the
// coordinates go to a binary file for the test to compare.
//   embed_driver <in.bin> <out.bin> <dim> <seed> [ml | via]
// "via": embedVia(As, hierarchy, d, anyToMultilevel(embedViaMinimization)), the
// reference's alternative multilevel embedder (src/embed.cpp:23-338).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "embed.hpp"
#include "export.hpp"
#include "partitioner.hpp"

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  std::ifstream in(argv[1], std::ios::binary);
  int n = 0, nnz = 0;
  in.read((char*)&n, sizeof(int));
  in.read((char*)&nnz, sizeof(int));
  std::vector<int> I(n + 1), J(nnz);
  std::vector<double> D(nnz);
  in.read((char*)I.data(), sizeof(int) * (n + 1));
  in.read((char*)J.data(), sizeof(int) * nnz);
  in.read((char*)D.data(), sizeof(double) * nnz);
  SparseMatrix A(I, J, D, n, n);
  const int dim = std::atoi(argv[3]);
  partition::setSeed((unsigned)std::strtoul(argv[4], nullptr, 10));

  double coarseningFactor = 0.1;
  std::vector<SparseMatrix> hierarchy = partition::partition(A, coarseningFactor);
  std::vector<SparseMatrix> As = {A};
  for (size_t level = 0; level < hierarchy.size(); level++) {
    SparseMatrix host = hierarchy[level].Mult(As[level]).Mult(hierarchy[level].Transpose());
    SparseMatrix dev = partition::galerkin(hierarchy[level], As[level]);
    if (host.GetIndptr() != dev.GetIndptr() || host.GetIndices() != dev.GetIndices() ||
        host.GetData() != dev.GetData()) {
      std::fprintf(stderr, "galerkin mismatch at level %zu\n", level);
      return 3;
    }
    As.push_back(dev);
  }
  std::vector<std::vector<double>> coords;
  if (argc > 5 && std::string(argv[5]) == "via") {
    using Embedder = std::vector<std::vector<double>> (*)(const SparseMatrix&, const int);
    coords = partition::embedVia(
        As, hierarchy, dim,
        partition::anyToMultilevel(static_cast<Embedder>(partition::embedViaMinimization)));
  } else if (argc > 5) {
    std::vector<double> r_A;
    std::vector<std::vector<double>> coords_A;
    coords = partition::embedMultilevel(As, hierarchy, dim, 0, r_A, coords_A);
  } else {
    coords = partition::embed(As, hierarchy, dim);
  }
  std::ofstream out(argv[2], std::ios::binary);
  for (const auto& row : coords) out.write((const char*)row.data(), sizeof(double) * dim);
  partition::writeCoords(coords, std::string(argv[2]) + ".txt");
  partition::writeCoordsExact(coords, std::string(argv[2]) + ".exact.txt");
  return 0;
}
