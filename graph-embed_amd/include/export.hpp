// Drop-in for include/export.hpp (LLNL/graph-embed): the text writers of
// src/export.cpp:16-39, same format (default stream precision, one vertex per
// line, values separated and terminated by a space).
#ifndef EXPORT_HPP
#define EXPORT_HPP

#include <algorithm>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "matrixutils.hpp"

namespace partition {

inline void writePartition(const std::vector<int>& partition, const std::string& outputpath) {
  std::ofstream file(outputpath);
  for (int v : partition) file << v << "\n";
}

inline void writeCoords(const std::vector<std::vector<double>>& coords,
                        const std::string& outputpath) {
  std::ofstream file(outputpath);
  for (const auto& row : coords) {
    for (double x : row) file << x << " ";
    file << "\n";
  }
}

}  // namespace partition

#endif  // EXPORT_HPP
