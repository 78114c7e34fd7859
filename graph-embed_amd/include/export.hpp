// Drop-in for include/export.hpp (LLNL/graph-embed): the text writers of
// src/export.cpp:16-39, same format (default stream precision, one vertex per
// line, values separated and terminated by a space).  Extension: writeCoords
// with a `digits` argument writes that many significant digits; 17
// (std::numeric_limits<double>::max_digits10) round-trips every fp64 coordinate
// exactly, which the reference's 6-digit output does not.
#ifndef EXPORT_HPP
#define EXPORT_HPP

#include <algorithm>
#include <fstream>
#include <iostream>
#include <limits>
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

inline void writeCoords(const std::vector<std::vector<double>>& coords,
                        const std::string& outputpath, int digits) {
  std::ofstream file(outputpath);
  file.precision(digits);
  for (const auto& row : coords) {
    for (double x : row) file << x << " ";
    file << "\n";
  }
}

// Full precision: every coordinate reads back to the same double.
inline void writeCoordsExact(const std::vector<std::vector<double>>& coords,
                             const std::string& outputpath) {
  writeCoords(coords, outputpath, std::numeric_limits<double>::max_digits10);
}

}  // namespace partition

#endif  // EXPORT_HPP
