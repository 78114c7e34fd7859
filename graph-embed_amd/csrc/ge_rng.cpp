// ge_rng.cpp -- the reference's random initialisation, restated explicitly.
//
// The reference seeds std::mt19937 from std::random_device
// (include/forceatlas.hpp:104-108, :332-336) and draws
// std::uniform_real_distribution<double>(-1, 1).  libe replaces random_device
// with ge_fa_params.seed and reproduces libstdc++'s value stream exactly:
//   * mt19937: 32-bit Mersenne Twister, init_genrand seeding;
//   * generate_canonical<double, 53>: two draws g1, g2 ->
//     (double(g1) + double(g2) * 2^32) / 2^64, clamped below 1;
//   * uniform(-1, 1) = canonical * 2.0 + (-1.0).
// tests/test_host.py checks it against std:: through the oracle.

#include <cmath>
#include <cstdint>

#include "ge_internal.hpp"

namespace ge {

namespace {

class Mt19937 {
 public:
  explicit Mt19937(uint32_t seed) {
    s_[0] = seed;
    for (int i = 1; i < 624; ++i) s_[i] = 1812433253u * (s_[i - 1] ^ (s_[i - 1] >> 30)) + (uint32_t)i;
    k_ = 624;
  }
  uint32_t next() {
    if (k_ >= 624) refill();
    uint32_t y = s_[k_++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
  }

 private:
  void refill() {
    for (int i = 0; i < 624; ++i) {
      const uint32_t y = (s_[i] & 0x80000000u) | (s_[(i + 1) % 624] & 0x7FFFFFFFu);
      uint32_t v = s_[(i + 397) % 624] ^ (y >> 1);
      if (y & 1u) v ^= 0x9908B0DFu;
      s_[i] = v;
    }
    k_ = 0;
  }
  uint32_t s_[624];
  int k_;
};

}  // namespace

void uniform_stream(unsigned seed, size_t count, double* out) {
  Mt19937 g(seed);
  const double two32 = 4294967296.0;
  const double two64 = 18446744073709551616.0;
  for (size_t c = 0; c < count; ++c) {
    double sum = (double)g.next();
    sum += (double)g.next() * two32;
    double canon = sum / two64;
    if (canon >= 1.0) canon = std::nextafter(1.0, 0.0);
    out[c] = canon * 2.0 + (-1.0);
  }
}

}  // namespace ge
