// compat/linalgcpp.hpp -- see compat/sparsematrix.hpp and compat/parser.hpp
// (graph readers).  Also the Timer the reference's drivers use
// (examples/embedder.cpp:219-222).
#ifndef GE_COMPAT_LINALGCPP_HPP
#define GE_COMPAT_LINALGCPP_HPP

#include <chrono>
#include <vector>

#include "parser.hpp"
#include "sparsematrix.hpp"

namespace linalgcpp {

class Timer {
 public:
  enum class Start { True, False };
  explicit Timer(Start s = Start::False) {
    if (s == Start::True) Click();
  }
  void Click() {
    const auto now = std::chrono::steady_clock::now();
    if (started_) laps_.push_back(std::chrono::duration<double>(now - last_).count());
    last_ = now;
    started_ = true;
  }
  double operator[](int i) const { return laps_.at(i); }

 private:
  bool started_ = false;
  std::chrono::steady_clock::time_point last_;
  std::vector<double> laps_;
};

}  // namespace linalgcpp

#endif
