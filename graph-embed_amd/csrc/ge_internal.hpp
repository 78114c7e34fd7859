// ge_internal.hpp -- shared internals of libge.so (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "ge.h"

namespace ge {

// Error plumbing: internal code throws ge::Error; every extern "C" entry point
// catches it, records the message for ge_last_error() and returns the code.
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

#define GE_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t _e = (call);                                                           \
    if (_e != hipSuccess)                                                             \
      throw ::ge::Error(GE_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(_e) + \
                                        " (" __FILE__ ":" + std::to_string(__LINE__) + ")"); \
  } while (0)

#define GE_REQUIRE(cond, msg)                                 \
  do {                                                        \
    if (!(cond)) throw ::ge::Error(GE_ERR_ARG, (msg));        \
  } while (0)

template <class F>
int guarded(F&& f) {
  try {
    f();
    return GE_OK;
  } catch (const Error& e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    set_last_error("host allocation failed");
    return GE_ERR_NOMEM;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return GE_ERR_STATE;
  }
}

// RAII device buffer.
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  explicit DevBuf(size_t count) { alloc(count); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
    return *this;
  }
  ~DevBuf() { release(); }
  void alloc(size_t count) {
    release();
    n = count;
    if (count) GE_HIP(hipMalloc(&p, count * sizeof(T)));
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  void upload(const T* h, size_t count, hipStream_t s) {
    if (count) GE_HIP(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s));
  }
  void download(T* h, size_t count, hipStream_t s) const {
    if (count) GE_HIP(hipMemcpyAsync(h, p, count * sizeof(T), hipMemcpyDeviceToHost, s));
  }
};

}  // namespace ge

struct ge_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
};

// Host CSR (returned to callers through ge_csr*).
struct ge_csr {
  int rows = 0, cols = 0;
  std::vector<int> indptr, indices;
  std::vector<double> data;
};

struct ge_hier {
  std::vector<int> rows, cols;
  std::vector<std::vector<int>> indptr, indices;
};

namespace ge {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(const ge_ctx* c) {
    GE_HIP(hipGetDevice(&prev));
    if (prev != c->device) GE_HIP(hipSetDevice(c->device));
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

// libstdc++ uniform_real_distribution<double>(-1,1) over mt19937(seed); written
// out explicitly (see ge_rng.cpp) and tested equal to std:: in tests.
void uniform_stream(unsigned seed, size_t count, double* out);

// Device entry points implemented in the .hip files, called by host drivers.
void fa_run_device(ge_ctx* ctx, int n, int nnz, const int* d_ip, const int* d_ix,
                   const double* d_dx, int dim, double* d_x, int iterations,
                   const ge_fa_params& p);
void faml_run_device(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix, const double* d_dx,
                     int m, const int* h_pt_ip, const int* d_pt_ip, const int* d_pt_ix,
                     const int* d_vA, const double* d_cA, const double* d_rA,
                     const double* d_init, double* d_x, int dim, int iterations,
                     const ge_fa_params& p);
ge_hier* partition_incremental(int n, const int* I, const int* J, const double* Dv, double cf,
                               bool printing, bool positive, double stall, int matching);
// Device path (ge_partition_dev.hip); nullptr when the input needs the host path
// (non-integer weights, asymmetric A, rows not strictly ascending).
ge_hier* partition_device(ge_ctx* ctx, int n, const int* I, const int* J, const double* Dv,
                          double cf, bool printing, bool positive, double stall, int matching);
void ptap_device(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix, const double* d_dx,
                 int nnz, int m, const int* d_pt_ip, const int* d_pt_ix, ge_csr* out);

}  // namespace ge
