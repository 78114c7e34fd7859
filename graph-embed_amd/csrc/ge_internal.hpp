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

// Device copy of a host CSR.
struct DevCsr {
  DevBuf<int> ip, ix;
  DevBuf<double> dx;
  int n = 0, nnz = 0;
  DevCsr(int rows, const int* hip_, const int* hix, const double* hdx, hipStream_t s)
      : ip(rows + 1), ix(hip_[rows] > 0 ? hip_[rows] : 1), dx(hip_[rows] > 0 ? hip_[rows] : 1),
        n(rows), nnz(hip_[rows]) {
    ip.upload(hip_, rows + 1, s);
    ix.upload(hix, nnz, s);
    dx.upload(hdx, nnz, s);
  }
};

}  // namespace ge

struct ge_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
};

// A communicator (ge_dist.hip): RCCL, or a caller transport staged through host
// memory.  `nccl` is an ncclComm_t kept opaque here.
struct ge_comm {
  ge_ctx* ctx = nullptr;
  int nranks = 1, rank = 0;
  void* nccl = nullptr;
  ge_transport tp{};
};

namespace ge {
// Multi-GPU helpers (ge_dist.hip) used inside per-level plans.
void allgather_stream(ge_comm* c, hipStream_t s, const void* d_send, void* d_recv, size_t bytes);
void exchange_rows(ge_comm* c, hipStream_t s, int dim, const int* d_rows, const int* d_counts,
                   const int* d_first, const int* h_counts, const int* h_first, int width,
                   double* d_buf, double* d_x);
}  // namespace ge

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
// Host CSR validation (indptr, index range); throws GE_ERR_ARG.
void check_csr(int n, const int* ip, const int* ix, const double* dx);

// Device entry points implemented in the .hip files, called by host drivers.
// One launch of the symmetric all-pairs repulsion (ge_sym.hpp, faml_sym_repulse)
// over `nunits` units {aggregate, row tile, progress offset, kind}; queue and
// prog zeroed by the caller.  Defined in ge_faml.hip, shared with single-level
// forceAtlas (ge_fa.hip).  sym_blocks_per_cu: the resident blocks it is sized for.
void sym_repulse_launch(int dim, int blocks, hipStream_t s, int nunits, const int4* units,
                        int* queue, const int* seg, const double* X, const double* DP,
                        double repel, double* F, double* H, size_t hs, int* prog, int* err,
                        long long limit);
int sym_blocks_per_cu(int dim);

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
// Coarse rows [a0, a1) of P_T A P_T^T (a0 = 0, a1 = m: the whole matrix) into a
// host CSR of a1 - a0 rows and m columns.  h_pt_ip: P_T's indptr on the host.
void ptap_device(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix, const double* d_dx,
                 int nnz, int m, const int* h_pt_ip, const int* d_pt_ip, const int* d_pt_ix,
                 int a0, int a1, ge_csr* out);

// Host-array drivers (ge_host.cpp) and their sharded forms (ge_dist.hip).
void fa_host(ge_ctx* ctx, int n, const int* ip, const int* ix, const double* dx, int dim,
             double* X, bool init_random, int iterations, const ge_fa_params& p);
void faml_host(ge_ctx* ctx, int n, const int* ip, const int* ix, const double* dx, int m,
               const int* pip, const int* pix, const int* vA, const double* cA,
               const double* rA, double* X, int dim, int iterations, const ge_fa_params& p);
void normalize_host(double* X, int n, int dim);
// radius step (src/embed.cpp:615-777): host replay of the serial event loop
// (ge_host.cpp) and the device rounds (ge_radius.hip; false: a zero distance,
// the caller must use the host version)
void radius_step_host(int m, double* cA, double* rA, int dim, bool base, int mc, const int* PIc,
                      const int* PJc, const double* cAc, const double* rAc, const int* AcI,
                      const int* AcJ);
bool radius_step_device(ge_ctx* ctx, int m, double* cA, double* rA, int dim, bool base, int mc,
                        const int* PIc, const int* PJc, const double* cAc, const double* rAc,
                        const int* AcI, const int* AcJ);
void fa_host_dist(ge_comm* comm, int n, const int* ip, const int* ix, const double* dx, int dim,
                  double* X, bool init_random, int iterations, const ge_fa_params& p);
void faml_host_dist(ge_comm* comm, int n, const int* ip, const int* ix, const double* dx, int m,
                    const int* pip, const int* pix, const int* vA, const double* cA,
                    const double* rA, double* X, int dim, int iterations,
                    const ge_fa_params& p);
// the embed orchestration (src/embed.cpp:561-796); comm == nullptr: one GPU
void embed_impl(ge_ctx* ctx, ge_comm* comm, int levels, const int* a_n, const int* a_off,
                const int* a_nz_off, const int* a_ip, const int* a_ix, const double* a_dx,
                const int* p_rows, const int* p_off, const int* p_nz_off, const int* p_ip,
                const int* p_ix, int dim, int base_iterations, int ml_iterations,
                int print_progress, const ge_fa_params& p, double* coords_out);

}  // namespace ge
