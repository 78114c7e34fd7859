// ge_quality.hip -- modularity of a partition on the device.
//
// Reference: partition::modularity, src/partitioner.cpp:69-114.  Every weight is
// truncated to int (`int a_ij = D[k]`, :90) before it is summed, so d[A], out[A]
// and T are sums of integers: exact in any order while they stay below 2^53.
// They are accumulated here in 64-bit integer atomics (one per row and
// aggregate; T per block), then the O(M) final sum runs on the host in the
// reference's aggregate order with the reference's double arithmetic.

#include <hip/hip_runtime.h>

#include <vector>

#include "ge_internal.hpp"

namespace ge {
namespace {

constexpr int kQT = 256;

__global__ void __launch_bounds__(kQT)
modularity_rows(int n, const int* __restrict__ ip, const int* __restrict__ ix,
                const double* __restrict__ dx, const int* __restrict__ vA,
                unsigned long long* __restrict__ din, unsigned long long* __restrict__ dout,
                unsigned long long* __restrict__ total) {
  __shared__ long long red[kQT];
  const int i = blockIdx.x * kQT + threadIdx.x;
  long long lt = 0;
  if (i < n) {
    const int a = vA[i];
    long long li = 0, lo = 0;
    for (int e = ip[i]; e < ip[i + 1]; ++e) {
      const long long w = (int)dx[e];  // sic: truncation to int (:90)
      if (vA[ix[e]] == a) li += w;
      else lo += w;
      lt += w;
    }
    if (li) atomicAdd(&din[a], (unsigned long long)li);  // two's complement: signed sums
    if (lo) atomicAdd(&dout[a], (unsigned long long)lo);
  }
  red[threadIdx.x] = lt;
  __syncthreads();
  for (int s = kQT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0 && red[0]) atomicAdd(total, (unsigned long long)red[0]);
}

}  // namespace
}  // namespace ge

extern "C" int ge_modularity_device(ge_ctx* ctx, int n, const int* d_ip, const int* d_ix,
                                    const double* d_dx, int m, const int* d_vA, double* q) {
  return ge::guarded([&] {
    GE_REQUIRE(ctx && q && d_ip && d_vA && (n == 0 || (d_ix && d_dx)), "null argument");
    GE_REQUIRE(n >= 0 && m > 0, "bad sizes");
    ge::DeviceGuard g(ctx);
    hipStream_t s = ctx->stream;
    ge::DevBuf<unsigned long long> acc(2 * (size_t)m + 1);
    GE_HIP(hipMemsetAsync(acc.p, 0, sizeof(unsigned long long) * acc.n, s));
    if (n > 0) {
      hipLaunchKernelGGL(ge::modularity_rows, dim3((n + ge::kQT - 1) / ge::kQT), dim3(ge::kQT),
                         0, s, n, d_ip, d_ix, d_dx, d_vA, acc.p, acc.p + m, acc.p + 2 * m);
      GE_HIP(hipGetLastError());
    }
    std::vector<long long> h(acc.n);
    GE_HIP(hipMemcpyAsync(h.data(), acc.p, sizeof(long long) * acc.n, hipMemcpyDeviceToHost, s));
    GE_HIP(hipStreamSynchronize(s));
    const double T = (double)h[2 * (size_t)m];
    double sum = 0.0;
    for (int a = 0; a < m; ++a) {  // :103-108, aggregate order
      const double din = (double)h[a], dout = (double)h[(size_t)m + a];
      const double alpha = (din + dout) / T;
      sum += din / T - alpha * alpha;
    }
    *q = sum;
  });
}
