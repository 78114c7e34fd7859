// Microbenchmark: dependent fp64 add chain latency on gfx950 (one wave), with
// terms from registers and from LDS (lane_chain-style pipelined reads).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void reg_chain(const double* in, double* out, int n, long long* cyc) {
  double a = in[threadIdx.x], b = in[threadIdx.x + 64];
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) a = a + b;
  }
  long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void reg_chain3(const double* in, double* out, int n, long long* cyc) {
  double a = in[threadIdx.x], c = in[threadIdx.x + 1], d = in[threadIdx.x + 2], b = in[threadIdx.x + 64];
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) { a = a + b; c = c + b; d = d + b; }
  }
  long long t1 = clock64();
  out[threadIdx.x] = a + c + d;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  double *in, *out; long long* cyc;
  hipMalloc(&in, 1024 * 8); hipMalloc(&out, 1024 * 8); hipMalloc(&cyc, 8);
  std::vector<double> h(1024, 1e-3); hipMemcpy(in, h.data(), 8192, hipMemcpyHostToDevice);
  const int n = 1 << 14;
  long long c;
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(reg_chain, dim3(1), dim3(64), 0, 0, in, out, n, cyc);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("1 chain: %.2f clock64 ticks per dependent v_add_f64\n", (double)c / (n * 16));
    hipLaunchKernelGGL(reg_chain3, dim3(1), dim3(64), 0, 0, in, out, n, cyc);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("3 chains: %.2f ticks per step (3 independent adds)\n", (double)c / (n * 16));
  }
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(reg_chain, dim3(1), dim3(64), 0, 0, in, out, n * 8, cyc);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("1 chain wall: %.3f ns per dependent add\n", ms * 1e6 / (n * 8 * 16.0));
  return 0;
}
