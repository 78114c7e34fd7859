// Microbenchmark: issue cost of fp64 VALU instructions on gfx950 -- v_fma_f64,
// v_rcp_f64, v_rsq_f64 and the 60:3 mix of the symmetric repulsion step -- as
// SIMD cycles per wave-instruction, with 1 and 4 waves per SIMD (8 independent
// chains per lane).  One block on one CU; cycles from s_memtime (shader clock).
// build: hipcc --offload-arch=gfx950 -O3 f64_issue.hip -o f64_issue
#include <hip/hip_runtime.h>

#include <cstdio>

template <int KIND>
__global__ void issue(const double* in, double* out, int n, long long* cyc) {
  double v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = in[(threadIdx.x + u) & 255] + 1.0;
  const double b = in[300], c = in[301];
  __syncthreads();
  const long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    if (KIND == 0) {  // 16 fma per lane-iteration... 8 chains x 2
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_fma(v[u], b, c);
    } else if (KIND == 1) {  // 8 rcp
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = __builtin_amdgcn_rcp(v[u]);
    } else if (KIND == 2) {  // 8 rsq
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = __builtin_amdgcn_rsq(v[u]);
    } else {  // 20 fma + 1 rcp per chain pair: the repulsion step's 60:3
#pragma unroll
      for (int u = 0; u < 8; ++u) {
#pragma unroll
        for (int r = 0; r < 20; ++r) v[u] = __builtin_fma(v[u], b, c);
        v[u] = __builtin_amdgcn_rcp(v[u]);
      }
    }
  }
  const long long t1 = clock64();
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += v[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double *in, *out;
  long long* cyc;
  hipMalloc(&in, 4096 * sizeof(double));
  hipMalloc(&out, 1 << 24);
  hipMalloc(&cyc, 1024 * sizeof(long long));
  double h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = 1.0 + i * 1e-6;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const int n = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[4] = {"fma", "rcp", "rsq", "mix20fma+rcp"};
  const double per_iter[4] = {16, 8, 8, 168};  // wave-instructions per wave per iteration
  // whole chip: 256 CUs x B blocks of 256 threads (B waves per SIMD); wall time by
  // events, priced at 2.4 GHz
  for (int B : {1, 2, 4}) {
    for (int k = 0; k < 4; ++k) {
      const int grid = 256 * B;
      auto run = [&]() {
        switch (k) {
          case 0: hipLaunchKernelGGL(issue<0>, dim3(grid), dim3(256), 0, 0, in, out, n, cyc); break;
          case 1: hipLaunchKernelGGL(issue<1>, dim3(grid), dim3(256), 0, 0, in, out, n, cyc); break;
          case 2: hipLaunchKernelGGL(issue<2>, dim3(grid), dim3(256), 0, 0, in, out, n, cyc); break;
          default: hipLaunchKernelGGL(issue<3>, dim3(grid), dim3(256), 0, 0, in, out, n, cyc); break;
        }
      };
      run();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      run();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      long long c = 0;
      hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
      const double instr = per_iter[k] * n * B;  // wave-instructions per SIMD
      std::printf("%-14s waves/SIMD %d: %.2f cycles at 2.4 GHz per wave-instruction per SIMD "
                  "(%.3f ms; clock64 ticks per wave-instruction of wave 0: %.2f)\n",
                  names[k], B, ms * 1e-3 * 2.4e9 / instr, ms, (double)c / (per_iter[k] * n));
    }
  }
  return 0;
}
