// Microbenchmark: the coarsest level's packed adder (ge_fa.hip packed_iteration) in
// isolation -- lanes 0..11 of wave 0 add chunks of 96 terms from an LDS line each
// (stride 98 doubles), one dependent v_add_f64 per term, in batches of 16 16-byte
// reads prefetched one batch ahead; the other three waves idle or run fp64 work.
// Prints shader-clock cycles per chunk for: the adds from registers, the adds from
// LDS (prefetched), from LDS with a workgroup barrier per chunk, and with three
// busy waves beside it.  build: hipcc --offload-arch=gfx950 -O3 adder_chain.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int C = 96, S = 98, B = 16;

// the same, with the reads of batch b + 1 interleaved one per two adds of batch b
// (sched_group_barrier: 1 DS read, then 2 VALU, repeated)
__device__ __forceinline__ double chain_interleaved(double a, const double* p) {
  double v[2][B];
#pragma unroll
  for (int l = 0; l < B; l += 2) {
    const double2 x = *reinterpret_cast<const double2*>(p + l);
    v[0][l] = x.x;
    v[0][l + 1] = x.y;
  }
#pragma unroll
  for (int b = 0; b < C / B; ++b) {
    if (b + 1 < C / B) {
#pragma unroll
      for (int l = 0; l < B; l += 2) {
        const double2 x = *reinterpret_cast<const double2*>(p + (b + 1) * B + l);
        v[(b + 1) & 1][l] = x.x;
        v[(b + 1) & 1][l + 1] = x.y;
      }
    }
#pragma unroll
    for (int l = 0; l < B; ++l) a = a + v[b & 1][l];
    if (b + 1 < C / B) {
#pragma unroll
      for (int l = 0; l < B / 2; ++l) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // two VALU
      }
    }
  }
  return a;
}

// the shipped form (ge_fa.hip chain_prefetch): three batches ahead, runtime cnt
__device__ __forceinline__ double chain_shipped(double a, const double* p, int cnt) {
  constexpr int NB = C / B, P = 3, R = P + 1;
  double v[R][B];
#pragma unroll
  for (int b = 0; b < P && b < NB; ++b)
#pragma unroll
    for (int l = 0; l < B; l += 2) {
      const double2 x = *reinterpret_cast<const double2*>(p + b * B + l);
      v[b][l] = x.x;
      v[b][l + 1] = x.y;
    }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b + P < NB) {
#pragma unroll
      for (int l = 0; l < B; l += 2) {
        const double2 x = *reinterpret_cast<const double2*>(p + (b + P) * B + l);
        v[(b + P) % R][l] = x.x;
        v[(b + P) % R][l + 1] = x.y;
      }
    }
    if (cnt >= C) {
#pragma unroll
      for (int l = 0; l < B; ++l) a = a + v[b % R][l];
    } else {
#pragma unroll
      for (int l = 0; l < B; ++l) a = a + ((b * B + l < cnt) ? v[b % R][l] : 0.0);
    }
  }
  return a;
}

// the round-5 fix: no per-batch branch on the count (full chunks: plain adds)
__device__ __forceinline__ double chain_fixed(double a, const double* p) {
  constexpr int NB = C / B, P = 3, R = P + 1;
  double v[R][B];
#pragma unroll
  for (int b = 0; b < P && b < NB; ++b)
#pragma unroll
    for (int l = 0; l < B; l += 2) {
      const double2 x = *reinterpret_cast<const double2*>(p + b * B + l);
      v[b][l] = x.x;
      v[b][l + 1] = x.y;
    }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b + P < NB) {
#pragma unroll
      for (int l = 0; l < B; l += 2) {
        const double2 x = *reinterpret_cast<const double2*>(p + (b + P) * B + l);
        v[(b + P) % R][l] = x.x;
        v[(b + P) % R][l + 1] = x.y;
      }
    }
#pragma unroll
    for (int l = 0; l < B; ++l) a = a + v[b % R][l];
  }
  return a;
}

__device__ __forceinline__ double chain_prefetch(double a, const double* p) {
  double v[2][B];
#pragma unroll
  for (int l = 0; l < B; l += 2) {
    const double2 x = *reinterpret_cast<const double2*>(p + l);
    v[0][l] = x.x;
    v[0][l + 1] = x.y;
  }
#pragma unroll
  for (int b = 0; b < C / B; ++b) {
    if (b + 1 < C / B) {
#pragma unroll
      for (int l = 0; l < B; l += 2) {
        const double2 x = *reinterpret_cast<const double2*>(p + (b + 1) * B + l);
        v[(b + 1) & 1][l] = x.x;
        v[(b + 1) & 1][l + 1] = x.y;
      }
    }
#pragma unroll
    for (int l = 0; l < B; ++l) a = a + v[b & 1][l];
  }
  return a;
}

// MODE 0: registers only; 1: LDS, no barrier; 2: LDS + __syncthreads per chunk;
// 3: as 2 with waves 1-3 running 200 fp64 FMAs per chunk; 4: as 2, reads interleaved;
// 5: as 2 with waves 1-3 reading records and writing terms to LDS like the producers;
// 6: as 5 with the round-5 adder before the fix (three batches ahead, a per-lane count
// tested per batch); 7: as 6 without the count (the fix: full chunks add plainly)
template <int MODE>
__global__ void adder(const double* in, double* out, int chunks, long long* cyc) {
  __shared__ __attribute__((aligned(16))) double buf[2][12 * S];
  __shared__ __attribute__((aligned(16))) double rec[1024 * 4];  // MODE 5: producers' records
  for (int i = threadIdx.x; i < 2 * 12 * S; i += blockDim.x) (&buf[0][0])[i] = in[i & 1023] * 1e-3;
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) rec[i] = in[i & 1023];
  __syncthreads();
  const int tid = threadIdx.x;
  double a = 0.0, r = in[tid & 1023];
  double w[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) w[u] = in[(tid + u) & 1023];
  const long long t0 = clock64();
  for (int ch = 0; ch < chunks; ++ch) {
    if (tid < 12) {
      if (MODE == 0) {
#pragma unroll
        for (int l = 0; l < C; ++l) a = a + r;
      } else if (MODE == 4) {
        a = chain_interleaved(a, &buf[ch & 1][tid * S]);
      } else if (MODE == 7) {
        a = chain_fixed(a, &buf[ch & 1][tid * S]);
      } else if (MODE == 6) {
        a = chain_shipped(a, &buf[ch & 1][tid * S], chunks > 1 ? C - (ch == chunks - 1) : 1);
      } else {
        a = chain_prefetch(a, &buf[ch & 1][tid * S]);
      }
    } else if (MODE == 3 && tid >= 64) {
      for (int k = 0; k < 25; ++k)
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = __builtin_fma(w[u], r, 1e-3);
    } else if (MODE >= 5 && tid >= 64) {  // producer-like: 2 records in, 6 terms out, fp64 work
      const int p = tid - 64, pr = p / 48, pj = p % 48;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const double4 x = *reinterpret_cast<const double4*>(&rec[((ch * 96 + pj + 48 * u) & 1023) * 4]);
        double t = x.x + x.y + x.z + x.w;
        for (int k = 0; k < 12; ++k) t = __builtin_fma(t, r, 1e-3);
#pragma unroll
        for (int k = 0; k < 3; ++k) buf[(ch + 1) & 1][(pr * 3 + k) * S + pj + 48 * u] = t + k;
      }
    }
    if (MODE >= 2) __syncthreads();
  }
  const long long t1 = clock64();
  out[tid] = a + w[0] + w[7];
  if (tid == 0) *cyc = t1 - t0;
}

int main() {
  double *in, *out;
  long long* cyc;
  hipMalloc(&in, 1024 * 8);
  hipMalloc(&out, 1024 * 8);
  hipMalloc(&cyc, 8);
  double h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 1.0 + i * 1e-6;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const int chunks = 4096;
  long long c;
  const char* names[8] = {"registers", "LDS prefetched", "LDS + barrier", "LDS + barrier + 3 busy waves",
                          "LDS interleaved + barrier", "LDS + barrier + producer-like",
                          "shipped chain + producer-like", "fixed chain + producer-like"};
  for (int rep = 0; rep < 2; ++rep) {
    for (int m = 0; m < 8; ++m) {
      switch (m) {
        case 0: hipLaunchKernelGGL(adder<0>, dim3(1), dim3(256), 0, 0, in, out, chunks, cyc); break;
        case 1: hipLaunchKernelGGL(adder<1>, dim3(1), dim3(256), 0, 0, in, out, chunks, cyc); break;
        case 2: hipLaunchKernelGGL(adder<2>, dim3(1), dim3(256), 0, 0, in, out, chunks, cyc); break;
        case 3: hipLaunchKernelGGL(adder<3>, dim3(1), dim3(256), 0, 0, in, out, chunks, cyc); break;
        case 4: hipLaunchKernelGGL(adder<4>, dim3(1), dim3(256), 0, 0, in, out, chunks, cyc); break;
        case 5: hipLaunchKernelGGL(adder<5>, dim3(1), dim3(256), 0, 0, in, out, chunks, cyc); break;
        case 6: hipLaunchKernelGGL(adder<6>, dim3(1), dim3(256), 0, 0, in, out, chunks, cyc); break;
        case 7: hipLaunchKernelGGL(adder<7>, dim3(1), dim3(256), 0, 0, in, out, chunks, cyc); break;
      }
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      if (rep == 1) printf("%-30s %.0f cycles per chunk of %d adds (%.2f per add)\n", names[m],
                           (double)c / chunks, C, (double)c / chunks / C);
    }
  }
  return 0;
}
