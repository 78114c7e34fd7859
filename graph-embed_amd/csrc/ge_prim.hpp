// ge_prim.hpp -- device-wide scans and radix sorts through rocPRIM (the AMD
// primitives library, called directly; no CUB-shaped compatibility layer).
//
// Each call sizes its temporary storage, allocates it in a DevBuf (whose hipFree
// waits for the device) and runs on `st`.  rocPRIM's radix sorts are stable
// (LSD), which the P^T A P composite-key sort and the R-MAT symmetrisation rely on.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "ge_internal.hpp"

namespace ge {

// out[i] = in[0] + ... + in[i - 1], out[0] = 0
template <class T, class U>
void prim_exclusive_sum(hipStream_t st, const T* in, U* out, size_t count) {
  size_t tmp = 0;
  GE_HIP(rocprim::exclusive_scan(nullptr, tmp, in, out, U(0), count, rocprim::plus<U>(), st));
  DevBuf<unsigned char> scratch(std::max<size_t>(tmp, 1));
  GE_HIP(rocprim::exclusive_scan(scratch.p, tmp, in, out, U(0), count, rocprim::plus<U>(), st));
}

// out[i] = in[0] + ... + in[i]
template <class T>
void prim_inclusive_sum(hipStream_t st, const T* in, T* out, size_t count) {
  size_t tmp = 0;
  GE_HIP(rocprim::inclusive_scan(nullptr, tmp, in, out, count, rocprim::plus<T>(), st));
  DevBuf<unsigned char> scratch(std::max<size_t>(tmp, 1));
  GE_HIP(rocprim::inclusive_scan(scratch.p, tmp, in, out, count, rocprim::plus<T>(), st));
}

// Temporary bytes of one key sort of `count` keys (callers that sort many chunks
// allocate once for the largest).
template <class K>
size_t prim_sort_keys_bytes(hipStream_t st, const K* in, K* out, size_t count, int end_bit) {
  size_t tmp = 0;
  GE_HIP(rocprim::radix_sort_keys(nullptr, tmp, in, out, count, 0, end_bit, st));
  return std::max<size_t>(tmp, 1);
}

template <class K>
void prim_sort_keys(hipStream_t st, void* scratch, size_t bytes, const K* in, K* out,
                    size_t count, int end_bit) {
  GE_HIP(rocprim::radix_sort_keys(scratch, bytes, in, out, count, 0, end_bit, st));
}

// Stable sort of (key, value) pairs by the low end_bit bits of the key.
template <class K, class V>
void prim_sort_pairs(hipStream_t st, const K* kin, K* kout, const V* vin, V* vout, size_t count,
                     int end_bit) {
  size_t tmp = 0;
  GE_HIP(rocprim::radix_sort_pairs(nullptr, tmp, kin, kout, vin, vout, count, 0, end_bit, st));
  DevBuf<unsigned char> scratch(std::max<size_t>(tmp, 1));
  GE_HIP(rocprim::radix_sort_pairs(scratch.p, tmp, kin, kout, vin, vout, count, 0, end_bit, st));
}

}  // namespace ge
