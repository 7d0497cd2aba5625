// orbx_fastcore.cuh — FAST-9/16 pieces shared by the per-cell FAST kernel
// (orbx_fast.hip) and the fused front kernel (orbx_front.hip): OpenCV 3.x's
// cornerScore<16> and the 9-contiguous arc test on a 16-bit ring mask.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbx {

// popcount of the bits of m below this lane
__device__ __forceinline__ int mbcnt64(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// FAST-9/16 "cornerScore<16>" of OpenCV 3.x, d[k] = v - ring[k].
__device__ __forceinline__ int corner_score16(const int (&d)[16], int threshold) {
  auto D = [&](int k) { return d[k & 15]; };
  int a0 = threshold;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int a = min(D(k + 1), D(k + 2));
    a = min(a, D(k + 3));
    if (a <= a0) continue;
    a = min(a, D(k + 4));
    a = min(a, D(k + 5));
    a = min(a, D(k + 6));
    a = min(a, D(k + 7));
    a = min(a, D(k + 8));
    a0 = max(a0, min(a, D(k)));
    a0 = max(a0, min(a, D(k + 9)));
  }
  int b0 = -a0;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int b = max(D(k + 1), D(k + 2));
    b = max(b, D(k + 3));
    b = max(b, D(k + 4));
    b = max(b, D(k + 5));
    if (b >= b0) continue;
    b = max(b, D(k + 6));
    b = max(b, D(k + 7));
    b = max(b, D(k + 8));
    b0 = min(b0, max(b, D(k)));
    b0 = min(b0, max(b, D(k + 9)));
  }
  return -b0 - 1;
}

// 9 contiguous set bits in a circular 16-bit mask
__device__ __forceinline__ bool has_arc9(uint32_t m) {
  const uint32_t x = m | (m << 16);
  uint32_t a = x & (x >> 1);  // runs of 2
  a &= a >> 2;                // runs of 4
  a &= a >> 4;                // runs of 8
  a &= x >> 8;                // runs of 9
  return (a & 0xFFFFu) != 0;
}

}  // namespace orbx
