// orbx_fastcore.cuh — FAST-9/16 pieces of the per-cell FAST kernel
// (orbx_fast.hip): the ordered-compaction lane count and OpenCV 3.x's
// cornerScore<16> for two pixels in packed i16x2 arithmetic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orbx_wave.cuh"

namespace orbx {


// FAST-9/16 "cornerScore<16>" of OpenCV 3.x (d[k] = v - ring[k]) for two pixels at once,
// packed i16x2 (one pixel per half).
// Branch-free restatement: cornerScore<16>'s early `continue`s skip only
// updates that cannot change a0 / b0 (the partial arc minimum already bounds
// the full one), so
//   a0 = max(t, max over the 16 arcs of 9 of min(d)),
//   b0 = min(-a0, min over the 16 arcs of 9 of max(d)),  score = -b0 - 1
//      = max(t, max over arcs of min(d), -(min over arcs of max(d))) - 1.
// Computed from the ring pixels p[k] themselves (u16x2, one pixel per half)
// and the centre v: min over an arc of (v - p) = v - max over the arc of p
// (exact in integers), so with A = min over arcs of (max of p) and
// B = max over arcs of (min of p), score = max(t, v - A, B - v) - 1. A pixel
// is FAST-detected at t iff its score is >= t; the max with t only lifts
// pixels that are not detected, so it is dropped: the value returned equals
// cornerScore<16> for every detected pixel and is < t for the others.
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ i16x2 corner_score16_x2_ring(const u16x2_t (&P)[16], u16x2_t v) {
  u16x2_t hi[8], lo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // runs of 2 from odd start s = 2j + 1
    hi[j] = __builtin_elementwise_max(P[2 * j + 1], P[(2 * j + 2) & 15]);
    lo[j] = __builtin_elementwise_min(P[2 * j + 1], P[(2 * j + 2) & 15]);
  }
  u16x2_t hi4[8], lo4[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // runs of 4
    hi4[j] = __builtin_elementwise_max(hi[j], hi[(j + 1) & 7]);
    lo4[j] = __builtin_elementwise_min(lo[j], lo[(j + 1) & 7]);
  }
  // runs of 8 from s = 2j + 1, extended to the two 9-arcs from s - 1 and s:
  // min(max(r, p[s-1]), max(r, p[s+8])) = max(r, min(p[s-1], p[s+8])), so a
  // pair of arcs costs two ops and 8 pair extrema meet in the trees
  u16x2_t ta[8], tb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const u16x2_t a = __builtin_elementwise_max(hi4[j], hi4[(j + 2) & 7]);
    const u16x2_t b = __builtin_elementwise_min(lo4[j], lo4[(j + 2) & 7]);
    const u16x2_t e0 = P[2 * j], e1 = P[(2 * j + 9) & 15];
    ta[j] = __builtin_elementwise_max(a, __builtin_elementwise_min(e0, e1));
    tb[j] = __builtin_elementwise_min(b, __builtin_elementwise_max(e0, e1));
  }
#pragma unroll
  for (int w = 4; w >= 1; w >>= 1)
#pragma unroll
    for (int j = 0; j < w; ++j) {
      ta[j] = __builtin_elementwise_min(ta[j], ta[j + w]);
      tb[j] = __builtin_elementwise_max(tb[j], tb[j + w]);
    }
  const u16x2_t A = ta[0], B = tb[0];
  const i16x2 vs = __builtin_bit_cast(i16x2, v);
  const i16x2 one = {1, 1};
  return __builtin_elementwise_max(vs - __builtin_bit_cast(i16x2, A), __builtin_bit_cast(i16x2, B) - vs) - one;
}

}  // namespace orbx
