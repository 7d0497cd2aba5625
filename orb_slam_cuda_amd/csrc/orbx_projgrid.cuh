// orbx_projgrid.cuh — the LDS-resident keypoint grid of the projection
// searches (orbx_project.hip, orbx_project_pose.hip).
//
// Frame::AssignFeaturesToGrid / PosInGrid (src/Frame.cc:228-243, 381-391) and
// KeyFrame's copy of the same grid: 64 x 48 cells over the image bounds, each
// cell holding its keypoint indices in ascending order. Here the keypoints are
// sorted stably by cell (cell = ix * 48 + iy, the order GetFeaturesInArea
// visits, src/Frame.cc:350-376) and their positions, octave, uRight and
// descriptors copied to LDS in that order, so the cells ix*48 + cy0 ..
// ix*48 + cy1 of one grid column are one contiguous run of positions.
#pragma once
#include "orbx_device.cuh"
#include "orbx_wave.cuh"

namespace orbx {

constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS  include/Frame.h:37-38
constexpr int kGridCells = kGridCols * kGridRows;

// LDS carve-up shared by the projection kernels (dynamic shared memory):
//   s_cell [kGridCells + 1] cell offsets, s_kd [2K] descriptors by position,
//   s_kp [K] (x, y, octave bits, uRight), s_kid [K] keypoint index by position,
//   s_mark [K] per-keypoint scratch of the caller.
struct ProjGridLds {
  int* cell;
  uint4* kd;
  float4* kp;
  int* kid;
  int* mark;
};

__host__ __device__ inline size_t proj_grid_lds_bytes(int kp_pitch) {
  return (size_t)((kGridCells + 1 + 3) & ~3) * 4 + (size_t)kp_pitch * (32 + 16 + 4 + 4);
}

__device__ inline ProjGridLds proj_grid_carve(int* s_dyn, int K) {
  ProjGridLds g;
  g.cell = s_dyn;
  g.kd = (uint4*)(s_dyn + ((kGridCells + 1 + 3) & ~3));
  g.kp = (float4*)(g.kd + 2 * K);
  g.kid = (int*)(g.kp + K);
  g.mark = g.kid + K;
  return g;
}

// Stable grid sort of n keypoints (KP, D, UR may be null) into g. Leaves
// g.mark[i] = cell of keypoint i (-1 outside the grid). Ends with a barrier.
template <int NT>
__device__ void proj_grid_sort(const ProjGridLds& g, const orbx_kp* __restrict__ KP, const uint8_t* __restrict__ D,
                               const float* __restrict__ UR, int n, float minX, float minY, float invW, float invH,
                               int* s_tmp) {
  const int tid = threadIdx.x;
  for (int c = tid; c <= kGridCells; c += NT) g.cell[c] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += NT) {
    const float x = KP[i].x, y = KP[i].y;
    // PosInGrid: round((kp.x - mnMinX) * mfGridElementWidthInv)
    const int px = (int)roundf(__fmul_rn(__fsub_rn(x, minX), invW));
    const int py = (int)roundf(__fmul_rn(__fsub_rn(y, minY), invH));
    int c = -1;
    if (!(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows)) {
      c = px * kGridRows + py;
      __hip_atomic_fetch_add(&g.cell[c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    g.mark[i] = c;
  }
  __syncthreads();
  block_scan_excl<NT>(g.cell, kGridCells + 1, s_tmp);
  // rank within the cell = number of smaller indices in the same cell (cells
  // hold a handful of keypoints; the O(n) count only runs for shared cells)
  for (int i = tid; i < n; i += NT) {
    const int c = g.mark[i];
    if (c < 0) continue;
    int rank = 0;
    const int cnt = g.cell[c + 1] - g.cell[c];
    if (cnt > 1)
      for (int j = 0; j < i; ++j) rank += g.mark[j] == c;
    const int q = g.cell[c] + rank;
    const orbx_kp k = KP[i];
    g.kp[q] = make_float4(k.x, k.y, __int_as_float(k.octave), UR ? UR[i] : -1.f);
    g.kid[q] = i;
    g.kd[2 * q] = ((const uint4*)(D + (size_t)i * 32))[0];
    g.kd[2 * q + 1] = ((const uint4*)(D + (size_t)i * 32))[1];
  }
  __syncthreads();
}

// The window of GetFeaturesInArea (src/Frame.cc:330-346; KeyFrame.cc:583-597):
// false when it is empty.
__device__ inline bool proj_window(float x, float y, float r, float minX, float minY, float invW, float invH, int& cx0,
                                   int& cx1, int& cy0, int& cy1) {
  cx0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(x, minX), r), invW)));
  if (cx0 >= kGridCols) return false;
  cx1 = min(kGridCols - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(x, minX), r), invW)));
  if (cx1 < 0) return false;
  cy0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(y, minY), r), invH)));
  if (cy0 >= kGridRows) return false;
  cy1 = min(kGridRows - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(y, minY), r), invH)));
  if (cy1 < 0) return false;
  return true;
}

__device__ inline int hamming256(uint4 a, uint4 b, uint4 m0, uint4 m1) {
  return __popc(a.x ^ m0.x) + __popc(a.y ^ m0.y) + __popc(a.z ^ m0.z) + __popc(a.w ^ m0.w) + __popc(b.x ^ m1.x) +
         __popc(b.y ^ m1.y) + __popc(b.z ^ m1.z) + __popc(b.w ^ m1.w);
}

}  // namespace orbx
