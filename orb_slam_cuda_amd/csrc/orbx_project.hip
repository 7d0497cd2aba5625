// orbx_project.hip — ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th)
// on the GPU (the local-map search of Tracking::SearchLocalPoints,
// src/Tracking.cc:1277).
//
// Reference: src/ORBmatcher.cc:45-118 (+ RadiusByViewingCos :120-126,
// Frame::GetFeaturesInArea src/Frame.cc:326-379, the 64 x 48 grid of
// Frame::AssignFeaturesToGrid / PosInGrid :228-243, 381-391). Map points are
// visited in order; each takes the keypoint with the smallest Hamming distance
// among the unblocked candidates of its window (first one in grid order on
// ties), subject to TH_HIGH and, when best and second are on one level, the
// ratio test. A keypoint holding a map point with Observations() > 0 is
// blocked, and every assignment of a point with observations blocks the
// keypoint for the points after it: a sequential, order-dependent process.
//
// One 1024-thread workgroup per frame:
//   * stable grid sort of the keypoints (cell = ix * 48 + iy, the iteration
//     order of GetFeaturesInArea), positions, octave, uRight and descriptors
//     copied to LDS in that order;
//   * one map point per lane; the candidates of its window are walked in the
//     reference's order;
//   * the sequential blocking is resolved as a fixed point: in round t, point
//     j treats keypoint k as blocked iff it was blocked on entry or some point
//     i < j with observations picked k in round t-1 (an LDS atomic-min table).
//     The system is triangular, so its fixed point is unique and equals the
//     sequential result; rounds stop when no pick changes (a sequential pass
//     by one lane resolves it if P.max_rounds is reached).
#include "orbx_device.cuh"
#include "orbx_wave.cuh"

namespace orbx {

constexpr int kProjThreads = 1024;
constexpr int kProjMaxMp = 8 * kProjThreads;  // map points per frame held in registers
constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS  include/Frame.h:37-38
constexpr int kProjTHigh = 100;               // ORBmatcher::TH_HIGH

size_t proj_lds_bytes(int kp_pitch) {
  return (size_t)(kGridCols * kGridRows + 1) * 4 + (size_t)kp_pitch * (16 + 32 + 4 + 4) + 64;
}

__global__ __launch_bounds__(kProjThreads) void search_proj_kernel(ProjParams P, const orbx_kp* __restrict__ kps,
                                                                   const uint8_t* __restrict__ desc,
                                                                   const int* __restrict__ d_n,
                                                                   const float* __restrict__ uright,
                                                                   const uint8_t* __restrict__ blocked,
                                                                   const orbm_map_point_proj* __restrict__ mps,
                                                                   const uint8_t* __restrict__ mpdesc,
                                                                   const int* __restrict__ d_nmp,
                                                                   int* __restrict__ out, int* __restrict__ nmatches) {
  extern __shared__ __attribute__((aligned(16))) int s_dyn[];
  __shared__ int s_tmp[kProjThreads / 64];
  __shared__ int s_flag;
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int K = P.kp_pitch, n = d_n[f], nmp = min(d_nmp[f], kProjMaxMp);
  constexpr int NC = kGridCols * kGridRows;
  int* s_cell = s_dyn;                                      // [NC + 1]
  uint4* s_kd = (uint4*)(s_cell + ((NC + 1 + 3) & ~3));     // [2K] descriptors by position
  float4* s_kp = (float4*)(s_kd + 2 * K);                   // [K] x, y, octave (bits), uRight
  int* s_kid = (int*)(s_kp + K);                            // [K] keypoint index by position
  int* s_mark = s_kid + K;                                  // [K] by keypoint index: cell / min picker
  const orbx_kp* KP = kps + (size_t)f * K;
  const uint8_t* D = desc + (size_t)f * K * 32;
  const float* UR = P.has_uright ? uright + (size_t)f * K : nullptr;
  const uint8_t* BL = blocked + (size_t)f * K;

  // ---- stable grid sort (AssignFeaturesToGrid: cells hold indices ascending)
  for (int c = tid; c <= NC; c += kProjThreads) s_cell[c] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += kProjThreads) {
    const float x = KP[i].x, y = KP[i].y;
    const int px = (int)roundf((x - P.minX) * P.invW), py = (int)roundf((y - P.minY) * P.invH);
    int c = -1;
    if (!(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows)) {
      c = px * kGridRows + py;
      __hip_atomic_fetch_add(&s_cell[c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    s_mark[i] = c;
  }
  __syncthreads();
  block_scan_excl<kProjThreads>(s_cell, NC + 1, s_tmp);
  // each cell's keypoints in ascending index: rank within the cell by a count of
  // smaller indices in the same cell (cells hold a handful of keypoints)
  for (int i = tid; i < n; i += kProjThreads) {
    const int c = s_mark[i];
    if (c < 0) continue;
    int rank = 0;
    const int cnt = s_cell[c + 1] - s_cell[c];
    if (cnt > 1)
      for (int j = 0; j < i; ++j) rank += s_mark[j] == c;  // O(n) only for shared cells
    const int q = s_cell[c] + rank;
    const orbx_kp k = KP[i];
    s_kp[q] = make_float4(k.x, k.y, __int_as_float(k.octave), UR ? UR[i] : -1.f);
    s_kid[q] = i;
    s_kd[2 * q] = ((const uint4*)(D + (size_t)i * 32))[0];
    s_kd[2 * q + 1] = ((const uint4*)(D + (size_t)i * 32))[1];
  }
  __syncthreads();

  long long* prof = P.prof ? P.prof + (size_t)f * 64 : nullptr;  // diagnostics (ORBX_PROJ_PROF)
  if (prof && tid == 0) prof[0] = (long long)__builtin_readcyclecounter();
  // ---- this lane's map points (j = tid + kProjThreads * r)
  constexpr int R = kProjMaxMp / kProjThreads;
  int pick[R];
#pragma unroll
  for (int r = 0; r < R; ++r) pick[r] = -2;  // -2: not computed, -1: no match
  const bool bFactor = P.th != 1.0f;
  const orbm_map_point_proj* MP = mps + (size_t)f * P.mp_pitch;
  const uint8_t* MD = mpdesc + (size_t)f * P.mp_pitch * 32;

  // one map point against the keypoints, given the blocking table
  auto search = [&](int j) -> int {
    const orbm_map_point_proj mp = MP[j];
    if (!mp.track_in_view) return -1;
    const int lvl = mp.predicted_level;
    float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos
    if (bFactor) r = r * P.th;
    const float rad = r * P.scale[min(max(lvl, 0), kMaxLevels - 1)];
    const float x = mp.proj_x, y = mp.proj_y;
    const int cx0 = max(0, (int)floorf((x - P.minX - rad) * P.invW));
    if (cx0 >= kGridCols) return -1;
    const int cx1 = min(kGridCols - 1, (int)ceilf((x - P.minX + rad) * P.invW));
    if (cx1 < 0) return -1;
    const int cy0 = max(0, (int)floorf((y - P.minY - rad) * P.invH));
    if (cy0 >= kGridRows) return -1;
    const int cy1 = min(kGridRows - 1, (int)ceilf((y - P.minY + rad) * P.invH));
    if (cy1 < 0) return -1;
    const int minLevel = lvl - 1, maxLevel = lvl;
    const bool check = (minLevel > 0) || (maxLevel >= 0);
    const uint4* md = (const uint4*)(MD + (size_t)j * 32);
    const uint4 m0 = md[0], m1 = md[1];
    int best = 256, lv = -1, best2 = 256, lv2 = -1, bidx = -1;
    // cells ix*48 + cy0 .. ix*48 + cy1 of one grid column are adjacent in the
    // sorted order: one flat run of positions per column (same visiting order)
    for (int ix = cx0; ix <= cx1; ++ix) {
      const int qe = s_cell[ix * kGridRows + cy1 + 1];
      for (int q = s_cell[ix * kGridRows + cy0]; q < qe; ++q) {
        const float4 k = s_kp[q];
        const int o = __float_as_int(k.z);
        if (check && (o < minLevel || (maxLevel >= 0 && o > maxLevel))) continue;
        if (!(fabsf(k.x - x) < rad && fabsf(k.y - y) < rad)) continue;
        const int idx = s_kid[q];
        // F.mvpMapPoints[idx]->Observations() > 0: on entry (mark -1) or taken by an earlier point
        if (s_mark[idx] < j) continue;
        if (k.w > 0) {
          const float er = fabsf(mp.proj_xr - k.w);
          if (er > rad) continue;
        }
        const uint4 a = s_kd[2 * q], b = s_kd[2 * q + 1];
        const int d = __popc(a.x ^ m0.x) + __popc(a.y ^ m0.y) + __popc(a.z ^ m0.z) + __popc(a.w ^ m0.w) +
                      __popc(b.x ^ m1.x) + __popc(b.y ^ m1.y) + __popc(b.z ^ m1.z) + __popc(b.w ^ m1.w);
        if (d < best) {
          best2 = best;
          best = d;
          lv2 = lv;
          lv = o;
          bidx = idx;
        } else if (d < best2) {
          lv2 = o;
          best2 = d;
        }
      }
    }
    if (best <= kProjTHigh) {
      if (lv == lv2 && (float)best > P.nnratio * (float)best2) return -1;
      return bidx;
    }
    return -1;
  };

  // ---- fixed-point rounds over the blocking table (s_mark: min picker with observations)
  bool converged = false;
  for (int round = 0; round < P.max_rounds; ++round) {
    for (int i = tid; i < n; i += kProjThreads) s_mark[i] = BL[i] ? -1 : INT_MAX;
    if (tid == 0) s_flag = 0;
    __syncthreads();
    if (round > 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int j = tid + kProjThreads * r;
        if (j < nmp && pick[r] >= 0 && MP[j].obs_positive)
          __hip_atomic_fetch_min(&s_mark[pick[r]], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __syncthreads();
    }
    int changed = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = tid + kProjThreads * r;
      if (j < nmp) {
        const int np = search(j);
        changed |= np != pick[r];
        pick[r] = np;
      }
    }
    if (changed) s_flag = 1;
    __syncthreads();
    const int any = s_flag;
    __syncthreads();
    if (prof && tid == 0) prof[1 + min(round, 40)] = (long long)__builtin_readcyclecounter();
    if (!any) {
      converged = true;
      break;
    }
  }
  if (!converged) {
    // sequential resolution (a safety net; keeps the result exact): one lane
    // visits the points in order and records, per keypoint, the first point
    // with observations that takes it; with that table every point's search
    // sees exactly the keypoints blocked before it
    if (tid == 0) {
      for (int i = 0; i < n; ++i) s_mark[i] = BL[i] ? -1 : INT_MAX;
      for (int j = 0; j < nmp; ++j) {
        const int pk = search(j);
        if (pk >= 0 && MP[j].obs_positive && s_mark[pk] == INT_MAX) s_mark[pk] = j;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = tid + kProjThreads * r;
      if (j < nmp) pick[r] = search(j);
    }
    __syncthreads();
  }

  // ---- outputs: per keypoint the last point that wrote it, and the count
  for (int i = tid; i < n; i += kProjThreads) s_mark[i] = -1;
  if (tid == 0) s_flag = 0;
  __syncthreads();
  int cnt = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = tid + kProjThreads * r;
    if (j < nmp && pick[r] >= 0) {
      ++cnt;
      __hip_atomic_fetch_max(&s_mark[pick[r]], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  cnt = wave_sum_dpp(cnt);
  if (lane == 0 && cnt) __hip_atomic_fetch_add(&s_flag, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  for (int i = tid; i < n; i += kProjThreads) out[(size_t)f * K + i] = s_mark[i];
  if (tid == 0) nmatches[f] = s_flag;
}

int launch_search_proj(const ProjParams& P, const orbx_kp* kps, const uint8_t* desc, const int* n,
                       const float* uright, const uint8_t* blocked, const orbm_map_point_proj* mps,
                       const uint8_t* mpdesc, const int* nmp, int frames, int* out, int* nmatches, void* stream) {
  const size_t lds = proj_lds_bytes(P.kp_pitch);
  static size_t attr = 0;
  if (lds > attr) {
    if (hipFuncSetAttribute((const void*)search_proj_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return ORBX_EDEVICE;
    attr = lds;
  }
  hipLaunchKernelGGL(search_proj_kernel, dim3(frames), dim3(kProjThreads), lds, (hipStream_t)stream, P, kps, desc, n,
                     uright, blocked, mps, mpdesc, nmp, out, nmatches);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
