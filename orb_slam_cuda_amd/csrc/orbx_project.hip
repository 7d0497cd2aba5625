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
#include "orbx_projgrid.cuh"

namespace orbx {

constexpr int kProjThreads = 1024;
constexpr int kProjMaxMp = 8 * kProjThreads;  // map points per frame held in registers
constexpr int kProjTHigh = 100;               // ORBmatcher::TH_HIGH

size_t proj_lds_bytes(int kp_pitch) { return proj_grid_lds_bytes(kp_pitch); }

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
  const ProjGridLds g = proj_grid_carve(s_dyn, K);
  int* s_cell = g.cell;
  uint4* s_kd = g.kd;
  float4* s_kp = g.kp;
  int* s_kid = g.kid;
  int* s_mark = g.mark;  // by keypoint index: cell / min picker
  const orbx_kp* KP = kps + (size_t)f * K;
  const uint8_t* D = desc + (size_t)f * K * 32;
  const float* UR = P.has_uright ? uright + (size_t)f * K : nullptr;
  const uint8_t* BL = blocked + (size_t)f * K;

  // ---- stable grid sort (AssignFeaturesToGrid: cells hold indices ascending)
  proj_grid_sort<kProjThreads>(g, KP, D, UR, n, P.minX, P.minY, P.invW, P.invH, s_tmp);

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
    int cx0, cx1, cy0, cy1;
    if (!proj_window(x, y, rad, P.minX, P.minY, P.invW, P.invH, cx0, cx1, cy0, cy1)) return -1;
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
        const int d = hamming256(a, b, m0, m1);
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
  if (raise_lds_limit((const void*)search_proj_kernel, lds)) return ORBX_EDEVICE;
  hipLaunchKernelGGL(search_proj_kernel, dim3(frames), dim3(kProjThreads), lds, (hipStream_t)stream, P, kps, desc, n,
                     uright, blocked, mps, mpdesc, nmp, out, nmatches);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
