// orbx_project_pose.hip — the ORBmatcher::SearchByProjection overloads that
// project MapPoint world positions with a pose, on the GPU:
//   LAST_FRAME  SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame,
//               th, bMono)  src/ORBmatcher.cc:1328-1470 (every tracked frame,
//               Tracking::TrackWithMotionModel src/Tracking.cc:962)
//   KEYFRAME    SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th,
//               ORBdist)  src/ORBmatcher.cc:1472-1599 (Tracking::Relocalization)
//   SIM3        SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)
//               src/ORBmatcher.cc:290-403 (LoopClosing::ComputeSim3)
//   FUSE        Fuse(KeyFrame*, vpMapPoints, th), matching part  :825-930
//               (LocalMapping::SearchInNeighbors)
//   FUSE_SIM3   Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint), matching
//               part  :977-1081 (LoopClosing::SearchAndFuse)
//   SIM3_MATCH  SearchBySim3, one direction  :1102-1292 (LoopClosing::ComputeSim3)
//
// Per point (in order): project with the pose (R*x + t as OpenCV's 3x3 gemm
// small-matrix path: float dot, then a double add of t), the image / depth /
// distance / viewing-angle tests of the overload, PredictScale (level from
// precomputed logf thresholds, see orbm_predict_scale_thresholds), the grid
// window of GetFeaturesInArea with the overload's level band, then the
// nearest unblocked descriptor (first one in grid order on ties) under the
// distance threshold. Assignments block keypoints for the points after them
// (LAST_FRAME: points with observations; KEYFRAME, SIM3: every point), so the
// result is order-dependent; as in orbx_project.hip it is resolved as the
// unique fixed point of the triangular blocking system (rounds over an LDS
// atomic-min table, a one-lane sequential pass past max_rounds). LAST_FRAME
// and KEYFRAME then apply the rotation-consistency check (three largest
// histogram bins, ComputeThreeMaxima src/ORBmatcher.cc:1601-1642).
//
// One 1024-thread workgroup per frame; the keypoint grid lives in LDS
// (orbx_projgrid.cuh); picks are kept per point in a global scratch array so
// the number of points per frame is not bounded by registers.
#include "orbx_projgrid.cuh"

namespace orbx {

constexpr int kPoseThreads = 1024;
constexpr int kHisto = 30;  // ORBmatcher::HISTO_LENGTH

size_t pose_lds_bytes(int kp_pitch) { return proj_grid_lds_bytes(kp_pitch); }

// R*x + t, row r of the 3x4 T: gemm's small-matrix path (float dot products,
// then (float)(t*1.0 + c*1.0) in double)
__device__ inline float pose_row(const float* T, int r, float x, float y, float z) {
  const float t = __fadd_rn(__fadd_rn(__fmul_rn(T[4 * r], x), __fmul_rn(T[4 * r + 1], y)), __fmul_rn(T[4 * r + 2], z));
  return __double2float_rn(__dadd_rn((double)t, (double)T[4 * r + 3]));
}

// cv::norm (NORM_L2) of 3 floats: sqrt of the double sum of squares
__device__ inline float norm3(float a, float b, float c) {
  const double s = __dadd_rn(__dadd_rn(__dmul_rn((double)a, (double)a), __dmul_rn((double)b, (double)b)),
                             __dmul_rn((double)c, (double)c));
  return __double2float_rn(__dsqrt_rn(s));
}

// MapPoint::PredictScale (src/MapPoint.cc:390-422) from the host's thresholds
__device__ inline int predict_level(const PoseParams& P, float maxd, float dist) {
  const float ratio = __fdiv_rn(maxd, dist);
  if (__builtin_isinf(ratio)) return 0;  // ceil(log(inf)) -> int: INT_MIN on x86, clamped to 0
  int l = 0;
#pragma unroll
  for (int k = 0; k < kMaxLevels - 1; ++k) l += (k < P.L - 1 && ratio >= P.pred_thr[k]) ? 1 : 0;
  return l;
}

struct PoseQuery {
  float u, v, rad, ur;  // window centre and radius; ur: right-image coordinate (LAST_FRAME stereo)
  int minL, maxL;       // level band (GetFeaturesInArea semantics: check if minL > 0 || maxL >= 0)
  bool ok;
};

// modes whose output is per point (no blocking, no per-keypoint epilogue)
__host__ __device__ constexpr bool per_point(int mode) {
  return mode == ORBM_PROJ_FUSE || mode == ORBM_PROJ_FUSE_SIM3 || mode == ORBM_PROJ_SIM3_MATCH;
}

template <int MODE>
__device__ inline PoseQuery pose_query(const PoseParams& P, const orbm_pose& C, const orbm_map_point_world& mp) {
  PoseQuery q;
  q.ok = false;
  if (!mp.valid) return q;
  const float X = mp.pos[0], Y = mp.pos[1], Z = mp.pos[2];
  float xc = pose_row(C.Rt, 0, X, Y, Z), yc = pose_row(C.Rt, 1, X, Y, Z), zc = pose_row(C.Rt, 2, X, Y, Z);
  if (MODE == ORBM_PROJ_SIM3_MATCH) {  // p3Dc2 = sR21*p3Dc1 + t21 (:1156-1157)
    const float a = xc, b = yc, c = zc;
    xc = pose_row(C.Rt2, 0, a, b, c);
    yc = pose_row(C.Rt2, 1, a, b, c);
    zc = pose_row(C.Rt2, 2, a, b, c);
  }
  float invz;
  if (MODE == ORBM_PROJ_SIM3 || MODE == ORBM_PROJ_FUSE || MODE == ORBM_PROJ_FUSE_SIM3 ||
      MODE == ORBM_PROJ_SIM3_MATCH) {
    if (zc < 0.0f) return q;
    // float 1/z (:321, :854) or double 1.0/z (:1014, :1164)
    invz = (MODE == ORBM_PROJ_SIM3 || MODE == ORBM_PROJ_FUSE) ? __fdiv_rn(1.0f, zc)
                                                                : __double2float_rn(__ddiv_rn(1.0, (double)zc));
    q.u = __fadd_rn(__fmul_rn(C.fx, __fmul_rn(xc, invz)), C.cx);
    q.v = __fadd_rn(__fmul_rn(C.fy, __fmul_rn(yc, invz)), C.cy);
    // KeyFrame::IsInImage (src/KeyFrame.cc:619-622)
    if (!(q.u >= P.minX && q.u < P.maxX && q.v >= P.minY && q.v < P.maxY)) return q;
    q.ur = __fsub_rn(q.u, __fmul_rn(C.mbf, invz));  // Fuse: ur = u - bf*invz
  } else {
    invz = __double2float_rn(__ddiv_rn(1.0, (double)zc));
    if (MODE == ORBM_PROJ_LAST_FRAME && invz < 0.0f) return q;
    q.u = __fadd_rn(__fmul_rn(__fmul_rn(C.fx, xc), invz), C.cx);
    q.v = __fadd_rn(__fmul_rn(__fmul_rn(C.fy, yc), invz), C.cy);
    if (q.u < P.minX || q.u > P.maxX) return q;
    if (q.v < P.minY || q.v > P.maxY) return q;
    q.ur = __fsub_rn(q.u, __fmul_rn(C.mbf, invz));
  }
  if (MODE == ORBM_PROJ_LAST_FRAME) {
    const int lo = min(max((int)mp.octave, 0), kMaxLevels - 1);
    q.rad = __fmul_rn(P.th, P.scale[lo]);
    if (C.level_mode == 1) {  // bForward
      q.minL = lo;
      q.maxL = -1;
    } else if (C.level_mode == 2) {  // bBackward
      q.minL = 0;
      q.maxL = lo;
    } else {
      q.minL = lo - 1;
      q.maxL = lo + 1;
    }
  } else {
    float dist, PO0, PO1, PO2;
    if (MODE == ORBM_PROJ_SIM3_MATCH) {  // cv::norm(p3Dc2): camera coordinates
      dist = norm3(xc, yc, zc);
      PO0 = PO1 = PO2 = 0.0f;
    } else {  // PO = p3Dw - Ow
      PO0 = __fsub_rn(X, C.Ow[0]);
      PO1 = __fsub_rn(Y, C.Ow[1]);
      PO2 = __fsub_rn(Z, C.Ow[2]);
      dist = norm3(PO0, PO1, PO2);
    }
    const float maxDistance = __fmul_rn(1.2f, mp.max_distance);  // GetMaxDistanceInvariance
    const float minDistance = __fmul_rn(0.8f, mp.min_distance);  // GetMinDistanceInvariance
    if (dist < minDistance || dist > maxDistance) return q;
    if (MODE == ORBM_PROJ_SIM3 || MODE == ORBM_PROJ_FUSE || MODE == ORBM_PROJ_FUSE_SIM3) {
      // PO.dot(Pn) < 0.5*dist: viewing angle over 60 degrees (double dot product)
      const double dot = __dadd_rn(__dadd_rn(__dmul_rn((double)PO0, (double)mp.normal[0]),
                                             __dmul_rn((double)PO1, (double)mp.normal[1])),
                                   __dmul_rn((double)PO2, (double)mp.normal[2]));
      if (dot < 0.5 * (double)dist) return q;
    }
    const int lvl = predict_level(P, mp.max_distance, dist);
    q.rad = __fmul_rn(P.th, P.scale[lvl]);
    if (MODE == ORBM_PROJ_KEYFRAME) {
      q.minL = lvl - 1;
      q.maxL = lvl + 1;
    } else {  // KeyFrame::GetFeaturesInArea has no level band; the matchers keep lvl-1..lvl
      q.minL = lvl - 1;
      q.maxL = lvl;
    }
  }
  q.ok = true;
  return q;
}

template <int MODE>
__global__ __launch_bounds__(kPoseThreads) void search_pose_kernel(
    PoseParams P, const orbx_kp* __restrict__ kps, const uint8_t* __restrict__ desc, const int* __restrict__ d_n,
    const float* __restrict__ uright, const uint8_t* __restrict__ blocked, const orbm_pose* __restrict__ poses,
    const orbm_map_point_world* __restrict__ mps, const uint8_t* __restrict__ mpdesc, const int* __restrict__ d_nmp,
    int* __restrict__ picks, int* __restrict__ out, int* __restrict__ nmatches) {
  extern __shared__ __attribute__((aligned(16))) int s_dyn[];
  __shared__ int s_tmp[kPoseThreads / 64];
  __shared__ int s_flag, s_cnt, s_rej;
  __shared__ int s_hist[kHisto], s_ind[3];
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int K = P.kp_pitch, n = d_n[f], nmp = d_nmp[f];
  const ProjGridLds g = proj_grid_carve(s_dyn, K);
  const orbx_kp* KP = kps + (size_t)f * K;
  const uint8_t* D = desc + (size_t)f * K * 32;
  const float* UR = P.has_uright ? uright + (size_t)f * K : nullptr;
  const uint8_t* BL = blocked + (size_t)f * K;
  const orbm_map_point_world* MP = mps + (size_t)f * P.mp_pitch;
  const uint8_t* MD = mpdesc + (size_t)f * P.mp_pitch * 32;
  int* PK = picks + (size_t)f * P.mp_pitch;
  const orbm_pose C = poses[f];

  proj_grid_sort<kPoseThreads>(g, KP, D, UR, n, P.minX, P.minY, P.invW, P.invH, s_tmp);
  const bool stereo = MODE == ORBM_PROJ_LAST_FRAME && UR != nullptr;
  const bool has_ur = UR != nullptr;

  // point j against the keypoints, given the blocking table g.mark
  auto search = [&](int j) -> int {
    const orbm_map_point_world mp = MP[j];
    const PoseQuery q = pose_query<MODE>(P, C, mp);
    if (!q.ok) return -1;
    int cx0, cx1, cy0, cy1;
    if (!proj_window(q.u, q.v, q.rad, P.minX, P.minY, P.invW, P.invH, cx0, cx1, cy0, cy1)) return -1;
    const bool check = (q.minL > 0) || (q.maxL >= 0);
    const uint4* md = (const uint4*)(MD + (size_t)j * 32);
    const uint4 m0 = md[0], m1 = md[1];
    int best = 256, bidx = -1;
    for (int ix = cx0; ix <= cx1; ++ix) {
      const int qe = g.cell[ix * kGridRows + cy1 + 1];
      for (int p = g.cell[ix * kGridRows + cy0]; p < qe; ++p) {
        const float4 k = g.kp[p];
        const int o = __float_as_int(k.z);
        if (check && (o < q.minL || (q.maxL >= 0 && o > q.maxL))) continue;
        if (!(fabsf(__fsub_rn(k.x, q.u)) < q.rad && fabsf(__fsub_rn(k.y, q.v)) < q.rad)) continue;
        const int idx = g.kid[p];
        if (g.mark[idx] < j) continue;  // blocked on entry (-1) or taken by an earlier blocking point
        if (stereo && k.w > 0) {
          const float er = fabsf(__fsub_rn(q.ur, k.w));
          if (er > q.rad) continue;
        }
        if (MODE == ORBM_PROJ_FUSE) {  // reprojection error (src/ORBmatcher.cc:900-925)
          const float ex = __fsub_rn(q.u, k.x), ey = __fsub_rn(q.v, k.y);
          float e2 = __fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey));
          const bool st = has_ur && k.w >= 0.0f;
          if (st) {
            const float er = __fsub_rn(q.ur, k.w);
            e2 = __fadd_rn(e2, __fmul_rn(er, er));
          }
          if ((double)__fmul_rn(e2, P.inv_sigma2[min(max(o, 0), kMaxLevels - 1)]) > (st ? 7.8 : 5.99)) continue;
        }
        const int d = hamming256(g.kd[2 * p], g.kd[2 * p + 1], m0, m1);
        if (d < best) {
          best = d;
          bidx = idx;
        }
      }
    }
    return best <= P.dist_th ? bidx : -1;
  };
  auto blocks = [&](int j) -> bool { return MODE != ORBM_PROJ_LAST_FRAME || MP[j].obs_positive; };
  constexpr bool kPerPoint = per_point(MODE);

  // ---- fixed-point rounds (g.mark[k] = least blocking point that picked k last round)
  bool converged = false;
  for (int round = 0; round < P.max_rounds; ++round) {
    for (int i = tid; i < n; i += kPoseThreads) g.mark[i] = BL[i] ? -1 : INT_MAX;
    if (tid == 0) s_flag = 0;
    __syncthreads();
    if (round > 0) {
      for (int j = tid; j < nmp; j += kPoseThreads) {
        const int pk = PK[j];
        if (pk >= 0 && blocks(j))
          __hip_atomic_fetch_min(&g.mark[pk], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __syncthreads();
    }
    int changed = 0;
    for (int j = tid; j < nmp; j += kPoseThreads) {
      const int np = search(j);
      changed |= (round == 0) || np != PK[j];
      PK[j] = np;
    }
    if (changed) s_flag = 1;
    __syncthreads();
    const int any = s_flag;
    __syncthreads();
    if (!any || kPerPoint) {  // per-point modes: no blocking, one round is the result
      converged = true;
      break;
    }
  }
  if (!converged) {
    // one lane visits the points in order, recording per keypoint the first
    // blocking point that takes it; then every point searches once more
    if (tid == 0) {
      for (int i = 0; i < n; ++i) g.mark[i] = BL[i] ? -1 : INT_MAX;
      for (int j = 0; j < nmp; ++j) {
        const int pk = search(j);
        if (pk >= 0 && blocks(j) && g.mark[pk] == INT_MAX) g.mark[pk] = j;
      }
    }
    __syncthreads();
    for (int j = tid; j < nmp; j += kPoseThreads) PK[j] = search(j);
    __syncthreads();
  }

  if (kPerPoint) {  // ---- outputs: per point, the keypoint it matched
    int* O = out + (size_t)f * P.mp_pitch;
    int cnt = 0;
    for (int j = tid; j < nmp; j += kPoseThreads) {
      const int pk = PK[j];
      O[j] = pk;
      cnt += pk >= 0;
    }
    cnt = wave_sum_dpp(cnt);
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    if (lane == 0 && cnt) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (tid == 0) nmatches[f] = s_cnt;
    return;
  }
  // ---- outputs: per keypoint the last point that stored itself there
  for (int i = tid; i < n; i += kPoseThreads) {
    g.mark[i] = -1;
    g.kid[i] = 0;  // reused: cleared by the rotation check
  }
  if (tid < kHisto) s_hist[tid] = 0;
  if (tid == 0) {
    s_cnt = 0;
    s_rej = 0;
  }
  __syncthreads();
  const bool rot = MODE != ORBM_PROJ_SIM3 && P.check_ori;
  const float factor = 1.0f / kHisto;
  int cnt = 0;
  for (int j = tid; j < nmp; j += kPoseThreads) {
    const int pk = PK[j];
    if (pk < 0) continue;
    ++cnt;
    __hip_atomic_fetch_max(&g.mark[pk], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (rot) {
      float r = __fsub_rn(MP[j].angle, KP[pk].angle);
      if (r < 0.0f) r = __fadd_rn(r, 360.0f);
      int bin = (int)roundf(__fmul_rn(r, factor));
      if (bin == kHisto) bin = 0;
      atomicAdd(&s_hist[bin], 1);
    }
  }
  cnt = wave_sum_dpp(cnt);
  if (lane == 0 && cnt) atomicAdd(&s_cnt, cnt);
  __syncthreads();
  if (rot) {
    if (tid == 0) {  // ComputeThreeMaxima (src/ORBmatcher.cc:1601-1642)
      int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
      for (int i = 0; i < kHisto; i++) {
        const int s = s_hist[i];
        if (s > max1) {
          max3 = max2; max2 = max1; max1 = s;
          ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
          max3 = max2; max2 = s;
          ind3 = ind2; ind2 = i;
        } else if (s > max3) {
          max3 = s;
          ind3 = i;
        }
      }
      if (max2 < __fmul_rn(0.1f, (float)max1)) {
        ind2 = -1;
        ind3 = -1;
      } else if (max3 < __fmul_rn(0.1f, (float)max1)) {
        ind3 = -1;
      }
      s_ind[0] = ind1;
      s_ind[1] = ind2;
      s_ind[2] = ind3;
    }
    __syncthreads();
    const int i1 = s_ind[0], i2 = s_ind[1], i3 = s_ind[2];
    int rej = 0;
    for (int j = tid; j < nmp; j += kPoseThreads) {
      const int pk = PK[j];
      if (pk < 0) continue;
      float r = __fsub_rn(MP[j].angle, KP[pk].angle);
      if (r < 0.0f) r = __fadd_rn(r, 360.0f);
      int bin = (int)roundf(__fmul_rn(r, factor));
      if (bin == kHisto) bin = 0;
      if (bin == i1 || bin == i2 || bin == i3) continue;
      ++rej;
      g.kid[pk] = 1;  // mvpMapPoints[rotHist[i][j]] = NULL
    }
    rej = wave_sum_dpp(rej);
    if (lane == 0 && rej) atomicAdd(&s_rej, rej);
    __syncthreads();
  }
  int* O = out + (size_t)f * K;
  for (int i = tid; i < n; i += kPoseThreads) O[i] = g.kid[i] ? -2 : g.mark[i];
  if (tid == 0) nmatches[f] = s_cnt - s_rej;
}

int launch_search_pose(const PoseParams& P, const orbx_kp* kps, const uint8_t* desc, const int* n,
                       const float* uright, const uint8_t* blocked, const orbm_pose* poses,
                       const orbm_map_point_world* mps, const uint8_t* mpdesc, const int* nmp, int frames, int* picks,
                       int* out, int* nmatches, void* stream) {
  const size_t lds = pose_lds_bytes(P.kp_pitch);
  const void* fns[7] = {nullptr,
                        (const void*)search_pose_kernel<ORBM_PROJ_LAST_FRAME>,
                        (const void*)search_pose_kernel<ORBM_PROJ_KEYFRAME>,
                        (const void*)search_pose_kernel<ORBM_PROJ_SIM3>,
                        (const void*)search_pose_kernel<ORBM_PROJ_FUSE>,
                        (const void*)search_pose_kernel<ORBM_PROJ_FUSE_SIM3>,
                        (const void*)search_pose_kernel<ORBM_PROJ_SIM3_MATCH>};
  if (P.mode < 1 || P.mode > 6) return ORBX_EINVAL;
  const void* fn = fns[P.mode];
  if (raise_lds_limit(fn, lds)) return ORBX_EDEVICE;
#define ORBX_POSE_LAUNCH(M)                                                                                       \
  hipLaunchKernelGGL(search_pose_kernel<M>, dim3(frames), dim3(kPoseThreads), lds, (hipStream_t)stream, P, kps, \
                     desc, n, uright, blocked, poses, mps, mpdesc, nmp, picks, out, nmatches)
  switch (P.mode) {
    case ORBM_PROJ_LAST_FRAME: ORBX_POSE_LAUNCH(ORBM_PROJ_LAST_FRAME); break;
    case ORBM_PROJ_KEYFRAME: ORBX_POSE_LAUNCH(ORBM_PROJ_KEYFRAME); break;
    case ORBM_PROJ_SIM3: ORBX_POSE_LAUNCH(ORBM_PROJ_SIM3); break;
    case ORBM_PROJ_FUSE: ORBX_POSE_LAUNCH(ORBM_PROJ_FUSE); break;
    case ORBM_PROJ_FUSE_SIM3: ORBX_POSE_LAUNCH(ORBM_PROJ_FUSE_SIM3); break;
    default: ORBX_POSE_LAUNCH(ORBM_PROJ_SIM3_MATCH); break;
  }
#undef ORBX_POSE_LAUNCH
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
