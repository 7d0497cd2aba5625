// orbx_stereo.hip — stereo matching of a rectified pair, Frame::ComputeStereoMatches.
//
// Reference: src/Frame.cc:465-639. For every left keypoint: the right
// keypoints whose row band [floor(y - 2 s), ceil(y + 2 s)] (s = scale of the
// right keypoint's octave) holds the left keypoint's row, whose octave is
// within one of the left one and whose x lies in [uL - mbf/mb, uL], are
// compared by Hamming distance (best = strict '<', TH_HIGH = 100 start); a
// best below thOrbDist = 75 is refined by an 11 x 11 SAD block match of
// mean-removed patches (mean = the patch centre pixel) over 11 shifts on the
// keypoint's pyramid level, a parabola through the SAD minimum, and kept if
// the disparity is in [0, mbf/mb). Finally every match whose SAD is at least
// 1.5 * 1.4 * median(SAD) is dropped.
//
// Two kernels per batch of frame pairs:
//   stereo_match_kernel   grid (groups, pairs). Each workgroup buckets the
//                         pair's right keypoints by row in LDS (counting sort
//                         on floor(y)) and runs one left keypoint per
//                         wavefront at a time: one lane per candidate in the
//                         row window, (dist << 16 | iR) wave minimum (= the
//                         reference's first strict minimum in iR order), then
//                         the SAD on 44 lanes (11 shifts x 4 row groups, quad
//                         DPP sum). Writes uRight, depth and the SAD per left
//                         keypoint (-1 when none).
//   stereo_median_kernel  one workgroup per pair: median of the kept SADs by
//                         two 256-bin radix-select passes, then the rejection.
//
// Float expressions follow the reference's evaluation order with the
// translation unit's -ffp-contract=off; SADs are integers (< 2^16), exact in
// the reference's float accumulation.
#include "orbx_device.cuh"
#include "orbx_wave.cuh"

namespace orbx {

constexpr int kStThreads = 256;
constexpr int kStWaves = kStThreads / 64;
constexpr int kStTHigh = 100;                  // ORBmatcher::TH_HIGH  src/ORBmatcher.cc:37
constexpr int kStThOrbDist = (100 + 50) / 2;   // (TH_HIGH + TH_LOW) / 2  src/Frame.cc:467

__device__ __forceinline__ int hamming256(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

size_t stereo_lds_bytes(int nrows, int kp_pitch) {
  return (size_t)(2 * nrows + 1) * 4 + (size_t)kp_pitch * 12;
}

__global__ __launch_bounds__(kStThreads) void stereo_match_kernel(StereoParams P, const orbx_kp* __restrict__ kpL,
                                                                  const uint8_t* __restrict__ descL,
                                                                  const int* __restrict__ nLp,
                                                                  const orbx_kp* __restrict__ kpR,
                                                                  const uint8_t* __restrict__ descR,
                                                                  const int* __restrict__ nRp,
                                                                  float* __restrict__ uRight,
                                                                  float* __restrict__ depth, int* __restrict__ sad) {
  extern __shared__ int s_dyn[];
  __shared__ float s_r2[kMaxLevels];
  __shared__ int s_tmp[kStWaves];
  const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int g = wg % gridDim.x, p = wg / gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int K = P.kp_pitch, nrows = P.nrows;
  int* s_row = s_dyn;                 // [nrows + 1] row starts (counts before the scan)
  int* s_cur = s_row + nrows + 1;     // [nrows] scatter cursors
  float* s_rx = (float*)(s_cur + nrows);
  float* s_ry = s_rx + K;
  int* s_ri = (int*)(s_ry + K);       // iR | octave << 16
  const int nL = nLp[p], nR = nRp[p];
  const orbx_kp* KL = kpL + (long long)p * K;
  const orbx_kp* KR = kpR + (long long)p * K;
  const uint8_t* DL = descL + (long long)p * K * 32;
  const uint8_t* DR = descR + (long long)p * K * 32;

  // ---- right keypoints bucketed by floor(y) (the row table of :477-491, one entry per keypoint)
  if (tid < kMaxLevels) s_r2[tid] = 2.0f * P.scale[min(tid, P.L - 1)];
  for (int i = tid; i <= nrows; i += kStThreads) s_row[i] = 0;
  __syncthreads();
  for (int i = tid; i < nR; i += kStThreads) {
    const int r = min(max((int)floorf(KR[i].y), 0), nrows - 1);
    __hip_atomic_fetch_add(&s_row[r], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  block_scan_excl<kStThreads>(s_row, nrows + 1, s_tmp);
  for (int i = tid; i < nrows; i += kStThreads) s_cur[i] = s_row[i];
  __syncthreads();
  for (int i = tid; i < nR; i += kStThreads) {
    const orbx_kp k = KR[i];
    const int r = min(max((int)floorf(k.y), 0), nrows - 1);
    const int q = __hip_atomic_fetch_add(&s_cur[r], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    s_rx[q] = k.x;
    s_ry[q] = k.y;
    s_ri[q] = i | (k.octave << 16);
  }
  __syncthreads();

  const float minZ = P.mb, minD = 0.f, maxD = __fdiv_rn(P.mbf, minZ);
  const int nw = gridDim.x * kStWaves;
  for (int iL = g * kStWaves + wid; iL < nL; iL += nw) {
    const orbx_kp kl = KL[iL];
    const int oL = kl.octave;
    const float vL = kl.y, uL = kl.x;
    const float minU = uL - maxD, maxU = uL - minD;
    int best = INT_MAX;
    const bool rowok = vL >= 0.f && vL < (float)nrows && !(maxU < 0);
    if (rowok) {
      const int yi = (int)vL;
      const uint4 dl0 = ((const uint4*)(DL + (long long)iL * 32))[0];
      const uint4 dl1 = ((const uint4*)(DL + (long long)iL * 32))[1];
      const int p0 = s_row[max(yi - P.rwin, 0)], p1 = s_row[min(yi + P.rwin, nrows - 1) + 1];
      for (int b = p0; b < p1; b += 64) {
        const int q = b + lane;
        int key = INT_MAX;
        if (q < p1) {
          const float x = s_rx[q], y = s_ry[q];
          const int ri = s_ri[q], o = ri >> 16;
          const float r = s_r2[o];
          const int maxr = (int)ceilf(y + r), minr = (int)floorf(y - r);
          if (yi >= minr && yi <= maxr && o >= oL - 1 && o <= oL + 1 && x >= minU && x <= maxU) {
            const int iR = ri & 0xFFFF;
            const uint4* dr = (const uint4*)(DR + (long long)iR * 32);
            const int d = hamming256(dl0, dl1, dr[0], dr[1]);
            if (d < kStTHigh) key = (d << 16) | iR;
          }
        }
        best = min(best, key);
      }
      best = wave_min_dpp(best);
    }

    // ---- SAD block match around the best (:549-606)
    float outU = -1.f, outD = -1.f;
    int outS = -1;
    bool sad_ok = best != INT_MAX && (best >> 16) < kStThOrbDist;
    int ul = 0, vl = 0, ur0 = 0;
    float scaleduR0 = 0.f;
    if (sad_ok) {
      const float uR0 = KR[best & 0xFFFF].x;
      const float sf = P.inv_scale[oL];
      const float scaleduL = roundf(uL * sf), scaledvL = roundf(vL * sf);
      scaleduR0 = roundf(uR0 * sf);
      const float iniu = scaleduR0 + 5.f - 5.f, endu = scaleduR0 + 5.f + 5.f + 1.f;
      ul = (int)scaleduL;
      vl = (int)scaledvL;
      ur0 = (int)scaleduR0;
      sad_ok = !(iniu < 0 || endu >= (float)P.lw[oL]) &&
               // windows reaching off the level: an OpenCV range assertion in the reference
               ur0 >= 10 && ul >= 5 && ul + 5 < P.lw[oL] && vl >= 5 && vl + 5 < P.lh[oL];
    }
    if (sad_ok) {
      const uint8_t* bl = P.pl.base[oL] + p * P.pl.fstride[oL] + (long long)vl * P.pl.pitch[oL] + ul;
      const uint8_t* brc = P.pr.base[oL] + p * P.pr.fstride[oL] + (long long)vl * P.pr.pitch[oL] + ur0;
      const int pl = P.pl.pitch[oL], pr = P.pr.pitch[oL];
      int acc = 0;
      if (lane < 44) {
        const int s = lane >> 2, gq = lane & 3;
        const uint8_t* br = brc + (s - 5);
        const int cL = bl[0], cR = br[0];
        const int r0 = gq * 3 - 5, r1 = min(gq * 3 + 3, 11) - 5;
        for (int r = r0; r < r1; ++r) {
          const uint8_t* a = bl + r * pl - 5;
          const uint8_t* c = br + r * pr - 5;
#pragma unroll
          for (int k = 0; k < 11; ++k) acc += abs((a[k] - cL) - (c[k] - cR));
        }
      }
      acc += dpp_i<kDppQuad1032>(0, acc);
      acc += dpp_i<kDppQuad2301>(0, acc);
      int vd[11];
#pragma unroll
      for (int s = 0; s < 11; ++s) vd[s] = __builtin_amdgcn_readlane(acc, 4 * s);
      int bestDist = INT_MAX, bestinc = 0;
#pragma unroll
      for (int s = 0; s < 11; ++s)
        if (vd[s] < bestDist) {
          bestDist = vd[s];
          bestinc = s - 5;
        }
      if (bestinc != -5 && bestinc != 5) {
        const float dist1 = (float)vd[bestinc + 4], dist2 = (float)vd[bestinc + 5], dist3 = (float)vd[bestinc + 6];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (!(deltaR < -1 || deltaR > 1)) {
          float bestuR = P.scale[oL] * (scaleduR0 + (float)bestinc + deltaR);
          float disparity = uL - bestuR;
          if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
              disparity = (float)0.01;
              bestuR = (float)((double)uL - 0.01);
            }
            outD = P.mbf / disparity;
            outU = bestuR;
            outS = bestDist;
          }
        }
      }
    }
    if (lane == 0) {
      const long long o = (long long)p * K + iL;
      uRight[o] = outU;
      depth[o] = outD;
      sad[o] = outS;
    }
  }
}

// Outlier rejection by the median SAD (:620-638), one workgroup per pair.
__global__ __launch_bounds__(kStThreads) void stereo_median_kernel(int K, const int* __restrict__ nLp,
                                                                   float* __restrict__ uRight,
                                                                   float* __restrict__ depth,
                                                                   const int* __restrict__ sad,
                                                                   int* __restrict__ nkept) {
  __shared__ int s_hist[256];
  __shared__ int s_sel[4];  // n, bin, rank within bin, rejected
  const int p = blockIdx.x, tid = threadIdx.x;
  const int nL = nLp[p];
  const long long base = (long long)p * K;
  s_hist[tid] = 0;
  if (tid < 4) s_sel[tid] = 0;
  __syncthreads();
  int n = 0;
  for (int i = tid; i < nL; i += kStThreads) {
    const int s = sad[base + i];
    if (s >= 0) {
      ++n;
      __hip_atomic_fetch_add(&s_hist[s >> 8], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  n = wave_sum_dpp(n);
  if ((tid & 63) == 0) __hip_atomic_fetch_add(&s_sel[0], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  const int total = s_sel[0];
  if (total == 0) {  // the reference indexes an empty vector here
    if (tid == 0) nkept[p] = 0;
    return;
  }
  const int k = total / 2;  // vDistIdx[size / 2] after an ascending sort
  if (tid == 0) {
    int c = 0, b = 0;
    while (c + s_hist[b] <= k) c += s_hist[b++];
    s_sel[1] = b;
    s_sel[2] = k - c;
  }
  __syncthreads();
  const int hi = s_sel[1], k2 = s_sel[2];
  __syncthreads();
  s_hist[tid] = 0;
  __syncthreads();
  for (int i = tid; i < nL; i += kStThreads) {
    const int s = sad[base + i];
    if (s >= 0 && (s >> 8) == hi)
      __hip_atomic_fetch_add(&s_hist[s & 255], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  if (tid == 0) {
    int c = 0, b = 0;
    while (c + s_hist[b] <= k2) c += s_hist[b++];
    s_sel[1] = (hi << 8) | b;
  }
  __syncthreads();
  const float median = (float)s_sel[1];
  const float thDist = 1.5f * 1.4f * median;
  int rej = 0;
  for (int i = tid; i < nL; i += kStThreads) {
    const int s = sad[base + i];
    if (s >= 0 && !((float)s < thDist)) {
      uRight[base + i] = -1.f;
      depth[base + i] = -1.f;
      ++rej;
    }
  }
  rej = wave_sum_dpp(rej);
  if ((tid & 63) == 0) __hip_atomic_fetch_add(&s_sel[3], rej, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  if (tid == 0) nkept[p] = total - s_sel[3];
}

int launch_stereo(const StereoParams& P, const orbx_kp* kpL, const uint8_t* descL, const int* nL,
                  const orbx_kp* kpR, const uint8_t* descR, const int* nR, int pairs, float* uRight,
                  float* depth, int* sad, int* nkept, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = stereo_lds_bytes(P.nrows, P.kp_pitch);
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)stereo_match_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024) != hipSuccess)
      return ORBX_EDEVICE;
    attr_set = true;
  }
  dim3 grid(P.groups, pairs);
  hipLaunchKernelGGL(stereo_match_kernel, grid, dim3(kStThreads), lds, s, P, kpL, descL, nL, kpR, descR, nR,
                     uRight, depth, sad);
  hipLaunchKernelGGL(stereo_median_kernel, dim3(pairs), dim3(kStThreads), 0, s, P.kp_pitch, nL, uRight, depth,
                     sad, nkept);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
