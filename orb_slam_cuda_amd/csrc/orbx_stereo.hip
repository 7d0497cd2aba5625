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

constexpr int kStThreads = 1024;
constexpr int kStWaves = kStThreads / 64;
constexpr int kMedThreads = 256;
constexpr int kStTHigh = 100;                  // ORBmatcher::TH_HIGH  src/ORBmatcher.cc:37
constexpr int kStThOrbDist = (100 + 50) / 2;   // (TH_HIGH + TH_LOW) / 2  src/Frame.cc:467

__device__ __forceinline__ int hamming256(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ uint32_t sad_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm volatile("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

size_t stereo_lds_bytes(int nrows, int kp_pitch, int jobs_cap) {
  return (size_t)(2 * nrows + 1) * 4 + (size_t)kp_pitch * (12 + 32) + 16 + (size_t)jobs_cap * 28;
}

__global__ __launch_bounds__(kStThreads) void stereo_match_kernel(StereoParams P, const orbx_kp* __restrict__ kpL,
                                                                  const uint8_t* __restrict__ descL,
                                                                  const int* __restrict__ nLp,
                                                                  const orbx_kp* __restrict__ kpR,
                                                                  const uint8_t* __restrict__ descR,
                                                                  const int* __restrict__ nRp,
                                                                  float* __restrict__ uRight,
                                                                  float* __restrict__ depth, int* __restrict__ sad) {
  extern __shared__ __attribute__((aligned(16))) int s_dyn[];
  __shared__ float s_r2[kMaxLevels];
  __shared__ int s_rwin[kMaxLevels];
  __shared__ int s_tmp[kStWaves];
  __shared__ const uint8_t* s_lb[2][kMaxLevels];  // pair p's level bases (left, right)
  __shared__ int s_lp[2][kMaxLevels];
  __shared__ float s_scale[kMaxLevels], s_iscale[kMaxLevels];
  __shared__ int s_lw[kMaxLevels], s_lh[kMaxLevels];
  __shared__ int s_njobs;
  const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int g = wg % gridDim.x, p = wg / gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int K = P.kp_pitch, nrows = P.nrows;
  int* s_row = s_dyn;                 // [nrows + 1] row starts (counts before the scan)
  int* s_cur = s_row + nrows + 1;     // [nrows] scatter cursors
  float* s_rx = (float*)(s_cur + nrows);
  float* s_ry = s_rx + K;
  int* s_ri = (int*)(s_ry + K);       // iR | octave << 16
  uint4* s_dr = (uint4*)(s_ri + K + ((-(2 * nrows + 1 + 3 * K)) & 3));  // descriptors by bucket position
  int4* s_job = (int4*)(s_dr + 2 * K);  // SAD jobs
  float* s_juL = (float*)(s_job + P.jobs_cap);
  int* s_qbest = (int*)(s_juL + P.jobs_cap);     // phase A1 result per keypoint slot
  float* s_qbx = (float*)(s_qbest + P.jobs_cap);
  const int nL = nLp[p], nR = nRp[p];
  const orbx_kp* KL = kpL + (long long)p * K;
  const orbx_kp* KR = kpR + (long long)p * K;
  const uint8_t* DL = descL + (long long)p * K * 32;
  const uint8_t* DR = descR + (long long)p * K * 32;

  // ---- right keypoints bucketed by floor(y) (the row table of :477-491, one entry per keypoint)
  if (tid < kMaxLevels) {
    const int l = min(tid, P.L - 1);
    s_r2[tid] = 2.0f * P.scale[l];
    // row half-window for a left keypoint of octave l: candidates have octave
    // <= l + 1, so floor(y) lies within ceil(2 * scale[l + 1]) + 2 rows of its row
    s_rwin[tid] = (int)ceilf(2.0f * P.scale[min(l + 1, P.L - 1)]) + 2;
    s_scale[tid] = P.scale[l];
    s_iscale[tid] = P.inv_scale[l];
    s_lw[tid] = P.lw[l];
    s_lh[tid] = P.lh[l];
    s_lb[0][tid] = P.pl.base[l] + p * P.pl.fstride[l];
    s_lb[1][tid] = P.pr.base[l] + p * P.pr.fstride[l];
    s_lp[0][tid] = P.pl.pitch[l];
    s_lp[1][tid] = P.pr.pitch[l];
  }
  if (tid == 0) s_njobs = 0;
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
    s_dr[2 * q] = ((const uint4*)(DR + (long long)i * 32))[0];
    s_dr[2 * q + 1] = ((const uint4*)(DR + (long long)i * 32))[1];
  }
  __syncthreads();

  const float minZ = P.mb, minD = 0.f, maxD = __fdiv_rn(P.mbf, minZ);
  if (P.stop == 1) return;

  // ---- phase A1: the Hamming search (:503-545), one left keypoint per
  // wavefront at a time (iL = g + groups * m, m = w + 16 k): a lane per
  // candidate of the row window, (dist << 16 | iR) wave minimum = the
  // reference's first strict minimum in iR order. The result goes to LDS slot
  // m; the per-keypoint epilogue runs lane-parallel in A2.
  const int nq = nL > g ? (nL - g + P.groups - 1) / P.groups : 0;  // this workgroup's keypoints
  // the next keypoint's descriptor and (x, y, octave) are prefetched with one
  // VECTOR load per lane (scalar loads would share lgkmcnt with the LDS reads)
  const int fo = lane < 8 ? lane * 4 : (lane < 10 ? (lane - 8) * 4 : 20);
  auto fetch = [&](int m) -> uint32_t {
    const int i = max(min(g + P.groups * m, nL - 1), 0);
    const uint8_t* a = lane < 8 ? DL + (long long)i * 32 : (const uint8_t*)(KL + i);
    return *(const uint32_t*)(a + fo);
  };
  uint32_t nxt = fetch(wid);
  for (int m = wid; m < nq; m += kStWaves) {
    const uint32_t cur = nxt;
    nxt = fetch(m + kStWaves);
    uint32_t rl[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) rl[k] = (uint32_t)__builtin_amdgcn_readlane((int)cur, k);
    const uint4 dl0 = make_uint4(rl[0], rl[1], rl[2], rl[3]), dl1 = make_uint4(rl[4], rl[5], rl[6], rl[7]);
    const float uL = __int_as_float(__builtin_amdgcn_readlane((int)cur, 8));
    const float vL = __int_as_float(__builtin_amdgcn_readlane((int)cur, 9));
    const int oL = __builtin_amdgcn_readlane((int)cur, 10);
    const float minU = uL - maxD, maxU = uL - minD;
    int best = INT_MAX;
    float bestx = 0.f;
    if (vL >= 0.f && vL < (float)nrows && !(maxU < 0)) {
      const int yi = (int)vL;
      const int rw = s_rwin[min(max(oL, 0), kMaxLevels - 1)];
      const int p0 = s_row[max(yi - rw, 0)], p1 = s_row[min(yi + rw, nrows - 1) + 1];
      for (int b = p0; b < p1; b += 64) {
        const int q = b + lane;
        if (q < p1) {
          const int ri = s_ri[q], o = ri >> 16;
          if (o >= oL - 1 && o <= oL + 1) {
            const float x = s_rx[q], y = s_ry[q];
            const float r = s_r2[o];
            if (yi >= (int)floorf(y - r) && yi <= (int)ceilf(y + r) && x >= minU && x <= maxU) {
              const int d = hamming256(dl0, dl1, s_dr[2 * q], s_dr[2 * q + 1]);
              const int key = (d << 16) | (ri & 0xFFFF);
              if (d < kStTHigh && key < best) {
                best = key;
                bestx = x;
              }
            }
          }
        }
      }
      const int wbest = wave_min_dpp(best);
      // keys are unique (iR), so exactly one lane holds the winner and its x
      const uint64_t win = __ballot(best == wbest && wbest != INT_MAX);
      bestx = win ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bestx), __builtin_ctzll(win))) : 0.f;
      best = wbest;
    }
    if (lane == 0) {
      s_qbest[m] = best;
      s_qbx[m] = bestx;
    }
  }
  __syncthreads();

  // ---- phase A2: per keypoint, lane-parallel: the SAD window (:549-575),
  // job list for phase B, "no match" outputs
  for (int m0 = 0; m0 < nq; m0 += kStThreads) {
    const int m = m0 + tid;
    bool sad_ok = false;
    int ul = 0, vl = 0, ur0 = 0, oL = 0, iL = 0;
    float uL = 0.f;
    if (m < nq) {
      iL = g + P.groups * m;
      const int best = s_qbest[m];
      if (best != INT_MAX && (best >> 16) < kStThOrbDist && P.stop != 2) {
        const orbx_kp kl = KL[iL];
        oL = kl.octave;
        uL = kl.x;
        const float sf = s_iscale[oL];
        const float scaleduL = roundf(uL * sf), scaledvL = roundf(kl.y * sf);
        const float scaleduR0 = roundf(s_qbx[m] * sf);
        const float iniu = scaleduR0 + 5.f - 5.f, endu = scaleduR0 + 5.f + 5.f + 1.f;
        ul = (int)scaleduL;
        vl = (int)scaledvL;
        ur0 = (int)scaleduR0;
        const int lw = s_lw[oL], lh = s_lh[oL];
        sad_ok = !(iniu < 0 || endu >= (float)lw) &&
                 // windows reaching off the level: an OpenCV range assertion in the reference
                 ur0 >= 10 && ul >= 5 && ul + 5 < lw && vl >= 5 && vl + 5 < lh;
      }
      if (!sad_ok) {
        const long long o = (long long)p * K + iL;
        uRight[o] = -1.f;
        depth[o] = -1.f;
        sad[o] = -1;
      }
    }
    // append this wave's SAD jobs (one LDS atomic per wave)
    const uint64_t bal = __ballot(sad_ok);
    int base = 0;
    if (lane == 0 && bal)
      base = __hip_atomic_fetch_add(&s_njobs, __popcll(bal), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    base = __builtin_amdgcn_readfirstlane(base);
    if (sad_ok) {
      const int j = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
      s_job[j] = make_int4(iL, ul | (oL << 16), vl, ur0);
      s_juL[j] = uL;
    }
  }
  __syncthreads();

  // ---- phase B: the SAD block match (:549-617), four lanes per job: lane gq
  // of the quad sums rows 3gq .. 3gq+2 of the 11 (gq = 3: rows 9, 10) for all
  // 11 shifts, a quad DPP sum completes them. Each lane loads the centre row
  // and its rows as dwords in one burst and accumulates with v_sad_u32:
  // |(a - cL) - (b - cR_s)| = |(a + 1024) - (b + 1024 + cL - cR_s)|.
  const int njobs = s_njobs;
  for (int t = tid; t < 4 * njobs; t += kStThreads) {
    const int j = t >> 2, gq = t & 3;
    const int4 jb = s_job[j];
    const int iLj = jb.x, ul = jb.y & 0xFFFF, oL = jb.y >> 16, vl = jb.z, ur0 = jb.w;
    const int pl = s_lp[0][oL], pr = s_lp[1][oL];
    const uint8_t* bl = s_lb[0][oL] + (long long)(vl - 5) * pl + ul - 5;   // window row 0, col 0
    const uint8_t* br = s_lb[1][oL] + (long long)(vl - 5) * pr + ur0 - 10;
    // rows of this lane (index 3 = the centre row 5); row 11 would be a dummy
    int rr[4];
#pragma unroll
    for (int i = 0; i < 3; ++i) rr[i] = min(3 * gq + i, 10);
    rr[3] = 5;
    uint32_t a[4][3], bb[4][6];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // dword-aligned loads covering [al, al + 11) and [ar, ar + 21); dwords past
      // the last needed byte are clamped onto it (never read beyond the window)
      const uintptr_t al = (uintptr_t)(bl + (long long)rr[i] * pl), ar = (uintptr_t)(br + (long long)rr[i] * pr);
      const uint32_t* ql = (const uint32_t*)(al & ~(uintptr_t)3);
      const uint32_t* qr = (const uint32_t*)(ar & ~(uintptr_t)3);
      const int ol = (int)(al & 3), orr = (int)(ar & 3);
      const int lastl = (ol + 10) >> 2, lastr = (orr + 20) >> 2;
      uint32_t wl[4], wr[7];
#pragma unroll
      for (int k = 0; k < 4; ++k) wl[k] = ql[min(k, lastl)];
#pragma unroll
      for (int k = 0; k < 6; ++k) wr[k] = qr[min(k, lastr)];
      wr[6] = wr[5];
#pragma unroll
      for (int k = 0; k < 3; ++k) a[i][k] = __builtin_amdgcn_alignbyte(wl[k + 1], wl[k], ol);
#pragma unroll
      for (int k = 0; k < 6; ++k) bb[i][k] = __builtin_amdgcn_alignbyte(wr[k + 1], wr[k], orr);
    }
    auto byte_of = [](const uint32_t* w, int k) { return (int)((w[k >> 2] >> (8 * (k & 3))) & 0xFF); };
    const int cL = byte_of(a[3], 5);
    int E[11];
#pragma unroll
    for (int s = 0; s < 11; ++s) E[s] = 1024 + cL - byte_of(bb[3], s + 5);
    uint32_t acc[11];
#pragma unroll
    for (int s = 0; s < 11; ++s) acc[s] = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (3 * gq + i > 10) break;  // gq = 3 has two rows
      int A[11], Bv[21];
#pragma unroll
      for (int k = 0; k < 11; ++k) A[k] = byte_of(a[i], k) + 1024;
#pragma unroll
      for (int k = 0; k < 21; ++k) Bv[k] = byte_of(bb[i], k);
#pragma unroll
      for (int s = 0; s < 11; ++s)
#pragma unroll
        for (int k = 0; k < 11; ++k) acc[s] = sad_u32(A[k], Bv[k + s] + E[s], acc[s]);
    }
#pragma unroll
    for (int s = 0; s < 11; ++s) {
      int v = (int)acc[s];
      v += dpp_i<kDppQuad1032>(0, v);
      v += dpp_i<kDppQuad2301>(0, v);
      acc[s] = (uint32_t)v;
    }
    if (gq != 0) continue;
    const float uL = s_juL[j];
    int bestDist = INT_MAX, bestinc = 0;
#pragma unroll
    for (int s = 0; s < 11; ++s)
      if ((int)acc[s] < bestDist) {
        bestDist = (int)acc[s];
        bestinc = s - 5;
      }
    float outU = -1.f, outD = -1.f;
    int outS = -1;
    if (bestinc != -5 && bestinc != 5) {
      float dist1 = 0.f, dist2 = 0.f, dist3 = 0.f;
#pragma unroll
      for (int s = 0; s < 11; ++s) {  // register-resident select, no dynamic indexing
        if (s == bestinc + 4) dist1 = (float)acc[s];
        if (s == bestinc + 5) dist2 = (float)acc[s];
        if (s == bestinc + 6) dist3 = (float)acc[s];
      }
      const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
      if (!(deltaR < -1 || deltaR > 1)) {
        float bestuR = s_scale[oL] * ((float)ur0 + (float)bestinc + deltaR);
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
    const long long o = (long long)p * K + iLj;
    uRight[o] = outU;
    depth[o] = outD;
    sad[o] = outS;
  }
}

// Outlier rejection by the median SAD (:620-638), one workgroup per pair.
__global__ __launch_bounds__(kMedThreads) void stereo_median_kernel(int K, const int* __restrict__ nLp,
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
  for (int i = tid; i < nL; i += kMedThreads) {
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
  for (int i = tid; i < nL; i += kMedThreads) {
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
  for (int i = tid; i < nL; i += kMedThreads) {
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
  const size_t lds = stereo_lds_bytes(P.nrows, P.kp_pitch, P.jobs_cap);
  if (raise_lds_limit((const void*)stereo_match_kernel, lds)) return ORBX_EDEVICE;
  dim3 grid(P.groups, pairs);
  hipLaunchKernelGGL(stereo_match_kernel, grid, dim3(kStThreads), lds, s, P, kpL, descL, nL, kpR, descR, nR,
                     uRight, depth, sad);
  hipLaunchKernelGGL(stereo_median_kernel, dim3(pairs), dim3(kMedThreads), 0, s, P.kp_pitch, nL, uRight, depth,
                     sad, nkept);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
