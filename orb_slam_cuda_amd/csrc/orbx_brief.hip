// orbx_brief.hip — orientation, rBRIEF descriptors and keypoint assembly.
//
// Reference: computeOrientation/IC_Angle (src/ORBextractor.cc:164-191,
// 822-829) on the unblurred level; computeOrbDescriptor (:195-233) on the
// blurred level with the 256-test bit_pattern_31_ table (:236-494, fork
// value at entry 96, see orbx_pattern.h); keypoint scaling/assembly
// (:1314-1324, 1793-1803): pt *= mvScaleFactor[level] for level > 0,
// size = (int)(31 * scale), octave = level, class_id = -1, output in
// level-major order.
//
// One wavefront per keypoint: IC moments over the r=15 circular patch with
// lanes = patch columns (wave-reduced), cv::fastAtan2 in float without
// contraction, then 4 rBRIEF tests per lane packed by four 64-bit ballots
// straight into the 32 descriptor bytes (bit j of byte i = test 8i+j).
#include "orbx_device.cuh"
#include "orbx_pattern.h"
#include "orbx_sincosf.h"

namespace orbx {

__constant__ signed char c_brief_x[512];
__constant__ signed char c_brief_y[512];

__global__ __launch_bounds__(256) void orient_brief_kernel(ExtractParams P, LevelPtrs lp,
                                                           const uint8_t* __restrict__ blur,
                                                           const uint32_t* __restrict__ qkeys,
                                                           const int* __restrict__ qcounts,
                                                           const int* __restrict__ umax,
                                                           orbx_kp* __restrict__ out_kps,
                                                           uint8_t* __restrict__ out_desc,
                                                           int* __restrict__ out_counts) {
  const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int bx = wg % gridDim.x, f = wg / gridDim.x, lane = threadIdx.x & 63;
  const int slot = bx * 4 + (threadIdx.x >> 6);
  const int* cnt = qcounts + f * P.L;
  if (bx == 0 && threadIdx.x == 0) {
    int tot = 0;
    for (int i = 0; i < P.L; ++i) tot += cnt[i];
    out_counts[f] = tot;
  }
  if (slot >= P.kp_per_frame) return;
  int l = 0;
  while (l + 1 < P.L && slot >= P.lv[l + 1].kbase) ++l;
  const LevelGeom& g = P.lv[l];
  const int idx = slot - g.kbase;
  if (idx >= cnt[l]) return;
  int outpos = idx;
  for (int i = 0; i < l; ++i) outpos += cnt[i];
  const uint32_t key = qkeys[(long long)f * P.kp_per_frame + slot];
  const int x = key_x(key) + g.minBX, y = key_y(key) + g.minBY;

  // IC_Angle: lanes 0..30 -> column u = lane-15, rows v = 0 (centre) and 1..7;
  //           lanes 32..62 -> u = lane-47, rows v = 8..15.
  const int pitch = lp.pitch[l];
  const uint8_t* center = lp.base[l] + f * lp.fstride[l] + (long long)y * pitch + x;
  int m10 = 0, m01 = 0;
  {
    const int half = lane >> 5, u = (lane & 31) - 15;
    if ((lane & 31) < 31) {
      if (half == 0) m10 += u * center[u];
      const int vb = half ? 8 : 1, ve = half ? 15 : 7;
      for (int v = vb; v <= ve; ++v) {
        const int d = umax[v];
        if (u >= -d && u <= d) {
          const int vp = center[u + v * pitch], vm = center[u - v * pitch];
          m01 += v * (vp - vm);
          m10 += u * (vp + vm);
        }
      }
    }
  }
  m10 = wave_sum(m10);
  m01 = wave_sum(m01);
  const float angle = fast_atan2_dev((float)m01, (float)m10);

  // computeOrbDescriptor: a = (float)cos(angle*pi/180), b = (float)sin(...)
  // with glibc's cosf/sinf (orbx_sincosf.h)
  const float factorPI = (float)(M_PI / 180.f);
  const float ang = __fmul_rn(angle, factorPI);
  float a, b;
  glibc_sincosf(ang, &b, &a);
  const uint8_t* bc = blur + g.off + f * g.plane + (long long)y * g.pitch + x;
  const int step = g.pitch;
  uint64_t words[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int test = w * 64 + lane;
    int px0 = c_brief_x[2 * test];
    const int py0 = c_brief_y[2 * test];
    const int px1 = c_brief_x[2 * test + 1], py1 = c_brief_y[2 * test + 1];
    if (P.pattern_upstream && 2 * test == kBriefForkPoint) px0 = kBriefUpstreamX;
    // GET_VALUE(idx): center[cvRound(x*b + y*a)*step + cvRound(x*a - y*b)]
    const int ry0 = __float2int_rn(__fadd_rn(__fmul_rn((float)px0, b), __fmul_rn((float)py0, a)));
    const int rx0 = __float2int_rn(__fsub_rn(__fmul_rn((float)px0, a), __fmul_rn((float)py0, b)));
    const int ry1 = __float2int_rn(__fadd_rn(__fmul_rn((float)px1, b), __fmul_rn((float)py1, a)));
    const int rx1 = __float2int_rn(__fsub_rn(__fmul_rn((float)px1, a), __fmul_rn((float)py1, b)));
    words[w] = __ballot(bc[ry0 * step + rx0] < bc[ry1 * step + rx1]);
  }
  const long long o = (long long)f * P.kp_per_frame + outpos;
  if (lane < 4) ((uint64_t*)(out_desc + o * 32))[lane] = words[lane];
  if (lane == 0) {
    orbx_kp kp;
    float fxp = (float)x, fyp = (float)y;
    if (l != 0) {
      fxp = __fmul_rn(fxp, g.scale);
      fyp = __fmul_rn(fyp, g.scale);
    }
    kp.x = fxp;
    kp.y = fyp;
    kp.size = g.size;
    kp.angle = angle;
    kp.response = (float)key_score(key);
    kp.octave = l;
    kp.class_id = -1;
    out_kps[o] = kp;
  }
}

static bool g_pattern_uploaded = false;

int launch_orient_brief(const ExtractParams& P, const LevelPtrs& lp, const ExtractBuffers& X, orbx_kp* kps,
                        uint8_t* desc, int* counts, int batch, hipStream_t s) {
  if (!g_pattern_uploaded) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_brief_x), kBriefPointX, 512) != hipSuccess) return ORBX_EDEVICE;
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_brief_y), kBriefPointY, 512) != hipSuccess) return ORBX_EDEVICE;
    g_pattern_uploaded = true;
  }
  dim3 grid((P.kp_per_frame + 3) / 4, batch);
  hipLaunchKernelGGL(orient_brief_kernel, grid, dim3(256), 0, s, P, lp, X.blur, X.qkeys, X.qcounts, X.umax, kps, desc,
                     counts);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
