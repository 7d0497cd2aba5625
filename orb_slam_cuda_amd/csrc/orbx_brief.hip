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
// Two keypoints per wavefront, 32 lanes each. Every global access of a
// keypoint is issued in one burst after its key is known: the 31 rows of the
// IC patch (lane = patch column, one byte load per row, coalesced across the
// lanes) and the 39 x 64-byte blurred patch that the rotated BRIEF pattern
// can reach (radius <= 19), staged in LDS with 16-byte loads. Moments are
// reduced across the 32 lanes with DPP, cv::fastAtan2 and glibc sin/cos are
// evaluated per lane, and 8 tests per lane (test t = lane + 32k) give, by
// one ballot per k, descriptor dword k of both keypoints at once
// (bit j of byte i = test 8i + j).
#include <atomic>
#include <mutex>

#include "orbx_device.cuh"
#include "orbx_pattern.h"
#include "orbx_sincosf.h"
#include "orbx_wave.cuh"

namespace orbx {

// test t: {x0, y0, x1, y1} as floats (fork and upstream tables), converted once
// on the host so a test costs one 16-byte LDS read instead of 4 byte
// extracts + 4 int->float conversions per lane
__constant__ float4 c_brief_tests[2][256];

#ifndef ORBX_OB_THREADS
#define ORBX_OB_THREADS 256
#endif
constexpr int kObThreads = ORBX_OB_THREADS;  // 256: 4 waves, 8 keypoints
constexpr int kObKps = kObThreads / 32;
static_assert(kObKps == kKpGroup, "a workgroup's keypoints must lie in one level's slot range");
constexpr int kObRadius = 19;                // |rotated pattern offset| <= 18.4, rounded
constexpr int kObRows = 2 * kObRadius + 1;   // 39
// staged row stride: the 4 x 16-byte chunks of a row, padded so that the
// rotated pattern's byte gathers spread over the banks (bank = dword mod 32:
// 64-byte rows put every other row on the same 16 banks)
#ifndef ORBX_OB_STRIDE
#define ORBX_OB_STRIDE 64
#endif
constexpr int kObStride = ORBX_OB_STRIDE;
static_assert(kObStride >= 64 && kObStride % 8 == 0, "rows hold 4 chunks, 8-byte aligned");
// IC coefficient rows in LDS: 24 dwords each, read as 6 ds_read_b128 per lane
// (bank = dword mod 64, 16-lane groups); at a stride of 28 dwords (4 x odd)
// the 16 |v| rows start on 16 distinct multiples of 4 banks, so a group's
// reads never share a bank (24 put rows 4 apart on one bank: LDS bank-conflict
// cycles per 32-frame launch 4.58 M -> 3.91 M, time equal; round 5)
#ifndef ORBX_OB_ICSTRIDE
#define ORBX_OB_ICSTRIDE 28
#endif
constexpr int kIcStride = ORBX_OB_ICSTRIDE;

// IC_Angle coefficient dwords per |v| (0..15): byte j of dword k is column
// u = 4k + j - 15; {u if 0 < u <= umax[|v|]}, {-u if -umax <= u < 0}, {1 if |u| <= umax}
__constant__ uint32_t c_ic_coef[16 * 24];

// sum over the 32 lanes of each half-wave; the half's total is returned to all its lanes
__device__ __forceinline__ int half_sum(int v) {
  v += dpp_i<kDppQuad1032>(0, v);
  v += dpp_i<kDppQuad2301>(0, v);
  v += dpp_i<kDppHalfMirror>(0, v);
  v += dpp_i<kDppMirror>(0, v);
  v += dpp_i<kDppBcast15, 0xa>(0, v);
  const int lo = __builtin_amdgcn_readlane(v, 31), hi = __builtin_amdgcn_readlane(v, 63);
  return (threadIdx.x & 32) ? hi : lo;
}

// kLv: the level loops' unrolled length (8 covers the usual 8-level
// pyramid in half the scalar bookkeeping of kMaxLevels)
template <int kLv>
__global__ __launch_bounds__(kObThreads) void orient_brief_kernel(ExtractParams P, LevelPtrs lp,
                                                                  const uint8_t* __restrict__ blur,
                                                                  const uint32_t* __restrict__ qkeys,
                                                                  const int* __restrict__ qcounts,
                                                                  const int* __restrict__ /*umax*/,
                                                                  orbx_kp* __restrict__ out_kps,
                                                                  uint8_t* __restrict__ out_desc,
                                                                  int* __restrict__ out_counts) {
  __shared__ __attribute__((aligned(16))) uint8_t s_patch[kObKps][kObRows * kObStride];
  __shared__ float4 s_tests[256];
  __shared__ uint32_t s_ictab[16 * kIcStride];
  const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int bx = wg % gridDim.x, f = wg / gridDim.x, tid = threadIdx.x;
  const int lane = tid & 31, hk = tid >> 5;  // keypoint of this half-wave within the workgroup
  const int slot = bx * kObKps + hk;

  // ---- the loads that depend on nothing are issued together: the key, the
  // frame's level counts (uniform; the buffer is padded to kMaxLevels), the
  // test table and the IC coefficient table (written to LDS after the patch
  // loads are in flight)
  const uint32_t key_raw = slot < P.kp_per_frame ? qkeys[(long long)f * P.kp_per_frame + slot] : 0u;
  const int* cnt = qcounts + f * P.L;
  int c[kLv];
#pragma unroll
  for (int i = 0; i < kLv; ++i) c[i] = cnt[i];
  constexpr int kTestsPer = (256 + kObThreads - 1) / kObThreads, kIcPer = (16 * 24 + kObThreads - 1) / kObThreads;
  float4 test_v[kTestsPer];
  uint32_t ic_v[kIcPer];
#pragma unroll
  for (int k = 0; k < kTestsPer; ++k) test_v[k] = c_brief_tests[P.pattern_upstream ? 1 : 0][min(tid + k * kObThreads, 255)];
#pragma unroll
  for (int k = 0; k < kIcPer; ++k) ic_v[k] = c_ic_coef[min(tid + k * kObThreads, 16 * 24 - 1)];

  // the workgroup's level, in scalar code: level slot ranges start at
  // multiples of kKpGroup (= kObKps) slots, so all of a workgroup's keypoints
  // share one level
  const int slot0 = bx * kObKps;
  int l = 0;
#pragma unroll
  for (int i = 1; i < kLv; ++i)
    if (i < P.L && slot0 >= P.lv[i].kbase) l = i;
  const LevelGeom& g = P.lv[l];
  const int g_kbase = g.kbase, g_minBX = g.minBX, g_minBY = g.minBY, g_w = g.w, g_h = g.h, g_pitch = g.pitch;
  const long long g_off = g.off, g_plane = g.plane;
  const float g_scale = g.scale, g_size = g.size;
  const int lpitch = lp.pitch[l];
  const uint8_t* lbase = lp.base[l];
  const long long lfstride = lp.fstride[l];
  // keypoints of the levels before l, its own count, the frame's total (scalar)
  int cnt_l = 0, before = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kLv; ++i) {
    const int ci = i < P.L ? c[i] : 0;
    if (i == l) cnt_l = ci;
    if (i < l) before += ci;
    tot += ci;
  }
  if (bx == 0 && tid == 0) {
    out_counts[f] = tot;
    // the earlier stages' status word beside the count (single-frame calls:
    // one read-back carries both; they finished before this launch began)
    if (P.status_dst && f == 0) *P.status_dst = *P.status_src;
  }

  // ---- the keypoint of this half-wave
  const int idx = slot - g_kbase;
  const bool valid = slot < P.kp_per_frame && idx < cnt_l;
  const uint32_t key = valid ? key_raw : 0u;
  // an empty slot works on a dummy keypoint at the level centre (never stored)
  const int x = valid ? key_x(key) + g_minBX : g_w / 2, y = valid ? key_y(key) + g_minBY : g_h / 2;

  // ---- one burst of loads: blurred patch (16-byte chunks, five per lane) and
  // IC rows (lane v - 15 = patch row: the row's 31 pixels within 9 dwords from
  // the dword boundary below x - 15; they reach at most byte x + 20 <= w of a
  // row <= h - 5, so they stay inside the level). Every load is unconditional
  // (an empty slot reads around its dummy keypoint, the IC rows the level
  // start) so that no branch join waits for them.
  const int c0 = (x - kObRadius) & ~15;
  const int pitch = lpitch;
  constexpr int kChunks = kObRows * 4, kPerLane = (kChunks + 31) / 32;
  uint4 pv[kPerLane];
  // lane -> (row lane / 4 of an 8-row block, chunk lane % 4): load k is row
  // block k at the lane's offset + 8k * pitch (one add) through one
  // descriptor over the frame's level plane, so no lane computes a 64-bit
  // address per load. Chunks past a row end read the next row, and the row
  // below the patch reads 0 past the plane end (the range check covers the
  // VGPR offset); neither is sampled.
  static_assert(kPerLane * 8 >= kObRows, "row blocks cover the patch");
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(blur + g_off + f * g_plane), (short)0, (int)g_plane, 0x00020000);
  const int pvoff = (y - kObRadius + (lane >> 2)) * g_pitch + c0 + (lane & 3) * 16;
#pragma unroll
  for (int k = 0; k < kPerLane; ++k) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 t = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, pvoff + 8 * k * g_pitch, 0, 0));
    pv[k] = make_uint4(t.x, t.y, t.z, t.w);
  }
  const uint8_t* rp = lbase + f * lfstride + (long long)(y - kHalfPatch + min(lane, kPatchSize - 1)) * pitch +
                      (x - kHalfPatch);
  const uint32_t* q = valid ? (const uint32_t*)((uintptr_t)rp & ~(uintptr_t)3) : (const uint32_t*)lbase;
  const int sh = (int)((uintptr_t)rp & 3);
  uint32_t w[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) w[k] = q[k];
#pragma unroll
  for (int k = 0; k < kTestsPer; ++k)
    if (tid + k * kObThreads < 256) s_tests[tid + k * kObThreads] = test_v[k];
#pragma unroll
  for (int k = 0; k < kIcPer; ++k)
    if (tid + k * kObThreads < 16 * 24) {
      const int i = tid + k * kObThreads;
      s_ictab[(i / 24) * kIcStride + i % 24] = ic_v[k];
    }
  // an empty slot writes its own unused patch; the loads hold row
  // (lane / 4) + 8k, and the rows past the patch are not stored
  {
    uint8_t* dst = s_patch[hk];
#pragma unroll
    for (int k = 0; k < kPerLane; ++k) {
      const int i = lane + 32 * k, r = i >> 2, ch = i & 3;
      if ((k + 1) * 32 > kChunks && i >= kChunks) continue;
      if constexpr (kObStride % 16 == 0) {
        *(uint4*)(dst + r * kObStride + ch * 16) = pv[k];
      } else {  // 8-byte aligned rows: two b64 stores (a misaligned b128 store replays)
        *(uint2*)(dst + r * kObStride + ch * 16) = make_uint2(pv[k].x, pv[k].y);
        *(uint2*)(dst + r * kObStride + ch * 16 + 8) = make_uint2(pv[k].z, pv[k].w);
      }
    }
  }
  __syncthreads();  // staged patch, test table, IC coefficient table

  // ---- IC_Angle (:164-191): per row, the pixels weighted with v_dot4_u32_u8
  // against coefficient dwords (u for u > 0 / -u for u < 0 / 1, inside the
  // circle umax[|v|]); the 31 row sums are reduced over the half-wave
  int m10 = 0, m01 = 0;
  if (valid && lane < kPatchSize) {
    const int v = lane - kHalfPatch, av = v < 0 ? -v : v;
    const uint32_t* tp = s_ictab + av * kIcStride;
    uint32_t pos = 0, neg = 0, sum = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t d = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
      pos = __builtin_amdgcn_udot4(d, tp[k], pos, false);
      neg = __builtin_amdgcn_udot4(d, tp[8 + k], neg, false);
      sum = __builtin_amdgcn_udot4(d, tp[16 + k], sum, false);
    }
    m10 = (int)pos - (int)neg;
    m01 = v * (int)sum;
  }
  m10 = half_sum(m10);
  m01 = half_sum(m01);
  const float angle = fast_atan2_dev((float)m01, (float)m10);

  // computeOrbDescriptor: a = cosf(angle*pi/180), b = sinf(...), glibc's (orbx_sincosf.h)
  const float factorPI = (float)(M_PI / 180.f);
  float a, b;
  glibc_sincosf(__fmul_rn(angle, factorPI), &b, &a);

  // GET_VALUE(idx): center[cvRound(x*b + y*a)*step + cvRound(x*a - y*b)]
  const uint8_t* pc = s_patch[hk] + kObRadius * kObStride + (x - c0);
  uint32_t dword[8];
  // a test's two points as packed float pairs (the table holds {x0, x1, y0,
  // y1}): each product and sum rounded as the reference rounds it (packed
  // v_pk_mul_f32 / v_pk_add_f32, no contraction), then cvRound as one more
  // add: fl(v + 1.5 * 2^23) holds round-half-even(v) in its low mantissa bits
  // (|v| < 2^22), so the patch offset ry * stride + rx is an integer
  // multiply-add of the two sums' bit patterns, the magic constant's share
  // folded into the patch pointer (32-bit wrap-around arithmetic)
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const f32x2_t aa = {a, a}, bb = {b, b}, mg = {12582912.0f, 12582912.0f};
  const uint8_t* pcm = pc - (uint32_t)(0x4B400000u * (uint32_t)(kObStride + 1));
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float4 t = s_tests[lane + 32 * k];
    const f32x2_t X = {t.x, t.y}, Y = {t.z, t.w};
    const f32x2_t fy = (X * bb + Y * aa) + mg, fx = (X * aa - Y * bb) + mg;
    const uint32_t i0 = __float_as_uint(fy.x) * (uint32_t)kObStride + __float_as_uint(fx.x);
    const uint32_t i1 = __float_as_uint(fy.y) * (uint32_t)kObStride + __float_as_uint(fx.y);
    const uint64_t m = __ballot(pcm[i0] < pcm[i1]);
    dword[k] = (uint32_t)((tid & 32) ? (m >> 32) : m);
  }

  if (!valid) return;
  const long long o = (long long)f * P.kp_per_frame + before + idx;
  if (lane < 2) {
    uint4* d = (uint4*)(out_desc + o * 32) + lane;
    *d = lane ? make_uint4(dword[4], dword[5], dword[6], dword[7])
              : make_uint4(dword[0], dword[1], dword[2], dword[3]);
  } else if (lane == 2) {
    orbx_kp kp;
    float fxp = (float)x, fyp = (float)y;
    if (l != 0) {
      fxp = __fmul_rn(fxp, g_scale);
      fyp = __fmul_rn(fyp, g_scale);
    }
    kp.x = fxp;
    kp.y = fyp;
    kp.size = g_size;
    kp.angle = angle;
    kp.response = (float)key_score(key);
    kp.octave = l;
    kp.class_id = -1;
    out_kps[o] = kp;
  }
}

// Test i of pattern mode m (0 fork, 1 upstream) as {x0, y0, x1, y1}: points
// 2i and 2i+1 of the 512-point table (ORBextractor ctor :534-536).
static void brief_test(int m, int i, int t[4]) {
  t[0] = kBriefPointX[2 * i];
  if (m == 1 && 2 * i == kBriefForkPoint) t[0] = kBriefUpstreamX;
  t[1] = kBriefPointY[2 * i];
  t[2] = kBriefPointX[2 * i + 1];
  t[3] = kBriefPointY[2 * i + 1];
}

// Per device (constant memory is per device). Two extractor handles may run on
// two host threads, as the reference's stereo Frame does (src/Frame.cc:77-80):
// the first launch on a device uploads under the lock, later ones only read the
// flag (acquire pairs with the release store after the upload).
static std::atomic<bool> g_pattern_uploaded[64];
static std::mutex g_pattern_mutex;

int launch_orient_brief(const ExtractParams& P, const LevelPtrs& lp, const ExtractBuffers& X, orbx_kp* kps,
                        uint8_t* desc, int* counts, int batch, hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return ORBX_EDEVICE;
  if (!g_pattern_uploaded[dev].load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> lock(g_pattern_mutex);
    if (!g_pattern_uploaded[dev].load(std::memory_order_relaxed)) {
      float4 t[2][256];
      for (int m = 0; m < 2; ++m)
        for (int i = 0; i < 256; ++i) {
          int q[4];
          brief_test(m, i, q);
          t[m][i] = make_float4((float)q[0], (float)q[2], (float)q[1], (float)q[3]);  // {x0, x1, y0, y1}

        }
      if (hipMemcpyToSymbol(HIP_SYMBOL(c_brief_tests), t, sizeof(t)) != hipSuccess) return ORBX_EDEVICE;
      // umax of the r = 15 circle (ORBextractor ctor :540-555; PATCH_SIZE is fixed at 31)
      constexpr int kUmax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
      uint32_t coef[16 * 24] = {};
      for (int av = 0; av < 16; ++av)
        for (int b = 0; b < 32; ++b) {
          const int u = b - kHalfPatch, au = u < 0 ? -u : u;
          if (au > kUmax[av] || b >= kPatchSize) continue;
          const int k = b >> 2, sh = 8 * (b & 3);
          if (u > 0) coef[av * 24 + k] |= (uint32_t)u << sh;
          if (u < 0) coef[av * 24 + 8 + k] |= (uint32_t)(-u) << sh;
          coef[av * 24 + 16 + k] |= 1u << sh;
        }
      if (hipMemcpyToSymbol(HIP_SYMBOL(c_ic_coef), coef, sizeof(coef)) != hipSuccess) return ORBX_EDEVICE;
      g_pattern_uploaded[dev].store(true, std::memory_order_release);
    }
  }
  dim3 grid((P.kp_per_frame + kObKps - 1) / kObKps, batch);
  if (P.L <= 8)
    hipLaunchKernelGGL(orient_brief_kernel<8>, grid, dim3(kObThreads), 0, s, P, lp, X.blur, X.qkeys, X.qcounts,
                       X.umax, kps, desc, counts);
  else
    hipLaunchKernelGGL(orient_brief_kernel<kMaxLevels>, grid, dim3(kObThreads), 0, s, P, lp, X.blur, X.qkeys,
                       X.qcounts, X.umax, kps, desc, counts);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx

extern "C" int orbx_get_pattern(int pattern_mode, int* out1024) {
  if (!out1024 || (pattern_mode != ORBX_PATTERN_FORK && pattern_mode != ORBX_PATTERN_UPSTREAM)) return ORBX_EINVAL;
  for (int i = 0; i < 256; ++i) orbx::brief_test(pattern_mode, i, out1024 + 4 * i);
  return ORBX_OK;
}
