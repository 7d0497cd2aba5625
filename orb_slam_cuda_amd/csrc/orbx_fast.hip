// orbx_fast.hip — FAST-9/16 per grid cell with per-cell non-max suppression.
//
// Reference: ComputeKeyPointsOctTree's FAST stage (src/ORBextractor.cc:1258-1298)
// calls cv::FAST(ROI, iniThFAST, nonmax) on every cell ROI (cell + 3-px halo
// on each side) and, if that finds nothing, cv::FAST(ROI, minThFAST). FAST on
// a ROI only scores pixels in [3, n-3) of the ROI and its 3x3 NMS sees 0 for
// everything outside that band, so suppression is per cell; cells' bands
// tile the level exactly.
//
// One wavefront per (frame, cell). The ROI is staged in LDS (16-byte loads
// when the level is 16-byte aligned), then a three-step funnel keeps lanes
// busy on the pixels that matter:
//   (a) every band pixel: centre + 4 compass ring pixels; a 9-arc always
//       covers two compass points, so pixels without two agreeing compass
//       points cannot be corners at t_low = min(iniTh, minTh);
//   (b) survivors: OpenCV's cornerScore<16> (the largest threshold at which
//       the pixel is still detected, minus 1), two pixels per lane in packed
//       i16x2 arithmetic; a pixel is detected at t iff its score is >= t, so
//       the score is the detection test (no separate 16-pixel ring test) and
//       detected pixels write it to a score map.
// One score map serves both thresholds. NMS then visits only detected pixels, records the
// survivors at iniThFAST and minThFAST as ballots, keeps the iniThFAST set
// unless it is empty, and writes the keys in row-major order (the order
// cv::FAST emits them) into the cell's fixed slot range. Every compaction is
// an ordered ballot compaction, so row-major order is preserved throughout.
#if (defined(ORBX_FAST_SAMEROI) || defined(ORBX_FAST_LCAP)) && !defined(ORBX_DIAG)
#error "result-changing diagnostic switches need -DORBX_DIAG"
#endif
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "orbx_device.cuh"
#include "orbx_fastcore.cuh"

namespace orbx {

#define LDSP __attribute__((address_space(3)))

// ROI row stride in LDS: 44 when every cell ROI fits 3 + rw <= 44 bytes (cells
// of <= 35 px: KITTI), 48 when it fits 48 (cells of <= 39 px: EuRoC, whose
// top level has 36-px cells), staged with dword loads from the dword below
// the ROI; else 80 (>= 65-px ROI + 15 bytes of 16-B alignment slack, 16-byte
// staging, the scalar compass). The tight strides keep a wave's LDS near
// 6 KB instead of ~8 KB and run the dword compass (compass4).
constexpr int kTightE = 4;  // staging element of the tight strides
#ifndef ORBX_FAST_T1
#define ORBX_FAST_T1 44  // tight strides (bank-conflict experiments: tools/variant.sh)
#endif
#ifndef ORBX_FAST_T2
#define ORBX_FAST_T2 48
#endif
constexpr int kRoiTight = ORBX_FAST_T1, kRoiTight2 = ORBX_FAST_T2, kRoiWide = 80;
static_assert(kRoiTight < kRoiTight2 && kRoiTight2 < kRoiWide && kRoiTight % 4 == 0 && kRoiTight2 % 4 == 0,
              "tight strides in increasing order, whole dwords");

// the FAST grid's border box starts at EDGE_THRESHOLD - 3 on every level
// (minBorderX/Y, src/ORBextractor.cc:1133-1134)
constexpr int kFastMinB = kEdgeThreshold - 3;

// 24-bit multiply (full-rate v_mul_u32_u24; the compiler cannot prove the
// operand ranges and otherwise picks the quarter-rate 32/64-bit forms)
__device__ __forceinline__ int u24mul(int a, int b) { return (int)__umul24((unsigned)a, (unsigned)b); }

// Bresenham ring of radius 3, k = 0..15 (cv::makeOffsets, pattern 16)
template <int kRoiStride>
__device__ __forceinline__ int ring_off(int k) {
  constexpr int rx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
  constexpr int ry[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
  return ry[k] * kRoiStride + rx[k];
}

// (a) of the tight-stride kernel on dword LDS reads: a lane tests 4
// horizontally adjacent band pixels (G = ceil(bw / 4) lanes per band row,
// 64 / G rows per pass). Band pixel (y, x) is ROI byte (y + 3) * S + OX + 3 + x
// (OX = the cell's byte offset in its first staged dword, a template
// parameter so every byte extraction is one v_alignbyte_b32 with a constant
// shift). Pixels split into even / odd u16x2 pairs for the packed compass
// network; per-pixel ballots give the row-major ordered compaction.
template <int S, int OX>
__device__ __forceinline__ int compass4(const LDSP uint8_t* roi, LDSP uint16_t* list, int bw, int bh, int t,
                                        int lane) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  // byte offsets, from the group's first dword, of the group's centres, +3 and -3 neighbours
  constexpr int kC = OX + 3, kN4 = OX + 6, kN12 = OX;
  // 64 / G and lane / G by one reciprocal: G <= 15, so (n + 0.5) / G is at
  // least 1/30 from an integer and rcp's 1-ulp error cannot move the floor
  const int G = (bw + 3) >> 2;
  const float rg = __builtin_amdgcn_rcpf((float)G);
  const int RP = __builtin_amdgcn_readfirstlane((int)(64.5f * rg));  // uniform: the pass loop stays scalar
  const int r = (int)(((float)lane + 0.5f) * rg), g = lane - r * G, x = 4 * g;
  const bool lane_ok = r < RP;
  uint64_t colm[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) colm[j] = __ballot(lane_ok && x + j < bw);
  const u16x2 tt = {(unsigned short)t, (unsigned short)t};
  int n1 = 0;
  // one pass over RP band rows; kFull: every row of the pass is inside the
  // band, so the row mask is the lane mask already folded into colm
  auto pass = [&](int by0, auto full) {
    constexpr bool kFull = decltype(full)::value;
    const int by = by0 + r;
    const uint64_t rowm = kFull ? ~0ull : __ballot(by < bh);
    const LDSP uint32_t* rc = (const LDSP uint32_t*)(roi + u24mul((kFull ? by : min(by, bh - 1)) + 3, S)) + g;
    const LDSP uint32_t* ru = rc - 3 * S / 4;  // 3 rows up: ring pixel 8
    const LDSP uint32_t* rd = rc + 3 * S / 4;  // 3 rows down: ring pixel 0
    uint32_t dc[4], du[2], dd[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) dc[k] = k <= ((kN4 + 3) >> 2) ? rc[k] : 0u;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      du[k] = (kC >> 2) + k <= ((kC + 3) >> 2) ? ru[(kC >> 2) + k] : 0u;
      dd[k] = (kC >> 2) + k <= ((kC + 3) >> 2) ? rd[(kC >> 2) + k] : 0u;
    }
    u16x2 any[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // h = 0: pixels 0 and 2, h = 1: pixels 1 and 3
      // bytes o + h and o + h + 2 of a staged run as a u16x2 pair: one v_perm_b32
      auto pair = [h](const uint32_t* d, int o) -> u16x2 {
        const int b = (o & 3) + h;
        const uint32_t sel = (uint32_t)b | 0x0C00u | ((uint32_t)(b + 2) << 16) | 0x0C000000u;
        return __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(d[(o >> 2) + 1], d[o >> 2], sel));
      };
      const u16x2 v = pair(dc, kC);
      const u16x2 a0 = pair(dd, kC & 3), a4 = pair(dc, kN4);
      const u16x2 a8 = pair(du, kC & 3), a12 = pair(dc, kN12);
      const u16x2 s1 = __builtin_elementwise_min(a0, a4), l1 = __builtin_elementwise_max(a0, a4);
      const u16x2 s2 = __builtin_elementwise_min(a8, a12), l2 = __builtin_elementwise_max(a8, a12);
      const u16x2 a = __builtin_elementwise_max(s1, s2), b = __builtin_elementwise_min(l1, l2);
      const u16x2 dk = __builtin_elementwise_sub_sat(__builtin_elementwise_sub_sat(v, tt), __builtin_elementwise_min(a, b));
      const u16x2 br = __builtin_elementwise_sub_sat(__builtin_elementwise_max(a, b), v + tt);
      any[h] = dk | br;
    }
    uint64_t m0 = __ballot(any[0].x != 0) & colm[0], m1 = __ballot(any[1].x != 0) & colm[1];
    uint64_t m2 = __ballot(any[0].y != 0) & colm[2], m3 = __ballot(any[1].y != 0) & colm[3];
    if (!kFull) {
      m0 &= rowm;
      m1 &= rowm;
      m2 &= rowm;
      m3 &= rowm;
    }
    int pos = n1 + mbcnt64(m0) + mbcnt64(m1) + mbcnt64(m2) + mbcnt64(m3);
    const uint16_t e = (uint16_t)((by << 8) | x);
#ifdef ORBX_FAST_LCAP  // timing experiment (diagnostics builds): a capped list, results incomplete
#define LIST_AT(i) list[min((i), ORBX_FAST_LCAP - 1)]
#else
#define LIST_AT(i) list[i]
#endif
    // the masks themselves predicate the stores (inverse ballot: no per-lane bit test)
    if (__builtin_amdgcn_inverse_ballot_w64(m0)) LIST_AT(pos++) = e;
    if (__builtin_amdgcn_inverse_ballot_w64(m1)) LIST_AT(pos++) = (uint16_t)(e + 1);
    if (__builtin_amdgcn_inverse_ballot_w64(m2)) LIST_AT(pos++) = (uint16_t)(e + 2);
    if (__builtin_amdgcn_inverse_ballot_w64(m3)) LIST_AT(pos) = (uint16_t)(e + 3);
#undef LIST_AT
    n1 += __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
  };
  int by0 = 0;
  for (; by0 + RP <= bh; by0 += RP) pass(by0, std::true_type{});
  if (by0 < bh) pass(by0, std::false_type{});
  return n1;
}

#ifndef ORBX_FAST_PK
#define ORBX_FAST_PK 1  // packed-u16 compass pre-test (0: the scalar form, for A/B)
#endif
#ifndef ORBX_FAST_WAVES
#define ORBX_FAST_WAVES 8  // VGPR budget: 8 waves per SIMD (<= 64 VGPRs; 41 used)
#endif
// kProf: the ORBX_FAST_PROF instantiation with the phase stamps (the shipped
// one carries no diagnostics code)
template <int kRoiStride, bool kProf>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ORBX_FAST_WAVES))) void fast_cells_kernel(ExtractParams P, LevelPtrs lp,
                                                        const CellGeom* __restrict__ cells,
                                                        const uint8_t* __restrict__ pyr,
                                                        uint32_t* __restrict__ slots,
                                                        int* __restrict__ cell_counts, int* dbg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned long long t_begin = kProf ? __builtin_amdgcn_s_memtime() : 0ull;
  auto stamp = [&](int k) {
    if (kProf && threadIdx.x == 0)
      dbg[(blockIdx.x + blockIdx.y * gridDim.x) * 8 + k] = (int)(__builtin_amdgcn_s_memtime() - t_begin);
  };
  const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  // the frame by a multiply-high with the plan's magic (exact for every id
  // of the launch, checked at plan time), the cell by one multiply-add: no
  // division on the path to the cell record load
  const int f = P.ncells_magic ? (int)__umulhi((unsigned)wg, P.ncells_magic) : wg / P.ncells_total;
  const int cell = wg - f * P.ncells_total, lane = threadIdx.x;
  CellGeom cg;
  int row_off, rec_pitch, rec_fstride, geo;
  {
    // the whole 32-byte cell record in one scalar load (int16 fields unpacked
    // from it, so no 16-bit vector load sits on the critical path); with the
    // level's staging parameters inside it, nothing after it is indexed by level
    const int4 raw = ((const int4*)cells)[2 * cell], raw2 = ((const int4*)cells)[2 * cell + 1];
    // both record halves and level 0's kernel arguments in one burst of
    // scalar loads (else the compiler defers the second half and the
    // arguments past the skipped-cell test: a second memory latency)
    asm volatile("" ::"s"(raw.x), "s"(raw.y), "s"(raw.z), "s"(raw.w), "s"(raw2.x), "s"(raw2.y), "s"(raw2.z), "s"(raw2.w), "s"(lp.pitch[0]),
                 "s"(lp.aligned16[0]), "s"(lp.base[0]), "s"(lp.fstride[0]), "s"(pyr));
    cg.c0 = (int16_t)(raw.x & 0xFFFF);
    cg.r0 = (int16_t)(raw.x >> 16);
    cg.c1 = (int16_t)(raw.y & 0xFFFF);
    cg.r1 = (int16_t)(raw.y >> 16);
    cg.slot_off = raw.z;
    cg.cap = (int16_t)(raw.w & 0xFFFF);
    cg.level = (int16_t)(raw.w >> 16);
    row_off = raw2.x;
    rec_pitch = raw2.y;
    rec_fstride = raw2.z;
    geo = raw2.w;
    // diagnostics: clock at which the cell record arrived (the test waits for it)
    if (kProf && threadIdx.x == 0 && raw.w != -1)
      dbg[(blockIdx.x + blockIdx.y * gridDim.x) * 8 + 7] = (int)(__builtin_amdgcn_s_memtime() - t_begin);
  }
  int* cnt = cell_counts + (long long)f * P.ncells_total + cell;
  const int rw = cg.c1 - cg.c0, rh = cg.r1 - cg.r0;
  const int bw = rw - 6, bh = rh - 6;
  if (cg.cap == 0 || bw <= 0 || bh <= 0) {
    if (lane == 0) *cnt = 0;
    return;
  }
  // LDS-typed pointers: 32-bit offsets in every address computation
  LDSP unsigned char* sp = (LDSP unsigned char*)smem;
  auto take = [&](size_t bytes) { LDSP unsigned char* r = sp; sp += (bytes + 15) & ~(size_t)15; return r; };
  LDSP uint8_t* roi = (LDSP uint8_t*)take((size_t)P.fast_rh_max * kRoiStride);
  // score map with a zero ring, row stride bw + 1: the right border of a row
  // is the left border of the next, which no score is ever written to
  LDSP uint8_t* sc = (LDSP uint8_t*)take((size_t)(P.fast_bw_max + 1) * (P.fast_bh_max + 2) + 1);
  LDSP uint16_t* list = (LDSP uint16_t*)take(2ull * P.fast_bw_max * P.fast_bh_max);
  // the NMS ballots live in the ROI's LDS: the ROI is dead once the scores are
  // written (phase (d) reads only the list and the score map)
  LDSP uint64_t* ball = (LDSP uint64_t*)roi;

  // level 0 (pitch 0 in the record) is the caller's frames: its base, frame
  // stride and row stride are kernel arguments at fixed offsets, loaded
  // beside the record; levels >= 1 are all in the record
  const bool lvl0 = rec_pitch == 0;
  const int pitch = lvl0 ? lp.pitch[0] : rec_pitch;
  const bool aligned16 = lvl0 ? lp.aligned16[0] != 0 : true;
#ifdef ORBX_FAST_SAMEROI  // diagnostics (tools/variant.sh): every cell of a level stages frame 0's first ROI
  const uint8_t* rows = (lvl0 ? lp.base[0] : pyr + (row_off - cg.r0 * pitch)) + (long long)kFastMinB * pitch +
                        (kFastMinB - cg.c0);
#else
  const uint8_t* rows = lvl0 ? lp.base[0] + f * lp.fstride[0] + (long long)row_off * pitch
                             : pyr + (long long)f * rec_fstride + row_off;
#endif
  constexpr bool kDword = kRoiStride == kRoiTight || kRoiStride == kRoiTight2;  // dword staging
  constexpr bool kTight = kRoiStride != kRoiWide;                                 // the dword compass
  const int a0 = kDword ? (cg.c0 & ~(kTightE - 1)) : (cg.c0 & ~15), ox = cg.c0 - a0;
  if (aligned16 && kDword) {
    // whole rows per load instruction: lane -> (row lq < kRP, dword ld), so
    // load k is row block k at the lane's offset + k * kRP * pitch (one add)
    // and LDS offset k * kRP * stride (the instruction's immediate): no
    // per-piece index math. The buffer range (which checks the VGPR offset)
    // ends at the level plane's last readable byte, so the row blocks past a
    // short ROI read 0 beyond the plane instead of faulting; they land in LDS
    // below the ROI, in the score map cleared afterwards.
    constexpr int kPR = kRoiStride / kTightE, kRP = 64 / kPR;
    const int lq0 = lane / kPR, lq = min(lq0, kRP - 1), ld = lq0 < kRP ? lane - lq0 * kPR : kPR - 1;
    const int voff = u24mul(lq, pitch) + 4 * ld, roff = lq * kRoiStride + 4 * ld;
    const int nrec = (geo & 0xFFFF) * pitch + (geo >> 16) - a0;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(rows + a0), (short)0, nrec, 0x00020000);
    const int nk = (rh + kRP - 1) / kRP;
    constexpr int kK = (41 + kRP - 1) / kRP;  // a 41-row ROI in one burst, taller ones loop
    // unconditional: a shorter ROI's extra row blocks stay inside the wave's
    // LDS (ROI + score map) and inside the buffer range (else they read 0)
    static_assert(kK * kRP * kRoiStride <= 41 * kRoiStride + 1024, "extra row blocks stay in the wave's LDS");
    uint32_t v[kK];
#pragma unroll
    for (int k = 0; k < kK; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + k * kRP * pitch, 0, 0);
#pragma unroll
    for (int k = 0; k < kK; ++k) *(LDSP uint32_t*)(roi + roff + k * kRP * kRoiStride) = v[k];
    for (int k = kK; k < nk; ++k)
      *(LDSP uint32_t*)(roi + roff + k * kRP * kRoiStride) = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + k * kRP * pitch, 0, 0);
  } else if (aligned16) {
    // the ROI's 16-byte chunks, 4 per lane (tall cells loop for the rest)
    const int nch = (cg.c1 - a0 + 15) >> 4, total = rh * nch;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // (HIP's uint4 here ends up in scratch)
    u32x4 v[4];
    int ro[4], lo[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = min(lane + 64 * k, total - 1);
      const int r = i / nch, ch = i - r * nch;
      ro[k] = r * kRoiStride + ch * 16;
      lo[k] = r * pitch + ch * 16;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = *(const u32x4*)(rows + a0 + lo[k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) *(LDSP u32x4*)(roi + ro[k]) = v[k];
    for (int i = lane + 256; i < total; i += 64) {
      const int r = i / nch, ch = i - r * nch;
      *(LDSP u32x4*)(roi + r * kRoiStride + ch * 16) = *(const u32x4*)(rows + (long long)r * pitch + a0 + ch * 16);
    }
  } else {
    for (int r = 0; r < rh; ++r)
      for (int c = lane; c < rw; c += 64) roi[r * kRoiStride + ox + c] = rows[(long long)r * pitch + cg.c0 + c];
  }
  const int sw = bw + 1;
  for (int i = lane; i < (sw * (bh + 2) + 1 + 3) >> 2; i += 64) ((LDSP uint32_t*)sc)[i] = 0;
  __syncthreads();
  stamp(0);

  const int t = P.t_low;
  const bool two = bw <= 32;  // 2 rows x 32 lanes, else 1 row x 64 lanes (bw <= 59)
  const int lr = two ? (lane >> 5) : 0, lc = two ? (lane & 31) : lane;
  const int rstep = two ? 2 : 1;
  const LDSP uint8_t* band = roi + 3 * kRoiStride + ox + 3;  // band pixel (0,0)

  // (a) compass pre-test over all band pixels, row-major ordered compaction
  int n1 = 0;
  if constexpr (kTight) {
    const LDSP uint8_t* roi4 = roi + (ox & ~3);  // the dword holding the ROI's first byte
    switch (ox & 3) {
      case 0: n1 = compass4<kRoiStride, 0>(roi4, list, bw, bh, t, lane); break;
      case 1: n1 = compass4<kRoiStride, 1>(roi4, list, bw, bh, t, lane); break;
      case 2: n1 = compass4<kRoiStride, 2>(roi4, list, bw, bh, t, lane); break;
      default: n1 = compass4<kRoiStride, 3>(roi4, list, bw, bh, t, lane); break;
    }
#ifdef ORBX_FAST_LCAP
    n1 = min(n1, ORBX_FAST_LCAP);
#endif
  } else {
    // four row groups per step so their LDS reads are in flight together
    for (int by0 = 0; by0 < bh; by0 += 4 * rstep) {
      bool fl[4];
#if ORBX_FAST_PK
      // two row groups per packed u16x2 register: the min/max network, the
      // thresholds (saturating subtract) and the tests run as v_pk_* ops
      typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int q = 0; q < 4; q += 2) {
        const int byA = by0 + q * rstep + lr, byB = byA + rstep;
        const LDSP uint8_t* cA = band + u24mul(min(byA, bh - 1), kRoiStride) + min(lc, bw - 1);
        const LDSP uint8_t* cB = band + u24mul(min(byB, bh - 1), kRoiStride) + min(lc, bw - 1);
        auto pk = [](int lo, int hi) { return (u16x2){(unsigned short)lo, (unsigned short)hi}; };
        const u16x2 v = pk(cA[0], cB[0]);
        const u16x2 n0 = pk(cA[3 * kRoiStride], cB[3 * kRoiStride]), n4 = pk(cA[3], cB[3]);
        const u16x2 n8 = pk(cA[-3 * kRoiStride], cB[-3 * kRoiStride]), n12 = pk(cA[-3], cB[-3]);
        const u16x2 s1 = __builtin_elementwise_min(n0, n4), l1 = __builtin_elementwise_max(n0, n4);
        const u16x2 s2 = __builtin_elementwise_min(n8, n12), l2 = __builtin_elementwise_max(n8, n12);
        const u16x2 a = __builtin_elementwise_max(s1, s2), b = __builtin_elementwise_min(l1, l2);
        const u16x2 tt = {(unsigned short)t, (unsigned short)t};
        // min(a,b) < v - t  <=>  sat(sat(v - t) - min(a,b)) != 0;  max(a,b) > v + t  <=>  sat(max(a,b) - (v + t)) != 0
        const u16x2 dk = __builtin_elementwise_sub_sat(__builtin_elementwise_sub_sat(v, tt), __builtin_elementwise_min(a, b));
        const u16x2 br = __builtin_elementwise_sub_sat(__builtin_elementwise_max(a, b), v + tt);
        const u16x2 any = dk | br;
        fl[q] = (int)(byA < bh) & (int)(lc < bw) & (int)(any.x != 0);
        fl[q + 1] = (int)(byB < bh) & (int)(lc < bw) & (int)(any.y != 0);
      }
#else
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int by = by0 + q * rstep + lr;
        const LDSP uint8_t* c = band + u24mul(min(by, bh - 1), kRoiStride) + min(lc, bw - 1);
        const int v = c[0];
        const int n0 = c[3 * kRoiStride], n4 = c[3], n8 = c[-3 * kRoiStride], n12 = c[-3];
        // >= 2 of the 4 compass pixels darker than v - t  <=>  their 2nd smallest is;
        // >= 2 brighter than v + t  <=>  their 2nd largest is
        const int s1 = min(n0, n4), l1 = max(n0, n4), s2 = min(n8, n12), l2 = max(n8, n12);
        const int a = max(s1, s2), b = min(l1, l2);
        // bitwise, not short-circuit: the reads are clamped, so all four row
        // groups' loads can be in flight before the first use
        fl[q] = (int)(by < bh) & (int)(lc < bw) & ((int)(min(a, b) < v - t) | (int)(max(a, b) > v + t));
      }
#endif
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int by = by0 + q * rstep + lr;
        const uint64_t m = __ballot(fl[q]);
        if (fl[q]) list[n1 + mbcnt64(m)] = (uint16_t)((by << 8) | lc);
        n1 += __popcll(m);
      }
    }
  }
  stamp(1);
  int n2 = 0;
  // (b) cornerScore<16> of every compass survivor, two per lane as packed
  // i16x2 (entries i and i + 64 of a 128-entry chunk): detected iff score >= t,
  // so the score replaces the ring test. Detected pixels keep their score in
  // the map and are compacted in place, row-major (chunk reads precede writes).
  for (int i0 = 0; i0 < n1; i0 += 128) {
    const int iA = i0 + lane, iB = iA + 64;
    const int eA = list[min(iA, n1 - 1)], eB = list[min(iB, n1 - 1)];
    const LDSP uint8_t* cA = band + u24mul(eA >> 8, kRoiStride) + (eA & 255);
    const LDSP uint8_t* cB = band + u24mul(eB >> 8, kRoiStride) + (eB & 255);
    const u16x2_t v = {(unsigned short)cA[0], (unsigned short)cB[0]};
    u16x2_t R[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) R[k] = (u16x2_t){(unsigned short)cA[ring_off<kRoiStride>(k)], (unsigned short)cB[ring_off<kRoiStride>(k)]};
    const i16x2 s = corner_score16_x2_ring(R, v);
    // the chunk's valid entries as uniform lane masks (no per-lane compare),
    // the stores predicated by the masks themselves
    const int nA = n1 - i0, nB = nA - 64;
    const uint64_t vA = nA >= 64 ? ~0ull : (1ull << nA) - 1, vB = nB >= 64 ? ~0ull : nB <= 0 ? 0ull : (1ull << nB) - 1;
    const uint64_t mA = __ballot(s.x >= t) & vA, mB = __ballot(s.y >= t) & vB;
    const bool dA = __builtin_amdgcn_inverse_ballot_w64(mA), dB = __builtin_amdgcn_inverse_ballot_w64(mB);
    if (dA) {
      list[n2 + mbcnt64(mA)] = (uint16_t)eA;
      sc[u24mul((eA >> 8) + 1, sw) + (eA & 255) + 1] = (uint8_t)s.x;
    }
    n2 += __popcll(mA);
    if (dB) {
      list[n2 + mbcnt64(mB)] = (uint16_t)eB;
      sc[u24mul((eB >> 8) + 1, sw) + (eB & 255) + 1] = (uint8_t)s.y;
    }
    n2 += __popcll(mB);
  }
  stamp(2);
  __syncthreads();
  stamp(3);
  // (d) 3x3 NMS at both thresholds (neighbours below a threshold count as 0)
  const int ti = P.t_ini, tm = P.t_min;
  const int nch2 = (n2 + 63) >> 6;
  auto nms = [&](int i, bool* ki, bool* km) {  // detected entry i kept at iniThFAST / minThFAST
    const int e = list[i];
    const LDSP uint8_t* q = sc + u24mul((e >> 8) + 1, sw) + (e & 255) + 1;
    const int s = q[0];
    bool gi = s >= ti && s > 0, gm = s >= tm && s > 0;
    const int nbv[8] = {q[-1], q[1], q[-sw - 1], q[-sw], q[-sw + 1], q[sw - 1], q[sw], q[sw + 1]};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int x = nbv[j];
      if (x >= ti && x >= s) gi = false;
      if (x >= tm && x >= s) gm = false;
    }
    *ki = gi;
    *km = gm;
  };
  uint32_t* out = slots + (long long)f * P.slots_per_frame + cg.slot_off;
  auto emit = [&](int e, int pos) {  // the kept pixel's key, row-major position pos in the cell's slots
    const int by = e >> 8, bx = e & 255;
    const int x = cg.c0 + 3 + bx - kFastMinB, y = cg.r0 + 3 + by - kFastMinB;
    if (pos < cg.cap) out[pos] = pack_key(x, y, sc[(by + 1) * sw + bx + 1]);
  };
  int base = 0;
  if (nch2 <= 1) {
    // at most 64 detected pixels (the common case): the ballots stay in registers
    bool ki = false, km = false;
    if (lane < n2) nms(lane, &ki, &km);
    const uint64_t bi = __ballot(ki), bm = __ballot(km);
    const uint64_t m = bi ? bi : bm;
    if (__builtin_amdgcn_inverse_ballot_w64(m)) emit(list[lane], mbcnt64(m));
    base = __popcll(m);
  } else {
    int n_ini = 0;
    for (int ch = 0; ch < nch2; ++ch) {
      const int i = ch * 64 + lane;
      bool ki = false, km = false;
      if (i < n2) nms(i, &ki, &km);
      const uint64_t bi = __ballot(ki), bm = __ballot(km);
      if (lane == 0) {
        ball[2 * ch] = bi;
        ball[2 * ch + 1] = bm;
      }
      n_ini += __popcll(bi);
    }
    __syncthreads();
    const int which = n_ini > 0 ? 0 : 1;
    for (int ch = 0; ch < nch2; ++ch) {
      const uint64_t m = ball[2 * ch + which];
      if (__builtin_amdgcn_inverse_ballot_w64(m)) emit(list[ch * 64 + lane], base + mbcnt64(m));
      base += __popcll(m);
    }
  }
  if (lane == 0) *cnt = min(base, (int)cg.cap);
  stamp(4);
  if (kProf && lane == 0) {
    dbg[(blockIdx.x + blockIdx.y * gridDim.x) * 8 + 5] = n1;
    dbg[(blockIdx.x + blockIdx.y * gridDim.x) * 8 + 6] = n2;
  }
}

// the ROI row stride of a plan's launch: the tightest that holds every cell ROI
// (+ the 3 bytes of its first staged dword below c0)
static int fast_stride(const ExtractParams& P) {
  const int need = P.fast_bw_max + 6 + kTightE - 1;
  return need <= kRoiTight ? kRoiTight : need <= kRoiTight2 ? kRoiTight2 : kRoiWide;
}

size_t fast_lds_bytes(const ExtractParams& P) {
  auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t band = (size_t)P.fast_bw_max * P.fast_bh_max;
  const int stride = fast_stride(P);
#ifdef ORBX_FAST_LCAP
  const size_t list = std::min(band, (size_t)ORBX_FAST_LCAP);
#else
  const size_t list = band;
#endif
#ifndef ORBX_FAST_LDS_PAD
#define ORBX_FAST_LDS_PAD 0  // residency experiments (tools/variant.sh): extra LDS per wave
#endif
  return r16(std::max((size_t)P.fast_rh_max * stride, 16 * ((band + 63) / 64))) +
         r16((size_t)(P.fast_bw_max + 1) * (P.fast_bh_max + 2) + 1) + r16(2 * list) + ORBX_FAST_LDS_PAD;
}

int launch_fast(const ExtractParams& P, const LevelPtrs& lp, const CellGeom* cells, uint32_t* slots,
                int* cell_counts, int batch, hipStream_t s) {
  static int* dbg = nullptr;  // diagnostics only: per-cell phase cycles (ORBX_FAST_PROF=1)
  static const bool prof = getenv("ORBX_FAST_PROF") && getenv("ORBX_FAST_PROF")[0] == '1';
  const int nwg = P.ncells_total * batch;
  if (prof && !dbg) (void)hipMalloc(&dbg, (size_t)nwg * 32);
  if (prof) (void)hipMemsetAsync(dbg, 0, (size_t)nwg * 32, s);
  // diagnostics: ORBX_FAST_TWICE=1 runs the (idempotent) kernel twice, so the
  // second run's phase clocks show FAST on cache-warm levels
#ifdef ORBX_DIAG  // diagnostics builds only (tools/variant.sh)
  static const int reps = getenv("ORBX_FAST_TWICE") && getenv("ORBX_FAST_TWICE")[0] == '1' ? 2 : 1;
#else
  constexpr int reps = 1;
#endif
  // the pyramid buffer the cell records' level >= 1 offsets refer to
  const uint8_t* pyr = P.L > 1 ? lp.base[1] - P.lv[1].off : nullptr;
  for (int rep = 0; rep < reps; ++rep) {
    const int stride = fast_stride(P);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(P.ncells_total, batch), dim3(64), fast_lds_bytes(P), s, P, lp, cells, pyr,
                         slots, cell_counts, dbg);
    };
    if (stride == kRoiTight) prof ? go(fast_cells_kernel<kRoiTight, true>) : go(fast_cells_kernel<kRoiTight, false>);
    else if (stride == kRoiTight2) prof ? go(fast_cells_kernel<kRoiTight2, true>) : go(fast_cells_kernel<kRoiTight2, false>);
    else prof ? go(fast_cells_kernel<kRoiWide, true>) : go(fast_cells_kernel<kRoiWide, false>);
  }
  if (prof) {
    std::vector<int> h((size_t)nwg * 8);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), dbg, h.size() * 4, hipMemcpyDeviceToHost);
    double t[8] = {0};
    int n = 0;
    for (int w = 0; w < nwg; ++w) {
      if (h[w * 8 + 4] == 0) continue;  // skipped cell
      ++n;
      for (int k = 0; k < 8; ++k) t[k] += h[w * 8 + k];
    }
    n = n ? n : 1;
    fprintf(stderr, "fast: %d cells; avg cycles at stage end: record %.0f staged %.0f compass %.0f score %.0f synced %.0f done %.0f; avg n1 %.1f n2 %.1f\n",
            n, t[7] / n, t[0] / n, t[1] / n, t[2] / n, t[3] / n, t[4] / n, t[5] / n, t[6] / n);
  }
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
