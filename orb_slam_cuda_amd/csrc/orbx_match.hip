// orbx_match.hip — Hamming matchers of ORBmatcher for gfx950.
//
//   hamming_top2_kernel   dense best/second search (the inner loop shared by
//                         every ORBmatcher search), lane-per-query, candidate
//                         rows broadcast from LDS, 8 x v_bcnt per pair
//   (SearchForInitialization: orbx_init.hip)
//   search_bow_kernel     SearchByBoW (KF-F :159-288, KF-KF :522-655)
//
// The reference resolves matches greedily in a fixed order (a later query can
// steal a frame feature from an earlier one, SearchForInitialization
// :444-445,463-470; matched features drop out of SearchByBoW :205-210). The
// kernels keep that order exactly: candidate lists and all 256-bit distances
// are computed in parallel; SearchForInitialization's order-dependent
// resolution is solved as a triangular fixed point by parallel rounds (with
// a sequential wavefront as the fallback), SearchByBoW's per-node greedy
// loops run one wavefront per node with the best/second reduction across
// lanes.
#if (defined(ORBX_M_NOMFMA)) && !defined(ORBX_DIAG)
#error "result-changing diagnostic switches need -DORBX_DIAG"
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "orbx_device.cuh"
#include "orbx_internal.h"
#include "orbx_wave.cuh"

namespace orbx {

constexpr int kGridCols = 64;  // FRAME_GRID_COLS include/Frame.h:38
constexpr int kGridRows = 48;  // FRAME_GRID_ROWS include/Frame.h:37
constexpr int kHistoLength = 30;
constexpr int kThLow = 50;

__device__ __forceinline__ int hamming256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// ------------------------------------------------------------ dense top-2
constexpr int kTopQueries = 256;  // queries per workgroup, two per lane
#ifndef ORBX_TOP_SPLIT
#define ORBX_TOP_SPLIT 8
#endif
constexpr int kTopSplit = ORBX_TOP_SPLIT;  // candidate ranges per query (two waves each)
constexpr int kTopThreads = 128 * kTopSplit;
constexpr int kTopChunk = kTopThreads / (2 * kTopSplit);  // candidates per range per staged chunk (64)
// popcount(x) + acc as ONE v_bcnt_u32_b32 (the compiler otherwise splits the
// chain into bcnt(x, 0) and v_add3)
__device__ __forceinline__ int bcnt_acc(uint32_t x, int acc) {
  int r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
  return r;
}
__device__ __forceinline__ int med3_i32(int a, int b, int c) {
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Best / second of (distance, candidate) keys: key = d << 16 | j orders by
// distance, then by index, so min() keeps the first candidate on ties and
// med3() the second key (whose distance is the reference's bestDist2, ties
// included). Per pair 8 v_xor + 8 v_bcnt + v_lshl_or + v_min + v_med3.
struct Top2Acc {
  uint4 a0, a1;  // query descriptor
  uint32_t k1, k2;
  __device__ __forceinline__ void score(const uint4& r0, const uint4& r1, int j) {
    int d = bcnt_acc(a0.x ^ r0.x, 0);
    d = bcnt_acc(a0.y ^ r0.y, d);
    d = bcnt_acc(a0.z ^ r0.z, d);
    d = bcnt_acc(a0.w ^ r0.w, d);
    d = bcnt_acc(a1.x ^ r1.x, d);
    d = bcnt_acc(a1.y ^ r1.y, d);
    d = bcnt_acc(a1.z ^ r1.z, d);
    d = bcnt_acc(a1.w ^ r1.w, d);
    const uint32_t key = ((uint32_t)d << 16) | (uint32_t)j;
    k2 = med3_u32(key, k1, k2);
    k1 = min(key, k1);
  }
};
constexpr uint32_t kTopNone = (256u << 16) | 0xFFFFu;  // distance 256, no candidate

// Two queries per lane against wave-uniform candidate rows. The candidates
// are split in kTopSplit contiguous ranges, two waves per range (so that 8
// waves per SIMD are resident); each range stages chunks in LDS (one 16-byte
// load per thread per chunk) that its lanes read back as broadcast loads, one
// pair of row reads serving two queries. A pair costs 8 v_xor + 8 v_bcnt + 3
// top-2 updates on (distance << 16 | index) keys (Top2Acc). The partial
// results merge exactly because the keys carry the index (the earlier
// candidate wins ties, as the sequential scan would).
__global__ __launch_bounds__(kTopThreads) void hamming_top2_kernel(const uint8_t* __restrict__ A, long long a_pitch,
                                                                   const int* __restrict__ nA, int a_cap,
                                                                   const uint8_t* __restrict__ B, long long b_pitch,
                                                                   const int* __restrict__ nB,
                                                                   int* __restrict__ best_idx, int* __restrict__ best,
                                                                   int* __restrict__ second, int* err) {
  __shared__ uint4 sB[kTopSplit][kTopChunk][2];
  __shared__ uint2 part[kTopSplit][kTopQueries];
  const int p = blockIdx.y, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int k = wv >> 1, h = wv & 1;
  const int qa = h * 64 + lane, qb = 128 + h * 64 + lane;  // this lane's two queries (of 256)
  const int base = blockIdx.x * kTopQueries;
  // candidate indices live in the low 16 key bits; rows past a_cap have no output slot
  const int na = min(nA[p], a_cap), nb = min(nB[p], 65535);
  if (tid == 0 && blockIdx.x == 0 && (nB[p] > 65535 || nA[p] > a_cap)) atomicOr(err, 16);
  if (base >= na) return;
  const uint4* Ap = (const uint4*)(A + p * a_pitch);
  const uint4* Bp = (const uint4*)(B + p * b_pitch);
  Top2Acc x{make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), kTopNone, kTopNone};
  Top2Acc y = x;
  if (base + qa < na) {
    x.a0 = Ap[2 * (base + qa)];
    x.a1 = Ap[2 * (base + qa) + 1];
  }
  if (base + qb < na) {
    y.a0 = Ap[2 * (base + qb)];
    y.a1 = Ap[2 * (base + qb) + 1];
  }
  const int per = (nb + kTopSplit - 1) / kTopSplit;
  // wave-uniform range (scalar registers: the key's index operand stays an SGPR)
  const int jb = __builtin_amdgcn_readfirstlane(min(k * per, nb)), je = __builtin_amdgcn_readfirstlane(min(jb + per, nb));
  // loader role of this thread: range lk, row lr, half lh
  const int lk = tid / (2 * kTopChunk), lr = (tid >> 1) % kTopChunk, lh = tid & 1;
  const int ljb = min(lk * per, nb), lje = min(ljb + per, nb);
  for (int c0 = 0; c0 < per; c0 += kTopChunk) {
    __syncthreads();
    if (ljb + c0 + lr < lje) sB[lk][lr][lh] = Bp[2 * (ljb + c0 + lr) + lh];
    __syncthreads();
    const int n = __builtin_amdgcn_readfirstlane(min(kTopChunk, je - (jb + c0)));  // wave-uniform
    int j = 0;
    for (; j + 2 <= n; j += 2) {  // two rows' LDS reads in flight, then four (row, query) pairs
      const uint4 r0 = sB[k][j][0], r1 = sB[k][j][1], r2 = sB[k][j + 1][0], r3 = sB[k][j + 1][1];
      x.score(r0, r1, jb + c0 + j);
      y.score(r0, r1, jb + c0 + j);
      x.score(r2, r3, jb + c0 + j + 1);
      y.score(r2, r3, jb + c0 + j + 1);
    }
    if (j < n) {
      const uint4 r0 = sB[k][j][0], r1 = sB[k][j][1];
      x.score(r0, r1, jb + c0 + j);
      y.score(r0, r1, jb + c0 + j);
    }
  }
  part[k][qa] = make_uint2(x.k1, x.k2);
  part[k][qb] = make_uint2(y.k1, y.k2);
  __syncthreads();
  if (tid >= kTopQueries || base + tid >= na) return;
  // merge the ranges: keys are globally ordered (distance, index), so the
  // best / second keys of the union are min / the second smallest
  uint2 r = part[0][tid];
#pragma unroll
  for (int s = 1; s < kTopSplit; ++s) {
    const uint2 o = part[s][tid];
    r.y = min(min(max(r.x, o.x), r.y), o.y);
    r.x = min(r.x, o.x);
  }
  if (base + tid >= na) return;
  const long long o = (long long)p * a_cap + base + tid;
  const int d1 = (int)(r.x >> 16);
  best_idx[o] = d1 < 256 ? (int)(r.x & 0xFFFFu) : -1;
  best[o] = d1;
  second[o] = (int)(r.y >> 16);
}

// ------------------------------------------------ dense top-2 on the matrix cores
// The all-pairs distance matrix is a GEMM: with bits mapped to +-1, the dot
// product of two descriptors is 256 - 2 * Hamming. The kernel runs it on the
// block-scaled FP4 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, e2m1 operands:
// 0x2 = +1.0, 0xA = -1.0; 4x the BF16 rate), K = 256 bits in four MFMAs.
//   candidates (A, rows):  bit set -> -1, clear -> +1, block scale 2^14
//   queries    (B, cols):  bit set -> +1, clear -> -1, block scale 2^0
// so A.B = 2^14 * (2h - 256), and with the accumulator seeded with
// 2^22 + 1 + (candidate index within a 32768 block) every result IS the sort
// key 32768 * h + index + 1, an integer in [1, 2^24), exact in f32 whatever the
// accumulation order. Per (candidate, query) value the lane then does one
// v_min_f32 + one v_med3_f32 (the best / second update of Top2Acc). The bit
// order inside K is free as long as A and B use the same one (dot products
// are order-independent): word w of a descriptor goes to the 16-byte
// fragment of MFMA step w >> 1, lane half w & 1, bit 4n + m to nibble n of
// dword m.
// C/D layout (gfx950, 32x32): lane l holds column l & 31 (the query) and
// rows (r & 3) + 8 (r >> 2) + 4 (l >> 5), r = 0..15 (the candidates).
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
#ifndef ORBX_M_QT
#define ORBX_M_QT 4
#endif
#ifndef ORBX_M_WPE
#define ORBX_M_WPE 2
#endif
#ifndef ORBX_M_CHUNK
#define ORBX_M_CHUNK 128
#endif
constexpr int kMqTiles = ORBX_M_QT;          // 32-query tiles per wave
#ifndef ORBX_M_WAVES
#define ORBX_M_WAVES 2
#endif
#ifndef ORBX_M_HALVES
#define ORBX_M_HALVES 2
#endif
constexpr int kMWaves = ORBX_M_WAVES;        // query waves per candidate range
constexpr int kMHalves = ORBX_M_HALVES;      // candidate ranges per workgroup
constexpr int kMQueries = 32 * kMqTiles * kMWaves;  // 256 queries per workgroup
constexpr int kMChunk = ORBX_M_CHUNK;        // candidates per staged chunk per half (a multiple of 128)
constexpr int kMRowsPerPass = 32 * kMWaves;  // staged rows per pass (two threads per row)
static_assert(kMChunk % kMRowsPerPass == 0, "a chunk is whole staging passes");
constexpr int kMThreads = 64 * kMWaves * kMHalves;
constexpr int kMBlock = 32768;               // candidate indices per float-key block
constexpr float kMNone = 3.0e38f;            // float key of "no candidate"

// 32 descriptor bits -> 32 e2m1 nibbles (bit 4n + m -> nibble n of dword m)
__device__ __forceinline__ i32x4_t fp4_expand(uint32_t w) {
  i32x4_t o;
  o[0] = (int)(((w << 3) & 0x88888888u) | 0x22222222u);
  o[1] = (int)(((w << 2) & 0x88888888u) | 0x22222222u);
  o[2] = (int)(((w << 1) & 0x88888888u) | 0x22222222u);
  o[3] = (int)((w & 0x88888888u) | 0x22222222u);
  return o;
}
__device__ __forceinline__ uint32_t top2_ukey(uint32_t kb, int base) {
  const float k = __builtin_bit_cast(float, kb);
  if (!(k < 1.0e30f)) return kTopNone;
  const int v = (int)k - 1;
  return ((uint32_t)(v >> 15) << 16) | (uint32_t)((v & (kMBlock - 1)) + base);
}
#ifndef ORBX_M_ILV
#define ORBX_M_ILV 1  // MFMA chains of the query tiles interleaved (0: tile-major, for A/B and the timing experiments)
#endif
#ifndef ORBX_M_PAIRS
#define ORBX_M_PAIRS 1  // top-2 update on pairs of results (0: one result per step, for A/B)
#endif
__device__ __forceinline__ void top2_merge(uint32_t& u1, uint32_t& u2, uint32_t x1, uint32_t x2) {
  u2 = min(min(max(u1, x1), u2), x2);
  u1 = min(u1, x1);
}

__global__ __launch_bounds__(kMThreads) __attribute__((amdgpu_waves_per_eu(ORBX_M_WPE))) void hamming_top2_mfma_kernel(
    const uint8_t* __restrict__ A, long long a_pitch, const int* __restrict__ nA, int a_cap,
    const uint8_t* __restrict__ B, long long b_pitch, const int* __restrict__ nB, int* __restrict__ best_idx,
    int* __restrict__ best, int* __restrict__ second, int* err) {
  __shared__ __attribute__((aligned(16))) i32x4_t sC[2][kMHalves][kMChunk / 32][4][64];  // [buffer][half][tile][step][lane]
  __shared__ uint2 part[kMHalves > 1 ? kMHalves - 1 : 1][kMQueries];
  // XCD-aware order: a pair's query blocks are consecutive logical ids, which
  // xcd_remap keeps on one XCD, so its candidates are fetched into one L2
  const int lg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int p = lg / gridDim.x, tid = threadIdx.x, lane = tid & 63;
  const int hf = tid / (64 * kMWaves), wv = (tid >> 6) % kMWaves, ht = tid % (64 * kMWaves);
  const int base = (lg % gridDim.x) * kMQueries;
  // final keys hold the index in 16 bits; rows past a_cap have no output slot
  const int na = min(nA[p], a_cap), nb = min(nB[p], 65535);
  if (tid == 0 && (lg % gridDim.x) == 0 && (nB[p] > 65535 || nA[p] > a_cap)) atomicOr(err, 16);
  if (base >= na) return;
  // queries (the B operand), this wave's kMqTiles tiles, held for the whole kernel
  const uint4* Ap = (const uint4*)(A + p * a_pitch);
  const uint4* Bp = (const uint4*)(B + p * b_pitch);
  const int hl = lane >> 5;
  i32x4_t qf[kMqTiles][4];
#pragma unroll
  for (int q = 0; q < kMqTiles; ++q) {
    const int qi = min(base + wv * 32 * kMqTiles + q * 32 + (lane & 31), na - 1);
    const uint4 d0 = Ap[2 * qi], d1 = Ap[2 * qi + 1];
    const uint32_t w[4] = {hl ? d0.y : d0.x, hl ? d0.w : d0.z, hl ? d1.y : d1.x, hl ? d1.w : d1.z};
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[q][s] = fp4_expand(~w[s]);
  }
  // running row keys: 2^22 + 1 + (index of this lane's row r in the next tile - blk);
  // the + 1 keeps every key >= 1, so no result is a signed zero (whose bit
  // pattern would order last)
  f32x16_t rk;
  auto rk_reset = [&]() {
#pragma unroll
    for (int r = 0; r < 16; ++r) rk[r] = 4194305.0f + (float)((r & 3) + 8 * (r >> 2) + 4 * hl);
  };
  rk_reset();
  uint32_t k1[kMqTiles], k2[kMqTiles];  // float keys as bit patterns
  uint32_t u1[kMqTiles], u2[kMqTiles];
  const uint32_t kNoneBits = __builtin_bit_cast(uint32_t, kMNone);
#pragma unroll
  for (int q = 0; q < kMqTiles; ++q) {
    k1[q] = k2[q] = kNoneBits;
    u1[q] = u2[q] = kTopNone;
  }
  const int per = (nb + kMHalves - 1) / kMHalves;
  const int jb = min(hf * per, nb), je = min(jb + per, nb);  // this half's candidates
  const int nchunks = (per + kMChunk - 1) / kMChunk;         // the same for both halves (barriers)
  int blk = jb;                                              // first index of the current key block
  const int sr = ht >> 1, spart = ht & 1;                    // staging role: row, 16-byte half
  // double-buffered staging: chunk c+1's global load is in flight while chunk
  // c is computed; one barrier per chunk (a wave writing buffer c & 1 has
  // passed the barrier every wave reaches only after computing chunk c - 2)
  constexpr int kRep = kMChunk / kMRowsPerPass;  // staged rows per thread per chunk
  uint4 pre[kRep];
#pragma unroll
  for (int i = 0; i < kRep; ++i) pre[i] = jb < je ? Bp[2 * min(jb + sr + kMRowsPerPass * i, je - 1) + spart] : make_uint4(0, 0, 0, 0);
  // top-2 update of query tile q with one tile's 16 results per lane: results
  // in pairs; with k1 <= k2, the second smallest of {k1, k2, x0, x1} is
  // min(med3(k1, x0, x1), k2) and the smallest min3(k1, x0, x1); two pairs
  // share one min3 into k2, so four values cost 5 integer VALU instead of 8
  // (positive floats order as their bit patterns; the medians as v_med3_f32,
  // so no integer min is shared with the new minimum's and each folds into
  // one v_min3_u32)
  auto top2_update = [&](int q, const f32x16_t& acc) {
#pragma unroll
    for (int r = 0; r < 16; r += 4) {
      const float xf0 = acc[r], xf1 = acc[r + 1], xf2 = acc[r + 2], xf3 = acc[r + 3];
      const uint32_t x0 = __float_as_uint(xf0), x1 = __float_as_uint(xf1);
      const uint32_t x2 = __float_as_uint(xf2), x3 = __float_as_uint(xf3);
      const uint32_t t0 = __float_as_uint(__builtin_amdgcn_fmed3f(xf0, xf1, __uint_as_float(k1[q])));
      const uint32_t m = min(min(k1[q], x0), x1);
      const uint32_t t1 = __float_as_uint(__builtin_amdgcn_fmed3f(xf2, xf3, __uint_as_float(m)));
      k1[q] = min(min(m, x2), x3);
      k2[q] = min(min(t0, t1), k2[q]);
    }
  };
  auto top2_tile = [&](const i32x8_t (&af)[4], const f32x16_t& rkt) {
#if ORBX_M_ILV && !defined(ORBX_M_NOMFMA) && !defined(ORBX_M_NOTOP2)
    // step-major: the four query tiles' accumulation chains interleaved
    // (34.3 -> 33.1 us per 64 pairs alone against tile-major chains)
    f32x16_t accs[kMqTiles];
#pragma unroll
    for (int q = 0; q < kMqTiles; ++q) accs[q] = rkt;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int q = 0; q < kMqTiles; ++q) {
        const i32x8_t bf = (i32x8_t){qf[q][s][0], qf[q][s][1], qf[q][s][2], qf[q][s][3], 0, 0, 0, 0};
        accs[q] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[s], bf, accs[q], 4, 4, 0, 141, 0, 127);
      }
    }
#pragma unroll
    for (int q = 0; q < kMqTiles; ++q) top2_update(q, accs[q]);
    return;
#endif
#pragma unroll
    for (int q = 0; q < kMqTiles; ++q) {
      f32x16_t acc = rkt;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const i32x8_t bf = (i32x8_t){qf[q][s][0], qf[q][s][1], qf[q][s][2], qf[q][s][3], 0, 0, 0, 0};
#if defined(ORBX_M_NOMFMA)  // timing experiment only: the top-2 update without MFMA
        acc[s] += __builtin_bit_cast(float, af[s][0] ^ bf[0]);
#else
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[s], bf, acc, 4, 4, 0, 141, 0, 127);
#endif
      }
#if defined(ORBX_M_NOTOP2)  // timing experiment only: MFMA without the top-2 update
      const float x0 = acc[0];
      k1[q] = min(__float_as_uint(x0), k1[q]);
#elif ORBX_M_PAIRS
      top2_update(q, acc);
#else
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        // positive floats order as their bit patterns: the best key is an
        // integer v_min_u32 and the second a v_med3_f32 (the target builtin);
        // fminf would first canonicalise every MFMA result with a v_max_f32.
        // (__float_as_uint of a float copy: ROCm 7.2 clang lowers
        // __builtin_bit_cast(uint32_t, acc[r]) of an ext_vector element to a
        // read of element 0)
        const float xf = acc[r];
        k2[q] = __float_as_uint(__builtin_amdgcn_fmed3f(xf, __uint_as_float(k1[q]), __uint_as_float(k2[q])));
        k1[q] = min(__float_as_uint(xf), k1[q]);
      }
#endif
    }
  };
  for (int c = 0; c < nchunks; ++c) {
    const int c0 = jb + c * kMChunk, buf = c & 1;
    if (c0 < je) {
#pragma unroll
      for (int k = 0; k < kRep; ++k) {
        const int row = sr + kMRowsPerPass * k;
        const uint32_t w[4] = {pre[k].x, pre[k].y, pre[k].z, pre[k].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int wi = 4 * spart + i;
          sC[buf][hf][row >> 5][wi >> 1][(row & 31) + 32 * (wi & 1)] = fp4_expand(w[i]);
        }
      }
      if (c0 + kMChunk < je) {
#pragma unroll
        for (int k = 0; k < kRep; ++k) pre[k] = Bp[2 * min(c0 + kMChunk + sr + kMRowsPerPass * k, je - 1) + spart];
      }
    }
    __syncthreads();
    if (c0 >= je) continue;
    if (c0 - blk >= kMBlock) {  // key block full: fold the float keys into the index keys
#pragma unroll
      for (int q = 0; q < kMqTiles; ++q) {
        top2_merge(u1[q], u2[q], top2_ukey(k1[q], blk), top2_ukey(k2[q], blk));
        k1[q] = k2[q] = kNoneBits;
      }
      blk = c0;
      rk_reset();
    }
    const int nval = min(kMChunk, je - c0);
#ifdef ORBX_M_PREF
    // the next tile's candidate fragments are read while this tile computes
    const int ntile = (nval + 31) >> 5;
    i32x4_t nx[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) nx[s] = sC[buf][hf][0][s][lane];
#endif
    for (int t = 0; t * 32 < nval; ++t) {
      i32x8_t af[4];
#ifdef ORBX_M_PREF
#pragma unroll
      for (int s = 0; s < 4; ++s) af[s] = (i32x8_t){nx[s][0], nx[s][1], nx[s][2], nx[s][3], 0, 0, 0, 0};
      const int tn = min(t + 1, ntile - 1);
#pragma unroll
      for (int s = 0; s < 4; ++s) nx[s] = sC[buf][hf][tn][s][lane];
#else
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const i32x4_t v = sC[buf][hf][t][s][lane];
        af[s] = (i32x8_t){v[0], v[1], v[2], v[3], 0, 0, 0, 0};
      }
#endif
      const int nrow = nval - 32 * t;  // valid rows of this tile
      if (nrow >= 32) {
        top2_tile(af, rk);
      } else {  // ragged last tile: rows past the end never win
        f32x16_t rkt;
#pragma unroll
        for (int r = 0; r < 16; ++r) rkt[r] = (r & 3) + 8 * (r >> 2) + 4 * hl < nrow ? rk[r] : kMNone;
        top2_tile(af, rkt);
      }
      rk += 32.0f;
    }
  }
  // fold the last block, then merge the two lane halves (rows 0-3 / 4-7 of each 8)
#pragma unroll
  for (int q = 0; q < kMqTiles; ++q) {
    top2_merge(u1[q], u2[q], top2_ukey(k1[q], blk), top2_ukey(k2[q], blk));
    const uint32_t o1 = __shfl_xor(u1[q], 32), o2 = __shfl_xor(u2[q], 32);
    top2_merge(u1[q], u2[q], o1, o2);
  }
  const int qloc = wv * 32 * kMqTiles + (lane & 31);
  if (hf >= 1 && lane < 32) {
#pragma unroll
    for (int q = 0; q < kMqTiles; ++q) part[hf - 1][qloc + 32 * q] = make_uint2(u1[q], u2[q]);
  }
  if (kMHalves > 1) __syncthreads();
  if (hf != 0 || lane >= 32) return;
#pragma unroll
  for (int q = 0; q < kMqTiles; ++q) {
    const int qi = base + qloc + 32 * q;
    if (qi >= na) continue;
    for (int h = 0; h + 1 < kMHalves; ++h) {  // ranges in index order: keys merge exactly in any order
      const uint2 o = part[h][qloc + 32 * q];
      top2_merge(u1[q], u2[q], o.x, o.y);
    }
    const long long oi = (long long)p * a_cap + qi;
    const int d1 = (int)(u1[q] >> 16);
    best_idx[oi] = d1 < 256 ? (int)(u1[q] & 0xFFFFu) : -1;
    best[oi] = d1;
    second[oi] = (int)(u2[q] >> 16);
  }
}

// ------------------------------------------------------------ wave helpers
__device__ __forceinline__ int wave_min(int v) { return wave_min_dpp(v); }
__device__ __forceinline__ int wave_sum_i(int v) { return wave_sum_dpp(v); }

// best / second of the multiset of valid distances, first position wins ties
// (the sequential "if(d<best){second=best;best=d;idx=i} else if(d<second)"
// loop computes exactly this). Returns wave-uniform values.
struct Top2 {
  int best, pos, second;
};
__device__ __forceinline__ Top2 wave_top2(bool valid, int dist, int pos) {
  const int BIG = INT_MAX;
  const int d = valid ? dist : BIG;
  const int b = wave_min(d);
  const uint64_t eq = __ballot(valid && d == b);
  Top2 r;
  r.best = b;
  if (eq == 0) {
    r.pos = -1;
    r.second = BIG;
    return r;
  }
  const int first_lane = __ffsll((long long)eq) - 1;
  r.pos = __builtin_amdgcn_readlane(pos, first_lane);
  if (__popcll(eq) >= 2) {
    r.second = b;
  } else {
    const int lane = threadIdx.x & 63;
    r.second = wave_min(lane == first_lane ? BIG : d);
  }
  return r;
}

// ------------------------------------------------------------ SearchByBoW
// Grid: pairs x G workgroups; workgroup g of a pair takes the pair's A nodes
// [g*nnA/G, (g+1)*nnA/G). Shared vocabulary nodes are independent: DBoW2 puts
// every feature in exactly one node, so a node's B features are touched by
// that node's A features only, the taken bits of a workgroup's nodes are
// private to it, and only the rotation histogram and the match count are the
// pair's (global atomics: hist[0..29] bins, hist[30] count;
// search_bow_finalize_kernel applies ComputeThreeMaxima after). An accepted
// match goes to the pair's row record, bin << 16 | matched index (16 bits: the
// entry points bound both frames' counts by 65536), in a
// scratch that is all -1 between calls (finalize writes `out` from it and
// resets it and the histogram, so no fill launches precede the kernel).
//
// Inside a node the reference is greedy (src/ORBmatcher.cc:186-262): A rows in
// node order, each taking the best untaken B row. The workgroup splits that
// into
//  (1) a data-parallel pass, one lane per A row: the node's B rows (staged in
//      LDS in node order, static filter applied) are scanned once and the
//      row's K smallest keys (distance << 16 | position in the node) kept;
//  (2) the greedy pass, one lane per node, in A order: the first two untaken
//      keys of the row's list ARE the reference's bestDist1/bestIdx and
//      bestDist2 (keys order ties by node position, as the strict `<` of
//      :211-226 does), so the pass is a few register operations per row; a
//      row whose list has fewer than two untaken keys left while it had more
//      than K candidates rescans its node (rare).
// A workgroup whose node range does not fit the LDS tables falls back to the
// per-wave greedy (a wave per node, the best/second reduced across lanes).
struct BowSide {
  const uint8_t* desc;  // pair p: desc + p * kp_pitch * 32
  const float* angle;   // keypoint i's angle at angle[p * kp_pitch * angle_stride + i * angle_stride]
  int angle_stride;     // 1 for an angle array, 7 for orbx_kp records
  const uint8_t* mp;    // has a (good) MapPoint, or null = all
  const int* n;         // features per pair
  const uint32_t* nodes;  // FeatureVector CSR: pair p at p * node_pitch (off: p * (node_pitch + 1))
  const int* off;
  const int* idx;
  const int* nn;        // nodes per pair
  long long kp_pitch, node_pitch;
};

#ifndef ORBX_BOW_GROUPS
#define ORBX_BOW_GROUPS 24
#endif
#ifndef ORBX_BOW_BALANCE
#define ORBX_BOW_BALANCE 1  // node ranges of equal estimated work (0: equal node counts)
#endif
// Workgroup shape (C3 + BoW bench, 64 KITTI pairs): alone, 8 ranges of <= 768
// rows on 512 threads are fastest (34.9 us; 256 threads 40.8 us), but in the
// pipelined step those 71 KB-LDS workgroups wait for CUs the extraction
// kernels hold (0.24 ms of event time per batch); 24 ranges of <= 256 rows
// (~26 KB) on 256 threads fit beside them: 0.135 ms, 106 k -> 118 k frames/s.
// Ranges past the caps take the per-wave fallback.
constexpr int kBowGroups = ORBX_BOW_GROUPS;  // workgroups per pair (node ranges)
#ifndef ORBX_BOW_THREADS
#define ORBX_BOW_THREADS 256
#endif
constexpr int kBowThreads = ORBX_BOW_THREADS;
constexpr int kBowK = 8;         // smallest keys kept per A row
#ifndef ORBX_BOW_CAP
#define ORBX_BOW_CAP 256
#endif
constexpr int kBowCapB = ORBX_BOW_CAP;      // B rows staged per workgroup
constexpr int kBowCapA = ORBX_BOW_CAP;      // A rows per workgroup
constexpr int kBowCapN = ORBX_BOW_CAP / 3;  // nodes per workgroup
constexpr int kBowMaxB = 256;    // fallback: B features of a node held in registers (4 chunks of 64 lanes)
constexpr uint32_t kBowNone = 0xFFFFFFFFu;
#ifndef ORBX_BOW_ROWCOST
#define ORBX_BOW_ROWCOST 64
#endif
constexpr int kBowRowCost = ORBX_BOW_ROWCOST;  // a row's fixed cost in candidate scans (range balance)
#ifndef ORBX_BOW_ROUNDS
#define ORBX_BOW_ROUNDS 16
#endif
constexpr int kBowRounds = ORBX_BOW_ROUNDS;  // default greedy fixed-point rounds before the sequential pass
// (ORBX_BOW_ROUNDS=<n> in the environment overrides it per call; 0: the sequential pass only; results are the same)

struct BowTables {  // the two-pass layout
  uint32_t bdesc[kBowCapB][8];  // the range's B rows, node by node
  int bidx[kBowCapB];           // their feature index, -1 = not a candidate (KF-KF without a good MapPoint)
  uint4 top[kBowCapA][2];       // per A row its kBowK = 8 smallest keys, ascending (kBowNone = empty)
  int nv[kBowCapA];             // candidates the row saw, -1 = row skipped (no good MapPoint);
                                // after the greedy pass: the matched staged position, or -1
  int match[kBowCapA];          // greedy rounds: the row's current choice (staged position, -1 = none)
  int claim[kBowCapB];          // greedy rounds: first row (in range order) choosing the position
  int rq[kBowCapA];             // the row's node: B rows [rq & 0xFFFF, rq >> 16)
  int boff[kBowCapN + 1];       // node j's B rows at [boff[j], boff[j+1])
  int aoff[kBowCapN + 1];       // node j's A rows at [aoff[j], aoff[j+1]) (relative to the range)
  int bsrc[kBowCapN];           // node j's B CSR start
  int sstart[kBowCapN + 1];     // phase (1) lane slots: the k-th node in slot order starts at sstart[k]
  int snode[kBowCapN];          // ... and is node snode[k]
  int rescan[kBowCapA];         // greedy rounds: rows whose list ran out, rescanned by whole waves
  uint32_t taken[kBowCapB / 32];  // by staged position
};
struct BowFallback {  // the per-wave layout
  uint32_t taken[2048];  // one bit per B feature
  uint32_t adesc[kBowThreads / 64][64][8];
  int aidx[kBowThreads / 64][64];
  int bidx[kBowThreads / 64][kBowMaxB];
};
union BowLds {
  BowTables t;
  BowFallback f;
};

template <int NT>
__global__ __launch_bounds__(NT) void search_bow_kernel(BowSide A, BowSide B, float nnratio, int check_ori,
                                                        int kf_vs_kf, int G, int max_rounds, long long out_pitch,
                                                        int* __restrict__ rec_all, int* __restrict__ hist_all,
                                                        int* __restrict__ err, int* dbg) {
  constexpr int kWaves = NT / 64;
  const unsigned long long t_begin = __builtin_amdgcn_s_memtime();
  auto stamp = [&](int k, int v) {  // diagnostics only (ORBX_BOW_PROF=1): per-workgroup phase cycles
    if (dbg && threadIdx.x == 0) dbg[blockIdx.x * 8 + k] = v < 0 ? (int)(__builtin_amdgcn_s_memtime() - t_begin) : v;
  };
  __shared__ BowLds S;
  __shared__ int s_scan[kWaves + 1];
  __shared__ int s_hist[32];
  __shared__ int s_queue;
  const int p = blockIdx.x / G, g = blockIdx.x - p * G;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nnA = A.nn[p], nnB = B.nn[p];
  const int* offA0 = A.off + p * (A.node_pitch + 1);
#if ORBX_BOW_BALANCE
  // The pair's nodes split into G contiguous ranges of equal estimated work
  // rather than equal node counts (node sizes are skewed: a few nodes hold
  // hundreds of features, and a range's time follows its largest nodes). A
  // node of n A rows costs about n x (n + kBowRowCost): the candidate scans
  // plus each row's fixed part (its node lookup and two dependent global
  // loads, worth ~64 candidates; with n x (n + 4) the first range of a pair
  // took ~540 rows, two passes of the workgroup's lanes). B's node sizes
  // follow A's in consecutive frames, so no B lookup is needed here: node j
  // goes to workgroup floor(excl_j x G / total), non-decreasing in j.
  int k0, k1;
  {
    // n clamped at 4096 in the estimate (it only drives the balance): with at
    // most 65536 rows per frame every sum below then stays far inside 32 bits
    auto work = [&](int j) {
      const int n = min(offA0[j + 1] - offA0[j], 4096);
      return n * (n + kBowRowCost);
    };
    int tot = 0;
    for (int j = tid; j < nnA; j += NT) tot += work(j);
    tot = wave_sum_dpp(tot);
    if (lane == 0) s_scan[wv] = tot;
    __syncthreads();
    long long W = 0;
    for (int w = 0; w < kWaves; ++w) W += s_scan[w];
    __syncthreads();
    int lt = 0, le = 0;
    long long carry = 0;
    for (int j0 = 0; j0 < nnA; j0 += NT) {
      const int j = j0 + tid;
      const int wj = j < nnA ? work(j) : 0;
      const int incl = wave_incl_scan_dpp(wj);
      if (lane == 63) s_scan[wv] = incl;
      __syncthreads();
      long long before = carry;
      for (int w = 0; w < wv; ++w) before += s_scan[w];
      const long long excl = before + incl - wj;
      if (j < nnA) {
        const int owner = W > 0 ? (int)min((long long)(G - 1), excl * G / W) : 0;
        lt += owner < g;
        le += owner <= g;
      }
      for (int w = 0; w < kWaves; ++w) carry += s_scan[w];
      __syncthreads();
    }
    lt = wave_sum_dpp(lt);
    le = wave_sum_dpp(le);
    if (lane == 0) {
      s_scan[wv] = lt;
      s_hist[wv] = le;
    }
    __syncthreads();
    k0 = k1 = 0;
    for (int w = 0; w < kWaves; ++w) {
      k0 += s_scan[w];
      k1 += s_hist[w];
    }
    __syncthreads();
  }
  const int nk = k1 - k0;
#else
  const int k0 = (int)((long long)g * nnA / G), k1 = (int)((long long)(g + 1) * nnA / G), nk = k1 - k0;
#endif
  const uint8_t* descA = A.desc + p * A.kp_pitch * 32;
  const uint8_t* descB = B.desc + p * B.kp_pitch * 32;
  const float* angA = A.angle + p * A.kp_pitch * A.angle_stride;
  const float* angB = B.angle + p * B.kp_pitch * B.angle_stride;
  const uint8_t* mpA = A.mp ? A.mp + p * A.kp_pitch : nullptr;
  const uint8_t* mpB = B.mp ? B.mp + p * B.kp_pitch : nullptr;
  const uint32_t* nodesA = A.nodes + p * A.node_pitch;
  const uint32_t* nodesB = B.nodes + p * B.node_pitch;
  const int* offA = A.off + p * (A.node_pitch + 1);
  const int* offB = B.off + p * (B.node_pitch + 1);
  const int* idxA = A.idx + p * A.node_pitch;
  const int* idxB = B.idx + p * B.node_pitch;
  int* rec = rec_all + p * out_pitch;
  int* hist = hist_all + p * 32;
  if (nk <= 0) return;
  // feature indices come from device CSR arrays the host cannot check: an
  // index outside [0, min(n, kp_pitch)) is not a candidate and sets status
  // bit 32 (it would address the next pair's rows or past the buffers)
  // (a side's pitch is 0 for the single-pair host entry; out rows are indexed by
  // the A feature for KF-KF and by the B feature for KF-F)
  auto extent = [&](const BowSide& X, bool out_side) {
    long long e = X.n[p];
    if (X.kp_pitch > 0) e = min(e, X.kp_pitch);
    if (out_side) e = min(e, out_pitch);
    return (int)e;
  };
  const int nAp = extent(A, kf_vs_kf), nBp = extent(B, !kf_vs_kf);
  if (tid == 0 && g == 0 && (A.n[p] > nAp || B.n[p] > nBp)) atomicOr(err, 32);
  auto in_a = [&](int i) {
    const bool ok = (unsigned)i < (unsigned)nAp;
    if (!ok) atomicOr(err, 32);
    return ok;
  };
  auto in_b = [&](int i) {
    const bool ok = (unsigned)i < (unsigned)nBp;
    if (!ok) atomicOr(err, 32);
    return ok;
  };
  const float factor = 1.0f / kHistoLength;
  // an accepted match: output, the pair's count and rotation histogram
  auto accept = [&](int idx1, int bestIdx2, int* h) {
    int bin = 0;
    atomicAdd(&h[30], 1);
    if (check_ori) {
      float rot = __fsub_rn(angA[(long long)idx1 * A.angle_stride], angB[(long long)bestIdx2 * B.angle_stride]);
      if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
      bin = (int)roundf(__fmul_rn(rot, factor));
      if (bin == kHistoLength) bin = 0;
      atomicAdd(&h[bin], 1);
    }
    if (kf_vs_kf) rec[idx1] = bin << 16 | bestIdx2;
    else rec[bestIdx2] = bin << 16 | idx1;
  };
  // lower_bound of a node id in B's node list (the lock-step walk of :180-264
  // meets exactly the shared ids); -1 when B lacks it
  auto find_b = [&](uint32_t id) {
    int lo = 0, hi = nnB;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (nodesB[mid] < id) lo = mid + 1;
      else hi = mid;
    }
    return (lo < nnB && nodesB[lo] == id) ? lo : -1;
  };
  const int a_base = offA[k0], na = offA[k1] - a_base;

  // ---- node table: B node per A node, staged B offsets (block scan of counts)
  bool fits = nk <= kBowCapN && na <= kBowCapA;
  if (fits) {
    // B's node list in LDS (the claim table is free until the greedy rounds):
    // the per-node lower_bound then waits on LDS, not on ~7 dependent global loads
    const bool nodes_lds = nnB <= kBowCapB;
    uint32_t* const snb = (uint32_t*)S.t.claim;
    if (nodes_lds)
      for (int i = tid; i < nnB; i += NT) snb[i] = nodesB[i];
    __syncthreads();
    auto find_b_lds = [&](uint32_t id) {
      int lo = 0, hi = nnB;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (snb[mid] < id) lo = mid + 1;
        else hi = mid;
      }
      return (lo < nnB && snb[lo] == id) ? lo : -1;
    };
    int carry = 0;
    for (int j0 = 0; j0 < nk; j0 += NT) {
      const int j = j0 + tid;
      int cnt = 0, src = 0;
      if (j < nk) {
        const uint32_t id = nodesA[k0 + j];
        const int kb = nodes_lds ? find_b_lds(id) : find_b(id);
        if (kb >= 0) {
          src = offB[kb];
          cnt = offB[kb + 1] - src;
        }
        S.t.bsrc[j] = src;
        S.t.aoff[j + 1] = offA[k0 + j + 1] - a_base;
      }
      const int incl = wave_incl_scan_dpp(cnt);
      if (lane == 63) s_scan[wv] = incl;
      __syncthreads();
      int before = carry;
      for (int w = 0; w < wv; ++w) before += s_scan[w];
      if (j < nk) S.t.boff[j + 1] = before + incl;
      int tot = 0;
      for (int w = 0; w < kWaves; ++w) tot += s_scan[w];
      carry += tot;
      __syncthreads();
    }
    if (tid == 0) S.t.boff[0] = S.t.aoff[0] = 0;
    fits = carry <= kBowCapB;  // uniform
  }
  stamp(1, -1);
  if (fits) {
    __syncthreads();
    const int nb = S.t.boff[nk];
    for (int i = tid; i < kBowCapB / 32; i += NT) S.t.taken[i] = 0;
    // the range's A feature indices (phase (1) then needs one dependent global load, not two)
    for (int i = tid; i < na; i += NT) S.t.match[i] = idxA[a_base + i];
    // ---- stage the range's B rows in node order (static filter: KF-KF needs a good MapPoint)
    for (int i = tid; i < nb; i += NT) {
      int lo = 0, hi = nk;  // node j with boff[j] <= i < boff[j+1]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (S.t.boff[mid] <= i) lo = mid;
        else hi = mid;
      }
      int i2 = idxB[S.t.bsrc[lo] + (i - S.t.boff[lo])];
      bool ok = in_b(i2);
      if (!ok) i2 = 0;
      ok = ok && (!kf_vs_kf || !mpB || mpB[i2] != 0);
      const uint4* d2 = (const uint4*)(descB + (long long)i2 * 32);
      const uint4 v0 = d2[0], v1 = d2[1];
      *(uint4*)&S.t.bdesc[i][0] = v0;
      *(uint4*)&S.t.bdesc[i][4] = v1;
      S.t.bidx[i] = ok ? i2 : -1;
    }
    __syncthreads();
    stamp(2, -1);
    // ---- (1) per A row, its kBowK smallest keys over the node's candidates.
    // A row of a node with nb B rows gets L = 1, 2, 4 or 8 adjacent lanes
    // (nb > 48, 96, 192), each scanning every L-th candidate; the L sorted
    // lists then merge by xor shuffles. Without the split one lane walks all
    // nb candidates and the largest node sets the workgroup's time. Lane
    // slots: nodes ordered by L descending (node order within), each row's L
    // slots contiguous and L-aligned (every block before has a multiple of
    // L slots).
    auto lanes_of = [](int nbn) { return nbn > 192 ? 8 : nbn > 96 ? 4 : nbn > 48 ? 2 : 1; };
    int nslots = 0;
    {
      int base = 0, rank0 = 0;  // slots and nodes of the classes before
      for (int Lc = 8; Lc >= 1; Lc >>= 1) {
        int carry = 0;
        for (int j0 = 0; j0 < nk; j0 += NT) {
          const int j = j0 + tid;
          const bool mine = j < nk && lanes_of(S.t.boff[j + 1] - S.t.boff[j]) == Lc;
          const int sz = mine ? (S.t.aoff[j + 1] - S.t.aoff[j]) * Lc : 0;
          const uint64_t bm = __ballot(mine);
          const int incl = wave_incl_scan_dpp(sz);
          if (lane == 63) s_scan[wv] = incl;
          if (lane == 0) s_hist[wv] = __popcll(bm);
          __syncthreads();
          int before = carry, rb = rank0;
          for (int w = 0; w < wv; ++w) {
            before += s_scan[w];
            rb += s_hist[w];
          }
          if (mine) {
            const int k = rb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
            S.t.sstart[k] = base + before + incl - sz;
            S.t.snode[k] = j;
          }
          for (int w = 0; w < kWaves; ++w) {
            carry += s_scan[w];
            rank0 += s_hist[w];
          }
          __syncthreads();
        }
        base += carry;
      }
      nslots = base;
      if (tid == 0) S.t.sstart[nk] = nslots;
    }
    __syncthreads();
    for (int s0 = 0; s0 < nslots; s0 += NT) {  // uniform trip count: the shuffles below see every lane
      const int sl = s0 + tid;
      const bool act = sl < nslots;
      int lo = 0, hi = nk;  // slot-order node k with sstart[k] <= sl < sstart[k+1]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (S.t.sstart[mid] <= min(sl, nslots - 1)) lo = mid;
        else hi = mid;
      }
      const int j = min(max(S.t.snode[lo], 0), nk - 1);  // (every rank is written; the clamp guards the indexing)
      const int q0 = S.t.boff[j], q1 = S.t.boff[j + 1];
      const int L = lanes_of(q1 - q0), rel = min(sl, nslots - 1) - S.t.sstart[lo];
      const int ia = S.t.aoff[j] + rel / L, sub = rel & (L - 1);
      const int i1 = S.t.match[ia];  // idxA[a_base + ia], staged
      uint32_t t0 = kBowNone, t1 = kBowNone, t2 = kBowNone, t3 = kBowNone;
      uint32_t t4 = kBowNone, t5 = kBowNone, t6 = kBowNone, t7 = kBowNone;
      int nv = -1;
      if (act && in_a(i1) && (!mpA || mpA[i1])) {  // (:191-197)
        nv = 0;
        const uint4* d1 = (const uint4*)(descA + (long long)i1 * 32);
        const uint4 a0 = d1[0], a1 = d1[1];
        auto insert = [&](uint32_t key) {  // into the ascending t0..t7
          uint32_t m;
          m = min(t0, key); key = max(t0, key); t0 = m;
          m = min(t1, key); key = max(t1, key); t1 = m;
          m = min(t2, key); key = max(t2, key); t2 = m;
          m = min(t3, key); key = max(t3, key); t3 = m;
          m = min(t4, key); key = max(t4, key); t4 = m;
          m = min(t5, key); key = max(t5, key); t5 = m;
          m = min(t6, key); key = max(t6, key); t6 = m;
          t7 = min(t7, key);
        };
        // two candidates per step: their LDS reads are in flight together
        int q = q0 + sub;
        for (; q + L < q1; q += 2 * L) {
          const int okA = S.t.bidx[q], okB = S.t.bidx[q + L];
          const uint4 b0 = *(const uint4*)&S.t.bdesc[q][0], b1 = *(const uint4*)&S.t.bdesc[q][4];
          const uint4 c0 = *(const uint4*)&S.t.bdesc[q + L][0], c1 = *(const uint4*)&S.t.bdesc[q + L][4];
          const uint32_t kA = ((uint32_t)hamming256(a0, a1, b0, b1) << 16) | (uint32_t)(q - q0);
          const uint32_t kB = ((uint32_t)hamming256(a0, a1, c0, c1) << 16) | (uint32_t)(q + L - q0);
          if (okA >= 0) insert(kA), ++nv;
          if (okB >= 0) insert(kB), ++nv;
        }
        if (q < q1 && S.t.bidx[q] >= 0) {
          ++nv;
          insert(((uint32_t)hamming256(a0, a1, *(const uint4*)&S.t.bdesc[q][0], *(const uint4*)&S.t.bdesc[q][4]) << 16) |
                 (uint32_t)(q - q0));
        }
      }
      // merge the row's L lists: with the partner's list reversed, the
      // elementwise minima are the 8 smallest of the union as a bitonic
      // sequence, sorted by three half-cleaner stages (both partners end with
      // the same list; keys are unique, so the merge is exact)
      for (int st = 1; st < 8; st <<= 1) {
        if (!__ballot(act && L > st)) break;  // wave-uniform
        const uint32_t u0 = __shfl_xor(t0, st), u1 = __shfl_xor(t1, st), u2 = __shfl_xor(t2, st);
        const uint32_t u3 = __shfl_xor(t3, st), u4 = __shfl_xor(t4, st), u5 = __shfl_xor(t5, st);
        const uint32_t u6 = __shfl_xor(t6, st), u7 = __shfl_xor(t7, st);
        const int unv = __shfl_xor(nv, st);
        if (L > st) {
          uint32_t m[8] = {min(t0, u7), min(t1, u6), min(t2, u5), min(t3, u4),
                           min(t4, u3), min(t5, u2), min(t6, u1), min(t7, u0)};
#pragma unroll
          for (int h = 4; h >= 1; h >>= 1)
#pragma unroll
            for (int i = 0; i < 8; ++i)
              if ((i & h) == 0) {
                const uint32_t x = m[i], y = m[i + h];
                m[i] = min(x, y);
                m[i + h] = max(x, y);
              }
          t0 = m[0]; t1 = m[1]; t2 = m[2]; t3 = m[3]; t4 = m[4]; t5 = m[5]; t6 = m[6]; t7 = m[7];
          nv = (nv < 0 || unv < 0) ? -1 : nv + unv;  // the row's lanes agree on validity
        }
      }
      if (act && sub == 0) {
        S.t.top[ia][0] = make_uint4(t0, t1, t2, t3);
        S.t.top[ia][1] = make_uint4(t4, t5, t6, t7);
        S.t.nv[ia] = nv;
        S.t.rq[ia] = q0 | (q1 << 16);
      }
    }
    __syncthreads();
    stamp(3, -1);
    // ---- (2) the greedy pass as a fixed point (Jacobi rounds). Row i's
    // decision depends only on which of its candidates earlier rows of its
    // node took; every round recomputes all rows in parallel from the previous
    // round's choices (a position counts as taken for row i when a row before
    // i chose it: claim = the first such row). Row 1 of a node is right in
    // round 0 and row i by round i - 1, and a round without changes is the
    // unique fixed point = the sequential result, so the rounds stop there.
    // Rows with a decision changing after max_rounds rounds fall back to the
    // sequential pass below.
    auto decide = [&](int ia, auto&& taken, bool defer = false) -> int {  // staged position, -1, or -2 = deferred rescan
      const int nv = S.t.nv[ia];
      if (nv < 0) return -1;
      const int rq = S.t.rq[ia], q0 = rq & 0xFFFF, q1 = rq >> 16;
      if (q0 == q1) return -1;
      const uint4 tA = S.t.top[ia][0], tB = S.t.top[ia][1];
      const uint32_t keys[kBowK] = {tA.x, tA.y, tA.z, tA.w, tB.x, tB.y, tB.z, tB.w};
      int d1 = 256, d2 = 256, p1 = -1, found = 0;
#pragma unroll
      for (int k = 0; k < kBowK; ++k) {
        const uint32_t key = keys[k];
        if (key == kBowNone || found == 2 || taken(ia, q0 + (int)(key & 0xFFFF))) continue;
        if (found == 0) {
          d1 = (int)(key >> 16);
          p1 = q0 + (int)(key & 0xFFFF);
        } else {
          d2 = (int)(key >> 16);
        }
        ++found;
      }
      if (found < 2 && nv > kBowK) {
        if (defer) return -2;
        // the list ran out under taken rows: rescan the node (strict < of :211-226)
        const int i1 = idxA[a_base + ia];
        const uint4* da = (const uint4*)(descA + (long long)i1 * 32);
        const uint4 a0 = da[0], a1 = da[1];
        d1 = 256;
        d2 = 256;
        p1 = -1;
        for (int q = q0; q < q1; ++q) {
          if (S.t.bidx[q] < 0 || taken(ia, q)) continue;
          const int dist = hamming256(a0, a1, *(const uint4*)&S.t.bdesc[q][0], *(const uint4*)&S.t.bdesc[q][4]);
          if (dist < d1) {
            d2 = d1;
            d1 = dist;
            p1 = q;
          } else if (dist < d2) {
            d2 = dist;
          }
        }
      }
      // d1 = 256 never passes; with d1 < 256 the reference's bestIdx is set
      const bool pass = kf_vs_kf ? (d1 < kThLow) : (d1 <= kThLow);
      return (pass && (float)d1 < __fmul_rn(nnratio, (float)min(d2, 256))) ? p1 : -1;
    };
    const int nb_ = S.t.boff[nk];
    for (int ia = tid; ia < na; ia += NT) S.t.match[ia] = decide(ia, [](int, int) { return false; });
    bool settled = false;
    int rounds = 0;
    for (int round = 0; round < max_rounds && !settled; ++round) {
      ++rounds;
      for (int q = tid; q < nb_; q += NT) S.t.claim[q] = INT_MAX;
      if (tid == 0) s_queue = 0;
      __syncthreads();
      for (int ia = tid; ia < na; ia += NT) {
        const int q = S.t.match[ia];
        if (q >= 0) atomicMin(&S.t.claim[q], ia);
      }
      __syncthreads();
      int changed = 0;
      for (int ia = tid; ia < na; ia += NT) {
        const int m = decide(ia, [&](int row, int q) { return S.t.claim[q] < row; }, true);
        if (m == -2) {
          S.t.rescan[atomicAdd(&s_queue, 1)] = ia;
        } else if (m != S.t.match[ia]) {
          S.t.match[ia] = m;
          changed = 1;
        }
      }
      __syncthreads();
      // rows whose list ran out: a wave per row, lanes over the node's
      // candidates (taken = claimed by an earlier row), two wave minima
      const int nq = s_queue;
      for (int qi = wv; qi < nq; qi += kWaves) {
        const int ia = S.t.rescan[qi];
        const int rq = S.t.rq[ia], q0 = rq & 0xFFFF, q1 = rq >> 16;
        const int i1 = idxA[a_base + ia];
        const uint4* da = (const uint4*)(descA + (long long)i1 * 32);
        const uint4 a0 = da[0], a1 = da[1];
        uint32_t b1k = 0x7FFFFFFFu, b2k = 0x7FFFFFFFu;
        for (int q = q0 + lane; q < q1; q += 64) {
          if (S.t.bidx[q] < 0 || S.t.claim[q] < ia) continue;
          const uint32_t k = ((uint32_t)hamming256(a0, a1, *(const uint4*)&S.t.bdesc[q][0],
                                                   *(const uint4*)&S.t.bdesc[q][4]) << 16) | (uint32_t)(q - q0);
          b2k = min(b2k, max(b1k, k));
          b1k = min(b1k, k);
        }
        const uint32_t m1 = (uint32_t)wave_min((int)b1k);  // keys < 2^25
        const uint32_t m2 = (uint32_t)wave_min((int)(b1k == m1 ? b2k : b1k));
        const int d1 = m1 == 0x7FFFFFFFu ? 256 : (int)(m1 >> 16);
        const int d2 = m2 == 0x7FFFFFFFu ? 256 : (int)(m2 >> 16);
        const bool pass = kf_vs_kf ? (d1 < kThLow) : (d1 <= kThLow);
        const int m = (pass && (float)d1 < __fmul_rn(nnratio, (float)min(d2, 256))) ? q0 + (int)(m1 & 0xFFFF) : -1;
        if (lane == 0 && m != S.t.match[ia]) {
          S.t.match[ia] = m;
          changed = 1;
        }
      }
      settled = !__syncthreads_or(changed);
    }
    if (settled) {
      for (int ia = tid; ia < na; ia += NT) S.t.nv[ia] = S.t.match[ia];
    } else {
      // sequential: a wave per node, A rows in node order. The node's taken
      // set is wave-uniform: four 64-bit masks (positions < 256 in the node;
      // larger nodes use the LDS bits for the rest). Lane k < 8 checks key k
      // of the row's list, a ballot gives the first two untaken keys, and the
      // next row's key is read while the current one is decided. A row whose
      // list ran out (fewer than two untaken keys left while it saw more than
      // kBowK candidates) rescans its node: lanes over the candidates, two
      // wave minima.
      for (int j = wv; j < nk; j += kWaves) {
        const int q0 = S.t.boff[j], q1 = S.t.boff[j + 1];
        const int r0 = S.t.aoff[j], r1 = S.t.aoff[j + 1];
        if (q0 == q1) {  // node absent from B (or empty)
          for (int ia = r0 + lane; ia < r1; ia += 64) S.t.nv[ia] = -1;
          continue;
        }
        uint64_t tk[4] = {0, 0, 0, 0};  // taken node positions 0..255 (uniform)
        auto is_taken = [&](int r) -> bool {  // r: position in the node (per lane)
          if (r < 256) {
            const uint64_t m = r < 128 ? (r < 64 ? tk[0] : tk[1]) : (r < 192 ? tk[2] : tk[3]);
            return (m >> (r & 63)) & 1ull;
          }
          const int q = q0 + r;
          return (S.t.taken[q >> 5] >> (q & 31)) & 1u;
        };
        uint32_t key_n = lane < kBowK ? ((const uint32_t*)S.t.top[r0])[lane] : kBowNone;
        int nv_n = S.t.nv[r0];
        for (int ia = r0; ia < r1; ++ia) {
          const uint32_t key = key_n;
          const int nv = nv_n;  // uniform
          if (ia + 1 < r1) {
            key_n = lane < kBowK ? ((const uint32_t*)S.t.top[ia + 1])[lane] : kBowNone;
            nv_n = S.t.nv[ia + 1];
          }
          int res = -1;
          if (nv >= 0) {
            const bool ok = key != kBowNone && !is_taken((int)(key & 0xFFFF));
            const uint64_t bm = __ballot(ok);
            int d1 = 256, d2 = 256, r1st = -1;
            if (bm) {
              const uint32_t k1 = (uint32_t)__builtin_amdgcn_readlane((int)key, __ffsll((long long)bm) - 1);
              d1 = (int)(k1 >> 16);
              r1st = (int)(k1 & 0xFFFF);
              const uint64_t bm2 = bm & (bm - 1);
              if (bm2) d2 = (int)((uint32_t)__builtin_amdgcn_readlane((int)key, __ffsll((long long)bm2) - 1) >> 16);
            }
            if (__popcll(bm) < 2 && nv > kBowK) {
              // the list ran out under taken rows: rescan the node (strict < of :211-226)
              const int i1 = idxA[a_base + ia];
              const uint4* da = (const uint4*)(descA + (long long)i1 * 32);
              const uint4 a0 = da[0], a1 = da[1];
              uint32_t b1k = 0x7FFFFFFFu, b2k = 0x7FFFFFFFu;  // the lane's two smallest keys
              for (int r = lane; r < q1 - q0; r += 64) {
                if (S.t.bidx[q0 + r] < 0 || is_taken(r)) continue;
                const uint32_t k = ((uint32_t)hamming256(a0, a1, *(const uint4*)&S.t.bdesc[q0 + r][0],
                                                         *(const uint4*)&S.t.bdesc[q0 + r][4]) << 16) | (uint32_t)r;
                b2k = min(b2k, max(b1k, k));
                b1k = min(b1k, k);
              }
              // keys < 2^25: the signed DPP minimum orders them
              const uint32_t m1 = (uint32_t)wave_min((int)b1k);
              const uint32_t m2 = (uint32_t)wave_min((int)(b1k == m1 ? b2k : b1k));
              d1 = m1 == 0x7FFFFFFFu ? 256 : (int)(m1 >> 16);
              d2 = m2 == 0x7FFFFFFFu ? 256 : (int)(m2 >> 16);
              r1st = m1 == 0x7FFFFFFFu ? -1 : (int)(m1 & 0xFFFF);
            }
            // d1 = 256 never passes; with d1 < 256 the reference's bestIdx is set
            const bool pass = kf_vs_kf ? (d1 < kThLow) : (d1 <= kThLow);
            if (pass && (float)d1 < __fmul_rn(nnratio, (float)min(d2, 256))) {
              res = q0 + r1st;
              if (r1st < 256) {
                const uint64_t bit = 1ull << (r1st & 63);
                tk[0] |= r1st < 64 ? bit : 0ull;
                tk[1] |= (r1st >> 6) == 1 ? bit : 0ull;
                tk[2] |= (r1st >> 6) == 2 ? bit : 0ull;
                tk[3] |= (r1st >> 6) == 3 ? bit : 0ull;
              } else if (lane == 0) {
                atomicOr(&S.t.taken[res >> 5], 1u << (res & 31));  // words shared with other waves' nodes
              }
            }
          }
          if (lane == 0) S.t.nv[ia] = res;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
        }
      }
    }
    __syncthreads();
    stamp(4, -1);
    // ---- the accepted matches: outputs, then count and rotation histogram
    // summed in LDS first (one global atomic per bin per workgroup)
    if (tid < 32) s_hist[tid] = 0;
    __syncthreads();
    for (int ia = tid; ia < na; ia += NT) {
      const int q = S.t.nv[ia];
      if (q >= 0) accept(idxA[a_base + ia], S.t.bidx[q], s_hist);
    }
    __syncthreads();
    if (tid < 32 && s_hist[tid]) atomicAdd(&hist[tid], s_hist[tid]);
    if (dbg) {
      __syncthreads();
      stamp(0, -1);
      stamp(5, nk + 1000 * (settled ? rounds : 99));  // diagnostics: nodes + 1000 x rounds (99: sequential)
      stamp(6, na);
      stamp(7, S.t.boff[nk]);
    }
    return;
  }

  // ---- fallback: a wave per node through a queue, best/second reduced across lanes
  stamp(5, -nk);
  __syncthreads();
  volatile uint32_t* s_taken = S.f.taken;
  for (int i = tid; i < 2048; i += NT) S.f.taken[i] = 0;
  if (tid == 0) s_queue = 0;
  __syncthreads();
  for (;;) {
    int qi = 0;
    if (lane == 0) qi = atomicAdd(&s_queue, 1);
    const int ka = k0 + __builtin_amdgcn_readfirstlane(qi);
    if (ka >= k1) break;
    const int lo = find_b(nodesA[ka]);
    if (lo < 0) continue;
    const int b0 = offB[lo], b1 = offB[lo + 1];
    const int a0i = offA[ka], a1i = offA[ka + 1];
    const int nbn = b1 - b0;
    if (nbn <= kBowMaxB) {
      // the node's B descriptors in registers (lane l holds positions l, l+64,
      // ...), A descriptors staged 64 at a time in LDS and read back as
      // broadcasts: the greedy loop over A waits on no global load
      constexpr int kC = kBowMaxB / 64;
      uint4 q0[kC], q1[kC];
      int bidx[kC];
      bool bok[kC];
#pragma unroll
      for (int c = 0; c < kC; ++c) {
        const int pos = c * 64 + lane;
        bidx[c] = -1;
        bok[c] = false;
        q0[c] = q1[c] = make_uint4(0, 0, 0, 0);
        if (pos < nbn) {
          int i2 = idxB[b0 + pos];
          if (!in_b(i2)) i2 = -1;
          bidx[c] = i2;
          bok[c] = i2 >= 0 && (!kf_vs_kf || !mpB || mpB[i2] != 0);
          if (i2 < 0) i2 = 0;
          const uint4* d2 = (const uint4*)(descB + (long long)i2 * 32);
          q0[c] = d2[0];
          q1[c] = d2[1];
          S.f.bidx[wv][pos] = bidx[c];
        }
      }
      for (int ac = a0i; ac < a1i; ac += 64) {
        const int nan_ = min(64, a1i - ac);
        __builtin_amdgcn_wave_barrier();
        if (lane < nan_) {
          int i1 = idxA[ac + lane];
          const bool in = in_a(i1);
          if (!in) i1 = 0;
          const bool ok = in && (!mpA || mpA[i1]);
          const uint4* d1 = (const uint4*)(descA + (long long)i1 * 32);
          const uint4 v0 = d1[0], v1 = d1[1];
          uint32_t* w = S.f.adesc[wv][lane];
          w[0] = v0.x; w[1] = v0.y; w[2] = v0.z; w[3] = v0.w;
          w[4] = v1.x; w[5] = v1.y; w[6] = v1.z; w[7] = v1.w;
          S.f.aidx[wv][lane] = ok ? i1 : -1;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int i = 0; i < nan_; ++i) {
          const int idx1 = S.f.aidx[wv][i];
          if (idx1 < 0) continue;  // (:191-197) uniform
          const uint32_t* w = S.f.adesc[wv][i];
          const uint4 a0 = make_uint4(w[0], w[1], w[2], w[3]), a1 = make_uint4(w[4], w[5], w[6], w[7]);
          // per lane the two smallest (distance << 16 | position) keys over its
          // chunks, then the wave's: position order = the node vector's order,
          // so equal distances resolve to the earlier candidate as in :211-226
          uint32_t k1 = 0x7FFFFFFFu, k2 = 0x7FFFFFFFu;
#pragma unroll
          for (int c = 0; c < kC; ++c) {
            if (c * 64 >= nbn) break;  // uniform
            const int i2 = bidx[c];
            const bool valid = i2 >= 0 && bok[c] && !((s_taken[i2 >> 5] >> (i2 & 31)) & 1u);
            if (valid) {
              const uint32_t key = ((uint32_t)hamming256(a0, a1, q0[c], q1[c]) << 16) | (uint32_t)(c * 64 + lane);
              k2 = min(k2, max(k1, key));
              k1 = min(k1, key);
            }
          }
          const uint32_t m1 = (uint32_t)wave_min((int)k1);
          const uint32_t m2 = (uint32_t)wave_min((int)(k1 == m1 ? k2 : k1));
          // merged with the initial best = second = 256 of the reference loop
          const int d1 = m1 == 0x7FFFFFFFu ? 256 : min((int)(m1 >> 16), 256);
          const int d2 = m2 == 0x7FFFFFFFu ? 256 : min((int)(m2 >> 16), 256);
          const bool pass = kf_vs_kf ? (d1 < kThLow) : (d1 <= kThLow);
          if (pass && (float)d1 < __fmul_rn(nnratio, (float)d2)) {
            if (lane == 0) {
              const int i2 = S.f.bidx[wv][m1 & 0xFFFF];
              atomicOr((unsigned*)&s_taken[i2 >> 5], 1u << (i2 & 31));
              accept(idx1, i2, hist);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
          }
        }
      }
      continue;
    }
    // very large nodes: candidates streamed from global memory 64 at a time
    for (int pa = a0i; pa < a1i; ++pa) {
      const int idx1 = idxA[pa];
      if (!in_a(idx1) || (mpA && !mpA[idx1])) continue;
      const uint4* d1 = (const uint4*)(descA + (long long)idx1 * 32);
      const uint4 a0 = d1[0], a1 = d1[1];
      Top2 acc{256, -1, 256};
      for (int q0 = b0; q0 < b1; q0 += 64) {
        const int q = q0 + lane;
        bool valid = false;
        int dist = 0, idx2 = -1;
        if (q < b1 && in_b(idxB[q])) {
          idx2 = idxB[q];
          const bool taken = (s_taken[idx2 >> 5] >> (idx2 & 31)) & 1u;
          valid = !taken && (!kf_vs_kf || !mpB || mpB[idx2] != 0);
          if (valid) {
            const uint4* d2 = (const uint4*)(descB + (long long)idx2 * 32);
            dist = hamming256(a0, a1, d2[0], d2[1]);
          }
        }
        const Top2 t = wave_top2(valid, dist, idx2);
        if (t.best < acc.best) {
          acc.second = min(acc.best, t.second);
          acc.best = t.best;
          acc.pos = t.pos;
        } else {
          acc.second = min(acc.second, t.best);
        }
      }
      const bool pass = kf_vs_kf ? (acc.best < kThLow) : (acc.best <= kThLow);
      if (pass && (float)acc.best < __fmul_rn(nnratio, (float)acc.second)) {
        if (lane == 0) {
          atomicOr((unsigned*)&s_taken[acc.pos >> 5], 1u << (acc.pos & 31));
          accept(idx1, acc.pos, hist);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
}

// Rotation consistency (src/ORBmatcher.cc:267-285, ComputeThreeMaxima :1601-1642)
// and the final count, one workgroup per pair: `out` rows from the row
// records (-1 for rows without a match, past the pair's extent, or whose bin
// is not one of the three maxima), then the records and the histogram go back
// to -1 / 0 for the next call.
__global__ __launch_bounds__(256) void search_bow_finalize_kernel(int check_ori, int* __restrict__ out_all,
                                                                  long long out_pitch, int* __restrict__ rec_all,
                                                                  int* __restrict__ hist_all, int* __restrict__ nmatches) {
  __shared__ int s_var[4];
  const int p = blockIdx.x, tid = threadIdx.x;
  int* hist = hist_all + p * 32;
  int count = 0;
  if (tid == 0) {
    count = hist[30];
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    if (check_ori) {
      for (int i = 0; i < kHistoLength; i++) {
        const int s = hist[i];
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
    }
    s_var[0] = ind1;
    s_var[1] = ind2;
    s_var[2] = ind3;
    s_var[3] = 0;
  }
  __syncthreads();
  if (tid < 32) hist[tid] = 0;
  const int ind1 = s_var[0], ind2 = s_var[1], ind3 = s_var[2];
  int* out = out_all + p * out_pitch;
  int* rec = rec_all + p * out_pitch;
  int removed = 0;
  for (long long i = tid; i < out_pitch; i += 256) {
    const int v = rec[i];
    int o = -1;
    if (v >= 0) {
      rec[i] = -1;
      const int b = v >> 16;
      if (!check_ori || b == ind1 || b == ind2 || b == ind3) o = v & 0xFFFF;
      else ++removed;
    }
    out[i] = o;
  }
  if (removed) atomicAdd(&s_var[3], removed);
  __syncthreads();
  if (tid == 0) nmatches[p] = count - s_var[3];
}

// rec_scratch / hist_scratch: the row records (all -1) and histograms (all 0)
// between calls when *clean; otherwise their first rec_ints / hist_ints (the
// whole buffers, so that a later call with more pairs or a wider pitch also
// finds them clean) are filled first. *clean is false from the search launch
// until its finalize is queued.
int launch_search_bow(const BowSide& A, const BowSide& B, int pairs, float nnratio, int check_ori, int kf_vs_kf,
                      int* out, long long out_pitch, int* nmatches, int* rec_scratch, size_t rec_ints,
                      int* hist_scratch, size_t hist_ints, bool* clean, int* err, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if ((size_t)pairs * out_pitch > rec_ints || (size_t)pairs * 32 > hist_ints) return ORBX_ECAPACITY;
  if (!*clean && (hipMemsetAsync(rec_scratch, 0xFF, rec_ints * 4, s) != hipSuccess ||
                  hipMemsetAsync(hist_scratch, 0, hist_ints * 4, s) != hipSuccess))
    return ORBX_EDEVICE;
  *clean = false;
  static int* dbg = nullptr;  // diagnostics only: per-workgroup phase cycles (ORBX_BOW_PROF=1)
  static const bool prof = getenv("ORBX_BOW_PROF") && getenv("ORBX_BOW_PROF")[0] == '1';
  const int nwg = pairs * kBowGroups;
  const char* rs = getenv("ORBX_BOW_ROUNDS");  // read per call (tests force the sequential pass with 0)
  const int rounds = rs ? std::max(0, std::min(atoi(rs), 1 << 16)) : kBowRounds;
  if (prof && !dbg) (void)hipMalloc(&dbg, (size_t)65536 * 32);
  if (prof) (void)hipMemsetAsync(dbg, 0, (size_t)nwg * 32, s);
  hipLaunchKernelGGL(search_bow_kernel<kBowThreads>, dim3(nwg), dim3(kBowThreads), 0, s, A, B, nnratio,
                     check_ori, kf_vs_kf, kBowGroups, rounds, out_pitch, rec_scratch, hist_scratch, err,
                     prof ? dbg : nullptr);
  if (prof) {
    std::vector<int> h((size_t)nwg * 8);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), dbg, h.size() * 4, hipMemcpyDeviceToHost);
    double t[8] = {0}, mx[8] = {0};
    int nfb = 0, nseq = 0, rsum = 0;
    for (int w = 0; w < nwg; ++w) {
      if (h[w * 8 + 5] < 0) ++nfb;
      if (h[w * 8 + 5] >= 0) {  // nodes + 1000 x rounds
        const int rd = h[w * 8 + 5] / 1000;
        nseq += rd == 99;
        rsum += rd == 99 ? 0 : rd;
        h[w * 8 + 5] %= 1000;
      }
      for (int k = 0; k < 8; ++k) t[k] += h[w * 8 + k], mx[k] = std::max(mx[k], (double)h[w * 8 + k]);
    }
    fprintf(stderr, "bow: %d WGs sequential greedy, the others settled in %.1f rounds on average\n", nseq,
            nwg > nseq ? (double)rsum / (nwg - nseq) : 0.0);
    fprintf(stderr, "bow: %d WGs (%d fallback); avg/max cycles at: table %.0f/%.0f staged %.0f/%.0f top %.0f/%.0f greedy %.0f/%.0f end %.0f/%.0f; avg nodes %.1f rows A %.1f B %.1f\n",
            nwg, nfb, t[1] / nwg, mx[1], t[2] / nwg, mx[2], t[3] / nwg, mx[3], t[4] / nwg, mx[4], t[0] / nwg, mx[0], t[5] / nwg, t[6] / nwg, t[7] / nwg);
    // the slowest workgroups: phase ends, nodes, A rows, B rows, and the pair's group index
    std::vector<int> order(nwg);
    for (int w = 0; w < nwg; ++w) order[w] = w;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return h[a * 8] > h[b * 8]; });
    for (int r = 0; r < std::min(nwg, 8); ++r) {
      const int w = order[r];
      fprintf(stderr, "bow slow[%d]: wg %d (pair %d group %d) table %d staged %d top %d greedy %d end %d; nodes %d A %d B %d\n",
              r, w, w / kBowGroups, w % kBowGroups, h[w * 8 + 1], h[w * 8 + 2], h[w * 8 + 3], h[w * 8 + 4], h[w * 8], h[w * 8 + 5],
              h[w * 8 + 6], h[w * 8 + 7]);
    }
  }
  hipLaunchKernelGGL(search_bow_finalize_kernel, dim3(pairs), dim3(256), 0, s, check_ori, out, out_pitch, rec_scratch,
                     hist_scratch, nmatches);
  if (hipGetLastError() != hipSuccess) return ORBX_EDEVICE;
  *clean = true;
  return ORBX_OK;
}

// ------------------------------------------------------------ launchers
int launch_hamming_top2(const uint8_t* A, size_t a_pitch, const int* nA, int a_cap, const uint8_t* B,
                        size_t b_pitch, const int* nB, int pairs, int* best_idx, int* best, int* second,
                        int* err, void* stream) {
  // ORBX_TOP2_VALU=1 selects the VALU kernel (A/B timing and the cross-check
  // in tests/test_gpu_match.py; read per call so a test can switch it)
  const char* ev = getenv("ORBX_TOP2_VALU");
  const bool valu = ev && ev[0] == '1';
  if (!valu) {
    dim3 grid((a_cap + kMQueries - 1) / kMQueries, pairs);
    hipLaunchKernelGGL(hamming_top2_mfma_kernel, grid, dim3(kMThreads), 0, (hipStream_t)stream, A, (long long)a_pitch,
                       nA, a_cap, B, (long long)b_pitch, nB, best_idx, best, second, err);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
  }
  dim3 grid((a_cap + kTopQueries - 1) / kTopQueries, pairs);
  hipLaunchKernelGGL(hamming_top2_kernel, grid, dim3(kTopThreads), 0, (hipStream_t)stream, A, (long long)a_pitch, nA, a_cap,
                     B, (long long)b_pitch, nB, best_idx, best, second, err);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}


}  // namespace orbx

// ============================================================ C ABI (matcher)
using namespace orbx;

namespace {
thread_local std::string g_merr;
int mfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_merr = buf;
  return code;
}
}  // namespace

extern "C" const char* orbm_last_error(void) { return g_merr.c_str(); }

#define MHIP(expr)                                                                             \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return mfail(ORBX_EDEVICE, "%s: %s", #expr, hipGetErrorString(e_));  \
  } while (0)

struct orbx_matcher {
  int device = 0, max_pairs = 0, max_kps = 0;
  int sortn = 1;
  int* init_ws = nullptr;  // SearchForInitialization: per-pair records, keys (init_ws_bytes_per_pair)
  size_t init_ws_pair = 0;  // bytes per pair
  int* host_init_ws = nullptr;  // orbm_search_for_initialization's own (its pitch is the call's)
  size_t host_init_ws_bytes = 0;
  int* err = nullptr;
  int* stereo_sad = nullptr;  // [max_pairs][max_kps] SAD per left keypoint (-1 = none)
  int* bow_hist = nullptr;    // [max_pairs][32] SearchByBoW rotation histogram (+ match count), 0 between calls
  int* bow_rec = nullptr;     // [max_pairs][max_kps] SearchByBoW row records, -1 between calls
  bool bow_clean = false;     // bow_hist / bow_rec hold their between-calls values
  int* pose_picks = nullptr;  // pose-projection picks per point (frames x mp_pitch)
  size_t pose_picks_cap = 0;
  hipStream_t stream = nullptr;
  WsOrder ws;  // stream order of cand / stereo_sad / pose_picks / bow_* across caller streams
  StreamMarks errm;  // streams of the launches that may set `err` (top-2, SearchByBoW)
  // staging for the synchronous entry points
  void* stage = nullptr;
  size_t stage_bytes = 0;
  void* h_stage = nullptr;  // pinned host staging (orbm_compute_stereo_matches_last)
  size_t h_stage_bytes = 0;
};

static int stage_reserve(orbx_matcher* m, size_t bytes) {
  if (m->stage_bytes >= bytes) return ORBX_OK;
  if (m->stage) (void)hipFree(m->stage);
  m->stage = nullptr;
  m->stage_bytes = 0;
  MHIP(hipMalloc(&m->stage, bytes));
  m->stage_bytes = bytes;
  return ORBX_OK;
}

static int host_stage_reserve(orbx_matcher* m, size_t bytes) {
  if (m->h_stage_bytes >= bytes) return ORBX_OK;
  if (m->h_stage) (void)hipHostFree(m->h_stage);
  m->h_stage = nullptr;
  m->h_stage_bytes = 0;
  MHIP(hipHostMalloc(&m->h_stage, bytes, hipHostMallocDefault));
  m->h_stage_bytes = bytes;
  return ORBX_OK;
}

static int search_init_launch(orbx_matcher* m, const orbx_kp* d_kp1, const uint8_t* d_desc1, const int* d_n1,
                              const orbx_kp* d_kp2, const uint8_t* d_desc2, const int* d_n2, int kp_pitch, int pairs,
                              orbm_grid_bounds b, float* d_prev_xy, int window, float nnratio, int check_ori,
                              int* d_matches12, int* d_nmatches, void* stream, int* ws) {
  InitParams P{};
  P.minX = b.min_x;
  P.maxX = b.max_x;
  P.minY = b.min_y;
  P.maxY = b.max_y;
  // mfGridElementWidthInv / HeightInv (src/Frame.cc:154-155)
  P.invW = static_cast<float>(kGridCols) / static_cast<float>(b.max_x - b.min_x);
  P.invH = static_cast<float>(kGridRows) / static_cast<float>(b.max_y - b.min_y);
  P.r = (float)window;
  P.nnratio = nnratio;
  P.check_ori = check_ori;
  P.kp_pitch = kp_pitch;
  if (m->ws.before((hipStream_t)stream)) return mfail(ORBX_EDEVICE, "stream wait on the workspace failed");
  const int rc = launch_search_init(P, d_kp1, d_desc1, d_n1, d_kp2, d_desc2, d_n2, d_prev_xy, ws, d_matches12,
                                    d_nmatches, pairs, stream);
  if (!rc && m->ws.after((hipStream_t)stream)) return mfail(ORBX_EDEVICE, "event record failed");
  if (rc == ORBX_ECAPACITY)
    return mfail(ORBX_ECAPACITY, "kp_pitch %d too large for SearchForInitialization at nnratio %g (<= %d)", kp_pitch,
                 (double)nnratio, search_init_max_pitch(nnratio));
  if (rc) return mfail(ORBX_EDEVICE, "search_init launch: %s", hipGetErrorString(hipGetLastError()));
  return ORBX_OK;
}

extern "C" {

int orbm_create(int device, int max_pairs, int max_kps, orbm_handle* out) {
  if (!out || max_pairs < 1 || max_kps < 1) return mfail(ORBX_EINVAL, "bad argument");
  if (max_kps > 65535) return mfail(ORBX_EINVAL, "max_kps must be <= 65535");
  MHIP(hipSetDevice(device));
  orbx_matcher* m = new orbx_matcher();
  m->device = device;
  m->max_pairs = max_pairs;
  m->max_kps = max_kps;
  while (m->sortn < max_kps) m->sortn <<= 1;
  m->init_ws_pair = init_ws_bytes_per_pair(max_kps);
  if (hipMalloc(&m->init_ws, (size_t)max_pairs * m->init_ws_pair) != hipSuccess ||
      hipMalloc(&m->err, 16) != hipSuccess ||
      hipMalloc(&m->stereo_sad, (size_t)max_pairs * max_kps * 4) != hipSuccess ||
      hipMalloc(&m->bow_hist, (size_t)max_pairs * 32 * 4) != hipSuccess ||
      hipMalloc(&m->bow_rec, (size_t)max_pairs * max_kps * 4) != hipSuccess) {
    orbm_destroy(m);
    return mfail(ORBX_ENOMEM, "matcher workspace allocation failed");
  }
  (void)hipMemset(m->err, 0, 16);
  *out = m;
  return ORBX_OK;
}

int orbm_destroy(orbm_handle m) {
  if (!m) return ORBX_OK;
  (void)hipSetDevice(m->device);
  if (m->stream) (void)hipStreamSynchronize(m->stream);
  if (m->ws.ev) (void)hipEventSynchronize(m->ws.ev);
  m->ws.release();
  (void)m->errm.wait();
  m->errm.release();
  if (m->init_ws) (void)hipFree(m->init_ws);
  if (m->host_init_ws) (void)hipFree(m->host_init_ws);
  if (m->err) (void)hipFree(m->err);
  if (m->stereo_sad) (void)hipFree(m->stereo_sad);
  if (m->bow_hist) (void)hipFree(m->bow_hist);
  if (m->bow_rec) (void)hipFree(m->bow_rec);
  if (m->pose_picks) (void)hipFree(m->pose_picks);
  if (m->stage) (void)hipFree(m->stage);
  if (m->h_stage) (void)hipHostFree(m->h_stage);
  if (m->stream) (void)hipStreamDestroy(m->stream);
  delete m;
  return ORBX_OK;
}

int orbm_get_status(orbm_handle m, int reset, int* status) {
  if (!m || !status) return mfail(ORBX_EINVAL, "null argument");
  MHIP(hipSetDevice(m->device));
  // the kernels that set the word ran on caller streams: wait for those
  // launches (their stream marks), not for the device
  if (m->errm.wait()) return mfail(ORBX_EDEVICE, "status: event wait failed");
  if (!m->stream) MHIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
  int e = 0;
  MHIP(hipMemcpyAsync(&e, m->err, 4, hipMemcpyDeviceToHost, m->stream));
  MHIP(hipStreamSynchronize(m->stream));
  if (reset && e) {
    MHIP(hipMemsetAsync(m->err, 0, 16, m->stream));
    MHIP(hipStreamSynchronize(m->stream));
  }
  *status = e;
  return ORBX_OK;
}

int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

int orbm_hamming_top2(orbm_handle m, const uint8_t* d_A, size_t a_pitch, const int* d_nA, int a_cap,
                      const uint8_t* d_B, size_t b_pitch, const int* d_nB, int pairs, int* d_best_idx, int* d_best,
                      int* d_second, void* stream) {
  if (!m || !d_A || !d_B || !d_nA || !d_nB || pairs < 1) return mfail(ORBX_EINVAL, "bad argument");
  if ((a_pitch | b_pitch) & 15) return mfail(ORBX_EINVAL, "pitches must be multiples of 16 bytes");
  MHIP(hipSetDevice(m->device));
  const int rc = launch_hamming_top2(d_A, a_pitch, d_nA, a_cap, d_B, b_pitch, d_nB, pairs, d_best_idx, d_best,
                                     d_second, m->err, stream);
  if (rc) return mfail(rc, "launch failed");
  return m->errm.mark((hipStream_t)stream) ? mfail(ORBX_EDEVICE, "event record failed") : ORBX_OK;
}

int orbm_search_for_initialization_batch(orbm_handle m, const orbx_kp* d_kp1, const uint8_t* d_desc1,
                                         const int* d_n1, const orbx_kp* d_kp2, const uint8_t* d_desc2,
                                         const int* d_n2, int kp_pitch, int pairs, orbm_grid_bounds b,
                                         float* d_prev_xy, int window, float nnratio, int check_ori,
                                         int* d_matches12, int* d_nmatches, void* stream) {
  if (!m || pairs < 1 || pairs > m->max_pairs || kp_pitch < 1 || kp_pitch > m->max_kps)
    return mfail(ORBX_EINVAL, "pairs/kp_pitch exceed the matcher workspace");
  MHIP(hipSetDevice(m->device));
  return search_init_launch(m, d_kp1, d_desc1, d_n1, d_kp2, d_desc2, d_n2, kp_pitch, pairs, b, d_prev_xy, window,
                            nnratio, check_ori, d_matches12, d_nmatches, stream, m->init_ws);
}

int orbm_search_for_initialization(orbm_handle m, const orbx_kp* kp1, const uint8_t* desc1, int n1,
                                   const orbx_kp* kp2, const uint8_t* desc2, int n2, orbm_grid_bounds bounds,
                                   float* prev_xy, int window, float nnratio, int check_ori, int* matches12,
                                   int* nmatches) {
  if (!m || !nmatches || n1 < 0 || n2 < 0) return mfail(ORBX_EINVAL, "bad argument");
  if ((n1 && (!kp1 || !desc1 || !prev_xy || !matches12)) || (n2 && (!kp2 || !desc2)))
    return mfail(ORBX_EINVAL, "null array");
  MHIP(hipSetDevice(m->device));
  // Only octave-0 keypoints take part (src/ORBmatcher.cc:424-428: level1 > 0 is
  // skipped; GetFeaturesInArea(.., level1, level1) returns octave-0 keypoints of
  // F2, src/Frame.cc:350-352), so both frames are compacted to them in index
  // order before the upload: the kernel's per-keypoint tables then scale with
  // the octave-0 counts, not with the frames' sizes, and every result maps back
  // through the index lists. Other keypoints keep matches12 = -1 and their
  // vbPrevMatched entry.
  std::vector<int> q1, q2;
  q1.reserve(n1);
  q2.reserve(n2);
  for (int i = 0; i < n1; ++i)
    if (kp1[i].octave == 0) q1.push_back(i);
  for (int i = 0; i < n2; ++i)
    if (kp2[i].octave == 0) q2.push_back(i);
  const int c1 = (int)q1.size(), c2 = (int)q2.size();
  for (int i = 0; i < n1; ++i) matches12[i] = -1;
  if (c1 == 0 || c2 == 0) {
    *nmatches = 0;
    return ORBX_OK;
  }
  const int pitch = std::max(c1, c2);
  if (pitch > 65535) return mfail(ORBX_ECAPACITY, "more than 65535 octave-0 keypoints");
  std::vector<orbx_kp> hk((size_t)c1 + c2);
  std::vector<uint8_t> hd(((size_t)c1 + c2) * 32);
  std::vector<float> hp((size_t)c1 * 2);
  for (int k = 0; k < c1; ++k) {
    hk[k] = kp1[q1[k]];
    memcpy(&hd[(size_t)k * 32], desc1 + (size_t)q1[k] * 32, 32);
    hp[2 * k] = prev_xy[2 * q1[k]];
    hp[2 * k + 1] = prev_xy[2 * q1[k] + 1];
  }
  for (int k = 0; k < c2; ++k) {
    hk[c1 + k] = kp2[q2[k]];
    memcpy(&hd[((size_t)c1 + k) * 32], desc2 + (size_t)q2[k] * 32, 32);
  }
  const size_t kpb = (size_t)pitch * sizeof(orbx_kp), db = (size_t)pitch * 32;
  const size_t bytes = 2 * kpb + 2 * db + (size_t)pitch * 8 + (size_t)pitch * 4 + 64;
  int rc;
  if ((rc = stage_reserve(m, bytes))) return rc;
  uint8_t* s = (uint8_t*)m->stage;
  orbx_kp* dk1 = (orbx_kp*)s;
  orbx_kp* dk2 = (orbx_kp*)(s + kpb);
  uint8_t* dd1 = s + 2 * kpb;
  uint8_t* dd2 = dd1 + db;
  float* dprev = (float*)(dd2 + db);
  int* dm = (int*)(dprev + 2 * pitch);
  int* dn = dm + pitch;  // n1, n2, nmatches
  if (!m->stream) MHIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));  // created on first use
  hipStream_t st = m->stream;
  const int hn[2] = {c1, c2};
  MHIP(hipMemcpyAsync(dk1, hk.data(), (size_t)c1 * sizeof(orbx_kp), hipMemcpyHostToDevice, st));
  MHIP(hipMemcpyAsync(dd1, hd.data(), (size_t)c1 * 32, hipMemcpyHostToDevice, st));
  MHIP(hipMemcpyAsync(dprev, hp.data(), (size_t)c1 * 8, hipMemcpyHostToDevice, st));
  MHIP(hipMemcpyAsync(dk2, hk.data() + c1, (size_t)c2 * sizeof(orbx_kp), hipMemcpyHostToDevice, st));
  MHIP(hipMemcpyAsync(dd2, hd.data() + (size_t)c1 * 32, (size_t)c2 * 32, hipMemcpyHostToDevice, st));
  MHIP(hipMemcpyAsync(dn, hn, 8, hipMemcpyHostToDevice, st));
  // the call's own workspace, sized for its pitch (the octave-0 counts)
  const size_t wsb = init_ws_bytes_per_pair(pitch);
  if (wsb > m->host_init_ws_bytes) {
    if (m->host_init_ws) {
      MHIP(hipStreamSynchronize(st));
      (void)hipFree(m->host_init_ws);
    }
    m->host_init_ws = nullptr;
    m->host_init_ws_bytes = 0;
    MHIP(hipMalloc(&m->host_init_ws, wsb));
    m->host_init_ws_bytes = wsb;
  }
  rc = search_init_launch(m, dk1, dd1, dn, dk2, dd2, dn + 1, pitch, 1, bounds, dprev, window, nnratio, check_ori, dm,
                          dn + 2, st, m->host_init_ws);
  if (rc) return rc;
  int nm = 0;
  std::vector<int> hm(c1);
  MHIP(hipMemcpyAsync(&nm, dn + 2, 4, hipMemcpyDeviceToHost, st));
  MHIP(hipMemcpyAsync(hm.data(), dm, (size_t)c1 * 4, hipMemcpyDeviceToHost, st));
  MHIP(hipMemcpyAsync(hp.data(), dprev, (size_t)c1 * 8, hipMemcpyDeviceToHost, st));
  MHIP(hipStreamSynchronize(st));
  for (int k = 0; k < c1; ++k) {
    const int i1 = q1[k];
    matches12[i1] = hm[k] >= 0 ? q2[hm[k]] : -1;
    prev_xy[2 * i1] = hp[2 * k];  // written by the kernel for matched queries, else the uploaded value
    prev_xy[2 * i1 + 1] = hp[2 * k + 1];
  }
  *nmatches = nm;
  return ORBX_OK;
}

int orbm_search_by_bow(orbm_handle m, const uint8_t* descA, const float* angleA, const uint8_t* mpA, int nA,
                       orbm_feature_vector fvA, const uint8_t* descB, const float* angleB, const uint8_t* mpB,
                       int nB, orbm_feature_vector fvB, float nnratio, int check_ori, int kf_vs_kf, int* out,
                       int* nmatches) {
  if (!m || !nmatches || nA < 0 || nB < 0) return mfail(ORBX_EINVAL, "bad argument");
  // DBoW2 precondition: each feature sits in at most one node; node ids ascending
  auto check_fv = [&](const orbm_feature_vector& fv, int n) -> bool {
    std::vector<char> seen(std::max(n, 1), 0);
    for (int k = 0; k < fv.n_nodes; ++k) {
      if (k && fv.nodes[k] <= fv.nodes[k - 1]) return false;
      for (int p = fv.off[k]; p < fv.off[k + 1]; ++p) {
        const int i = fv.idx[p];
        if (i < 0 || i >= n || seen[i]) return false;
        seen[i] = 1;
      }
    }
    return true;
  };
  // the row records keep the matched index in 16 bits (bin << 16 | index):
  // B's index in KF-KF mode, A's in KF-Frame mode; B's candidates are 16-bit too
  if (nB > 65536) return mfail(ORBX_EINVAL, "nB must be <= 65536");
  if (!kf_vs_kf && nA > 65536) return mfail(ORBX_EINVAL, "nA must be <= 65536 (KF-Frame row records)");
  if (!check_fv(fvA, nA) || !check_fv(fvB, nB))
    return mfail(ORBX_EINVAL, "FeatureVector must have ascending node ids and disjoint in-range indices");
  MHIP(hipSetDevice(m->device));
  const int nout = kf_vs_kf ? nA : nB;
  const int ia = fvA.n_nodes ? fvA.off[fvA.n_nodes] : 0, ib = fvB.n_nodes ? fvB.off[fvB.n_nodes] : 0;
  auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t sz[] = {r16((size_t)nA * 32), r16((size_t)nA * 4), r16((size_t)nA), r16((size_t)fvA.n_nodes * 4),
                       r16((size_t)(fvA.n_nodes + 1) * 4), r16((size_t)ia * 4), r16((size_t)nB * 32),
                       r16((size_t)nB * 4), r16((size_t)nB), r16((size_t)fvB.n_nodes * 4),
                       r16((size_t)(fvB.n_nodes + 1) * 4), r16((size_t)ib * 4), r16((size_t)std::max(nout, 1) * 4),
                       r16((size_t)std::max(nout, 1) * 4), 16, 16, 128};  // out / records: the launch's pitch
  size_t tot = 0;
  for (size_t v : sz) tot += v;
  int rc;
  if ((rc = stage_reserve(m, tot))) return rc;
  uint8_t* p = (uint8_t*)m->stage;
  void* d[17];
  for (int i = 0; i < 17; ++i) {
    d[i] = p;
    p += sz[i];
  }
  if (!m->stream) MHIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));  // created on first use
  hipStream_t st = m->stream;
  auto up = [&](void* dst, const void* src, size_t n) -> int {
    if (n && src) MHIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st));
    return ORBX_OK;
  };
  const int hn[4] = {nA, nB, fvA.n_nodes, fvB.n_nodes};
  if ((rc = up(d[0], descA, (size_t)nA * 32)) || (rc = up(d[1], angleA, (size_t)nA * 4)) ||
      (rc = up(d[2], mpA, (size_t)nA)) || (rc = up(d[3], fvA.nodes, (size_t)fvA.n_nodes * 4)) ||
      (rc = up(d[4], fvA.off, (size_t)(fvA.n_nodes + 1) * 4)) || (rc = up(d[5], fvA.idx, (size_t)ia * 4)) ||
      (rc = up(d[6], descB, (size_t)nB * 32)) || (rc = up(d[7], angleB, (size_t)nB * 4)) ||
      (rc = up(d[8], mpB, (size_t)nB)) || (rc = up(d[9], fvB.nodes, (size_t)fvB.n_nodes * 4)) ||
      (rc = up(d[10], fvB.off, (size_t)(fvB.n_nodes + 1) * 4)) || (rc = up(d[11], fvB.idx, (size_t)ib * 4)) ||
      (rc = up(d[15], hn, sizeof hn)))
    return rc;
  const int* dn = (const int*)d[15];
  BowSide A{(const uint8_t*)d[0], (const float*)d[1], 1, mpA ? (const uint8_t*)d[2] : nullptr, dn,
            (const uint32_t*)d[3], (const int*)d[4], (const int*)d[5], dn + 2, 0, 0};
  BowSide B{(const uint8_t*)d[6], (const float*)d[7], 1, mpB ? (const uint8_t*)d[8] : nullptr, dn + 1,
            (const uint32_t*)d[9], (const int*)d[10], (const int*)d[11], dn + 3, 0, 0};
  bool clean = false;  // staging memory: records and histogram filled first
  if ((rc = launch_search_bow(A, B, 1, nnratio, check_ori, kf_vs_kf, (int*)d[12], std::max(nout, 1), (int*)d[14],
                              (int*)d[13], (size_t)std::max(nout, 1), (int*)d[16], 32, &clean, m->err, st)))
    return mfail(rc, "search_bow launch: %s", hipGetErrorString(hipGetLastError()));
  if (m->errm.mark(st)) return mfail(ORBX_EDEVICE, "event record failed");
  int nm = 0;
  MHIP(hipMemcpyAsync(&nm, d[14], 4, hipMemcpyDeviceToHost, st));
  if (nout) MHIP(hipMemcpyAsync(out, d[12], (size_t)nout * 4, hipMemcpyDeviceToHost, st));
  MHIP(hipStreamSynchronize(st));
  *nmatches = nm;
  return ORBX_OK;
}

int orbm_search_by_bow_batch(orbm_handle m, int pairs, int kp_pitch, int node_pitch, const orbx_kp* d_kpA,
                             const uint8_t* d_descA, const int* d_nA, const uint8_t* d_mpA, const uint32_t* d_nodesA,
                             const int* d_offA, const int* d_idxA, const int* d_nnA, const orbx_kp* d_kpB,
                             const uint8_t* d_descB, const int* d_nB, const uint8_t* d_mpB, const uint32_t* d_nodesB,
                             const int* d_offB, const int* d_idxB, const int* d_nnB, float nnratio, int check_ori,
                             int kf_vs_kf, int* d_out, int* d_nmatches, void* stream) {
  if (!m || pairs < 1 || kp_pitch < 1 || node_pitch < 1 || !d_kpA || !d_descA || !d_nA || !d_nodesA || !d_offA ||
      !d_idxA || !d_nnA || !d_kpB || !d_descB || !d_nB || !d_nodesB || !d_offB || !d_idxB || !d_nnB || !d_out ||
      !d_nmatches)
    return mfail(ORBX_EINVAL, "bad argument");
  if (pairs > m->max_pairs || kp_pitch > m->max_kps)
    return mfail(ORBX_ECAPACITY, "pairs/kp_pitch above the matcher's max_pairs/max_kps");
  if (kp_pitch > 65536) return mfail(ORBX_EINVAL, "kp_pitch must be <= 65536");
  MHIP(hipSetDevice(m->device));
  // angles straight from the orbx_kp records (cv::KeyPoint::angle, float 3 of 7)
  BowSide A{d_descA, (const float*)d_kpA + 3, 7, d_mpA, d_nA, d_nodesA, d_offA, d_idxA, d_nnA, kp_pitch, node_pitch};
  BowSide B{d_descB, (const float*)d_kpB + 3, 7, d_mpB, d_nB, d_nodesB, d_offB, d_idxB, d_nnB, kp_pitch, node_pitch};
  hipStream_t s = (hipStream_t)stream;
  if (m->ws.before(s)) return mfail(ORBX_EDEVICE, "stream wait on the workspace failed");
  const int rc = launch_search_bow(A, B, pairs, nnratio, check_ori, kf_vs_kf, d_out, kp_pitch, d_nmatches, m->bow_rec,
                                   (size_t)m->max_pairs * m->max_kps, m->bow_hist, (size_t)m->max_pairs * 32,
                                   &m->bow_clean, m->err, stream);
  if (rc) return mfail(rc, "search_bow launch: %s", hipGetErrorString(hipGetLastError()));
  if (m->ws.after(s) || m->errm.mark(s)) return mfail(ORBX_EDEVICE, "event record failed");
  return ORBX_OK;
}

// sync: a synchronous caller that waits for the launch itself: its
// workspaces' earlier users are waited for only if still running, and no
// event is recorded after it (no barrier packets around its kernels)
static int stereo_batch(orbm_handle m, orbx_handle left, int left_frame0, orbx_handle right, int right_frame0,
                        const orbx_kp* d_kpL, const uint8_t* d_descL, const int* d_nL, const orbx_kp* d_kpR,
                        const uint8_t* d_descR, const int* d_nR, int kp_pitch, int pairs, float mb, float mbf,
                        float* d_uRight, float* d_depth, int* d_nkept, void* stream, bool sync) {
  if (!m || !left || !right || !d_kpL || !d_descL || !d_nL || !d_kpR || !d_descR || !d_nR || !d_uRight ||
      !d_depth || !d_nkept || pairs < 1 || kp_pitch < 1)
    return mfail(ORBX_EINVAL, "bad argument");
  if (pairs > m->max_pairs || kp_pitch > m->max_kps)
    return mfail(ORBX_ECAPACITY, "pairs/kp_pitch above the matcher's max_pairs/max_kps");
  if (!(mb > 0.f)) return mfail(ORBX_EINVAL, "baseline mb must be positive");
  MHIP(hipSetDevice(m->device));
  StereoParams P{};
  int wr[kMaxLevels], hr[kMaxLevels], LR = 0;
  float sr[kMaxLevels], isr[kMaxLevels];
  if (extractor_pyramid(left, left_frame0, pairs, &P.pl, P.lw, P.lh, P.scale, P.inv_scale, &P.L) ||
      extractor_pyramid(right, right_frame0, pairs, &P.pr, wr, hr, sr, isr, &LR))
    return mfail(ORBX_EINVAL, "stereo pyramid: %s", orbx_last_error());
  if (LR != P.L) return mfail(ORBX_EINVAL, "left and right extractors have different level counts");
  for (int l = 0; l < P.L; ++l)
    if (wr[l] != P.lw[l] || hr[l] != P.lh[l]) return mfail(ORBX_EINVAL, "left and right image sizes differ");
  P.nrows = P.lh[0];
  P.kp_pitch = kp_pitch;
  P.mb = mb;
  P.mbf = mbf;
  // ~256 workgroups (one per CU) over the batch, 8 per pair for batches of
  // 32+ pairs; each stages its pair's right keypoints and descriptors in LDS.
  // Few pairs (the stereo Frame's one) take up to 64 per pair: the left
  // keypoints each wave walks through one after another set the latency
  // (one pair: 0.107 ms with 8, 0.085 ms with 64, shim_latency's stereo_parts)
  P.groups = std::max(1, std::min(64, (256 + pairs - 1) / pairs));
  if (const char* e = getenv("ORBX_STEREO_GROUPS")) P.groups = std::max(1, atoi(e));  // tuning experiments
  P.stop = 0;
#ifdef ORBX_DIAG  // diagnostics builds only: stop after a phase, results incomplete
  if (const char* e = getenv("ORBX_STEREO_STOP")) P.stop = atoi(e);
#endif
  // workgroup g takes left keypoints iL = g + groups * m: at most this many
  P.jobs_cap = (kp_pitch + P.groups - 1) / P.groups;
  if (stereo_lds_bytes(P.nrows, kp_pitch, P.jobs_cap) > 156 * 1024)
    return mfail(ORBX_ECAPACITY, "stereo row table does not fit in LDS (rows %d, kp_pitch %d)", P.nrows, kp_pitch);
  // the SAD scratch is the matcher's, the pyramids the extractors': order
  // this launch after their last users and make their next users wait for it
  hipStream_t s = (hipStream_t)stream;
  WsOrder* wl = extractor_ws(left);
  WsOrder* wr2 = extractor_ws(right);
  if (sync ? (m->ws.before_pending(s) || wl->before_pending(s) || wr2->before_pending(s))
           : (m->ws.before(s) || wl->before(s) || wr2->before(s)))
    return mfail(ORBX_EDEVICE, "stream wait on the workspaces failed");
  if (launch_stereo(P, d_kpL, d_descL, d_nL, d_kpR, d_descR, d_nR, pairs, d_uRight, d_depth, m->stereo_sad, d_nkept,
                    stream) != ORBX_OK)
    return mfail(ORBX_EDEVICE, "stereo launch: %s", hipGetErrorString(hipGetLastError()));
  if (!sync && (m->ws.after(s) || wl->after(s) || wr2->after(s))) return mfail(ORBX_EDEVICE, "event record failed");
  return ORBX_OK;
}

int orbm_compute_stereo_matches_batch(orbm_handle m, orbx_handle left, int left_frame0, orbx_handle right,
                                      int right_frame0, const orbx_kp* d_kpL, const uint8_t* d_descL,
                                      const int* d_nL, const orbx_kp* d_kpR, const uint8_t* d_descR,
                                      const int* d_nR, int kp_pitch, int pairs, float mb, float mbf,
                                      float* d_uRight, float* d_depth, int* d_nkept, void* stream) {
  return stereo_batch(m, left, left_frame0, right, right_frame0, d_kpL, d_descL, d_nL, d_kpR, d_descR, d_nR,
                      kp_pitch, pairs, mb, mbf, d_uRight, d_depth, d_nkept, stream, false);
}

int orbm_compute_stereo_matches(orbm_handle m, orbx_handle left, orbx_handle right, const orbx_kp* kpL,
                                const uint8_t* descL, int nL, const orbx_kp* kpR, const uint8_t* descR, int nR,
                                float mb, float mbf, float* uRight, float* depth, int* nkept) {
  if (!m || !nkept || nL < 0 || nR < 0 || (nL && (!kpL || !descL || !uRight || !depth)) || (nR && (!kpR || !descR)))
    return mfail(ORBX_EINVAL, "bad argument");
  if (nL > m->max_kps || nR > m->max_kps) return mfail(ORBX_ECAPACITY, "more keypoints than max_kps");
  if (nR > 65535) return mfail(ORBX_ECAPACITY, "more than 65535 right keypoints");
  MHIP(hipSetDevice(m->device));
  const int pitch = std::max(std::max(nL, nR), 1);
  const size_t kpb = (size_t)pitch * sizeof(orbx_kp), db = (size_t)pitch * 32;
  const size_t bytes = 2 * kpb + 2 * db + (size_t)pitch * 8 + 64;
  int rc;
  if ((rc = stage_reserve(m, bytes))) return rc;
  uint8_t* s = (uint8_t*)m->stage;
  orbx_kp* dkl = (orbx_kp*)s;
  orbx_kp* dkr = (orbx_kp*)(s + kpb);
  uint8_t* ddl = s + 2 * kpb;
  uint8_t* ddr = ddl + db;
  float* du = (float*)(ddr + db);
  float* dd = du + pitch;
  int* dn = (int*)(dd + pitch);  // nL, nR, kept
  if (!m->stream) MHIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
  hipStream_t st = m->stream;
  const int hn[2] = {nL, nR};
  if (nL) {
    MHIP(hipMemcpyAsync(dkl, kpL, (size_t)nL * sizeof(orbx_kp), hipMemcpyHostToDevice, st));
    MHIP(hipMemcpyAsync(ddl, descL, (size_t)nL * 32, hipMemcpyHostToDevice, st));
  }
  if (nR) {
    MHIP(hipMemcpyAsync(dkr, kpR, (size_t)nR * sizeof(orbx_kp), hipMemcpyHostToDevice, st));
    MHIP(hipMemcpyAsync(ddr, descR, (size_t)nR * 32, hipMemcpyHostToDevice, st));
  }
  MHIP(hipMemcpyAsync(dn, hn, 8, hipMemcpyHostToDevice, st));
  rc = stereo_batch(m, left, 0, right, 0, dkl, ddl, dn, dkr, ddr, dn + 1, pitch, 1, mb, mbf, du, dd, dn + 2, st,
                    true);
  if (rc) return rc;
  int kept = 0;
  MHIP(hipMemcpyAsync(&kept, dn + 2, 4, hipMemcpyDeviceToHost, st));
  if (nL) {
    MHIP(hipMemcpyAsync(uRight, du, (size_t)nL * 4, hipMemcpyDeviceToHost, st));
    MHIP(hipMemcpyAsync(depth, dd, (size_t)nL * 4, hipMemcpyDeviceToHost, st));
  }
  MHIP(hipStreamSynchronize(st));
  *nkept = kept;
  return ORBX_OK;
}

// Frame::ComputeStereoMatches right after the stereo constructor's two
// extractions (src/Frame.cc:77-89): the keypoints and descriptors are read
// where the two orbx_extract calls left them on the device, so only mvuRight
// and mvDepth cross the link.
int orbm_compute_stereo_matches_last(orbm_handle m, orbx_handle left, orbx_handle right, float mb, float mbf,
                                     float* uRight, float* depth, int nL, int* nkept) {
  if (!m || !left || !right || !nkept || nL < 0 || (nL && (!uRight || !depth))) return mfail(ORBX_EINVAL, "bad argument");
  const int* dnL = nullptr;
  const int* dnR = nullptr;
  const orbx_kp *dkl = nullptr, *dkr = nullptr;
  const uint8_t *ddl = nullptr, *ddr = nullptr;
  int capL = 0, capR = 0;
  if (extractor_last_output(left, &dnL, &dkl, &ddl, &capL) || extractor_last_output(right, &dnR, &dkr, &ddr, &capR))
    return mfail(ORBX_EINVAL, "stereo (last extraction): %s", orbx_last_error());
  if (!dnL || !dnR) {
    // an empty left or right image: no right keypoints to match, every left
    // keypoint keeps uRight = depth = -1 (src/Frame.cc:465-470)
    if (!dnL && nL) return mfail(ORBX_EINVAL, "nL %d but the left extraction was of an empty image", nL);
    for (int i = 0; i < nL; ++i) uRight[i] = depth[i] = -1.f;
    *nkept = 0;
    return ORBX_OK;
  }
  if (capL != capR) return mfail(ORBX_EINVAL, "left and right extractors have different capacities");
  if (nL > capL) return mfail(ORBX_EINVAL, "nL %d above the left extraction's capacity %d", nL, capL);
  MHIP(hipSetDevice(m->device));
  // the device path sizes its LDS by the extractors' capacity; past the
  // matcher's limits (max_kps, or the stereo kernel's LDS for large
  // nFeatures) the keypoints come to the host and take the host-array path,
  // whose pitch is the actual counts
  auto host_fallback = [&]() -> int {
    int cnt[2] = {0, 0};
    MHIP(hipMemcpy(&cnt[0], dnL, 4, hipMemcpyDeviceToHost));
    MHIP(hipMemcpy(&cnt[1], dnR, 4, hipMemcpyDeviceToHost));
    if (nL > cnt[0]) return mfail(ORBX_EINVAL, "nL %d above the left extraction's count %d", nL, cnt[0]);
    std::vector<orbx_kp> kl(std::max(cnt[0], 1)), kr(std::max(cnt[1], 1));
    std::vector<uint8_t> dl((size_t)std::max(cnt[0], 1) * 32), dr((size_t)std::max(cnt[1], 1) * 32);
    MHIP(hipMemcpy(kl.data(), dkl, (size_t)cnt[0] * sizeof(orbx_kp), hipMemcpyDeviceToHost));
    MHIP(hipMemcpy(kr.data(), dkr, (size_t)cnt[1] * sizeof(orbx_kp), hipMemcpyDeviceToHost));
    MHIP(hipMemcpy(dl.data(), ddl, (size_t)cnt[0] * 32, hipMemcpyDeviceToHost));
    MHIP(hipMemcpy(dr.data(), ddr, (size_t)cnt[1] * 32, hipMemcpyDeviceToHost));
    return orbm_compute_stereo_matches(m, left, right, kl.data(), dl.data(), nL, kr.data(), dr.data(), cnt[1], mb, mbf,
                                       uRight, depth, nkept);
  };
  if (capL > m->max_kps) return host_fallback();
  // outputs {kept, -, -, -, uRight[nL], depth[nL]} in one block: one copy back
  // into the matcher's pinned staging
  const size_t bytes = 16 + (size_t)capL * 8;
  int rc;
  if ((rc = stage_reserve(m, bytes)) || (rc = host_stage_reserve(m, bytes))) return rc;
  int* dk = (int*)m->stage;
  float* du = (float*)m->stage + 4;  // uRight: capL floats (the kernels' pitch), then depth
  float* dd = du + capL;
  if (!m->stream) MHIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
  hipStream_t st = m->stream;
  rc = stereo_batch(m, left, 0, right, 0, dkl, ddl, dnL, dkr, ddr, dnR, capL, 1, mb, mbf, du, dd, dk, st, true);
  if (rc == ORBX_ECAPACITY) return host_fallback();  // checked before any launch
  if (rc) return rc;
  uint8_t* h = (uint8_t*)m->h_stage;
  MHIP(hipMemcpyAsync(h, dk, 16 + (size_t)capL * 8, hipMemcpyDeviceToHost, st));
  MHIP(hipStreamSynchronize(st));
  *nkept = ((const int*)h)[0];
  if (nL) {
    memcpy(uRight, h + 16, (size_t)nL * 4);
    memcpy(depth, h + 16 + (size_t)capL * 4, (size_t)nL * 4);
  }
  return ORBX_OK;
}

// orbm_stereo_frame's host phases (ORBX_STEREO_PROF=1): left staged, issued,
// right staged, issued, stereo issued, waited, copied out; medians of the
// calls after the first 20 per left handle, printed at exit
struct StereoProf {
  std::mutex mu;
  std::vector<std::pair<const void*, std::vector<double>>> per;  // per left handle: 7 phases per call
  void add(const void* key, const double* st) {
    std::lock_guard<std::mutex> lk(mu);
    size_t i = 0;
    while (i < per.size() && per[i].first != key) ++i;
    if (i == per.size()) per.push_back({key, {}});
    for (int k = 0; k < 7; ++k) per[i].second.push_back(st[k + 1] - st[k]);
  }
  ~StereoProf() {
    const char* names[7] = {"left staged", "issued", "right staged", "issued", "stereo issued", "wait", "copy-out"};
    for (auto& e : per) {
      const size_t n = e.second.size() / 7;
      if (n <= 20) continue;
      fprintf(stderr, "orbm_stereo_frame host phases, median of %zu calls (us):", n - 20);
      for (int k = 0; k < 7; ++k) {
        std::vector<double> v;
        for (size_t c = 20; c < n; ++c) v.push_back(e.second[c * 7 + k]);
        std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
        fprintf(stderr, " %s %.1f", names[k], v[v.size() / 2] * 1e6);
      }
      fprintf(stderr, "\n");
    }
  }
};
static StereoProf& stereo_prof() {
  static StereoProf p;
  return p;
}

// The stereo Frame's construction steps (src/Frame.cc:77-89: ExtractORB on
// threadLeft / threadRight, then ComputeStereoMatches :465-639) with one
// device round trip: both extraction chains are issued from the calling
// thread on the two handles' streams (they run concurrently), the stereo
// kernels follow on the right stream once both are done, and their {kept,
// uRight, depth} block comes back (a copy kernel into pinned memory) in the
// same wait as the two extractions' outputs. Results are those of
// orbx_extract x2 + orbm_compute_stereo_matches_last.
int orbm_stereo_frame(orbm_handle m, orbx_handle left, orbx_handle right, const uint8_t* img_left,
                      size_t stride_left, const uint8_t* img_right, size_t stride_right, int w, int h, float mb,
                      float mbf, orbx_kp* kps_left, int cap_left, uint8_t* desc_left, int* n_left,
                      orbx_kp* kps_right, int cap_right, uint8_t* desc_right, int* n_right, float* uRight,
                      float* depth, int* nkept) {
  if (!m || !left || !right || !n_left || !n_right || !nkept || w < 0 || h < 0) return mfail(ORBX_EINVAL, "bad argument");
  if (left == right) return mfail(ORBX_EINVAL, "left and right need two extractor handles");
  if (!(mb > 0.f)) return mfail(ORBX_EINVAL, "baseline mb must be positive");
  *nkept = 0;
  if (w == 0 || h == 0) {
    // empty images: the two calls' own semantics (no outputs, uRight = -1)
    if (orbx_extract(left, img_left, w, h, stride_left, kps_left, cap_left, desc_left, n_left) ||
        orbx_extract(right, img_right, w, h, stride_right, kps_right, cap_right, desc_right, n_right))
      return mfail(ORBX_EINVAL, "stereo frame: %s", orbx_last_error());
    return orbm_compute_stereo_matches_last(m, left, right, mb, mbf, uRight, depth, *n_left, nkept);
  }
  MHIP(hipSetDevice(m->device));
  int brc = ORBX_OK, cap = 0;
  auto between = [&](hipStream_t st) -> int {
    const int* dnL = nullptr;
    const int* dnR = nullptr;
    const orbx_kp *dkl = nullptr, *dkr = nullptr;
    const uint8_t *ddl = nullptr, *ddr = nullptr;
    int capR = 0;
    if (extractor_last_output(left, &dnL, &dkl, &ddl, &cap) || extractor_last_output(right, &dnR, &dkr, &ddr, &capR))
      return brc = mfail(ORBX_EINVAL, "stereo frame: %s", orbx_last_error());
    if (cap != capR) return brc = mfail(ORBX_EINVAL, "left and right extractors have different capacities");
    // past the matcher's limits: the host-array path after the extractions
    if (cap > m->max_kps) return (brc = ORBX_ECAPACITY), ORBX_OK;
    const size_t bytes = 16 + (size_t)cap * 8;
    int rc;
    if ((rc = stage_reserve(m, bytes)) || (rc = host_stage_reserve(m, bytes))) return brc = rc;
    int* dk = (int*)m->stage;
    float* du = (float*)m->stage + 4;
    float* dd = du + cap;
    rc = stereo_batch(m, left, 0, right, 0, dkl, ddl, dnL, dkr, ddr, dnR, cap, 1, mb, mbf, du, dd, dk, st, true);
    if (rc == ORBX_ECAPACITY) return (brc = ORBX_ECAPACITY), ORBX_OK;  // checked before any launch
    if (rc) return brc = rc;
    if ((rc = copy_to_host_async(m->h_stage, dk, bytes, st))) return brc = mfail(rc, "%s", orbx_last_error());
    return ORBX_OK;
  };
  // ORBX_STEREO_PROF=1 (diagnostics): host phases per call, medians printed at exit
  static const bool prof = getenv("ORBX_STEREO_PROF") && getenv("ORBX_STEREO_PROF")[0] == '1';
  double st[8];
  if (prof) st[0] = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  int rc = extract_pair(left, right, img_left, stride_left, img_right, stride_right, w, h, between, kps_left, cap_left,
                        desc_left, n_left, kps_right, cap_right, desc_right, n_right, prof ? st + 1 : nullptr);
  if (prof && !rc) stereo_prof().add(left, st);
  if (rc) return brc ? brc : mfail(rc, "stereo frame: %s", orbx_last_error());
  if (brc == ORBX_ECAPACITY)
    return orbm_compute_stereo_matches_last(m, left, right, mb, mbf, uRight, depth, *n_left, nkept);
  if (brc) return brc;
  const uint8_t* hs = (const uint8_t*)m->h_stage;
  *nkept = ((const int*)hs)[0];
  const int nL = *n_left;
  if (nL && (!uRight || !depth)) return mfail(ORBX_EINVAL, "null uRight/depth");
  if (nL) {
    memcpy(uRight, hs + 16, (size_t)nL * 4);
    memcpy(depth, hs + 16 + (size_t)cap * 4, (size_t)nL * 4);
  }
  return ORBX_OK;
}

int orbm_search_by_projection_batch(orbm_handle m, const orbx_kp* d_kps, const uint8_t* d_desc, const int* d_n,
                                    int kp_pitch, const float* d_uright, orbm_grid_bounds b, const float* scale,
                                    int nlevels, const uint8_t* d_blocked, const orbm_map_point_proj* d_mps,
                                    const uint8_t* d_mpdesc, const int* d_nmp, int mp_pitch, int frames, float th,
                                    float nnratio, int* d_out, int* d_nmatches, void* stream) {
  if (!m || !d_kps || !d_desc || !d_n || !scale || !d_blocked || !d_mps || !d_mpdesc || !d_nmp || !d_out ||
      !d_nmatches || frames < 1 || kp_pitch < 1 || mp_pitch < 1 || nlevels < 1 || nlevels > kMaxLevels)
    return mfail(ORBX_EINVAL, "bad argument");
  if (mp_pitch > 8192) return mfail(ORBX_ECAPACITY, "more than 8192 map points per frame");
  if (!(b.max_x > b.min_x) || !(b.max_y > b.min_y)) return mfail(ORBX_EINVAL, "empty grid bounds");
  if (proj_lds_bytes(kp_pitch) > 156 * 1024) return mfail(ORBX_ECAPACITY, "kp_pitch %d too large", kp_pitch);
  MHIP(hipSetDevice(m->device));
  ProjParams P{};
  P.minX = b.min_x;
  P.maxX = b.max_x;
  P.minY = b.min_y;
  P.maxY = b.max_y;
  // mfGridElementWidthInv = FRAME_GRID_COLS / (mnMaxX - mnMinX)  (src/Frame.cc:154-155)
  P.invW = 64.0f / (b.max_x - b.min_x);
  P.invH = 48.0f / (b.max_y - b.min_y);
  for (int l = 0; l < kMaxLevels; ++l) P.scale[l] = scale[std::min(l, nlevels - 1)];
  P.th = th;
  P.nnratio = nnratio;
  P.kp_pitch = kp_pitch;
  P.mp_pitch = mp_pitch;
  P.has_uright = d_uright != nullptr;
  P.max_rounds = 32;
  if (const char* e = getenv("ORBX_PROJ_ROUNDS")) P.max_rounds = atoi(e);  // tests: force the sequential pass
  static long long* prof = nullptr;  // ORBX_PROJ_PROF: phase clocks of frame 0 printed after the call
  const bool do_prof = getenv("ORBX_PROJ_PROF") != nullptr;
  if (do_prof) {
    if (!prof) MHIP(hipMalloc(&prof, (size_t)frames * 64 * 8));
    MHIP(hipMemset(prof, 0, (size_t)frames * 64 * 8));
    P.prof = prof;
  }
  if (launch_search_proj(P, d_kps, d_desc, d_n, d_uright, d_blocked, d_mps, d_mpdesc, d_nmp, frames, d_out,
                         d_nmatches, stream))
    return mfail(ORBX_EDEVICE, "search_proj launch: %s", hipGetErrorString(hipGetLastError()));
  if (do_prof) {
    long long h[64];
    MHIP(hipStreamSynchronize((hipStream_t)stream));
    MHIP(hipMemcpy(h, prof, sizeof h, hipMemcpyDeviceToHost));
    fprintf(stderr, "proj prof frame 0:");
    for (int i = 1; i < 42 && h[i]; ++i) fprintf(stderr, " r%d=%lld", i - 1, h[i] - h[0]);
    fprintf(stderr, "\n");
  }
  return ORBX_OK;
}

int orbm_search_by_projection(orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n, const float* uright,
                              orbm_grid_bounds b, const float* scale, int nlevels, const uint8_t* blocked,
                              const orbm_map_point_proj* mps, const uint8_t* mpdesc, int nmp, float th,
                              float nnratio, int* out, int* nmatches) {
  if (!m || !nmatches || n < 0 || nmp < 0 || (n && (!kps || !desc || !blocked || !out)) ||
      (nmp && (!mps || !mpdesc)))
    return mfail(ORBX_EINVAL, "bad argument");
  if (nmp > 8192) return mfail(ORBX_ECAPACITY, "more than 8192 map points");
  MHIP(hipSetDevice(m->device));
  const int kp = std::max(n, 1), mp = std::max(nmp, 1);
  const size_t sz[] = {(size_t)kp * sizeof(orbx_kp), (size_t)kp * 32, (size_t)kp * 4, (size_t)kp,
                       (size_t)mp * sizeof(orbm_map_point_proj), (size_t)mp * 32, (size_t)kp * 4, 16};
  size_t off[8], tot = 0;
  for (int i = 0; i < 8; ++i) {
    off[i] = tot;
    tot += (sz[i] + 255) & ~(size_t)255;
  }
  int rc;
  if ((rc = stage_reserve(m, tot))) return rc;
  uint8_t* s = (uint8_t*)m->stage;
  if (!m->stream) MHIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
  hipStream_t st = m->stream;
  int* cnt = (int*)(s + off[7]);  // n, nmp, nmatches
  const int hn[2] = {n, nmp};
  if (n) {
    MHIP(hipMemcpyAsync(s + off[0], kps, (size_t)n * sizeof(orbx_kp), hipMemcpyHostToDevice, st));
    MHIP(hipMemcpyAsync(s + off[1], desc, (size_t)n * 32, hipMemcpyHostToDevice, st));
    if (uright) MHIP(hipMemcpyAsync(s + off[2], uright, (size_t)n * 4, hipMemcpyHostToDevice, st));
    MHIP(hipMemcpyAsync(s + off[3], blocked, (size_t)n, hipMemcpyHostToDevice, st));
  }
  if (nmp) {
    MHIP(hipMemcpyAsync(s + off[4], mps, (size_t)nmp * sizeof(orbm_map_point_proj), hipMemcpyHostToDevice, st));
    MHIP(hipMemcpyAsync(s + off[5], mpdesc, (size_t)nmp * 32, hipMemcpyHostToDevice, st));
  }
  MHIP(hipMemcpyAsync(cnt, hn, 8, hipMemcpyHostToDevice, st));
  rc = orbm_search_by_projection_batch(m, (const orbx_kp*)(s + off[0]), s + off[1], cnt, kp,
                                       uright ? (const float*)(s + off[2]) : nullptr, b, scale, nlevels, s + off[3],
                                       (const orbm_map_point_proj*)(s + off[4]), s + off[5], cnt + 1, mp, 1, th,
                                       nnratio, (int*)(s + off[6]), cnt + 2, st);
  if (rc) return rc;
  int nm = 0;
  MHIP(hipMemcpyAsync(&nm, cnt + 2, 4, hipMemcpyDeviceToHost, st));
  if (n) MHIP(hipMemcpyAsync(out, s + off[6], (size_t)n * 4, hipMemcpyDeviceToHost, st));
  MHIP(hipStreamSynchronize(st));
  *nmatches = nm;
  return ORBX_OK;
}

// ---------------------------------------------- pose-projection overloads
namespace {

// R*x + t via gemm's small-matrix path (float dot, double add of t)
void host_rx_t(const float* T, const float* x, float* d) {
  for (int r = 0; r < 3; ++r) {
    const float t = T[4 * r] * x[0] + T[4 * r + 1] * x[1] + T[4 * r + 2] * x[2];
    d[r] = (float)((double)t * 1.0 + (double)T[4 * r + 3] * 1.0);
  }
}
// -R.t()*t via the general gemm path (double accumulation)
void host_neg_rt_t(const float* T, float* d) {
  for (int r = 0; r < 3; ++r) {
    double s = 0;
    for (int k = 0; k < 3; ++k) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
    d[r] = (float)(s * -1.0);
  }
}
// MapPoint::PredictScale's int level as a predicate of the ratio
int host_predict_direct(float ratio, float logsf, int L) {
  const float q = std::ceil(std::log(ratio) / logsf);  // float overloads (logf)
  int s = (q >= -2147483648.0f && q < 2147483648.0f) ? (int)q : INT_MIN;
  return s < 0 ? 0 : (s >= L ? L - 1 : s);
}

}  // namespace

int orbm_prepare_pose(int mode, const orbm_camera* cam, const float* Tlw, int mono, orbm_pose* out) {
  if (!cam || !out || mode < ORBM_PROJ_LAST_FRAME || mode > ORBM_PROJ_FUSE_SIM3 ||
      (mode == ORBM_PROJ_LAST_FRAME && !Tlw))
    return mfail(ORBX_EINVAL, "bad argument");
  orbm_pose p{};
  p.fx = cam->fx;
  p.fy = cam->fy;
  p.cx = cam->cx;
  p.cy = cam->cy;
  p.mbf = cam->mbf;
  if (mode == ORBM_PROJ_SIM3 || mode == ORBM_PROJ_FUSE_SIM3) {
    // scw = sqrt(sRcw.row(0).dot(sRcw.row(0))); Rcw = sRcw/scw; tcw = t/scw
    // (src/ORBmatcher.cc:298-303, 986-991): Mat::dot in double, Mat / s = convertTo(1/s)
    const float* S = cam->Tcw;
    const double d = (double)S[0] * S[0] + (double)S[1] * S[1] + (double)S[2] * S[2];
    const float scw = (float)std::sqrt(d);
    if (!(scw > 0)) return mfail(ORBX_EINVAL, "Scw has a zero scale");
    const float a = (float)(1.0 / (double)scw);
    for (int k = 0; k < 12; ++k) p.Rt[k] = S[k] * a + 0.0f;
  } else {
    for (int k = 0; k < 12; ++k) p.Rt[k] = cam->Tcw[k];
  }
  host_neg_rt_t(p.Rt, p.Ow);  // Ow = -Rcw.t()*tcw
  p.level_mode = 0;
  if (mode == ORBM_PROJ_LAST_FRAME) {
    // twc = -Rcw.t()*tcw; tlc = Rlw*twc + tlw (src/ORBmatcher.cc:1338-1349)
    float tlc[3];
    host_rx_t(Tlw, p.Ow, tlc);
    const bool bForward = tlc[2] > cam->mb && !mono;
    const bool bBackward = -tlc[2] > cam->mb && !mono;
    p.level_mode = bForward ? 1 : (bBackward ? 2 : 0);
  }
  *out = p;
  return ORBX_OK;
}

int orbm_prepare_sim3_match(const orbm_camera* cam1, const float* T1w, const float* T2w, float s12, const float* R12,
                            const float* t12, orbm_pose* out) {
  if (!cam1 || !T1w || !T2w || !R12 || !t12 || !out || !(s12 != 0.0f)) return mfail(ORBX_EINVAL, "bad argument");
  // sR12 = s12*R12; sR21 = (1.0/s12)*R12.t(); t21 = -sR21*t12 (src/ORBmatcher.cc:1118-1120):
  // scalar * Mat = convertTo(alpha) in float, -A*t = gemm small path with alpha -1
  const float a12 = (float)(double)s12, a21 = (float)(1.0 / (double)s12);
  float S12[12], S21[12];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      S12[4 * r + c] = R12[3 * r + c] * a12 + 0.0f;
      S21[4 * r + c] = R12[3 * c + r] * a21 + 0.0f;
    }
  for (int r = 0; r < 3; ++r) {
    S12[4 * r + 3] = t12[r];
    const float t = S21[4 * r] * t12[0] + S21[4 * r + 1] * t12[1] + S21[4 * r + 2] * t12[2];
    S21[4 * r + 3] = (float)((double)t * -1.0 + 0.0 * 0.0);
  }
  for (int d = 0; d < 2; ++d) {
    orbm_pose p{};
    p.fx = cam1->fx;
    p.fy = cam1->fy;
    p.cx = cam1->cx;
    p.cy = cam1->cy;
    p.mbf = cam1->mbf;
    std::memcpy(p.Rt, d == 0 ? T1w : T2w, sizeof p.Rt);
    std::memcpy(p.Rt2, d == 0 ? S21 : S12, sizeof p.Rt2);
    host_neg_rt_t(p.Rt, p.Ow);
    out[d] = p;
  }
  return ORBX_OK;
}

int orbm_predict_scale_thresholds(float scale_factor, int nlevels, float* thr) {
  if (!thr || nlevels < 1 || nlevels > kMaxLevels || !(scale_factor > 1.0f))
    return mfail(ORBX_EINVAL, "bad argument");
  const float logsf = std::log(scale_factor);  // Frame::mfLogScaleFactor (src/Frame.cc:70)
  for (int k = 1; k < nlevels; ++k) {
    // least positive float r with level(r) >= k; level is non-decreasing in r
    uint32_t lo = 0x00000001u, hi = 0x7f7fffffu;  // level(lo) = 0 < k <= level(FLT_MAX)
    auto at = [](uint32_t b) {
      float f;
      std::memcpy(&f, &b, 4);
      return f;
    };
    if (host_predict_direct(at(hi), logsf, nlevels) < k) return mfail(ORBX_EINVAL, "scale factor too small");
    while (hi - lo > 1) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (host_predict_direct(at(mid), logsf, nlevels) >= k)
        hi = mid;
      else
        lo = mid;
    }
    thr[k - 1] = at(hi);
  }
  for (int k = nlevels; k <= kMaxLevels; ++k) thr[k - 1 < kMaxLevels ? k - 1 : 0] = INFINITY;
  return ORBX_OK;
}

int orbm_predict_scale(float max_distance, float dist, float scale_factor, int nlevels) {
  float thr[kMaxLevels];
  if (orbm_predict_scale_thresholds(scale_factor, nlevels, thr)) return -1;
  const float ratio = max_distance / dist;
  if (std::isinf(ratio)) return 0;
  int l = 0;
  for (int k = 0; k < nlevels - 1; ++k) l += ratio >= thr[k];
  return l;
}

int orbm_search_by_projection_pose_batch(orbm_handle m, int mode, const orbx_kp* d_kps, const uint8_t* d_desc,
                                         const int* d_n, int kp_pitch, const float* d_uright, orbm_grid_bounds b,
                                         const float* scale, int nlevels, float scale_factor,
                                         const uint8_t* d_blocked, const orbm_pose* d_poses,
                                         const orbm_map_point_world* d_mps, const uint8_t* d_mpdesc,
                                         const int* d_nmp, int mp_pitch, int frames, float th, int dist_th,
                                         int check_ori, const float* inv_sigma2, int* d_out, int* d_nmatches,
                                         void* stream) {
  if (!m || !d_kps || !d_desc || !d_n || !scale || !d_blocked || !d_poses || !d_mps || !d_mpdesc || !d_nmp ||
      !d_out || !d_nmatches || frames < 1 || kp_pitch < 1 || mp_pitch < 1 || nlevels < 1 ||
      nlevels > kMaxLevels || mode < ORBM_PROJ_LAST_FRAME || mode > ORBM_PROJ_SIM3_MATCH ||
      (mode == ORBM_PROJ_FUSE && !inv_sigma2))
    return mfail(ORBX_EINVAL, "bad argument");
  if (!(b.max_x > b.min_x) || !(b.max_y > b.min_y)) return mfail(ORBX_EINVAL, "empty grid bounds");
  if (pose_lds_bytes(kp_pitch) > 156 * 1024) return mfail(ORBX_ECAPACITY, "kp_pitch %d too large", kp_pitch);
  MHIP(hipSetDevice(m->device));
  PoseParams P{};
  P.mode = mode;
  P.minX = b.min_x;
  P.maxX = b.max_x;
  P.minY = b.min_y;
  P.maxY = b.max_y;
  P.invW = 64.0f / (b.max_x - b.min_x);  // mfGridElementWidthInv (src/Frame.cc:154-155)
  P.invH = 48.0f / (b.max_y - b.min_y);
  for (int l = 0; l < kMaxLevels; ++l) P.scale[l] = scale[std::min(l, nlevels - 1)];
  if (mode != ORBM_PROJ_LAST_FRAME) {
    int rc = orbm_predict_scale_thresholds(scale_factor, nlevels, P.pred_thr);
    if (rc) return rc;
  }
  P.L = nlevels;
  P.th = th;
  P.dist_th = dist_th;
  P.check_ori = check_ori;
  P.kp_pitch = kp_pitch;
  P.mp_pitch = mp_pitch;
  P.has_uright = d_uright != nullptr && (mode == ORBM_PROJ_LAST_FRAME || mode == ORBM_PROJ_FUSE);
  for (int l = 0; l < kMaxLevels; ++l) P.inv_sigma2[l] = inv_sigma2 ? inv_sigma2[std::min(l, nlevels - 1)] : 0.f;
  P.max_rounds = 32;
  if (const char* e = getenv("ORBX_PROJ_ROUNDS")) P.max_rounds = atoi(e);  // tests: force the sequential pass
  const size_t need = (size_t)frames * mp_pitch;
  if (m->ws.before((hipStream_t)stream)) return mfail(ORBX_EDEVICE, "stream wait on the workspace failed");
  if (m->pose_picks_cap < need) {
    if (m->ws.ev) MHIP(hipEventSynchronize(m->ws.ev));
    if (m->pose_picks) MHIP(hipFree(m->pose_picks));
    m->pose_picks = nullptr;
    m->pose_picks_cap = 0;
    if (hipMalloc(&m->pose_picks, need * 4) != hipSuccess) return mfail(ORBX_ENOMEM, "pose picks workspace");
    m->pose_picks_cap = need;
  }
  if (launch_search_pose(P, d_kps, d_desc, d_n, d_uright, d_blocked, d_poses, d_mps, d_mpdesc, d_nmp, frames,
                         m->pose_picks, d_out, d_nmatches, stream))
    return mfail(ORBX_EDEVICE, "search_pose launch: %s", hipGetErrorString(hipGetLastError()));
  if (m->ws.after((hipStream_t)stream)) return mfail(ORBX_EDEVICE, "event record failed");
  return ORBX_OK;
}

namespace {
// One frame through orbm_search_by_projection_pose_batch from host buffers.
int pose_sync(orbm_handle m, int mode, const orbx_kp* kps, const uint8_t* desc, int n, const float* uright,
              orbm_grid_bounds b, const float* scale, int nlevels, float scale_factor, const uint8_t* blocked,
              const orbm_pose& pose, const orbm_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th,
              int dist_th, int check_ori, int* out, int* nmatches, const float* inv_sigma2 = nullptr) {
  const bool pp = mode == ORBM_PROJ_FUSE || mode == ORBM_PROJ_FUSE_SIM3 || mode == ORBM_PROJ_SIM3_MATCH;
  if (!m || !nmatches || n < 0 || nmp < 0 || (n && (!kps || !desc)) || (nmp && (!mps || !mpdesc)) ||
      ((pp ? nmp : n) && !out))
    return mfail(ORBX_EINVAL, "bad argument");
  MHIP(hipSetDevice(m->device));
  const int kp = std::max(n, 1), mp = std::max(nmp, 1);
  const size_t sz[] = {(size_t)kp * sizeof(orbx_kp), (size_t)kp * 32, (size_t)kp * 4, (size_t)kp,
                       (size_t)mp * sizeof(orbm_map_point_world), (size_t)mp * 32, (size_t)(pp ? mp : kp) * 4, 16,
                       sizeof(orbm_pose)};
  size_t off[9], tot = 0;
  for (int i = 0; i < 9; ++i) {
    off[i] = tot;
    tot += (sz[i] + 255) & ~(size_t)255;
  }
  int rc;
  if ((rc = stage_reserve(m, tot))) return rc;
  uint8_t* s = (uint8_t*)m->stage;
  if (!m->stream) MHIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
  hipStream_t st = m->stream;
  int* cnt = (int*)(s + off[7]);  // n, nmp, nmatches
  const int hn[2] = {n, nmp};
  std::vector<uint8_t> bl(kp, 0);
  if (blocked && n) std::memcpy(bl.data(), blocked, n);
  if (n) {
    MHIP(hipMemcpyAsync(s + off[0], kps, (size_t)n * sizeof(orbx_kp), hipMemcpyHostToDevice, st));
    MHIP(hipMemcpyAsync(s + off[1], desc, (size_t)n * 32, hipMemcpyHostToDevice, st));
    if (uright) MHIP(hipMemcpyAsync(s + off[2], uright, (size_t)n * 4, hipMemcpyHostToDevice, st));
  }
  MHIP(hipMemcpyAsync(s + off[3], bl.data(), (size_t)kp, hipMemcpyHostToDevice, st));
  if (nmp) {
    MHIP(hipMemcpyAsync(s + off[4], mps, (size_t)nmp * sizeof(orbm_map_point_world), hipMemcpyHostToDevice, st));
    MHIP(hipMemcpyAsync(s + off[5], mpdesc, (size_t)nmp * 32, hipMemcpyHostToDevice, st));
  }
  MHIP(hipMemcpyAsync(cnt, hn, 8, hipMemcpyHostToDevice, st));
  MHIP(hipMemcpyAsync(s + off[8], &pose, sizeof pose, hipMemcpyHostToDevice, st));
  rc = orbm_search_by_projection_pose_batch(
      m, mode, (const orbx_kp*)(s + off[0]), s + off[1], cnt, kp, uright ? (const float*)(s + off[2]) : nullptr, b,
      scale, nlevels, scale_factor, s + off[3], (const orbm_pose*)(s + off[8]),
      (const orbm_map_point_world*)(s + off[4]), s + off[5], cnt + 1, mp, 1, th, dist_th, check_ori, inv_sigma2,
      (int*)(s + off[6]), cnt + 2, st);
  if (rc) return rc;
  int nm = 0;
  MHIP(hipMemcpyAsync(&nm, cnt + 2, 4, hipMemcpyDeviceToHost, st));
  const int nout = pp ? nmp : n;
  if (nout) MHIP(hipMemcpyAsync(out, s + off[6], (size_t)nout * 4, hipMemcpyDeviceToHost, st));
  MHIP(hipStreamSynchronize(st));
  *nmatches = nm;
  return ORBX_OK;
}
}  // namespace

int orbm_search_by_projection_last_frame(orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n,
                                         const float* uright, orbm_grid_bounds b, const float* scale, int nlevels,
                                         const uint8_t* blocked, const orbm_camera* cur, const float* Tlw,
                                         const orbm_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th,
                                         int mono, int check_ori, int* out, int* nmatches) {
  orbm_pose pose;
  int rc = orbm_prepare_pose(ORBM_PROJ_LAST_FRAME, cur, Tlw, mono, &pose);
  if (rc) return rc;
  return pose_sync(m, ORBM_PROJ_LAST_FRAME, kps, desc, n, uright, b, scale, nlevels, 1.2f, blocked, pose, mps,
                   mpdesc, nmp, th, 100 /* TH_HIGH */, check_ori, out, nmatches);
}

int orbm_search_by_projection_keyframe(orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n,
                                       orbm_grid_bounds b, const float* scale, int nlevels, float scale_factor,
                                       const uint8_t* has_mp, const orbm_camera* cur,
                                       const orbm_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th,
                                       int orb_dist, int check_ori, int* out, int* nmatches) {
  orbm_pose pose;
  int rc = orbm_prepare_pose(ORBM_PROJ_KEYFRAME, cur, nullptr, 0, &pose);
  if (rc) return rc;
  return pose_sync(m, ORBM_PROJ_KEYFRAME, kps, desc, n, nullptr, b, scale, nlevels, scale_factor, has_mp, pose,
                   mps, mpdesc, nmp, th, orb_dist, check_ori, out, nmatches);
}

int orbm_search_by_projection_sim3(orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n,
                                   orbm_grid_bounds b, const float* scale, int nlevels, float scale_factor,
                                   const orbm_camera* kf, const orbm_map_point_world* mps, const uint8_t* mpdesc,
                                   int nmp, int th, const int* matched, int* out, int* nmatches) {
  orbm_pose pose;
  int rc = orbm_prepare_pose(ORBM_PROJ_SIM3, kf, nullptr, 0, &pose);
  if (rc) return rc;
  std::vector<uint8_t> bl(std::max(n, 1), 0);
  if (matched)
    for (int i = 0; i < n; ++i) bl[i] = matched[i] >= 0;  // vpMatched[idx] set on entry
  return pose_sync(m, ORBM_PROJ_SIM3, kps, desc, n, nullptr, b, scale, nlevels, scale_factor, bl.data(), pose, mps,
                   mpdesc, nmp, (float)th, 50 /* TH_LOW */, 0, out, nmatches);
}

int orbm_fuse(orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n, const float* uright, orbm_grid_bounds b,
              const float* scale, const float* inv_sigma2, int nlevels, float scale_factor, const orbm_camera* kf,
              const orbm_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th, int* out, int* nfused) {
  if (!inv_sigma2) return mfail(ORBX_EINVAL, "bad argument");
  orbm_pose pose;
  int rc = orbm_prepare_pose(ORBM_PROJ_FUSE, kf, nullptr, 0, &pose);
  if (rc) return rc;
  return pose_sync(m, ORBM_PROJ_FUSE, kps, desc, n, uright, b, scale, nlevels, scale_factor, nullptr, pose, mps,
                   mpdesc, nmp, th, 50 /* TH_LOW */, 0, out, nfused, inv_sigma2);
}

int orbm_fuse_sim3(orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n, orbm_grid_bounds b,
                   const float* scale, int nlevels, float scale_factor, const orbm_camera* kf,
                   const orbm_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th, int* out, int* nfused) {
  orbm_pose pose;
  int rc = orbm_prepare_pose(ORBM_PROJ_FUSE_SIM3, kf, nullptr, 0, &pose);
  if (rc) return rc;
  return pose_sync(m, ORBM_PROJ_FUSE_SIM3, kps, desc, n, nullptr, b, scale, nlevels, scale_factor, nullptr, pose,
                   mps, mpdesc, nmp, th, 50 /* TH_LOW */, 0, out, nfused);
}

int orbm_search_by_sim3(orbm_handle m, const orbx_kp* kps1, const uint8_t* desc1, int n1, orbm_grid_bounds b1,
                        const float* T1w, const orbm_map_point_world* mps1, const uint8_t* mpdesc1,
                        const orbx_kp* kps2, const uint8_t* desc2, int n2, orbm_grid_bounds b2, const float* T2w,
                        const orbm_map_point_world* mps2, const uint8_t* mpdesc2, const float* scale, int nlevels,
                        float scale_factor, const orbm_camera* cam1, float s12, const float* R12, const float* t12,
                        float th, int* match12, int* nfound) {
  if (!nfound || n1 < 0 || n2 < 0 || (n1 && !match12)) return mfail(ORBX_EINVAL, "bad argument");
  orbm_pose pz[2];
  int rc = orbm_prepare_sim3_match(cam1, T1w, T2w, s12, R12, t12, pz);
  if (rc) return rc;
  // direction 1: pKF1's points into pKF2 (vnMatch1); direction 2: pKF2's into pKF1 (vnMatch2)
  std::vector<int> vn1(std::max(n1, 1), -1), vn2(std::max(n2, 1), -1);
  int c1 = 0, c2 = 0;
  if ((rc = pose_sync(m, ORBM_PROJ_SIM3_MATCH, kps2, desc2, n2, nullptr, b2, scale, nlevels, scale_factor, nullptr,
                      pz[0], mps1, mpdesc1, n1, th, 100 /* TH_HIGH */, 0, vn1.data(), &c1)))
    return rc;
  if ((rc = pose_sync(m, ORBM_PROJ_SIM3_MATCH, kps1, desc1, n1, nullptr, b1, scale, nlevels, scale_factor, nullptr,
                      pz[1], mps2, mpdesc2, n2, th, 100 /* TH_HIGH */, 0, vn2.data(), &c2)))
    return rc;
  // Check agreement (:1295-1312)
  int nFound = 0;
  for (int i1 = 0; i1 < n1; i1++) {
    match12[i1] = -1;
    const int idx2 = vn1[i1];
    if (idx2 >= 0 && idx2 < n2 && vn2[idx2] == i1) {
      match12[i1] = idx2;
      nFound++;
    }
  }
  *nfound = nFound;
  return ORBX_OK;
}

int orbm_prepare_triangulation(const float* cw1, const float* T2w, const float* cam2, const float* F12,
                               orbm_tri_pair* out) {
  if (!cw1 || !T2w || !cam2 || !F12 || !out) return mfail(ORBX_EINVAL, "bad argument");
  // C2 = R2w*Cw + t2w; invz = 1.0f/C2.z; ex = fx*C2.x*invz + cx (src/ORBmatcher.cc:664-670)
  float C2[3];
  host_rx_t(T2w, cw1, C2);
  const float invz = 1.0f / C2[2];
  orbm_tri_pair t{};
  std::memcpy(t.F12, F12, sizeof t.F12);
  t.ex = cam2[0] * C2[0] * invz + cam2[2];
  t.ey = cam2[1] * C2[1] * invz + cam2[3];
  *out = t;
  return ORBX_OK;
}

int orbm_search_for_triangulation_batch(
    orbm_handle m, const orbx_kp* d_kps1, const uint8_t* d_desc1, const float* d_uright1, const uint8_t* d_has_mp1,
    const int* d_n1, const uint32_t* d_nodes1, const int* d_off1, const int* d_idx1, const int* d_nn1, int kp_pitch1,
    int node_pitch1, const orbx_kp* d_kps2, const uint8_t* d_desc2, const float* d_uright2, const uint8_t* d_has_mp2,
    const int* d_n2, const uint32_t* d_nodes2, const int* d_off2, const int* d_idx2, const int* d_nn2, int kp_pitch2,
    int node_pitch2, const orbm_tri_pair* d_pairs, const float* scale2, const float* sigma2, int nlevels, int pairs,
    int only_stereo, int check_ori, int* d_matches12, int out_pitch, int* d_nmatches, void* stream) {
  if (!m || !d_kps1 || !d_desc1 || !d_uright1 || !d_has_mp1 || !d_n1 || !d_nodes1 || !d_off1 || !d_idx1 || !d_nn1 ||
      !d_kps2 || !d_desc2 || !d_uright2 || !d_has_mp2 || !d_n2 || !d_nodes2 || !d_off2 || !d_idx2 || !d_nn2 ||
      !d_pairs || !scale2 || !sigma2 || !d_matches12 || !d_nmatches || pairs < 1 || nlevels < 1 ||
      nlevels > kMaxLevels || kp_pitch1 < 0 || node_pitch1 < 0 || kp_pitch2 < 1 || node_pitch2 < 1 || out_pitch < 1 ||
      ((kp_pitch1 == 0) != (node_pitch1 == 0)))
    return mfail(ORBX_EINVAL, "bad argument");
  MHIP(hipSetDevice(m->device));
  TriParams P{};
  for (int l = 0; l < kMaxLevels; ++l) {
    P.scale2[l] = scale2[std::min(l, nlevels - 1)];
    P.sigma2[l] = sigma2[std::min(l, nlevels - 1)];
  }
  P.only_stereo = only_stereo;
  P.check_ori = check_ori;
  P.out_pitch = out_pitch;
  const TriSide A{d_kps1, d_desc1, d_uright1, d_has_mp1, d_n1, d_nodes1, d_off1, d_idx1, d_nn1, kp_pitch1,
                  node_pitch1};
  const TriSide B{d_kps2, d_desc2, d_uright2, d_has_mp2, d_n2, d_nodes2, d_off2, d_idx2, d_nn2, kp_pitch2,
                  node_pitch2};
  if (launch_search_tri(P, A, B, d_pairs, pairs, d_matches12, d_nmatches, stream))
    return mfail(ORBX_EDEVICE, "search_tri launch: %s", hipGetErrorString(hipGetLastError()));
  return ORBX_OK;
}

int orbm_search_for_triangulation(orbm_handle m, const orbx_kp* kps1, const uint8_t* desc1, const float* uright1,
                                  const uint8_t* has_mp1, int n1, orbm_feature_vector fv1, const orbx_kp* kps2,
                                  const uint8_t* desc2, const float* uright2, const uint8_t* has_mp2, int n2,
                                  orbm_feature_vector fv2, const float* cw1, const float* T2w, const float* cam2,
                                  const float* scale2, const float* sigma2, int nlevels, const float* F12,
                                  int only_stereo, int check_ori, int* matches12, int* nmatches) {
  if (!m || !nmatches || n1 < 0 || n2 < 0 || fv1.n_nodes < 0 || fv2.n_nodes < 0 ||
      (n1 && (!kps1 || !desc1 || !uright1 || !has_mp1 || !matches12)) ||
      (n2 && (!kps2 || !desc2 || !uright2 || !has_mp2)) || (fv1.n_nodes && (!fv1.nodes || !fv1.off)) ||
      (fv2.n_nodes && (!fv2.nodes || !fv2.off)))
    return mfail(ORBX_EINVAL, "bad argument");
  orbm_tri_pair tp;
  int rc = orbm_prepare_triangulation(cw1, T2w, cam2, F12, &tp);
  if (rc) return rc;
  const int f1 = fv1.n_nodes ? fv1.off[fv1.n_nodes] : 0, f2 = fv2.n_nodes ? fv2.off[fv2.n_nodes] : 0;
  if (f1 > n1 || f2 > n2) return mfail(ORBX_EINVAL, "feature vector holds more indices than keypoints");
  for (int i = 0; i < f1; ++i)
    if (fv1.idx[i] < 0 || fv1.idx[i] >= n1) return mfail(ORBX_EINVAL, "feature index out of range");
  for (int i = 0; i < f2; ++i)
    if (fv2.idx[i] < 0 || fv2.idx[i] >= n2) return mfail(ORBX_EINVAL, "feature index out of range");
  MHIP(hipSetDevice(m->device));
  const int k1 = std::max(n1, 1), k2 = std::max(n2, 1);
  const int nn1 = std::max(fv1.n_nodes, 1), nn2 = std::max(fv2.n_nodes, 1);
  // staging: kps, desc, uright, has_mp, nodes, off, idx per side; counts; pair
  const size_t sz[] = {(size_t)k1 * sizeof(orbx_kp), (size_t)k1 * 32, (size_t)k1 * 4, (size_t)k1,
                       (size_t)nn1 * 4, (size_t)(nn1 + 1) * 4, (size_t)k1 * 4,
                       (size_t)k2 * sizeof(orbx_kp), (size_t)k2 * 32, (size_t)k2 * 4, (size_t)k2,
                       (size_t)nn2 * 4, (size_t)(nn2 + 1) * 4, (size_t)k2 * 4,
                       32, sizeof(orbm_tri_pair), (size_t)k1 * 4};
  constexpr int NS = sizeof(sz) / sizeof(sz[0]);
  size_t off[NS], tot = 0;
  for (int i = 0; i < NS; ++i) {
    off[i] = tot;
    tot += (sz[i] + 255) & ~(size_t)255;
  }
  if ((rc = stage_reserve(m, tot))) return rc;
  uint8_t* s = (uint8_t*)m->stage;
  if (!m->stream) MHIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
  hipStream_t st = m->stream;
  auto up = [&](int slot, const void* src, size_t bytes) -> int {
    if (bytes) MHIP(hipMemcpyAsync(s + off[slot], src, bytes, hipMemcpyHostToDevice, st));
    return ORBX_OK;
  };
  const int zero = 0;
  const int cnt[6] = {n1, fv1.n_nodes, n2, fv2.n_nodes, 0, 0};
  if ((rc = up(0, kps1, (size_t)n1 * sizeof(orbx_kp))) || (rc = up(1, desc1, (size_t)n1 * 32)) ||
      (rc = up(2, uright1, (size_t)n1 * 4)) || (rc = up(3, has_mp1, (size_t)n1)) ||
      (rc = up(4, fv1.nodes, (size_t)fv1.n_nodes * 4)) ||
      (rc = up(5, fv1.n_nodes ? fv1.off : &zero, (size_t)(fv1.n_nodes + 1) * 4)) ||
      (rc = up(6, fv1.idx, (size_t)f1 * 4)) || (rc = up(7, kps2, (size_t)n2 * sizeof(orbx_kp))) ||
      (rc = up(8, desc2, (size_t)n2 * 32)) || (rc = up(9, uright2, (size_t)n2 * 4)) ||
      (rc = up(10, has_mp2, (size_t)n2)) || (rc = up(11, fv2.nodes, (size_t)fv2.n_nodes * 4)) ||
      (rc = up(12, fv2.n_nodes ? fv2.off : &zero, (size_t)(fv2.n_nodes + 1) * 4)) ||
      (rc = up(13, fv2.idx, (size_t)f2 * 4)) || (rc = up(14, cnt, sizeof cnt)) || (rc = up(15, &tp, sizeof tp)))
    return rc;
  int* c = (int*)(s + off[14]);
  rc = orbm_search_for_triangulation_batch(
      m, (const orbx_kp*)(s + off[0]), s + off[1], (const float*)(s + off[2]), s + off[3], c,
      (const uint32_t*)(s + off[4]), (const int*)(s + off[5]), (const int*)(s + off[6]), c + 1, k1, nn1,
      (const orbx_kp*)(s + off[7]), s + off[8], (const float*)(s + off[9]), s + off[10], c + 2,
      (const uint32_t*)(s + off[11]), (const int*)(s + off[12]), (const int*)(s + off[13]), c + 3, k2, nn2,
      (const orbm_tri_pair*)(s + off[15]), scale2, sigma2, nlevels, 1, only_stereo, check_ori,
      (int*)(s + off[16]), k1, c + 4, st);
  if (rc) return rc;
  int nm = 0;
  MHIP(hipMemcpyAsync(&nm, c + 4, 4, hipMemcpyDeviceToHost, st));
  if (n1) MHIP(hipMemcpyAsync(matches12, s + off[16], (size_t)n1 * 4, hipMemcpyDeviceToHost, st));
  MHIP(hipStreamSynchronize(st));
  *nmatches = nm;
  return ORBX_OK;
}

}  // extern "C"
