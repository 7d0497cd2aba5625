// orbx_front.hip — the front half of ORBextractor::operator() in one pass
// over each level's rows: ComputePyramid (src/ORBextractor.cc:1837-1863),
// the 7x7 GaussianBlur of every level (:1735-1749) and the FAST stage of
// ComputeKeyPointsOctTree (:1128-1299: per-cell cv::FAST at iniThFAST, then
// minThFAST if the cell found nothing, strict 3x3 NMS inside the cell).
//
// front_band_kernel: one workgroup per (frame, band of rows). Bands partition
// every level's rows exactly as the band pyramid does (orbx_pyramid.hip); a
// band also keeps its owned rows +-4 of each level in LDS (blur +-3, FAST
// ring 3 + NMS 1). Per level, with the rows in LDS once:
//   * level l >= 1 is resized from level l-1's rows (LDS to LDS), owned rows
//     written to the pyramid planes (mvImagePyramid);
//   * blur: row pass v_dot4_u32_u8, column pass v_dot2_u32_u16 over a
//     register window of row pairs, owned rows written to the blur planes;
//   * FAST: every wave streams (row pair, 64 columns) items through a compass
//     pre-test (two rows per packed u16x2 op) into a wave-private ring of
//     survivors; each full 64 of survivors gets the 16-pixel arc test, each
//     full 64 of detections gets cornerScore<16>, so lanes stay busy; scores
//     land in a zeroed LDS score map (owned rows +-1);
//   * NMS: per owned row, 32 pixels per thread, only at nonzero scores:
//     strict maximum over the 8 neighbours inside the pixel's cell band
//     (cv::FAST on the cell ROI sees 0 outside it) at both thresholds; the
//     two survivor sets go out as bit rows, the survivors' scores to a score
//     plane.
// cell_compact_kernel: one workgroup per (frame, level, cell row) turns the
// bit rows into the per-cell key lists of the per-stage FAST kernel (same
// slots, same order: row-major inside a cell, iniThFAST set unless empty),
// so the quadtree and everything after it is shared with that path.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orbx_device.cuh"
#include "orbx_fastcore.cuh"

namespace orbx {

#ifndef ORBX_FRONT_THREADS
#define ORBX_FRONT_THREADS 512
#endif
constexpr int kFrThreads = ORBX_FRONT_THREADS;
constexpr int kFrWaves = kFrThreads / 64;
constexpr int kFrRing = 128;  // per-wave ring entries (survivors / detections); must match front_lds_fixed()
static_assert(kFrWaves == 8, "front_lds_fixed() in orbx_host.hip sizes the rings for 8 waves");

typedef unsigned short fr_us2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t fr_dot4(uint32_t px, uint32_t taps, uint32_t acc) {
  return __builtin_amdgcn_udot4(px, taps, acc, false);
}
__device__ __forceinline__ uint32_t fr_dot2(uint32_t pair, uint32_t taps, uint32_t acc) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(fr_us2_t, pair), __builtin_bit_cast(fr_us2_t, taps), acc, false);
}

// Bresenham ring of radius 3, k = 0..15 (cv::makeOffsets, pattern 16)
__device__ __forceinline__ int fr_ring(int k, int pitch) {
  constexpr int rx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
  constexpr int ry[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
  return ry[k] * pitch + rx[k];
}

// Level l rows [cd.x, cd.y] from level l-1's rows in LDS (INTER_LINEAR fixed
// point, or the 2x2 area mean for an exact 2x step), owned rows also to HBM.
template <bool AREA2X>
__device__ __forceinline__ void front_rows(const ExtractParams& P, const LevelPtrs& lp, int l, int f,
                                           const uint8_t* src, uint8_t* dst, const int2* yt_rows, int src_lo,
                                           int2 cd, int2 own, int r0, int rstep, int xa, int xb, const int (&sx)[8],
                                           const int (&a0v)[8], const int (&a1v)[8]) {
  const LevelGeom& g = P.lv[l];
  const int spitch = P.lv[l - 1].fpitch, w = g.w;
  uint8_t* G0 = (uint8_t*)lp.base[l] + f * lp.fstride[l];
  for (int r = cd.x + r0; r <= cd.y; r += rstep) {
    const int2 yt = yt_rows[r - cd.x];
    const uint8_t* s0 = src + ((yt.x & 0xFFFF) - src_lo) * spitch + kFrontPad;
    const uint8_t* s1 = src + ((yt.x >> 16) - src_lo) * spitch + kFrontPad;
    int p00[8], p01[8], p10[8], p11[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      p00[q] = s0[sx[q]];
      p01[q] = s0[sx[q] + 1];
      p10[q] = s1[sx[q]];
      p11[q] = s1[sx[q] + 1];
    }
    int v[8];
    if (AREA2X) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = (p00[q] + p01[q] + p10[q] + p11[q] + 2) >> 2;
    } else {
      const int b0 = (short)(yt.y & 0xFFFF), b1 = (short)(yt.y >> 16);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int D0 = p00[q] * a0v[q] + p01[q] * a1v[q];
        const int D1 = p10[q] * a0v[q] + p11[q] * a1v[q];
        v[q] = sat_u8((D0 * b0 + D1 * b1 + (1 << 21)) >> 22);
      }
    }
    const uint32_t pa = pack4_u8(v[0], v[1], v[2], v[3]), pb = pack4_u8(v[4], v[5], v[6], v[7]);
    uint8_t* lrow = dst + (r - cd.x) * g.fpitch + kFrontPad;
    *(uint32_t*)(lrow + xa) = pa;
    *(uint32_t*)(lrow + xb) = pb;
    if (r >= own.x && r <= own.y) {
      uint8_t* drow = G0 + (long long)r * lp.pitch[l];
      if (xa + 4 <= w) *(uint32_t*)(drow + xa) = pa;
      else for (int q = 0; xa + q < w; ++q) drow[xa + q] = (uint8_t)(pa >> (8 * q));
      if (xb + 4 <= w) *(uint32_t*)(drow + xb) = pb;
      else for (int q = 0; xb + q < w; ++q) drow[xb + q] = (uint8_t)(pb >> (8 * q));
    }
  }
}

// Blur, FAST and NMS of level l, whose rows [cd.x, cd.y] are in `cur`; the
// score map goes to `oth` (the previous level's rows are no longer needed).
__device__ void front_level(const ExtractParams& P, int l, int f, uint8_t* cur, uint8_t* oth, int2 cd, int2 own,
                            uint8_t* __restrict__ blur, uint8_t* __restrict__ score, uint32_t* __restrict__ bitmaps,
                            uint32_t* ringS, uint32_t* ringD) {
  const LevelGeom& g = P.lv[l];
  const int w = g.w, h = g.h, fp = g.fpitch, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool has_own = own.x <= own.y;
  // FAST scores for the owned rows +-1 inside the detection rectangle; the
  // score map holds rows [fy0 - 1, fy1 + 1] (zero rows around them)
  const int fy0 = max(own.x - 1, g.dy0), fy1 = min(own.y + 1, g.dy1 - 1);
  const int sm_lo = fy0 - 1, sm_rows = fy1 - fy0 + 3;
  // ---- (1) reflect pads (x = -3..-1, w..w+2) of the level rows; zero score map
  for (int r = tid; r < cd.y - cd.x + 1; r += kFrThreads) {
    uint8_t* p = cur + r * fp + kFrontPad;
    p[-1] = p[1];
    p[-2] = p[2];
    p[-3] = p[3];
    p[w] = p[w - 2];
    p[w + 1] = p[w - 3];
    p[w + 2] = p[w - 4];
  }
  if (has_own && fy0 <= fy1) {
    uint4* z = (uint4*)oth;
    const int n16 = sm_rows * fp / 16;
    for (int i = tid; i < n16; i += kFrThreads) z[i] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  if (!has_own) return;  // uniform: the band owns no row of this level

  // ---- (2) blur of the owned rows (BORDER_REFLECT_101 rows via reflect101, columns via the pads)
  {
    const int* k = P.gauss;
    // row pass: outputs x..x+3 read bytes x-3..x+6 from the dwords A=[x-4,x), B=[x,x+4), C=[x+4,x+8)
    const uint32_t kA0 = (k[0] << 8) | (k[1] << 16) | (k[2] << 24), kB0 = k[3] | (k[4] << 8) | (k[5] << 16) | (k[6] << 24);
    const uint32_t kA1 = (k[0] << 16) | (k[1] << 24), kB1 = k[2] | (k[3] << 8) | (k[4] << 16) | (k[5] << 24), kC1 = k[6];
    const uint32_t kA2 = k[0] << 24, kB2 = k[1] | (k[2] << 8) | (k[3] << 16) | (k[4] << 24), kC2 = k[5] | (k[6] << 8);
    const uint32_t kB3 = k[0] | (k[1] << 8) | (k[2] << 16) | (k[3] << 24), kC3 = k[4] | (k[5] << 8) | (k[6] << 16);
    // column pass on row pairs {2m, 2m+1}: even output rows t01 t23 t45 t6, odd ones u0 u12 u34 u56
    const uint32_t t01 = k[0] | (k[1] << 16), t23 = k[2] | (k[3] << 16), t45 = k[4] | (k[5] << 16), t6 = k[6];
    const uint32_t u0 = k[0] << 16, u12 = k[1] | (k[2] << 16), u34 = k[3] | (k[4] << 16), u56 = k[5] | (k[6] << 16);
    const int G = (w + 3) >> 2, nown = own.y - own.x + 1;
    const int nseg = max(1, min(kFrThreads / G, (nown + 1) >> 1));
    const int seglen = (((nown + nseg - 1) / nseg) + 1) & ~1;
    uint8_t* D = blur + g.off + (long long)f * g.plane;
    for (int t = tid; t < G * nseg; t += kFrThreads) {
      const int cgi = t % G, seg = t / G, x = 4 * cgi;
      const int ob = own.x + seg * seglen, oe = min(ob + seglen, own.y + 1);
      if (ob >= oe) continue;
      auto rowpass = [&](int r, uint32_t (&o)[4]) {
        const uint8_t* p = cur + (reflect101(r, h) - cd.x) * fp + kFrontPad + x;
        const uint32_t A = *(const uint32_t*)(p - 4), B = *(const uint32_t*)p, C = *(const uint32_t*)(p + 4);
        o[0] = fr_dot4(B, kB0, fr_dot4(A, kA0, 0));
        o[1] = fr_dot4(C, kC1, fr_dot4(B, kB1, fr_dot4(A, kA1, 0)));
        o[2] = fr_dot4(C, kC2, fr_dot4(B, kB2, fr_dot4(A, kA2, 0)));
        o[3] = fr_dot4(C, kC3, fr_dot4(B, kB3, 0));
      };
      uint32_t P0[4], P1[4], P2[4], P3[4], ra[4], rb[4];
      rowpass(ob - 3, ra);
      rowpass(ob - 2, rb);
#pragma unroll
      for (int c = 0; c < 4; ++c) P0[c] = ra[c] | (rb[c] << 16);
      rowpass(ob - 1, ra);
      rowpass(ob, rb);
#pragma unroll
      for (int c = 0; c < 4; ++c) P1[c] = ra[c] | (rb[c] << 16);
      rowpass(ob + 1, ra);
      rowpass(ob + 2, rb);
#pragma unroll
      for (int c = 0; c < 4; ++c) P2[c] = ra[c] | (rb[c] << 16);
      for (int o = ob; o < oe; o += 2) {
        rowpass(o + 3, ra);
        rowpass(o + 4, rb);
        int va[4], vb[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          P3[c] = ra[c] | (rb[c] << 16);
          const uint32_t a = fr_dot2(P3[c], t6, fr_dot2(P2[c], t45, fr_dot2(P1[c], t23, fr_dot2(P0[c], t01, 1u << 15))));
          const uint32_t b = fr_dot2(P3[c], u56, fr_dot2(P2[c], u34, fr_dot2(P1[c], u12, fr_dot2(P0[c], u0, 1u << 15))));
          va[c] = min((int)(a >> 16), 255);
          vb[c] = min((int)(b >> 16), 255);
        }
        const uint32_t pa = pack4_u8(va[0], va[1], va[2], va[3]), pb = pack4_u8(vb[0], vb[1], vb[2], vb[3]);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int y = o + hh;
          if (y >= oe) break;
          const uint32_t packed = hh ? pb : pa;
          uint8_t* dst = D + (long long)y * g.pitch + x;
          if (x + 4 <= w) {
            *(uint32_t*)dst = packed;
          } else {
            for (int q = 0; q < 4 && x + q < w; ++q) dst[q] = (uint8_t)(packed >> (8 * q));
          }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          P0[c] = P1[c];
          P1[c] = P2[c];
          P2[c] = P3[c];
        }
      }
    }
  }

  // ---- (3) FAST scores of rows [fy0, fy1] into the score map
  if (fy0 <= fy1) {
    const int t = P.t_low;
    const int nch = (g.dx1 - g.dx0 + 63) >> 6, nrp = (fy1 - fy0 + 2) >> 1;
    int sH = 0, sT = 0, dH = 0, dT = 0;  // ring heads (consumed) and tails (appended), wave-uniform
    const uint8_t* lvl = cur - cd.x * fp + kFrontPad;  // pixel (x, y) at lvl[y * fp + x]
    uint8_t* smap = oth - sm_lo * fp + kFrontPad;
    // 16-pixel arc test of n <= 64 survivors; detections move to ringD
    auto ring_batch = [&](int n) {
      const uint32_t e = lane < n ? ringS[(sH + lane) & (kFrRing - 1)] : 0u;
      bool det = false;
      if (lane < n) {
        const uint8_t* c = lvl + (int)(e >> 16) * fp + (int)(e & 0xFFFF);
        const int v = c[0];
        uint32_t dk = 0, br = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int px = c[fr_ring(k, fp)];
          dk |= (uint32_t)(px < v - t) << k;
          br |= (uint32_t)(px > v + t) << k;
        }
        det = has_arc9(dk) || has_arc9(br);
      }
      sH += n;
      const uint64_t m = __ballot(det);
      if (det) ringD[(dT + mbcnt64(m)) & (kFrRing - 1)] = e;
      dT += __popcll(m);
      __builtin_amdgcn_wave_barrier();
    };
    // cornerScore<16> of n <= 64 detections
    auto score_batch = [&](int n) {
      if (lane < n) {
        const uint32_t e = ringD[(dH + lane) & (kFrRing - 1)];
        const int y = (int)(e >> 16), x = (int)(e & 0xFFFF);
        const uint8_t* c = lvl + y * fp + x;
        const int v = c[0];
        int d[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = v - c[fr_ring(k, fp)];
        smap[y * fp + x] = (uint8_t)corner_score16(d, t);
      }
      dH += n;
      __builtin_amdgcn_wave_barrier();
    };
    auto append = [&](bool flag, uint32_t key) {
      const uint64_t m = __ballot(flag);
      if (flag) ringS[(sT + mbcnt64(m)) & (kFrRing - 1)] = key;
      sT += __popcll(m);
      __builtin_amdgcn_wave_barrier();
      if (sT - sH >= 64) {
        ring_batch(64);
        if (dT - dH >= 64) score_batch(64);
      }
    };
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 tt = {(unsigned short)t, (unsigned short)t};
    for (int it = wave; it < nrp * nch; it += kFrWaves) {
      const int rp = it / nch, ch = it - rp * nch;
      const int y = fy0 + 2 * rp, x = g.dx0 + ch * 64 + lane;
      const bool vx = x < g.dx1, vb = y + 1 <= fy1;
      const uint8_t* cA = lvl + y * fp + min(x, g.dx1 - 1);
      const uint8_t* cB = vb ? cA + fp : cA;
      // compass pre-test, both rows in one packed u16x2 register: a 9-arc
      // covers two of the four compass pixels, so a corner at t_low has two
      // compass pixels darker than v - t or two brighter than v + t
      auto pk = [](int lo, int hi) { return (u16x2){(unsigned short)lo, (unsigned short)hi}; };
      const u16x2 v = pk(cA[0], cB[0]);
      const u16x2 n0 = pk(cA[3 * fp], cB[3 * fp]), n4 = pk(cA[3], cB[3]);
      const u16x2 n8 = pk(cA[-3 * fp], cB[-3 * fp]), n12 = pk(cA[-3], cB[-3]);
      const u16x2 s1 = __builtin_elementwise_min(n0, n4), l1 = __builtin_elementwise_max(n0, n4);
      const u16x2 s2 = __builtin_elementwise_min(n8, n12), l2 = __builtin_elementwise_max(n8, n12);
      const u16x2 a = __builtin_elementwise_max(s1, s2), b = __builtin_elementwise_min(l1, l2);
      const u16x2 dk = __builtin_elementwise_sub_sat(__builtin_elementwise_sub_sat(v, tt), __builtin_elementwise_min(a, b));
      const u16x2 br = __builtin_elementwise_sub_sat(__builtin_elementwise_max(a, b), v + tt);
      const u16x2 any = dk | br;
      append(vx && any.x != 0, (uint32_t)x | ((uint32_t)y << 16));
      append(vx && vb && any.y != 0, (uint32_t)x | ((uint32_t)(y + 1) << 16));
    }
    while (sT > sH) {
      ring_batch(min(64, sT - sH));
      if (dT - dH >= 64) score_batch(64);
    }
    while (dT > dH) score_batch(min(64, dT - dH));
  }
  __syncthreads();

  // ---- (4) per-cell NMS of the owned rows at iniThFAST and minThFAST
  const int ny0 = max(own.x, g.dy0), ny1 = min(own.y, g.dy1 - 1);
  if (ny0 <= ny1) {
    const int ndw = g.bm_ndw, nreal = (g.dx1 - g.dx0 + 31) >> 5;
    uint32_t* bmf = bitmaps + (long long)f * P.bm_per_frame + g.bm_off;
    uint8_t* scf = score + g.off + (long long)f * g.plane;
    const int ti = P.t_ini, tm = P.t_min;
    for (int it = tid; it < (ny1 - ny0 + 1) * ndw; it += kFrThreads) {
      const int r = it / ndw, d = it - r * ndw, y = ny0 + r;
      uint32_t bi = 0, bmn = 0;
      if (d < nreal) {
        const int x0 = g.dx0 + 32 * d, n = min(32, g.dx1 - x0);
        const uint8_t* srow = oth + (y - sm_lo) * fp + kFrontPad;
        // nonzero scores among x0 .. x0+n-1 from nine aligned dwords
        const int a = kFrontPad + x0, base = a & ~3, sh = a & 3;
        const uint8_t* row0 = oth + (y - sm_lo) * fp;
        uint64_t nz = 0;
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          const uint32_t wv = *(const uint32_t*)(row0 + base + 4 * q);
          uint32_t b7 = (((wv & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | wv) & 0x80808080u;
          const uint32_t nib = ((b7 >> 7) & 1u) | ((b7 >> 14) & 2u) | ((b7 >> 21) & 4u) | ((b7 >> 28) & 8u);
          nz |= (uint64_t)nib << (4 * q);
        }
        nz >>= sh;
        nz &= n >= 64 ? ~0ull : ((1ull << n) - 1);
        const int cy = (y - g.dy0) % g.hCell;
        const bool U = cy != 0, Dn = cy != g.hCell - 1 && y + 1 < g.dy1;
        while (nz) {
          const int kb = __builtin_ctzll(nz);
          nz &= nz - 1;
          const int x = x0 + kb, s = srow[x];
          const int cx = (x - g.dx0) % g.wCell;
          const bool Lf = cx != 0, Rt = cx != g.wCell - 1 && x + 1 < g.dx1;
          const uint8_t* up = srow - fp;
          const uint8_t* dn = srow + fp;
          const int nbv[8] = {Lf ? srow[x - 1] : 0,       Rt ? srow[x + 1] : 0,      (U && Lf) ? up[x - 1] : 0,
                              U ? up[x] : 0,              (U && Rt) ? up[x + 1] : 0, (Dn && Lf) ? dn[x - 1] : 0,
                              Dn ? dn[x] : 0,             (Dn && Rt) ? dn[x + 1] : 0};
          bool gi = s >= ti && s > 0, gm = s >= tm && s > 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int xv = nbv[j];
            if (xv >= ti && xv >= s) gi = false;
            if (xv >= tm && xv >= s) gm = false;
          }
          if (gi) bi |= 1u << kb;
          if (gm) bmn |= 1u << kb;
          if (gi || gm) scf[(long long)y * g.pitch + x] = (uint8_t)s;
        }
      }
      uint32_t* brow = bmf + (long long)(y - g.dy0) * 2 * ndw;
      brow[d] = bi;
      brow[ndw + d] = bmn;
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kFrThreads) void front_band_kernel(ExtractParams P, LevelPtrs lp,
                                                                const int2* __restrict__ rtab,
                                                                uint8_t* __restrict__ blur,
                                                                uint8_t* __restrict__ score,
                                                                uint32_t* __restrict__ bitmaps) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int nb = P.fr_nbands, L = P.L, tid = threadIdx.x, wave = tid >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int f = wg / nb, band = wg - f * nb;
  const int2* bt = rtab + P.fr_bands + (long long)band * L * 2;  // {comp}, {own} per level
  uint8_t* const bufA = smem;
  uint8_t* const bufB = smem + P.fr_lds_a;
  int2* const s_yt = (int2*)(smem + P.fr_lds_a + P.fr_lds_b);
  uint32_t* const ringS = (uint32_t*)(smem + P.fr_lds_a + P.fr_lds_b + P.fr_lds_y) + wave * 2 * kFrRing;
  uint32_t* const ringD = ringS + kFrRing;

  // the band's row coefficients of levels 1..L-1, one per thread, loaded
  // before the level-0 rows so both are in flight together
  int yrow = 0, ytot = 0, yarea = 1, ytab = 0;
#pragma unroll
  for (int l = 1; l < kMaxLevels; ++l) {
    const int2 cd = bt[2 * min(l, L - 1)];
    const int n = l < L ? max(cd.y - cd.x + 1, 0) : 0;
    if (tid >= ytot && tid < ytot + n) {
      yrow = cd.x + tid - ytot;
      yarea = P.lv[l].area2x;
      ytab = P.lv[l].ytab;
    }
    ytot += n;
  }
  int2 yval = make_int2(0, 0);
  if (tid < ytot) yval = yarea ? make_int2((2 * yrow) | ((2 * yrow + 1) << 16), 0) : rtab[ytab + yrow];
  for (int i = tid + kFrThreads; i < ytot; i += kFrThreads) {  // very tall bands only
    int rem = i;
    for (int l = 1; l < L; ++l) {
      const int2 cd = bt[2 * l];
      const int n = max(cd.y - cd.x + 1, 0);
      if (rem < n) {
        const LevelGeom& g = P.lv[l];
        const int r = cd.x + rem;
        s_yt[i] = g.area2x ? make_int2((2 * r) | ((2 * r + 1) << 16), 0) : rtab[g.ytab + r];
        break;
      }
      rem -= n;
    }
  }
  // ---- stage level-0 rows [comp_lo, comp_hi], full width
  {
    const int2 c0 = bt[0];
    const int rows = max(c0.y - c0.x + 1, 0), W0 = P.lv[0].w, fp0 = P.lv[0].fpitch, pitch = lp.pitch[0];
    const uint8_t* S = lp.base[0] + f * lp.fstride[0] + (long long)c0.x * pitch;
    if (lp.aligned16[0]) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const int nch = (W0 + 15) >> 4, total = rows * nch;
      for (int i0 = tid; i0 < total; i0 += 4 * kFrThreads) {
        u32x4 v[4];
        int so[4], lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = min(i0 + q * kFrThreads, total - 1);
          const int r = i / nch, ch = i - r * nch;
          lo[q] = r * pitch + ch * 16;
          so[q] = r * fp0 + kFrontPad + ch * 16;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = *(const u32x4*)(S + lo[q]);
#pragma unroll
        for (int q = 0; q < 4; ++q) *(u32x4*)(bufA + so[q]) = v[q];
      }
    } else {
      for (int r = 0; r < rows; ++r)
        for (int c = tid; c < W0; c += kFrThreads) bufA[r * fp0 + kFrontPad + c] = S[(long long)r * pitch + c];
    }
    if (tid < ytot) s_yt[tid] = yval;
  }
  // column coefficients: level l+1's are fetched while level l is processed
  int2 nxt[8];
  auto fetch_cols = [&](int l) {
    const LevelGeom& g = P.lv[l];
    const int G = (g.w + 7) >> 3, gi = tid % G;
#pragma unroll
    for (int q = 0; q < 8; ++q) nxt[q] = rtab[g.xtab2 + min(4 * (gi + (q >> 2) * G) + (q & 3), g.w - 1)];
  };
  if (L > 1) fetch_cols(1);
  __syncthreads();

  int yoff = 0;
  for (int l = 0; l < L; ++l) {
    uint8_t* cur = (l & 1) ? bufB : bufA;
    uint8_t* oth = (l & 1) ? bufA : bufB;
    const int2 cd = bt[2 * l], own = bt[2 * l + 1];
    if (l >= 1) {
      const LevelGeom& g = P.lv[l];
      const int2 cs = bt[2 * (l - 1)];
      const int G = (g.w + 7) >> 3, rstep = kFrThreads / G;
      const int gi = tid % G, r0 = tid / G;
      const int xa = 4 * gi, xb = 4 * (gi + G);
      int sx[8], a0v[8], a1v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        sx[q] = nxt[q].x;
        a0v[q] = (short)(nxt[q].y & 0xFFFF);
        a1v[q] = (short)(nxt[q].y >> 16);
      }
      if (l + 1 < L) fetch_cols(l + 1);
      if (r0 < rstep) {
        if (g.area2x)
          front_rows<true>(P, lp, l, f, oth, cur, s_yt + yoff, cs.x, cd, own, r0, rstep, xa, xb, sx, a0v, a1v);
        else
          front_rows<false>(P, lp, l, f, oth, cur, s_yt + yoff, cs.x, cd, own, r0, rstep, xa, xb, sx, a0v, a1v);
      }
      yoff += max(cd.y - cd.x + 1, 0);
      __syncthreads();
    }
    front_level(P, l, f, cur, oth, cd, own, blur, score, bitmaps, ringS, ringD);
  }
}

size_t front_lds_bytes(const ExtractParams& P) {
  return (size_t)P.fr_lds_a + P.fr_lds_b + P.fr_lds_y + (size_t)kFrWaves * 2 * kFrRing * 4;
}
const void* front_kernel_ptr() { return (const void*)front_band_kernel; }

// ----------------------------------------------------------- cell compaction
// Bits [a, a + n) (n <= 64) of a bit row (at least 2 dwords of zero pad).
__device__ __forceinline__ uint64_t bit_range(const uint32_t* row, int a, int n) {
  const int d = a >> 5, sh = a & 31;
  const uint64_t lo = (uint64_t)row[d] | ((uint64_t)row[d + 1] << 32);
  uint64_t v = lo >> sh;
  if (sh) v |= (uint64_t)row[d + 2] << (64 - sh);
  return n >= 64 ? v : v & ((1ull << n) - 1);
}

constexpr int kCcThreads = 256;
constexpr int kCcMaxSeg = 4096;  // segments (cell x band row) of one cell row
constexpr int kCcMaxCols = 160;

__global__ __launch_bounds__(kCcThreads) void cell_compact_kernel(ExtractParams P, const CellGeom* __restrict__ cells,
                                                                  const uint32_t* __restrict__ bitmaps,
                                                                  const uint8_t* __restrict__ score,
                                                                  uint32_t* __restrict__ slots,
                                                                  int* __restrict__ cell_counts) {
  __shared__ int s_seg[kCcMaxSeg + 1];
  __shared__ int s_ini[kCcMaxCols];
  __shared__ int s_tmp[kCcThreads / 64];
  const int wg = xcd_remap(blockIdx.x, gridDim.x), tid = threadIdx.x;
  const int f = wg / P.cr_per_frame;
  int i = wg - f * P.cr_per_frame, l = 0;
  for (; l < P.L - 1 && i >= P.lv[l].nRows; ++l) i -= P.lv[l].nRows;
  const LevelGeom& g = P.lv[l];
  const int nC = g.nCols, hm = g.hCell, nseg = nC * hm;
  const int sy = g.dy0 + i * g.hCell, ey = min(sy + g.hCell, g.dy1);
  const uint32_t* bm = bitmaps + (long long)f * P.bm_per_frame + g.bm_off;
  const int ndw = g.bm_ndw;
  for (int j = tid; j < nC; j += kCcThreads) s_ini[j] = 0;
  __syncthreads();
  auto seg_geom = [&](int s, int& y, int& a, int& n) {
    const int j = s / hm, r = s - j * hm;
    y = sy + r;
    const int x0 = g.dx0 + j * g.wCell;
    a = x0 - g.dx0;
    n = y < ey ? max(min(x0 + g.wCell, g.dx1) - x0, 0) : 0;
  };
  // iniThFAST survivors per cell
  for (int s = tid; s < nseg; s += kCcThreads) {
    int y, a, n;
    seg_geom(s, y, a, n);
    if (n > 0) {
      const int c = __popcll(bit_range(bm + (long long)(y - g.dy0) * 2 * ndw, a, n));
      if (c) atomicAdd(&s_ini[s / hm], c);
    }
  }
  __syncthreads();
  // the set each cell keeps (minThFAST if iniThFAST found nothing), counted per segment
  for (int s = tid; s < nseg; s += kCcThreads) {
    int y, a, n;
    seg_geom(s, y, a, n);
    int c = 0;
    if (n > 0) {
      const uint32_t* row = bm + (long long)(y - g.dy0) * 2 * ndw + (s_ini[s / hm] > 0 ? 0 : ndw);
      c = __popcll(bit_range(row, a, n));
    }
    s_seg[s] = c;
  }
  __syncthreads();
  const int total = block_scan_excl<kCcThreads>(s_seg, nseg, s_tmp);
  if (tid == 0) s_seg[nseg] = total;
  __syncthreads();
  uint32_t* fslots = slots + (long long)f * P.slots_per_frame;
  const uint8_t* scf = score + g.off + (long long)f * g.plane;
  const int cbase = g.cell0 + i * nC;
  for (int s = tid; s < nseg; s += kCcThreads) {
    int y, a, n;
    seg_geom(s, y, a, n);
    const int j = s / hm;
    const int4 raw = ((const int4*)cells)[cbase + j];
    const int slot_off = raw.z, cap = (int16_t)(raw.w & 0xFFFF);
    if (n <= 0 || cap == 0) continue;
    const uint32_t* row = bm + (long long)(y - g.dy0) * 2 * ndw + (s_ini[j] > 0 ? 0 : ndw);
    uint64_t bits = bit_range(row, a, n);
    int pos = s_seg[s] - s_seg[j * hm];
    while (bits) {
      const int kb = __builtin_ctzll(bits);
      bits &= bits - 1;
      const int x = g.dx0 + a + kb;
      if (pos < cap) fslots[slot_off + pos] = pack_key(x - g.minBX, y - g.minBY, scf[(long long)y * g.pitch + x]);
      ++pos;
    }
  }
  int* cnt = cell_counts + (long long)f * P.ncells_total + cbase;
  for (int j = tid; j < nC; j += kCcThreads) {
    const int cap = (int16_t)(((const int4*)cells)[cbase + j].w & 0xFFFF);
    cnt[j] = cap ? min(s_seg[(j + 1) * hm] - s_seg[j * hm], cap) : 0;
  }
}

int launch_front(const ExtractParams& P, const LevelPtrs& lp, const ExtractBuffers& X, int batch, hipStream_t s) {
  hipLaunchKernelGGL(front_band_kernel, dim3(P.fr_nbands * batch), dim3(kFrThreads), front_lds_bytes(P), s, P, lp,
                     X.rtab, X.blur, X.score, X.bitmaps);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

int launch_cell_compact(const ExtractParams& P, const ExtractBuffers& X, int batch, hipStream_t s) {
  hipLaunchKernelGGL(cell_compact_kernel, dim3(P.cr_per_frame * batch), dim3(kCcThreads), 0, s, P, X.cells,
                     X.bitmaps, X.score, X.slots, X.cell_counts);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

bool front_cells_fit(const ExtractParams& P) {
  for (int l = 0; l < P.L; ++l)
    if ((long long)P.lv[l].nCols * P.lv[l].hCell > kCcMaxSeg || P.lv[l].nCols > kCcMaxCols) return false;
  return true;
}

}  // namespace orbx
