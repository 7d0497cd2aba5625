// orbx_front.hip — GaussianBlur + the FAST stage of ComputeKeyPointsOctTree in
// ONE pass over each pyramid level (the pyramid itself is the band kernel of
// orbx_pyramid.hip, one launch before this one).
//
// Reference: the 7x7 GaussianBlur of every level (src/ORBextractor.cc:1735-1749)
// and the FAST stage (:1128-1299): cv::FAST(cell ROI, iniThFAST, nonmax) per
// grid cell, cv::FAST(ROI, minThFAST) if that found nothing, keypoints in
// row-major order per cell. FAST on a ROI scores pixels in [3, n-3) of it and
// its 3x3 NMS sees 0 outside that band, so suppression never leaves a cell.
//
// front_tile_kernel: one 256-thread workgroup per (frame, level, cell row,
// chunk of consecutive cells). Tiles partition every level (edge tiles also
// own the border rows/columns outside the detection rectangle, which only
// the blur needs). The tile's pixels +-3 are staged in LDS ONCE, then:
//   * blur of the owned rectangle: row pass v_dot4_u32_u8, column pass
//     v_dot2_u32_u16 over a register window of row pairs (the OpenCV 3.x 8U
//     fixed-point kernel [18,34,49,55,49,34,18], (acc + 2^15) >> 16);
//   * FAST over the cell bands in flat phases, each spread over all threads:
//     compass pre-test 32 pixels per item (dword reads realigned with
//     v_alignbyte, pixel pairs gathered by v_perm into packed u16x2 ops) ->
//     survivor bits; the survivors' 16-pixel arc test -> detection bits;
//     cornerScore<16> of the detections -> a zeroed LDS score map (entry
//     lists built from the bit maps by a block scan);
//   * NMS at iniThFAST and minThFAST (strict maximum over the neighbours in
//     the same cell band) into two LDS bit maps;
//   * per cell: the iniThFAST set unless it is empty, keys written row-major
//     into the cell's fixed slot range with its count (the layout the
//     quadtree reads; identical to the per-cell FAST kernel's output).
// Rejected variant (notes/front_band_rejected.md): fusing the pyramid into
// the same pass per row band makes every level's +-4 halo cascade up the
// resize chain (+-20 rows at level 0), 148 KB of LDS and 3x slower.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orbx_device.cuh"
#include "orbx_fastcore.cuh"

namespace orbx {

#ifndef ORBX_TILE_THREADS
#define ORBX_TILE_THREADS 512
#endif
constexpr int kTlThreads = ORBX_TILE_THREADS;
constexpr int kTlList = 2048;  // FAST survivors / detections handled per pass (u16 entries)

typedef unsigned short tl_us2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t tl_dot4(uint32_t px, uint32_t taps, uint32_t acc) {
  return __builtin_amdgcn_udot4(px, taps, acc, false);
}
__device__ __forceinline__ uint32_t tl_dot2(uint32_t pair, uint32_t taps, uint32_t acc) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(tl_us2_t, pair), __builtin_bit_cast(tl_us2_t, taps), acc, false);
}

// Bresenham ring of radius 3, k = 0..15 (cv::makeOffsets, pattern 16)
__device__ __forceinline__ int tl_ring(int k, int pitch) {
  constexpr int rx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
  constexpr int ry[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
  return ry[k] * pitch + rx[k];
}

// Bits [a, a + n) (n <= 64) of a bit row with >= 2 dwords of zero pad.
__device__ __forceinline__ uint64_t bit_range(const uint32_t* row, int a, int n) {
  const int d = a >> 5, sh = a & 31;
  const uint64_t lo = (uint64_t)row[d] | ((uint64_t)row[d + 1] << 32);
  uint64_t v = lo >> sh;
  if (sh) v |= (uint64_t)row[d + 2] << (64 - sh);
  return n >= 64 ? v : v & ((1ull << n) - 1);
}

// Tile geometry shared by the host plan and the kernel.
struct TileGeom {
  int sx0, tp;        // staged columns [sx0, sx0 + tp), 16-byte aligned
  int ry0, nrow;      // staged rows [ry0, ry0 + nrow) = owned rows +-3 (reflected at the edges)
  int cx0, cx1;       // band columns of the tile's cells
  int sy, ey;         // band rows of the cell row
  int ndw;            // dwords per bit-map row (+2 zero pad)
  int o_smap, o_bm, o_cnt, o_list, o_seg, bytes;  // LDS layout
};

__host__ __device__ inline TileGeom tile_geom(const LevelGeom& g, int i, int j0, int j1, int bx0, int bx1, int by0,
                                             int by1) {
  TileGeom t;
  t.sx0 = ((bx0 & ~3) - 4) & ~15;
  t.tp = ((bx1 + 8 + 15) & ~15) - t.sx0;
  t.ry0 = by0 - 3;
  t.nrow = by1 - by0 + 6;
  t.cx0 = g.dx0 + j0 * g.wCell;
  t.cx1 = g.dx0 + j1 * g.wCell < g.dx1 ? g.dx0 + j1 * g.wCell : g.dx1;
  t.sy = g.dy0 + i * g.hCell;
  t.ey = t.sy + g.hCell < g.dy1 ? t.sy + g.hCell : g.dy1;
  const int bw = t.cx1 > t.cx0 ? t.cx1 - t.cx0 : 0;
  t.ndw = (bw + 31) / 32 + 2;
  auto r16 = [](int b) { return (b + 15) & ~15; };
  // tile pixels | score map (band rows +-1) | 4 bit maps (survivors,
  // detections, kept at iniThFAST, kept at minThFAST) | per-item counts |
  // entry list | per-cell segment counts
  t.o_smap = r16(t.nrow * t.tp);
  t.o_bm = t.o_smap + r16((g.hCell + 2) * t.tp);
  t.o_cnt = t.o_bm + r16(4 * g.hCell * t.ndw * 4);
  t.o_list = t.o_cnt + r16((g.hCell * t.ndw + 1) * 4);
  t.o_seg = t.o_list + r16(kTlList * 2);
  const int nseg = (j1 - j0) * g.hCell;
  t.bytes = t.o_seg + r16((nseg + 1 + (j1 - j0) + 8 + 2 * (j1 - j0)) * 4);
  return t;
}

__global__ __launch_bounds__(kTlThreads) void front_tile_kernel(ExtractParams P, LevelPtrs lp,
                                                                const int4* __restrict__ tiles,
                                                                const CellGeom* __restrict__ cells,
                                                                uint8_t* __restrict__ blur,
                                                                uint32_t* __restrict__ slots,
                                                                int* __restrict__ cell_counts, int* dbg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x;
  // diagnostics (ORBX_FRONT_PROF=1): cycles per phase, thread 0 of each workgroup
  unsigned long long t_ph = __builtin_amdgcn_s_memtime();
  auto mark = [&](int ph) {
    if (!dbg) return;
    lds_sync();
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    if (tid == 0) dbg[blockIdx.x * 8 + ph] = (int)(n - t_ph);
    t_ph = n;
  };
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int f = wg / P.tl_per_frame, ti = wg - f * P.tl_per_frame;
  const int4 ta = tiles[2 * ti], tb = tiles[2 * ti + 1];
  const int l = ta.x, i = ta.y, j0 = ta.z, j1 = ta.w;
  const int bx0 = tb.x, bx1 = tb.y, by0 = tb.z, by1 = tb.w;
  const LevelGeom& g = P.lv[l];
  const int w = g.w, h = g.h;
  const TileGeom T = tile_geom(g, i, j0, j1, bx0, bx1, by0, by1);
  const int tp = T.tp;
  uint8_t* tile = smem;
  uint8_t* smap = smem + T.o_smap;                   // rows [sy - 1, ey + 1)
  uint32_t* bmS = (uint32_t*)(smem + T.o_bm);       // bit maps, rows [sy, ey) x ndw each
  uint32_t* bmD = bmS + g.hCell * T.ndw;
  uint32_t* bmI = bmD + g.hCell * T.ndw;
  uint32_t* bmM = bmI + g.hCell * T.ndw;
  int* s_cnt = (int*)(smem + T.o_cnt);
  uint16_t* list = (uint16_t*)(smem + T.o_list);
  int* s_seg = (int*)(smem + T.o_seg);
  int* s_ini = s_seg + (j1 - j0) * g.hCell + 1;
  int* s_tmp = s_ini + (j1 - j0);
  int2* s_cinfo = (int2*)(s_tmp + 8);  // {slot_off, cap} of the tile's cells
  const bool has_band = T.cx0 < T.cx1 && T.sy < T.ey;

  // ---- stage the tile: rows ry0 .. ry0+nrow-1 and columns sx0 .. sx0+tp-1,
  // BORDER_REFLECT_101 outside the level; chunks fully inside the level are
  // 16-byte loads, four in flight per thread, the rest byte gathers
  {
    const uint8_t* S = lp.base[l] + f * lp.fstride[l];
    const int pitch = lp.pitch[l], nch = tp >> 4, total = T.nrow * nch;
    const bool al = lp.aligned16[l];
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    for (int q0 = tid; q0 < total; q0 += 4 * kTlThreads) {
      u32x4 v[4];
      int so[4], gy[4], gx[4];
      bool direct[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = min(q0 + u * kTlThreads, total - 1);
        const int r = q / nch, c = q - r * nch;
        gy[u] = reflect101_clamped(T.ry0 + r, h);
        gx[u] = T.sx0 + 16 * c;
        so[u] = r * tp + 16 * c;
        direct[u] = al && gx[u] >= 0 && gx[u] + 16 <= w;
        v[u] = *(const u32x4*)(S + (long long)gy[u] * pitch + (direct[u] ? gx[u] : 0));
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (q0 + u * kTlThreads >= total) break;
        if (direct[u]) {
          *(u32x4*)(tile + so[u]) = v[u];
        } else {
          const uint8_t* row = S + (long long)gy[u] * pitch;
#pragma unroll
          for (int k = 0; k < 16; ++k) tile[so[u] + k] = row[reflect101_clamped(gx[u] + k, w)];
        }
      }
    }
    for (int j = tid; j < j1 - j0; j += kTlThreads) {
      const int4 raw = ((const int4*)cells)[g.cell0 + i * g.nCols + j0 + j];
      s_cinfo[j] = make_int2(raw.z, (int16_t)(raw.w & 0xFFFF));
    }
    // zero the score map and the bit maps
    if (has_band) {
      uint4* z = (uint4*)smap;
      const int n16 = (T.o_cnt - T.o_smap) >> 4;
      for (int q = tid; q < n16; q += kTlThreads) z[q] = make_uint4(0, 0, 0, 0);
    }
  }
  lds_sync();
  mark(0);
  // pixel (x, y) of the level
  const uint8_t* px = tile - T.ry0 * tp - T.sx0;

  if (!has_band) {
    // cells of a tile without band pixels (skipped by the reference) keep nothing
    for (int j = j0 + tid; j < j1; j += kTlThreads) cell_counts[(long long)f * P.ncells_total + g.cell0 + i * g.nCols + j] = 0;
  } else {

  // ---- FAST, in flat data-parallel phases (every phase spreads its items
  // over all 256 threads; no wave waits on a chain of its own results)
  const int ndw = T.ndw, nreal = (T.cx1 - T.cx0 + 31) >> 5, nr = T.ey - T.sy, nit = nr * nreal;
  {
    // (a) compass pre-test of every band pixel, 32 pixels (one bit-map dword)
    // per item: the centre row and rows +-3 are read as dwords, realigned with
    // v_alignbyte, and pixel pairs (p, p + 16) gathered into packed u16x2
    // registers with v_perm; a 9-arc covers two of the four compass pixels, so
    // a corner at t_low has two compass pixels darker than v - t or two
    // brighter than v + t
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const int t = P.t_low;
    const u16x2 tt = {(unsigned short)t, (unsigned short)t}, one = {1, 1};
    for (int it = tid; it < nit; it += kTlThreads) {
      const int r = it / nreal, d = it - r * nreal, x0 = T.cx0 + 32 * d, n = min(32, T.cx1 - x0);
      const uint8_t* rowc = tile + (T.sy + r - T.ry0) * tp;
      const int oc = x0 - 3 - T.sx0, on = x0 - T.sx0;
      const uint32_t* wc = (const uint32_t*)rowc + (oc >> 2);
      const uint32_t* wu = (const uint32_t*)(rowc - 3 * tp) + (on >> 2);
      const uint32_t* wd = (const uint32_t*)(rowc + 3 * tp) + (on >> 2);
      uint32_t Wc[11], Wu[9], Wd[9];
#pragma unroll
      for (int k = 0; k < 11; ++k) Wc[k] = wc[k];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        Wu[k] = wu[k];
        Wd[k] = wd[k];
      }
      const int shc = oc & 3, shn = on & 3;
      uint32_t Cs[10], Us[8], Ds[8];
#pragma unroll
      for (int k = 0; k < 10; ++k) Cs[k] = __builtin_amdgcn_alignbyte(Wc[k + 1], Wc[k], shc);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        Us[k] = __builtin_amdgcn_alignbyte(Wu[k + 1], Wu[k], shn);
        Ds[k] = __builtin_amdgcn_alignbyte(Wd[k + 1], Wd[k], shn);
      }
      // bytes q and q + 16 of a stream as u16x2 {lo = byte q, hi = byte q+16}
      auto pair = [](const uint32_t* S, int q) {
        const uint32_t b = q & 3, sel = b | (0x0Cu << 8) | ((4u + b) << 16) | (0x0Cu << 24);
        return __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(S[(q >> 2) + 4], S[q >> 2], sel));
      };
      uint32_t bits = 0;
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const u16x2 v = pair(Cs, p + 3), n12 = pair(Cs, p), n4 = pair(Cs, p + 6);
        const u16x2 n0 = pair(Ds, p), n8 = pair(Us, p);
        const u16x2 s1 = __builtin_elementwise_min(n0, n4), l1 = __builtin_elementwise_max(n0, n4);
        const u16x2 s2 = __builtin_elementwise_min(n8, n12), l2 = __builtin_elementwise_max(n8, n12);
        const u16x2 a = __builtin_elementwise_max(s1, s2), b = __builtin_elementwise_min(l1, l2);
        const u16x2 dk =
            __builtin_elementwise_sub_sat(__builtin_elementwise_sub_sat(v, tt), __builtin_elementwise_min(a, b));
        const u16x2 br = __builtin_elementwise_sub_sat(__builtin_elementwise_max(a, b), v + tt);
        const u16x2 m = __builtin_elementwise_min(dk | br, one);
        bits |= __builtin_bit_cast(uint32_t, m) << p;
      }
      bits &= n >= 32 ? ~0u : (1u << n) - 1;
      bmS[r * ndw + d] = bits;
      s_cnt[it] = __popc(bits);
    }
  }
  lds_sync();
  mark(2);
  // entries of bit map `bm` with global index [base, base + kTlList) -> list
  // (u16: band row << 10 | tile column); s_cnt holds the items' exclusive offsets
  auto build_list = [&](const uint32_t* bm, int base) {
    for (int it = tid; it < nit; it += kTlThreads) {
      const int r = it / nreal, d = it - r * nreal;
      uint32_t bits = bm[r * ndw + d];
      int pos = s_cnt[it] - base;
      if (pos >= kTlList || pos + __popc(bits) <= 0) continue;
      const int xo = T.cx0 + 32 * d - T.sx0;
      while (bits) {
        const int kb = __builtin_ctz(bits);
        bits &= bits - 1;
        if (pos >= 0 && pos < kTlList) list[pos] = (uint16_t)((r << 10) | (xo + kb));
        ++pos;
      }
    }
  };
  auto set_bit = [&](uint32_t* bm, int r, int xo) {
    const int b = xo + T.sx0 - T.cx0;
    atomicOr(&bm[r * ndw + (b >> 5)], 1u << (b & 31));
  };
  {
    // (b) 16-pixel arc test of the survivors -> detection bit map
    const int t = P.t_low;
    const int nsurv = block_scan_excl<kTlThreads, true>(s_cnt, nit, s_tmp);
    for (int base = 0; base < nsurv; base += kTlList) {
      build_list(bmS, base);
      lds_sync();
      mark(7);
      const int nl = min(kTlList, nsurv - base);
      for (int e = tid; e < nl; e += kTlThreads) {
        const int ent = list[e], r = ent >> 10, xo = ent & 1023;
        const uint8_t* c = tile + (T.sy + r - T.ry0) * tp + xo;
        const int v = c[0];
        uint32_t dk = 0, br = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int p = c[tl_ring(k, tp)];
          dk |= (uint32_t)(p < v - t) << k;
          br |= (uint32_t)(p > v + t) << k;
        }
        if (has_arc9(dk) || has_arc9(br)) set_bit(bmD, r, xo);
      }
      lds_sync();
    }
    mark(3);
    // (c) cornerScore<16> of the detections -> score map; (d) NMS at
    // iniThFAST and minThFAST inside each cell band -> kept bit maps
    for (int it = tid; it < nit; it += kTlThreads) {
      const int r = it / nreal, d = it - r * nreal;
      s_cnt[it] = __popc(bmD[r * ndw + d]);
    }
    lds_sync();
    const int ndet = block_scan_excl<kTlThreads, true>(s_cnt, nit, s_tmp);
    for (int base = 0; base < ndet; base += kTlList) {
      build_list(bmD, base);
      lds_sync();
      const int nl = min(kTlList, ndet - base);
      for (int e = tid; e < nl; e += kTlThreads) {
        const int ent = list[e], r = ent >> 10, xo = ent & 1023;
        const uint8_t* c = tile + (T.sy + r - T.ry0) * tp + xo;
        const int v = c[0];
        int dd[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) dd[k] = v - c[tl_ring(k, tp)];
        smap[(r + 1) * tp + xo] = (uint8_t)corner_score16(dd, t);
      }
      lds_sync();
    }
    mark(4);
    const int ti = P.t_ini, tm = P.t_min;
    for (int base = 0; base < ndet; base += kTlList) {
      if (ndet > kTlList) {  // the list holds the last pass: rebuild
        build_list(bmD, base);
        lds_sync();
      }
      const int nl = min(kTlList, ndet - base);
      for (int e = tid; e < nl; e += kTlThreads) {
        const int ent = list[e], r = ent >> 10, xo = ent & 1023;
        const int y = T.sy + r, x = xo + T.sx0;
        const uint8_t* q = smap + (r + 1) * tp + xo;
        const int s = q[0];
        const int cy = (y - g.dy0) % g.hCell, cx = (x - g.dx0) % g.wCell;
        const bool U = cy != 0, Dn = cy != g.hCell - 1 && y + 1 < g.dy1;
        const bool Lf = cx != 0, Rt = cx != g.wCell - 1 && x + 1 < g.dx1;
        const int nbv[8] = {Lf ? q[-1] : 0,          Rt ? q[1] : 0,       (U && Lf) ? q[-tp - 1] : 0,
                            U ? q[-tp] : 0,          (U && Rt) ? q[-tp + 1] : 0, (Dn && Lf) ? q[tp - 1] : 0,
                            Dn ? q[tp] : 0,          (Dn && Rt) ? q[tp + 1] : 0};
        bool gi = s >= ti && s > 0, gm = s >= tm && s > 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int xv = nbv[j];
          if (xv >= ti && xv >= s) gi = false;
          if (xv >= tm && xv >= s) gm = false;
        }
        if (gi) set_bit(bmI, r, xo);
        if (gm) set_bit(bmM, r, xo);
      }
      lds_sync();
    }
  }
  mark(5);

  // ---- per cell: the iniThFAST set unless empty, keys row-major into the cell's slots
  {
    const int nc = j1 - j0, hm = g.hCell, nseg = nc * hm;
    for (int j = tid; j < nc; j += kTlThreads) s_ini[j] = 0;
    lds_sync();
    auto seg_geom = [&](int s, int& r, int& a, int& n) {
      const int j = s / hm;
      r = s - j * hm;
      const int x0 = g.dx0 + (j0 + j) * g.wCell;
      a = x0 - T.cx0;
      n = T.sy + r < T.ey ? max(min(x0 + g.wCell, g.dx1) - x0, 0) : 0;
    };
    for (int s = tid; s < nseg; s += kTlThreads) {
      int r, a, n;
      seg_geom(s, r, a, n);
      if (n > 0) {
        const int c = __popcll(bit_range(bmI + r * ndw, a, n));
        if (c) atomicAdd(&s_ini[s / hm], c);
      }
    }
    lds_sync();
    for (int s = tid; s < nseg; s += kTlThreads) {
      int r, a, n;
      seg_geom(s, r, a, n);
      s_seg[s] = n > 0 ? __popcll(bit_range((s_ini[s / hm] > 0 ? bmI : bmM) + r * ndw, a, n)) : 0;
    }
    lds_sync();
    const int total = block_scan_excl<kTlThreads, true>(s_seg, nseg, s_tmp);
    if (tid == 0) s_seg[nseg] = total;
    lds_sync();
    uint32_t* fslots = slots + (long long)f * P.slots_per_frame;
    const int cbase = g.cell0 + i * g.nCols + j0;
    for (int s = tid; s < nseg; s += kTlThreads) {
      int r, a, n;
      seg_geom(s, r, a, n);
      const int j = s / hm;
      const int slot_off = s_cinfo[j].x, cap = s_cinfo[j].y;
      if (n <= 0 || cap == 0) continue;
      uint64_t bits = bit_range((s_ini[j] > 0 ? bmI : bmM) + r * ndw, a, n);
      int pos = s_seg[s] - s_seg[j * hm];
      const int y = T.sy + r;
      while (bits) {
        const int kb = __builtin_ctzll(bits);
        bits &= bits - 1;
        const int x = T.cx0 + a + kb;
        if (pos < cap) fslots[slot_off + pos] = pack_key(x - g.minBX, y - g.minBY, smap[(r + 1) * tp + x - T.sx0]);
        ++pos;
      }
    }
    int* cnt = cell_counts + (long long)f * P.ncells_total + cbase;
    for (int j = tid; j < nc; j += kTlThreads) {
      const int cap = s_cinfo[j].y;
      cnt[j] = cap ? min(s_seg[(j + 1) * hm] - s_seg[j * hm], cap) : 0;
    }
  }
  mark(6);
  }  // has_band

  // The blur runs last: its global stores count in the same vmcnt as loads
  // (gfx9), so any load issued after them would first wait for the whole
  // blur tile to drain to memory.
  // ---- blur of the owned rectangle [bx0, bx1) x [by0, by1)
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
    const int xg0 = bx0 & ~3, G = (bx1 - xg0 + 3) >> 2, nown = by1 - by0;
    const int nseg = max(1, min(kTlThreads / G, (nown + 1) >> 1));
    const int seglen = (((nown + nseg - 1) / nseg) + 1) & ~1;
    uint8_t* D = blur + g.off + (long long)f * g.plane;
    for (int t = tid; t < G * nseg; t += kTlThreads) {
      const int cgi = t % G, seg = t / G, x = xg0 + 4 * cgi;
      const int ob = by0 + seg * seglen, oe = min(ob + seglen, by1);
      if (ob >= oe) continue;
      auto rowpass = [&](int r, uint32_t (&o)[4]) {
        const uint8_t* p = px + r * tp + x;
        const uint32_t A = *(const uint32_t*)(p - 4), B = *(const uint32_t*)p, C = *(const uint32_t*)(p + 4);
        o[0] = tl_dot4(B, kB0, tl_dot4(A, kA0, 0));
        o[1] = tl_dot4(C, kC1, tl_dot4(B, kB1, tl_dot4(A, kA1, 0)));
        o[2] = tl_dot4(C, kC2, tl_dot4(B, kB2, tl_dot4(A, kA2, 0)));
        o[3] = tl_dot4(C, kC3, tl_dot4(B, kB3, 0));
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
      const bool full = x >= bx0 && x + 4 <= bx1;
      for (int o = ob; o < oe; o += 2) {
        rowpass(o + 3, ra);
        rowpass(min(o + 4, T.ry0 + T.nrow - 1), rb);  // row o+4 only feeds output o+1 < oe
        int va[4], vb[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          P3[c] = ra[c] | (rb[c] << 16);
          const uint32_t a = tl_dot2(P3[c], t6, tl_dot2(P2[c], t45, tl_dot2(P1[c], t23, tl_dot2(P0[c], t01, 1u << 15))));
          const uint32_t b = tl_dot2(P3[c], u56, tl_dot2(P2[c], u34, tl_dot2(P1[c], u12, tl_dot2(P0[c], u0, 1u << 15))));
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
          if (full) {
            *(uint32_t*)dst = packed;
          } else {
            for (int q = 0; q < 4; ++q)
              if (x + q >= bx0 && x + q < bx1) dst[q] = (uint8_t)(packed >> (8 * q));
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
  mark(1);
}

// Host: the tile list of a plan (2 int4 per tile: {level, cell row, j0, j1},
// {bx0, bx1, by0, by1}) and the largest tile's LDS bytes; 0 if no plan.
int plan_tiles(ExtractParams& P, std::vector<int4>& tl, int target_px) {
  tl.clear();
  int lds = 0;
  for (int l = 0; l < P.L; ++l) {
    const LevelGeom& g = P.lv[l];
    if (g.dx1 <= g.dx0 || g.dy1 <= g.dy0) return 0;
    // cells per tile: about target_px columns, spread evenly over the row
    const int want = std::max(1, target_px / std::max(g.wCell, 1));
    const int nchunk = (g.nCols + want - 1) / want;
    for (int i = 0; i < g.nRows; ++i)
      for (int c = 0; c < nchunk; ++c) {
        const int j0 = c * g.nCols / nchunk, j1 = (c + 1) * g.nCols / nchunk;
        if (j0 >= j1) continue;
        const int bx0 = j0 == 0 ? 0 : g.dx0 + j0 * g.wCell, bx1 = j1 == g.nCols ? g.w : g.dx0 + j1 * g.wCell;
        const int by0 = i == 0 ? 0 : g.dy0 + i * g.hCell, by1 = i == g.nRows - 1 ? g.h : g.dy0 + (i + 1) * g.hCell;
        if (bx1 <= bx0 || by1 <= by0) return 0;
        const TileGeom T = tile_geom(g, i, j0, j1, bx0, bx1, by0, by1);
        lds = std::max(lds, T.bytes);
        tl.push_back(make_int4(l, i, j0, j1));
        tl.push_back(make_int4(bx0, bx1, by0, by1));
      }
  }
  P.tl_per_frame = (int)tl.size() / 2;
  P.tl_lds = lds;
  return lds <= 64 * 1024 ? lds : 0;
}

const void* front_tile_kernel_ptr() { return (const void*)front_tile_kernel; }

int launch_front_tiles(const ExtractParams& P, const LevelPtrs& lp, const ExtractBuffers& X, int batch,
                       hipStream_t s) {
  static int* dbg = nullptr;  // diagnostics only: per-workgroup phase cycles (ORBX_FRONT_PROF=1)
  static int dbg_cap = 0;
  static const bool prof = getenv("ORBX_FRONT_PROF") && getenv("ORBX_FRONT_PROF")[0] == '1';
  const int nwg = P.tl_per_frame * batch;
  if (prof) {
    if (nwg > dbg_cap) {
      if (dbg) (void)hipFree(dbg);
      (void)hipMalloc(&dbg, (size_t)nwg * 32);
      dbg_cap = nwg;
    }
    (void)hipMemsetAsync(dbg, 0, (size_t)nwg * 32, s);
  }
  hipLaunchKernelGGL(front_tile_kernel, dim3(nwg), dim3(kTlThreads), P.tl_lds, s, P, lp, X.tiles, X.cells, X.blur,
                     X.slots, X.cell_counts, prof ? dbg : nullptr);
  if (prof) {
    std::vector<int> h((size_t)nwg * 8);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), dbg, h.size() * 4, hipMemcpyDeviceToHost);
    double a[8] = {0};
    for (int w = 0; w < nwg; ++w)
      for (int k = 0; k < 8; ++k) a[k] += h[w * 8 + k];
    fprintf(stderr,
            "front tiles: %d WGs, lds %d; avg cycles stage %.0f blur %.0f compass %.0f scan+list %.0f arc %.0f "
            "score %.0f nms %.0f cells %.0f\n",
            nwg, P.tl_lds, a[0] / nwg, a[1] / nwg, a[2] / nwg, a[7] / nwg, a[3] / nwg, a[4] / nwg, a[5] / nwg,
            a[6] / nwg);
  }
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
