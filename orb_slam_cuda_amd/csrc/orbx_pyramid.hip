// orbx_pyramid.hip — ComputePyramid (src/ORBextractor.cc:1837-1863).
//
// Level l = cv::resize(level l-1, size_l, INTER_LINEAR), chained. OpenCV 3.x
// evaluates INTER_LINEAR on u8 in fixed point: 11-bit horizontal and vertical
// coefficients (tables built on the host from the same float expressions,
// orbx_host.hip resize_tables), an int32 horizontal pass, and the vertical
// pass (D0*b0 + D1*b1 + 2^21) >> 22; columns at or beyond `xmax` replicate
// the source pixel (x2048). An exact 2x downscale switches to the 2x2 area
// mean, as cv::resize does. The 19-px border the reference pads each level
// with is never read by extraction and is not built.
//
// pyr_resize_kernel: one launch per level (each level depends on the
// previous), used when a level's band does not fit LDS. A 256-thread
// block produces a 16-row x 256-column output tile: the source rows/columns
// the tile touches are staged in LDS with 16-byte loads, then each thread
// computes a 4x4 output block from LDS and writes 4 x 32-bit stores.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orbx_device.cuh"

namespace orbx {

constexpr int kPyrTW = 256, kPyrTH = 16;
constexpr int kPyrMaxSrcW = 576;  // >= 256 * 2 (scale <= 2) + 2 + 16 alignment + 16 slack
constexpr int kPyrMaxSrcH = 36;   // >= 16 * 2 + 2 + slack

__global__ __launch_bounds__(256) void pyr_resize_kernel(
    const uint8_t* __restrict__ src, long long src_fs, int src_pitch, int sw, int sh, uint8_t* __restrict__ dst,
    long long dst_fs, int dst_pitch, int dw, int dh, const int2* __restrict__ xtab, const int2* __restrict__ ytab,
    int xmax, int area2x, int src_aligned16) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kPyrMaxSrcH][kPyrMaxSrcW];
  __shared__ int2 s_xt[kPyrTW];
  __shared__ int2 s_yt[kPyrTH];
  const int wg = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                           gridDim.x * gridDim.y * gridDim.z);
  const int f = wg / (gridDim.x * gridDim.y), tid = threadIdx.x;
  const int x0 = (wg % gridDim.x) * kPyrTW, y0 = ((wg / gridDim.x) % gridDim.y) * kPyrTH;
  const int nx = min(kPyrTW, dw - x0), ny = min(kPyrTH, dh - y0);
  const uint8_t* S = src + f * src_fs;
  // source footprint of the tile
  int sx_lo, sx_hi, sy_lo, sy_hi;  // inclusive
  if (area2x) {
    if (tid < nx) s_xt[tid] = make_int2(2 * (x0 + tid), 0);
    if (tid < ny) s_yt[tid] = make_int2(2 * (y0 + tid) | ((2 * (y0 + tid) + 1) << 16), 0);
    sx_lo = 2 * x0;
    sx_hi = 2 * (x0 + nx - 1) + 1;
    sy_lo = 2 * y0;
    sy_hi = 2 * (y0 + ny - 1) + 1;
  } else {
    if (tid < nx) s_xt[tid] = xtab[x0 + tid];
    if (tid < ny) s_yt[tid] = ytab[y0 + tid];
    sx_lo = xtab[x0].x;
    sx_hi = min(xtab[x0 + nx - 1].x + 1, sw - 1);
    sy_lo = ytab[y0].x & 0xFFFF;
    sy_hi = ytab[y0 + ny - 1].x >> 16;
  }
  const int a0 = src_aligned16 ? (sx_lo & ~15) : sx_lo;
  const int nrow = sy_hi - sy_lo + 1;
  // stage source rows [sy_lo, sy_hi], columns [a0, sx_hi]
  if (src_aligned16) {
    const int nch = (sx_hi - a0 + 16) >> 4;
    for (int i = tid; i < nrow * nch; i += 256) {
      const int r = i / nch, ch = i - r * nch;
      const uint8_t* g = S + (long long)(sy_lo + r) * src_pitch + a0 + ch * 16;
      if (a0 + ch * 16 + 16 <= src_pitch) {
        *(uint4*)&tile[r][ch * 16] = *(const uint4*)g;
      } else {  // never read past the row's pitch (the last row may end the buffer)
        for (int k = 0; k < 16 && a0 + ch * 16 + k < sw; ++k) tile[r][ch * 16 + k] = g[k];
      }
    }
  } else {
    const int ncol = sx_hi - a0 + 1;
    for (int i = tid; i < nrow * ncol; i += 256) {
      const int r = i / ncol, c = i - r * ncol;
      tile[r][c] = S[(long long)(sy_lo + r) * src_pitch + a0 + c];
    }
  }
  __syncthreads();
  // thread -> 4 columns x 4 rows
  const int cx = (tid & 63) * 4, ry = (tid >> 6) * 4;
  if (cx >= nx) return;
  int sxl[4], a0v[4], a1v[4], rep[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = min(cx + q, nx - 1);
    const int2 xt = s_xt[c];
    sxl[q] = xt.x - a0;
    a0v[q] = (short)(xt.y & 0xFFFF);
    a1v[q] = (short)(xt.y >> 16);
    rep[q] = area2x ? 0 : (x0 + c >= xmax);
  }
  uint8_t* D = dst + f * dst_fs + (long long)(y0 + ry) * dst_pitch + x0 + cx;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    if (ry + rr >= ny) break;
    const int2 yt = s_yt[ry + rr];
    const uint8_t* r0 = tile[(yt.x & 0xFFFF) - sy_lo];
    const uint8_t* r1 = tile[(yt.x >> 16) - sy_lo];
    int v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int s = sxl[q];
      if (area2x) {
        v[q] = (r0[s] + r0[s + 1] + r1[s] + r1[s + 1] + 2) >> 2;
      } else {
        int D0, D1;
        if (!rep[q]) {
          D0 = __mul24((int)r0[s], a0v[q]) + __mul24((int)r0[s + 1], a1v[q]);
          D1 = __mul24((int)r1[s], a0v[q]) + __mul24((int)r1[s + 1], a1v[q]);
        } else {
          D0 = r0[s] * 2048;
          D1 = r1[s] * 2048;
        }
        const int b0 = (short)(yt.y & 0xFFFF), b1 = (short)(yt.y >> 16);
        v[q] = sat_u8((__mul24(D0, b0) + __mul24(D1, b1) + (1 << 21)) >> 22);
      }
    }
    const uint32_t packed = pack4_u8(v[0], v[1], v[2], v[3]);
    uint8_t* drow = D + (long long)rr * dst_pitch;
    if (cx + 4 <= nx) {
      *(uint32_t*)drow = packed;  // dst pitch, x0 and cx are multiples of 4
    } else {
      for (int q = 0; cx + q < nx; ++q) drow[q] = (uint8_t)(packed >> (8 * q));
    }
  }
}

// ---------------------------------------------------------------- band pyramid
// All levels in ONE launch: a workgroup owns a tile of the last level (a
// band of rows x a column tile) and, walking the chain back, the rows and
// columns of every level that tile depends on. It stages the level-0 tile
// once (16-byte loads, all in flight), then builds level 1, 2, ... in LDS,
// each from the previous level's tile in LDS, and writes to HBM only the rows
// and columns it owns at each level (tiles partition every level; the few
// source rows and columns two tiles share are recomputed by both instead of
// exchanged). Ranges per (band, level) and (column tile, level) come from the
// host (orbx_host.hip plan_band_pyramid / plan_pyr_cols): comp = computed,
// own = written. Column tiles let a single frame (or a small batch) spread
// over more workgroups than row bands alone allow, at a few recomputed
// columns per tile edge.
#ifndef ORBX_PYR_THREADS
#define ORBX_PYR_THREADS 512
#endif
constexpr int kPyrBandThreads = ORBX_PYR_THREADS;
// waves per SIMD the band kernel is compiled for (5: <= 96 VGPRs, two
// 512-thread workgroups per CU; 6 would allow three at <= 53 KB of LDS)
#ifndef ORBX_PYR_WPE
#define ORBX_PYR_WPE 5
#endif

// Rows of one level for one thread: all 32 source bytes of a row pair are
// read before any is used, so one LDS wait covers them.
// A thread's 8 output columns are kPyrRuns runs of 8 / kPyrRuns: run k starts
// at column (8 / kPyrRuns) * (gi + k * G), G = ceil(w / 8). With runs of 2
// (default) the 32 lanes of an LDS half-wave read source bytes within ~77
// bytes (20 dwords, distinct banks of ds_read_u8); runs of 4 spread them over
// ~154 bytes (39 dwords on 32 banks: 2-way conflicts).
#ifndef ORBX_PYR_RUN
#define ORBX_PYR_RUN 2
#endif
#ifndef ORBX_PYR_ROWFAST
#define ORBX_PYR_ROWFAST 0  // A/B: thread -> (column group, row) with rows fastest
#endif
constexpr int kPyrRun = ORBX_PYR_RUN, kPyrRuns = 8 / kPyrRun;
static_assert(kPyrRun == 2 || kPyrRun == 4, "runs of 2 or 4 columns");
__device__ __forceinline__ int pyr_col(int gi, int G, int q) { return kPyrRun * (gi + (q / kPyrRun) * G) + q % kPyrRun; }

// One level of a (band, column tile): rows cd of the level, columns x0 ..
// x0 + 8G - 1 (G = ceil(comp width / 8) thread groups; sx[] are LDS-relative
// source columns). Rows and columns owned by the tile go to HBM as well.
template <bool AREA2X>
__device__ __forceinline__ void band_rows(const LevelPtrs& lp, int l, int f, const uint8_t* src, int spitch,
                                          uint8_t* dst, int dpitch, const int2* yt_rows, int src_lo, int2 cd,
                                          int2 own, int2 ownx, int x0, int r0, int rstep, int gi, int G,
                                          const int (&sx)[8], const int (&a0v)[8], const int (&a1v)[8]) {
  uint8_t* G0 = (uint8_t*)lp.base[l] + f * lp.fstride[l];
  for (int r = cd.x + r0; r <= cd.y; r += rstep) {
    const int2 yt = yt_rows[r - cd.x];
    const uint8_t* s0 = src + __mul24((yt.x & 0xFFFF) - src_lo, spitch);
    const uint8_t* s1 = src + __mul24((yt.x >> 16) - src_lo, spitch);
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
      // every factor fits 24 bits (u8 x 11-bit coefficients, D < 2^20): full-rate
      // v_mad_i32_i24 instead of the quarter-rate 32-bit multiply
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int D0 = __mul24(p00[q], a0v[q]) + __mul24(p01[q], a1v[q]);
        const int D1 = __mul24(p10[q], a0v[q]) + __mul24(p11[q], a1v[q]);
        v[q] = sat_u8((__mul24(D0, b0) + __mul24(D1, b1) + (1 << 21)) >> 22);
      }
    }
    uint8_t* lrow = dst + __mul24(r - cd.x, dpitch);
    const bool owned = r >= own.x && r <= own.y;
    uint8_t* drow = G0 + (long long)r * lp.pitch[l];
    if constexpr (kPyrRun == 4) {
      const int xa = pyr_col(gi, G, 0), xb = pyr_col(gi, G, 4);
      const uint32_t pa = pack4_u8(v[0], v[1], v[2], v[3]), pb = pack4_u8(v[4], v[5], v[6], v[7]);
      *(uint32_t*)(lrow + xa) = pa;
      *(uint32_t*)(lrow + xb) = pb;
      if (owned) {
        for (int q = 0; q < 4; ++q) {
          const int ga = x0 + xa + q, gb = x0 + xb + q;
          if (ga >= ownx.x && ga <= ownx.y) drow[ga] = (uint8_t)(pa >> (8 * q));
          if (gb >= ownx.x && gb <= ownx.y) drow[gb] = (uint8_t)(pb >> (8 * q));
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPyrRuns; ++k) {
        const int xk = pyr_col(gi, G, 2 * k);
        const uint16_t pk = (uint16_t)(sat_u8(v[2 * k]) | (sat_u8(v[2 * k + 1]) << 8));
        *(uint16_t*)(lrow + xk) = pk;  // the LDS row holds the run even past the computed columns
        // owned ranges start at even columns (plan_pyr_cols), so a run is
        // owned whole or not at all, but at the level's last column
        const int gx = x0 + xk;
        if (owned && gx >= ownx.x && gx <= ownx.y) {
          if (gx < ownx.y) *(uint16_t*)(drow + gx) = pk;
          else drow[gx] = (uint8_t)pk;
        }
      }
    }
  }
}

__global__ __launch_bounds__(kPyrBandThreads) __attribute__((amdgpu_waves_per_eu(ORBX_PYR_WPE))) void pyr_band_kernel(ExtractParams P, LevelPtrs lp,
                                                                   const int2* __restrict__ rtab, int* dbg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const unsigned long long t_begin = __builtin_amdgcn_s_memtime();
  const int nb = P.pyr_nbands, nct = P.pyr_nct, L = P.L, tid = threadIdx.x;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int f = wg / (nb * nct), tile = wg - f * (nb * nct), band = tile / nct, ct = tile - band * nct;
  const int2* bt = rtab + P.pyr_bands + (long long)band * L * 2;  // {comp}, {own} rows per level
  const int2* xt = rtab + P.pyr_ctiles + (long long)ct * L * 3;   // {comp}, {own} columns, {LDS pitch, origin}
  uint8_t* const bufA = smem;
  uint8_t* const bufB = smem + P.pyr_lds_a;
  // the band's row coefficients of every level, staged once: a global load
  // per output row would put one memory latency on every row iteration
  int2* const s_yt = (int2*)(smem + P.pyr_lds_a + P.pyr_lds_b);
  // one staged row coefficient per thread (rows of levels 1..L-1 flattened;
  // bands hold far fewer than kPyrBandThreads rows, larger ones loop), its
  // load issued before the level-0 loads so that both are in flight together
  // (no early exit and constant level indices: the band table and level
  // fields are scalar loads issued together)
  int yrow = 0, ytot = 0, yarea = 1, ytab = 0;
#pragma unroll
  for (int l = 1; l < kMaxLevels; ++l) {
    const int2 cd = bt[2 * min(l, L - 1)];
    const int n = l < L ? cd.y - cd.x + 1 : 0;
    if (tid >= ytot && tid < ytot + n) {
      yrow = cd.x + tid - ytot;
      yarea = P.lv[l].area2x;
      ytab = P.lv[l].ytab;
    }
    ytot += n;
  }
  int2 yval = make_int2(0, 0);
  if (tid < ytot) yval = yarea ? make_int2((2 * yrow) | ((2 * yrow + 1) << 16), 0) : rtab[ytab + yrow];
  for (int i = tid + kPyrBandThreads; i < ytot; i += kPyrBandThreads) {  // very tall bands only
    int rem = i;
    for (int l = 1; l < L; ++l) {
      const int2 cd = bt[2 * l];
      const int n = cd.y - cd.x + 1;
      if (rem < n) {
        const LevelGeom& g = P.lv[l];
        const int r = cd.x + rem;
        s_yt[i] = g.area2x ? make_int2((2 * r) | ((2 * r + 1) << 16), 0) : rtab[g.ytab + r];
        break;
      }
      rem -= n;
    }
  }

  // ---- stage level-0 rows [comp_lo, comp_hi] x the tile's columns, 4 loads in flight per thread
  {
    const int2 c0 = bt[0], x0c = xt[0], x0p = xt[2];
    const int rows = c0.y - c0.x + 1, lp0 = x0p.x, org = x0p.y, pitch = lp.pitch[0];
    // the last staged column: the tile's last computed one, inside the image
    // (a source column past it is only read with weight 0)
    const int xe = min(x0c.y, P.lv[0].w - 1);
    const uint8_t* S = lp.base[0] + f * lp.fstride[0] + (long long)c0.x * pitch + org;
    if (lp.aligned16[0]) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const int nch = ((xe - org) >> 4) + 1, total = rows * nch;
      // unpredicated (indices past the end repeat the last chunk)
      for (int i0 = tid; i0 < total; i0 += 4 * kPyrBandThreads) {
        u32x4 v[4];
        int so[4], lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = min(i0 + q * kPyrBandThreads, total - 1);
          const int r = i / nch, ch = i - r * nch;
          lo[q] = r * pitch + ch * 16;
          so[q] = r * lp0 + ch * 16;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = *(const u32x4*)(S + lo[q]);
        if (i0 == tid && tid < ytot) s_yt[tid] = yval;
#pragma unroll
        for (int q = 0; q < 4; ++q) *(u32x4*)(bufA + so[q]) = v[q];
      }
      if (tid >= total && tid < ytot) s_yt[tid] = yval;
    } else {
      if (tid < ytot) s_yt[tid] = yval;
      const int ncol = xe - org + 1;
      for (int r = 0; r < rows; ++r)
        for (int c = tid; c < ncol; c += kPyrBandThreads) bufA[r * lp0 + c] = S[(long long)r * pitch + c];
    }
  }

  // column coefficients: level l+1's are fetched while level l is computed
  int2 nxt[8];
  // a thread's 8 columns are kPyrRuns runs (pyr_col) with G = ceil(width/8)
  // over the tile's computed columns: neighbouring lanes read source bytes a
  // run's width x 1.2 apart
  auto fetch_cols = [&](int l) {
    const LevelGeom& g = P.lv[l];
    const int2 xc = xt[3 * l];
#if ORBX_PYR_ROWFAST
    const int G = (xc.y - xc.x + 1 + 7) >> 3, gi = min(tid / (kPyrBandThreads / G), G - 1);
#else
    const int G = (xc.y - xc.x + 1 + 7) >> 3, gi = tid % G;
#endif
#pragma unroll
    for (int q = 0; q < 8; ++q) nxt[q] = rtab[g.xtab2 + min(xc.x + pyr_col(gi, G, q), g.w - 1)];
  };
  fetch_cols(1);
  lds_sync();  // LDS only: the owned rows written to HBM are not read back here
  if (dbg && tid == 0) dbg[blockIdx.x * 16] = (int)(__builtin_amdgcn_s_memtime() - t_begin);

  // ---- levels 1 .. L-1: thread -> 8 output columns (runs of 2), rows strided
  int yoff = 0;
  for (int l = 1; l < L; ++l) {
    const LevelGeom& g = P.lv[l];
    const uint8_t* src = (l & 1) ? bufA : bufB;
    uint8_t* dst = (l & 1) ? bufB : bufA;
    const int2 cs = bt[2 * (l - 1)], cd = bt[2 * l], own = bt[2 * l + 1];
    const int2 xc = xt[3 * l], xo = xt[3 * l + 1], sp = xt[3 * (l - 1) + 2], dp = xt[3 * l + 2];
    const int G = (xc.y - xc.x + 1 + 7) >> 3, rstep = kPyrBandThreads / G;
#if ORBX_PYR_ROWFAST
    // rows fastest: a half-wave's lanes read one column group of ~rstep rows
    const int gi = tid / rstep, r0 = tid < rstep * G ? tid - gi * rstep : rstep;
#else
    const int gi = tid % G, r0 = tid / G;
#endif
    int sx[8], a0v[8], a1v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sx[q] = nxt[q].x - sp.y;  // LDS-relative: the source level's row starts at column sp.y
      a0v[q] = (short)(nxt[q].y & 0xFFFF);
      a1v[q] = (short)(nxt[q].y >> 16);
    }
    if (l + 1 < L) fetch_cols(l + 1);
    if (r0 < rstep) {
      if (g.area2x)
        band_rows<true>(lp, l, f, src, sp.x, dst, dp.x, s_yt + yoff, cs.x, cd, own, xo, xc.x, r0, rstep, gi, G, sx,
                        a0v, a1v);
      else
        band_rows<false>(lp, l, f, src, sp.x, dst, dp.x, s_yt + yoff, cs.x, cd, own, xo, xc.x, r0, rstep, gi, G, sx,
                         a0v, a1v);
    }
    yoff += cd.y - cd.x + 1;
    lds_sync();
    if (dbg && tid == 0) dbg[blockIdx.x * 16 + l] = (int)(__builtin_amdgcn_s_memtime() - t_begin);
  }
}

size_t pyr_band_lds_bytes(const ExtractParams& P) { return (size_t)P.pyr_lds_a + P.pyr_lds_b + P.pyr_lds_y + 16; }
const void* pyr_band_kernel_ptr() { return (const void*)pyr_band_kernel; }
int pyr_band_occupancy(size_t lds) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pyr_band_kernel, kPyrBandThreads, lds) != hipSuccess) return 1;
  return std::max(1, n);
}

static int launch_band(const ExtractParams& P, const LevelPtrs& lp, const int2* rtab, int batch, hipStream_t s) {
  static int* dbg = nullptr;  // diagnostics only: per-workgroup phase cycles (ORBX_PYR_PROF=1)
  static int dbg_cap = 0;
  static const bool prof = getenv("ORBX_PYR_PROF") && getenv("ORBX_PYR_PROF")[0] == '1';
  const int nwg = P.pyr_nbands * P.pyr_nct * batch;
  if (prof && nwg > dbg_cap) {
    if (dbg) (void)hipFree(dbg);
    (void)hipMalloc(&dbg, (size_t)nwg * 16 * 4);
    dbg_cap = nwg;
  }
  hipLaunchKernelGGL(pyr_band_kernel, dim3(nwg), dim3(kPyrBandThreads), pyr_band_lds_bytes(P), s, P, lp, rtab,
                     prof ? dbg : nullptr);
  if (prof) {
    std::vector<int> h((size_t)nwg * 16);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), dbg, h.size() * 4, hipMemcpyDeviceToHost);
    double avg[16] = {0};
    int mx[16] = {0};
    for (int w = 0; w < nwg; ++w)
      for (int k = 0; k < P.L; ++k) {
        avg[k] += h[w * 16 + k];
        mx[k] = std::max(mx[k], h[w * 16 + k]);
      }
    fprintf(stderr, "pyr_band plans (bands x tiles/cost/lds):");
    for (int i = 0; i < P.pyr_nplans; ++i)
      fprintf(stderr, " %dx%d/%d/%d", P.pyr_plan[i].nbands, P.pyr_plan[i].nct, P.pyr_plan[i].cost,
              P.pyr_plan[i].lds_a + P.pyr_plan[i].lds_b + P.pyr_plan[i].lds_y + 16);
    fprintf(stderr, "\n");
    fprintf(stderr, "pyr_band: %d WGs (%d bands x %d tiles); phase cycles avg/max:", nwg, P.pyr_nbands, P.pyr_nct);
    for (int k = 0; k < P.L; ++k) fprintf(stderr, " [%d] %.0f/%d", k, avg[k] / nwg, mx[k]);
    fprintf(stderr, "\n");
  }
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

int launch_pyramid(const ExtractParams& P, const LevelPtrs& lp, const int2* rtab, int batch, hipStream_t s) {
  if (P.L < 2) return ORBX_OK;
  if (P.pyr_fused) {
    // each plan's resident workgroups per CU (LDS and the kernel's registers)
    // were found at plan time
    static const int cus = [] {
      int dev = 0, n = 256;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      return n;
    }();
    // experiments and the per-plan parity test: read per launch (a captured
    // graph keeps the plan it was captured with)
    const char* fp = getenv("ORBX_PYR_PLAN");
    const int forced = fp ? atoi(fp) : -1;
    ExtractParams Q = P;
    select_pyr_plan(Q, forced >= 0 && forced < P.pyr_nplans
                           ? forced
                           : pick_pyr_plan(P, batch, cus));
    return launch_band(Q, lp, rtab, batch, s);
  }
  for (int l = 1; l < P.L; ++l) {
    const LevelGeom& sg = P.lv[l - 1];
    const LevelGeom& d = P.lv[l];
    dim3 grid((d.w + kPyrTW - 1) / kPyrTW, (d.h + kPyrTH - 1) / kPyrTH, batch);
    hipLaunchKernelGGL(pyr_resize_kernel, grid, dim3(256), 0, s, lp.base[l - 1], lp.fstride[l - 1], lp.pitch[l - 1],
                       sg.w, sg.h, (uint8_t*)lp.base[l], lp.fstride[l], lp.pitch[l], d.w, d.h, rtab + d.xtab,
                       rtab + d.ytab, d.xmax, d.area2x, lp.aligned16[l - 1]);
  }
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
