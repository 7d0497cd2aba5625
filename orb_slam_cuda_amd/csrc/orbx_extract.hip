// orbx_extract.hip — HIP kernels of ORBextractor::operator() for gfx950.
//
// Pipeline for a batch of B frames (one stream, no host round trip):
//   pyr_resize_kernel    x (L-1)  ComputePyramid         src/ORBextractor.cc:1837-1863
//   blur_kernel          x 1      GaussianBlur 7x7 s=2   src/ORBextractor.cc:1735-1749
//   fast_cells_kernel    x 1      per-cell FAST + NMS    src/ORBextractor.cc:1258-1298
//   quadtree_kernel      x 1      DistributeOctTree      src/ORBextractor.cc:889-1120
//   orient_brief_kernel  x 1      IC_Angle + rBRIEF +    src/ORBextractor.cc:164-233,
//                                 scale/assemble         1314-1324, 1760-1803
// All arithmetic is integer except the few float expressions the reference
// evaluates in float (fastAtan2, BRIEF sample rotation, keypoint scaling):
// those are written with explicit round-to-nearest intrinsics and the file is
// compiled with -ffp-contract=off so that no FMA contraction changes a bit.
#include <hip/hip_runtime.h>

#include "orbx_internal.h"
#include "orbx_pattern.h"

namespace orbx {

__constant__ signed char c_brief_x[512];
__constant__ signed char c_brief_y[512];

// ------------------------------------------------------------ helpers
__device__ __forceinline__ int sat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

__device__ __forceinline__ int reflect101(int p, int len) {
  // BORDER_REFLECT_101 (cv::borderInterpolate); levels are >= 30 px wide.
  if (p < 0) p = -p;
  if (p >= len) p = 2 * len - 2 - p;
  return p;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// cv::fastAtan2 (OpenCV 3.x polynomial), float arithmetic without contraction.
__device__ __forceinline__ float fast_atan2_dev(float y, float x) {
  const float p1 = __fmul_rn(0.9997878412794807f, (float)(180 / M_PI));
  const float p3 = __fmul_rn(-0.3258083974640975f, (float)(180 / M_PI));
  const float p5 = __fmul_rn(0.1555786518463281f, (float)(180 / M_PI));
  const float p7 = __fmul_rn(-0.04432655554792128f, (float)(180 / M_PI));
  const float eps = (float)2.220446049250313e-16;  // (float)DBL_EPSILON
  float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = __fdiv_rn(ay, __fadd_rn(ax, eps));
    c2 = __fmul_rn(c, c);
    a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
  } else {
    c = __fdiv_rn(ax, __fadd_rn(ay, eps));
    c2 = __fmul_rn(c, c);
    a = __fsub_rn(90.f, __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c));
  }
  if (x < 0) a = __fsub_rn(180.f, a);
  if (y < 0) a = __fsub_rn(360.f, a);
  return a;
}

// ------------------------------------------------------------ pyramid
// One output row segment per block; fixed-point INTER_LINEAR (OpenCV 3.x
// HResizeLinear<uchar,int,short,2048> + VResizeLinear FixedPtCast<22>), or
// the 2x2 area average when the reference switches to INTER_AREA.
__global__ __launch_bounds__(256) void pyr_resize_kernel(
    const uint8_t* __restrict__ src, long long src_fs, int src_pitch, int sw, int sh,
    uint8_t* __restrict__ dst, long long dst_fs, int dst_pitch, int dw, int dh,
    const int2* __restrict__ xtab, const int2* __restrict__ ytab, int xmax, int area2x) {
  const int f = blockIdx.z, dy = blockIdx.y;
  const int dx = blockIdx.x * blockDim.x + threadIdx.x;
  if (dx >= dw) return;
  const uint8_t* S = src + f * src_fs;
  uint8_t* D = dst + f * dst_fs + (long long)dy * dst_pitch;
  if (area2x) {
    const uint8_t* r0 = S + (long long)(2 * dy) * src_pitch + 2 * dx;
    const uint8_t* r1 = r0 + src_pitch;
    D[dx] = (uint8_t)((r0[0] + r0[1] + r1[0] + r1[1] + 2) >> 2);
    return;
  }
  const int2 yt = ytab[dy];
  const int2 xt = xtab[dx];
  const uint8_t* r0 = S + (long long)(yt.x & 0xFFFF) * src_pitch;
  const uint8_t* r1 = S + (long long)(yt.x >> 16) * src_pitch;
  const int b0 = (short)(yt.y & 0xFFFF), b1 = (short)(yt.y >> 16);
  const int sx = xt.x;
  int D0, D1;
  if (dx < xmax) {
    const int a0 = (short)(xt.y & 0xFFFF), a1 = (short)(xt.y >> 16);
    D0 = r0[sx] * a0 + r0[sx + 1] * a1;
    D1 = r1[sx] * a0 + r1[sx + 1] * a1;
  } else {
    D0 = r0[sx] * 2048;
    D1 = r1[sx] * 2048;
  }
  D[dx] = (uint8_t)sat_u8((D0 * b0 + D1 * b1 + (1 << 21)) >> 22);
}

// ------------------------------------------------------------ blur
// Separable 7-tap fixed-point Gaussian, BORDER_REFLECT_101 at the level edges.
// Tile = 128 x 32 outputs per 256-thread block. The input tile (+3 halo, 16-B
// aligned: columns [x0-16, x0+144)) is staged with 16-byte loads (byte loads
// with reflection only where a chunk leaves the image); the row pass keeps
// u16 sums (max 257*255 = 65535); each thread then produces a 4 x 4 output
// block from a sliding column window and stores 4 bytes per row.
constexpr int kBlurTW = 128, kBlurTH = 32, kBlurInW = kBlurTW + 32;
__global__ __launch_bounds__(256) void blur_kernel(ExtractParams P, LevelPtrs lp, uint8_t* __restrict__ blur) {
  __shared__ __attribute__((aligned(16))) uint8_t in[kBlurTH + 6][kBlurInW];
  __shared__ __attribute__((aligned(16))) uint16_t tmp[kBlurTH + 6][kBlurTW];
  const int f = blockIdx.y, tid = threadIdx.x;
  int t = blockIdx.x, l = 0;
  for (; l < P.L; ++l) {
    const LevelGeom& g = P.lv[l];
    const int n = ((g.w + kBlurTW - 1) / kBlurTW) * ((g.h + kBlurTH - 1) / kBlurTH);
    if (t < n) break;
    t -= n;
  }
  if (l >= P.L) return;
  const LevelGeom& g = P.lv[l];
  const int W = g.w, H = g.h;
  const int tx = (W + kBlurTW - 1) / kBlurTW;
  const int x0 = (t % tx) * kBlurTW, y0 = (t / tx) * kBlurTH;
  const uint8_t* S = lp.base[l] + f * lp.fstride[l];
  const int pitch = lp.pitch[l];
  // stage rows y0-3 .. y0+TH+2, columns x0-16 .. x0+TW+15
  constexpr int kChunks = kBlurInW / 16;
  for (int i = tid; i < (kBlurTH + 6) * kChunks; i += 256) {
    const int r = i / kChunks, ch = i - r * kChunks;
    const int gy = reflect101(min(max(y0 + r - 3, -(H - 1)), 2 * H - 2), H);
    const int gx = x0 - 16 + ch * 16;
    const uint8_t* src = S + (long long)gy * pitch;
    uint4 v;
    if (gx >= 0 && gx + 16 <= W && (((uintptr_t)(src + gx)) & 15) == 0) {
      v = *(const uint4*)(src + gx);
    } else {
      uint8_t b[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int xx = min(max(gx + k, -(W - 1)), 2 * W - 2);
        b[k] = src[reflect101(xx, W)];
      }
      v = *(const uint4*)b;
    }
    *(uint4*)&in[r][ch * 16] = v;
  }
  __syncthreads();
  const int* k = P.gauss;
  // row pass: 4 outputs per item, input bytes [x+13, x+23) of the staged row
  for (int i = tid; i < (kBlurTH + 6) * (kBlurTW / 4); i += 256) {
    const int r = i / (kBlurTW / 4), x = (i - r * (kBlurTW / 4)) * 4;
    const uint32_t w0 = *(const uint32_t*)&in[r][x + 12];
    const uint32_t w1 = *(const uint32_t*)&in[r][x + 16];
    const uint32_t w2 = *(const uint32_t*)&in[r][x + 20];
    int px[12];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      px[j] = (w0 >> (8 * j)) & 255;
      px[4 + j] = (w1 >> (8 * j)) & 255;
      px[8 + j] = (w2 >> (8 * j)) & 255;
    }
    uint32_t o01 = 0, o23 = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int acc = 0;
#pragma unroll
      for (int j = 0; j < 7; ++j) acc += k[j] * px[q + 1 + j];
      if (q < 2) o01 |= (uint32_t)acc << (16 * q);
      else o23 |= (uint32_t)acc << (16 * (q - 2));
    }
    *(uint2*)&tmp[r][x] = make_uint2(o01, o23);
  }
  __syncthreads();
  // column pass: thread -> 4 columns x 4 rows
  const int cx = (tid & 31) * 4, ry = (tid >> 5) * 4;
  int col[10][4];
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const uint2 v = *(const uint2*)&tmp[ry + j][cx];
    col[j][0] = v.x & 0xFFFF;
    col[j][1] = v.x >> 16;
    col[j][2] = v.y & 0xFFFF;
    col[j][3] = v.y >> 16;
  }
  uint8_t* D = blur + g.off + f * g.plane;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int y = y0 + ry + rr;
    uint32_t packed = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int acc = 0;
#pragma unroll
      for (int j = 0; j < 7; ++j) acc += k[j] * col[rr + j][q];
      packed |= (uint32_t)sat_u8((acc + (1 << 15)) >> 16) << (8 * q);
    }
    if (y < H) {
      const int x = x0 + cx;
      uint8_t* dst = D + (long long)y * g.pitch + x;
      if (x + 4 <= W) {
        *(uint32_t*)dst = packed;
      } else {
        for (int q = 0; q < 4 && x + q < W; ++q) dst[q] = (uint8_t)(packed >> (8 * q));
      }
    }
  }
}

// ------------------------------------------------------------ FAST
// FAST-9/16 "cornerScore<16>" of OpenCV 3.x, d[k] = v - ring[k].
__device__ __forceinline__ int corner_score16(const int (&d)[16], int threshold) {
  auto D = [&](int k) { return d[k & 15]; };
  int a0 = threshold;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int a = min(D(k + 1), D(k + 2));
    a = min(a, D(k + 3));
    if (a <= a0) continue;
    a = min(a, D(k + 4));
    a = min(a, D(k + 5));
    a = min(a, D(k + 6));
    a = min(a, D(k + 7));
    a = min(a, D(k + 8));
    a0 = max(a0, min(a, D(k)));
    a0 = max(a0, min(a, D(k + 9)));
  }
  int b0 = -a0;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int b = max(D(k + 1), D(k + 2));
    b = max(b, D(k + 3));
    b = max(b, D(k + 4));
    b = max(b, D(k + 5));
    if (b >= b0) continue;
    b = max(b, D(k + 6));
    b = max(b, D(k + 7));
    b = max(b, D(k + 8));
    b0 = min(b0, max(b, D(k)));
    b0 = min(b0, max(b, D(k + 9)));
  }
  return -b0 - 1;
}

// 9 contiguous set bits in a circular 16-bit mask
__device__ __forceinline__ bool has_arc9(uint32_t m) {
  uint32_t x = m | (m << 16);
  uint32_t a = x & (x >> 1);  // runs of 2
  a &= a >> 2;                // runs of 4
  a &= a >> 4;                // runs of 8
  a &= x >> 8;                // runs of 9
  return (a & 0xFFFFu) != 0;
}

// One wavefront per (frame, grid cell). The cell ROI (<= 65 x 65 with the
// 3-px FAST halo) is staged in LDS; lanes cover the detection band as
// 2 rows x 32 columns (band width <= 32, every KITTI/EuRoC level) or
// 1 row x 64 columns. Every band pixel gets its FAST score at t_low (one
// score map serves both thresholds: detected-at-t <=> score >= t); a pixel
// fails fast unless two of the four compass ring pixels agree (any 9-arc
// covers two of them). Non-max suppression sees only the cell's own band
// (neighbours outside it are 0), exactly like cv::FAST on the ROI; one pass
// records the survivors at iniThFAST and at minThFAST as row-major ballots,
// the cell keeps the iniThFAST set unless it is empty, and the survivors are
// written in row-major order into the cell's fixed slot range.
constexpr int kMaxBallots = 64;
__global__ __launch_bounds__(64) void fast_cells_kernel(ExtractParams P, LevelPtrs lp,
                                                        const CellGeom* __restrict__ cells,
                                                        uint32_t* __restrict__ slots,
                                                        int* __restrict__ cell_counts) {
  __shared__ uint8_t roi[kMaxRoi * kMaxRoi];
  __shared__ uint8_t sc[(kMaxRoi - 4) * (kMaxRoi - 4)];
  __shared__ uint64_t s_ball[2][kMaxBallots];
  const int cell = blockIdx.x, f = blockIdx.y, lane = threadIdx.x;
  const CellGeom cg = cells[cell];
  int* cnt = cell_counts + (long long)f * P.ncells_total + cell;
  const int rw = cg.c1 - cg.c0, rh = cg.r1 - cg.r0;
  const int bw = rw - 6, bh = rh - 6;
  if (cg.cap == 0 || bw <= 0 || bh <= 0) {
    if (lane == 0) *cnt = 0;
    return;
  }
  const int l = cg.level;
  const LevelGeom& g = P.lv[l];
  const int pitch = lp.pitch[l];
  const uint8_t* S = lp.base[l] + f * lp.fstride[l] + (long long)cg.r0 * pitch + cg.c0;
  // stage the ROI: lanes = columns
#pragma unroll 4
  for (int r = 0; r < rh; ++r) {
    if (lane < rw) roi[r * rw + lane] = S[(long long)r * pitch + lane];
    if (lane + 64 < rw) roi[r * rw + lane + 64] = S[(long long)r * pitch + lane + 64];
  }
  const int sw = bw + 2;  // score map with a zero ring
  for (int i = lane; i < sw * (bh + 2); i += 64) sc[i] = 0;
  __syncthreads();
  const bool two = bw <= 32;
  const int lr = two ? (lane >> 5) : 0, lc = two ? (lane & 31) : lane;
  const int rstep = two ? 2 : 1;
  const int t = P.t_low;
  for (int by = lr; by < bh; by += rstep) {
    if (lc >= bw) continue;
    const uint8_t* c0 = roi + (by + 3) * rw + (lc + 3);
    const int v = c0[0];
    // compass points k = 0, 4, 8, 12: (0,3) (3,0) (0,-3) (-3,0)
    const int n0 = c0[3 * rw], n4 = c0[3], n8 = c0[-3 * rw], n12 = c0[-3];
    const int lo = v - t, hi = v + t;
    const int nd = (n0 < lo) + (n4 < lo) + (n8 < lo) + (n12 < lo);
    const int nb = (n0 > hi) + (n4 > hi) + (n8 > hi) + (n12 > hi);
    int s = 0;
    if (nd >= 2 || nb >= 2) {
      int d[16];
      uint32_t dark = 0, bright = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        constexpr int rx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
        constexpr int ry[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
        const int x = c0[ry[k] * rw + rx[k]];
        d[k] = v - x;
        dark |= (uint32_t)(x < lo) << k;
        bright |= (uint32_t)(x > hi) << k;
      }
      if (has_arc9(dark) || has_arc9(bright)) s = corner_score16(d, t);
    }
    sc[(by + 1) * sw + lc + 1] = (uint8_t)s;
  }
  __syncthreads();
  // NMS at both thresholds in one pass; neighbours below a threshold count as 0
  const int ti = P.t_ini, tm = P.t_min;
  const int nit = (bh + rstep - 1) / rstep;
  int n_ini = 0;
  for (int it = 0; it < nit; ++it) {
    const int by = it * rstep + lr;
    bool ki = false, km = false;
    if (by < bh && lc < bw) {
      const uint8_t* q = sc + (by + 1) * sw + lc + 1;
      const int s = q[0];
      if (s > 0) {
        int m = 0;  // max neighbour
        const int nbv[8] = {q[-1], q[1], q[-sw - 1], q[-sw], q[-sw + 1], q[sw - 1], q[sw], q[sw + 1]};
        bool gi = s >= ti, gm = s >= tm;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int x = nbv[j];
          if (x >= ti && x >= s) gi = false;
          if (x >= tm && x >= s) gm = false;
          m = max(m, x);
        }
        (void)m;
        ki = gi;
        km = gm;
      }
    }
    const uint64_t bi = __ballot(ki), bm = __ballot(km);
    if (lane == 0) {
      s_ball[0][it] = bi;
      s_ball[1][it] = bm;
    }
    n_ini += __popcll(bi);
  }
  __syncthreads();
  const int which = n_ini > 0 ? 0 : 1;
  uint32_t* out = slots + (long long)f * P.slots_per_frame + cg.slot_off;
  int base = 0;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int it = 0; it < nit; ++it) {
    const uint64_t m = s_ball[which][it];
    if ((m >> lane) & 1ull) {
      const int by = it * rstep + lr;
      const int pos = base + __popcll(m & lt);
      const int x = cg.c0 + 3 + lc - g.minBX, y = cg.r0 + 3 + by - g.minBY;
      const int score = sc[(by + 1) * sw + lc + 1];
      if (pos < cg.cap) out[pos] = pack_key(x, y, score);
    }
    base += __popcll(m);
  }
  if (lane == 0) *cnt = min(base, (int)cg.cap);
}

// ------------------------------------------------------------ quadtree
// DistributeOctTree as data-parallel rounds (see DESIGN.md "Quadtree"):
// the std::list of the reference becomes a node table indexed by list
// position; one round splits a prefix of the candidate nodes (list order in
// the breadth phase, (size desc, creation desc) order in the "sorted" phase),
// and the new list is [children of split nodes, last split first, n4..n1]
// followed by the untouched nodes in their old order. Keys never move; each
// key carries its node index. Size ties in the sorted phase are broken by
// node creation order, the oracle's documented stand-in for the reference's
// heap-pointer order (src/ORBextractor.cc:1041).
__device__ int block_scan_excl(int* a, int n, int* s_tmp) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = (n + kQtThreads - 1) / kQtThreads;
  const int b = min(tid * per, n), e = min(b + per, n);
  int sum = 0;
  for (int i = b; i < e; ++i) sum += a[i];
  int x = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  int wpre = 0, total = 0;
#pragma unroll
  for (int i = 0; i < kQtThreads / 64; ++i) {
    const int v = s_tmp[i];
    if (i < w) wpre += v;
    total += v;
  }
  int run = wpre + x - sum;
  for (int i = b; i < e; ++i) {
    const int v = a[i];
    a[i] = run;
    run += v;
  }
  __syncthreads();
  return total;
}

struct QNode {
  int16_t x0, y0, x1, y1;
};

__device__ __forceinline__ int quadrant(const QNode& nd, int kx, int ky) {
  const int halfX = (int)ceilf(__fdiv_rn((float)(nd.x1 - nd.x0), 2.f));
  const int halfY = (int)ceilf(__fdiv_rn((float)(nd.y1 - nd.y0), 2.f));
  const bool right = kx >= nd.x0 + halfX;
  const bool bottom = ky >= nd.y0 + halfY;
  return (right ? 1 : 0) + (bottom ? 2 : 0);  // 0=n1 1=n2 2=n3 3=n4
}

__device__ __forceinline__ QNode child_box(const QNode& nd, int q) {
  const int halfX = (int)ceilf(__fdiv_rn((float)(nd.x1 - nd.x0), 2.f));
  const int halfY = (int)ceilf(__fdiv_rn((float)(nd.y1 - nd.y0), 2.f));
  const int mx = nd.x0 + halfX, my = nd.y0 + halfY;
  QNode c;
  c.x0 = (q & 1) ? mx : nd.x0;
  c.x1 = (q & 1) ? nd.x1 : mx;
  c.y0 = (q & 2) ? my : nd.y0;
  c.y1 = (q & 2) ? nd.y1 : my;
  return c;
}

__global__ __launch_bounds__(kQtThreads) void quadtree_kernel(ExtractParams P, const int* __restrict__ cell_counts,
                                                              const uint32_t* __restrict__ slots,
                                                              const CellGeom* __restrict__ cells,
                                                              uint32_t* __restrict__ qscratch,
                                                              uint16_t* __restrict__ qnscratch,
                                                              long long qscratch_per_fl,
                                                              uint32_t* __restrict__ qkeys,
                                                              int* __restrict__ qcounts, int* err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int l = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
  const LevelGeom& g = P.lv[l];
  const int MN = P.maxnodes, SN = P.sortn;
  // ---- LDS carve (all offsets 16-byte aligned)
  unsigned char* p = smem;
  auto take = [&](size_t bytes) { unsigned char* r = p; p += (bytes + 15) & ~(size_t)15; return r; };
  unsigned long long* s_sort = (unsigned long long*)take(8ull * SN);  // also best-per-node
  QNode* nodeA = (QNode*)take(sizeof(QNode) * MN);
  QNode* nodeB = (QNode*)take(sizeof(QNode) * MN);
  int* nkA = (int*)take(4ull * MN);
  int* nkB = (int*)take(4ull * MN);
  int* seqA = (int*)take(4ull * MN);
  int* seqB = (int*)take(4ull * MN);
  int4* cc = (int4*)take(16ull * MN);     // child key counts, later child positions
  int* tA = (int*)take(4ull * (MN + 1));
  int* tB = (int*)take(4ull * (MN + 1));
  int* rank = (int*)take(4ull * MN);      // processing rank or -1
  int* ord = (int*)take(4ull * MN);
  int* coff = (int*)take(4ull * (P.max_cells_level + 1));
  int* s_tmp = (int*)take(64);
  int* s_var = (int*)take(64);
  uint32_t* lkeys = (uint32_t*)take(4ull * P.kcap_lds);
  uint16_t* lnode = (uint16_t*)take(2ull * P.kcap_lds);

  // ---- gather the level's FAST keys in reference order (cells row-major)
  const int* cntp = cell_counts + (long long)f * P.ncells_total + g.cell0;
  for (int c = tid; c < g.ncells; c += kQtThreads) coff[c] = cntp[c];
  __syncthreads();
  const int K = block_scan_excl(coff, g.ncells, s_tmp);
  uint32_t* keys;
  uint16_t* knode;
  if (K <= P.kcap_lds) {
    keys = lkeys;
    knode = lnode;
  } else {
    keys = qscratch + (long long)f * P.slots_per_frame + g.slot0;
    knode = qnscratch + (long long)f * P.slots_per_frame + g.slot0;
  }
  const uint32_t* fslots = slots + (long long)f * P.slots_per_frame;
  {
    const int wv = tid >> 6, lane = tid & 63;
    for (int c = wv; c < g.ncells; c += kQtThreads / 64) {
      const int n = cntp[c], o = coff[c];
      const uint32_t* src = fslots + cells[g.cell0 + c].slot_off;
      for (int i = lane; i < n; i += 64) keys[o + i] = src[i];
    }
  }
  // ---- initial nodes: nIni columns of width hX (src/ORBextractor.cc:894-921)
  const int nIni = g.nIni;
  int* rootCnt = tA;  // nIni <= MN
  for (int i = tid; i < nIni; i += kQtThreads) rootCnt[i] = 0;
  __syncthreads();
  for (int k = tid; k < K; k += kQtThreads) {
    const int r = (int)__fdiv_rn((float)key_x(keys[k]), g.hX);
    knode[k] = (uint16_t)r;
    atomicAdd(&rootCnt[r], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int n = 0;
    for (int i = 0; i < nIni; ++i) {
      const int c = rootCnt[i];
      if (c > 0) {
        QNode nd;
        nd.x0 = (int16_t)(int)__fmul_rn(g.hX, (float)i);
        nd.x1 = (int16_t)(int)__fmul_rn(g.hX, (float)(i + 1));
        nd.y0 = 0;
        nd.y1 = (int16_t)g.boxH;
        nodeA[n] = nd;
        nkA[n] = c;
        seqA[n] = 0;
        rootCnt[i] = n++;
      } else {
        rootCnt[i] = -1;
      }
    }
    s_var[0] = n;  // list size
    s_var[1] = 0;  // phase 2 flag
  }
  __syncthreads();
  for (int k = tid; k < K; k += kQtThreads) knode[k] = (uint16_t)rootCnt[knode[k]];
  __syncthreads();

  const int N = g.N;
  for (int round = 0; round < 64; ++round) {
    const int size = s_var[0];
    const bool phase2 = s_var[1] != 0;
    // A/B: child key counts of every splittable node
    for (int n = tid; n < size; n += kQtThreads) cc[n] = make_int4(0, 0, 0, 0);
    __syncthreads();
    for (int k = tid; k < K; k += kQtThreads) {
      const int n = knode[k];
      if (nkA[n] > 1) {
        const uint32_t kk = keys[k];
        const int q = quadrant(nodeA[n], key_x(kk), key_y(kk));
        atomicAdd(((int*)&cc[n]) + q, 1);
      }
    }
    __syncthreads();
    auto nz = [](int4 c) { return (c.x > 0) + (c.y > 0) + (c.z > 0) + (c.w > 0); };
    // C: processing order and cut-off (split while list size < N)
    int m;  // number of nodes split this round
    if (!phase2) {
      for (int n = tid; n < size; n += kQtThreads) {
        const bool cand = nkA[n] > 1;
        tA[n] = cand ? nz(cc[n]) - 1 : 0;
        tB[n] = cand ? 1 : 0;
      }
      __syncthreads();
      block_scan_excl(tA, size, s_tmp);
      block_scan_excl(tB, size, s_tmp);
      if (tid == 0) s_var[2] = 0;
      __syncthreads();
      for (int n = tid; n < size; n += kQtThreads) {
        const bool cand = nkA[n] > 1;
        if (cand && size + tA[n] < N) {
          rank[n] = tB[n];
          ord[tB[n]] = n;
          atomicAdd(&s_var[2], 1);
        } else {
          rank[n] = -1;
        }
      }
      __syncthreads();
      m = s_var[2];
    } else {
      for (int i = tid; i < SN; i += kQtThreads) {
        unsigned long long key = 0;
        if (i < size && nkA[i] > 1)
          key = ((unsigned long long)nkA[i] << 40) | ((unsigned long long)seqA[i] << 16) | (unsigned long long)i;
        s_sort[i] = key;
      }
      __syncthreads();
      // bitonic sort, descending
      for (int kk = 2; kk <= SN; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
          for (int i = tid; i < SN; i += kQtThreads) {
            const int ixj = i ^ j;
            if (ixj > i) {
              const unsigned long long a = s_sort[i], b = s_sort[ixj];
              const bool desc = (i & kk) == 0;
              if (desc ? (a < b) : (a > b)) {
                s_sort[i] = b;
                s_sort[ixj] = a;
              }
            }
          }
          __syncthreads();
        }
      }
      if (tid == 0) s_var[3] = 0;
      for (int n = tid; n < size; n += kQtThreads) rank[n] = -1;
      __syncthreads();
      for (int j = tid; j < size; j += kQtThreads) {
        const unsigned long long key = s_sort[j];
        tA[j] = key ? nz(cc[(int)(key & 0xFFFF)]) - 1 : 0;
        if (key) atomicAdd(&s_var[3], 1);
      }
      __syncthreads();
      const int ncand = s_var[3];
      block_scan_excl(tA, ncand, s_tmp);
      if (tid == 0) s_var[2] = 0;
      __syncthreads();
      for (int j = tid; j < ncand; j += kQtThreads) {
        if (size + tA[j] < N) {
          const int n = (int)(s_sort[j] & 0xFFFF);
          rank[n] = j;
          ord[j] = n;
          atomicAdd(&s_var[2], 1);
        }
      }
      __syncthreads();
      m = s_var[2];
    }
    // D: positions of the children block (reverse processing order)
    for (int j = tid; j < m; j += kQtThreads) tA[j] = nz(cc[ord[j]]);
    __syncthreads();
    const int T = block_scan_excl(tA, m, s_tmp);  // tA[j] = E_j
    // E: positions of kept nodes
    for (int n = tid; n < size; n += kQtThreads) tB[n] = rank[n] < 0 ? 1 : 0;
    __syncthreads();
    const int nKept = block_scan_excl(tB, size, s_tmp);
    const int newSize = T + nKept;
    // F: new node table; cc[n] becomes the child positions of split node n
    for (int n = tid; n < size; n += kQtThreads) {
      const int j = rank[n];
      if (j < 0) {
        const int pos = T + tB[n];
        nodeB[pos] = nodeA[n];
        nkB[pos] = nkA[n];
        seqB[pos] = seqA[n];
      } else {
        const int4 c = cc[n];
        const int cnts[4] = {c.x, c.y, c.z, c.w};
        const int Cj = nz(c);
        const int base = T - (tA[j] + Cj);
        int pos4[4];
        int after = 0;  // nonempty children with a higher quadrant index
#pragma unroll
        for (int q = 3; q >= 0; --q) {
          if (cnts[q] > 0) {
            pos4[q] = base + after;
            ++after;
            nodeB[pos4[q]] = child_box(nodeA[n], q);
            nkB[pos4[q]] = cnts[q];
            seqB[pos4[q]] = j * 4 + q;
          } else {
            pos4[q] = -1;
          }
        }
        cc[n] = make_int4(pos4[0], pos4[1], pos4[2], pos4[3]);
      }
    }
    __syncthreads();
    // G: re-home keys
    for (int k = tid; k < K; k += kQtThreads) {
      const int n = knode[k];
      const int j = rank[n];
      if (j < 0) {
        knode[k] = (uint16_t)(T + tB[n]);
      } else {
        const uint32_t kk = keys[k];
        const int q = quadrant(nodeA[n], key_x(kk), key_y(kk));
        knode[k] = (uint16_t)((const int*)&cc[n])[q];
      }
    }
    __syncthreads();
    // swap tables
    for (int n = tid; n < newSize; n += kQtThreads) {
      nodeA[n] = nodeB[n];
      nkA[n] = nkB[n];
      seqA[n] = seqB[n];
    }
    if (tid == 0) {
      int nExp = 0;
      for (int n = 0; n < newSize; ++n) nExp += nkB[n] > 1;
      s_var[4] = nExp;
    }
    __syncthreads();
    bool finish = newSize >= N || newSize == size;
    if (!finish && !phase2 && newSize + 3 * s_var[4] > N) {
      if (tid == 0) s_var[1] = 1;
    }
    if (tid == 0) s_var[0] = newSize;
    __syncthreads();
    if (finish) break;
    if (round == 63 && tid == 0) atomicOr(err, 2);
  }
  // ---- keep the best (max FAST score, first in node order) key per node
  const int size = s_var[0];
  for (int n = tid; n < size; n += kQtThreads) s_sort[n] = 0;
  __syncthreads();
  for (int k = tid; k < K; k += kQtThreads) {
    const unsigned long long v =
        ((unsigned long long)key_score(keys[k]) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)k);
    atomicMax(&s_sort[knode[k]], v);
  }
  __syncthreads();
  uint32_t* out = qkeys + (long long)f * P.kp_per_frame + g.kbase;
  for (int n = tid; n < size && n < g.kcap; n += kQtThreads) {
    const uint32_t k = 0xFFFFFFFFu - (uint32_t)(s_sort[n] & 0xFFFFFFFFull);
    out[n] = keys[k];
  }
  if (tid == 0) {
    qcounts[f * P.L + l] = min(size, g.kcap);
    if (size > g.kcap) atomicOr(err, 4);
  }
}

// ------------------------------------------------------------ angle + BRIEF
// One wavefront per keypoint: IC_Angle moments over the r=15 circular patch
// of the unblurred level (lanes = patch columns, wave-reduced), cv::fastAtan2,
// then the 256 rBRIEF tests on the blurred level (4 tests per lane, packed by
// four 64-bit ballots straight into the 32 descriptor bytes), then the
// keypoint record scaled to level 0 in cv::KeyPoint layout.
__global__ __launch_bounds__(256) void orient_brief_kernel(ExtractParams P, LevelPtrs lp,
                                                           const uint8_t* __restrict__ blur,
                                                           const uint32_t* __restrict__ qkeys,
                                                           const int* __restrict__ qcounts,
                                                           const int* __restrict__ umax,
                                                           orbx_kp* __restrict__ out_kps,
                                                           uint8_t* __restrict__ out_desc,
                                                           int* __restrict__ out_counts) {
  const int f = blockIdx.y, lane = threadIdx.x & 63;
  const int slot = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int* cnt = qcounts + f * P.L;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
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
  const uint8_t* img = lp.base[l] + f * lp.fstride[l];
  const int pitch = lp.pitch[l];
  const uint8_t* center = img + (long long)y * pitch + x;
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

  // computeOrbDescriptor: a = (float)cos(angle*pi/180), b = sin(...)
  const float factorPI = (float)(M_PI / 180.f);
  const float ang = __fmul_rn(angle, factorPI);
  const float a = (float)cos((double)ang), b = (float)sin((double)ang);
  const uint8_t* bimg = blur + g.off + f * g.plane;
  const uint8_t* bc = bimg + (long long)y * g.pitch + x;
  const int step = g.pitch;
  uint64_t words[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int test = w * 64 + lane;
    int px[2], py[2];
    px[0] = c_brief_x[2 * test];
    py[0] = c_brief_y[2 * test];
    px[1] = c_brief_x[2 * test + 1];
    py[1] = c_brief_y[2 * test + 1];
    if (P.pattern_upstream && 2 * test == kBriefForkPoint) px[0] = kBriefUpstreamX;
    int val[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float fx = (float)px[s], fy = (float)py[s];
      const int ry = __float2int_rn(__fadd_rn(__fmul_rn(fx, b), __fmul_rn(fy, a)));
      const int rx = __float2int_rn(__fsub_rn(__fmul_rn(fx, a), __fmul_rn(fy, b)));
      val[s] = bc[ry * step + rx];
    }
    words[w] = __ballot(val[0] < val[1]);
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

// ------------------------------------------------------------ launcher
size_t quadtree_lds_bytes(const ExtractParams& P);
const void* quadtree_kernel_ptr() { return (const void*)quadtree_kernel; }

static bool g_pattern_uploaded = false;

int launch_extract(const ExtractParams& P, const ExtractBuffers& X, const uint8_t* d_frames, int batch,
                   size_t frame_pitch, size_t row_stride, orbx_kp* d_kps, uint8_t* d_desc,
                   int* d_counts, void* stream_, void** ev) {
  hipStream_t stream = (hipStream_t)stream_;
  if (!g_pattern_uploaded) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_brief_x), kBriefPointX, 512) != hipSuccess) return ORBX_EDEVICE;
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_brief_y), kBriefPointY, 512) != hipSuccess) return ORBX_EDEVICE;
    g_pattern_uploaded = true;
  }
  ExtractParams Q = P;
  Q.B = batch;
  LevelPtrs lp;
  lp.base[0] = d_frames;
  lp.fstride[0] = (long long)frame_pitch;
  lp.pitch[0] = (int)row_stride;
  for (int l = 1; l < P.L; ++l) {
    lp.base[l] = X.pyr + P.lv[l].off;
    lp.fstride[l] = P.lv[l].plane;
    lp.pitch[l] = P.lv[l].pitch;
  }
  auto rec = [&](int i) {
    if (ev) (void)hipEventRecord((hipEvent_t)ev[i], stream);
  };
  rec(0);
  for (int l = 1; l < P.L; ++l) {
    const LevelGeom& s = P.lv[l - 1];
    const LevelGeom& d = P.lv[l];
    dim3 grid((d.w + 255) / 256, d.h, batch);
    hipLaunchKernelGGL(pyr_resize_kernel, grid, dim3(256), 0, stream, lp.base[l - 1], lp.fstride[l - 1],
                       lp.pitch[l - 1], s.w, s.h, (uint8_t*)lp.base[l], lp.fstride[l], lp.pitch[l], d.w,
                       d.h, X.rtab + d.xtab, X.rtab + d.ytab, d.xmax, d.area2x);
  }
  rec(1);
  int tiles = 0;
  for (int l = 0; l < P.L; ++l)
    tiles += ((P.lv[l].w + kBlurTW - 1) / kBlurTW) * ((P.lv[l].h + kBlurTH - 1) / kBlurTH);
  hipLaunchKernelGGL(blur_kernel, dim3(tiles, batch), dim3(256), 0, stream, Q, lp, X.blur);
  rec(2);
  hipLaunchKernelGGL(fast_cells_kernel, dim3(P.ncells_total, batch), dim3(64), 0, stream, Q, lp, X.cells,
                     X.slots, X.cell_counts);
  rec(3);
  hipLaunchKernelGGL(quadtree_kernel, dim3(P.L, batch), dim3(kQtThreads), quadtree_lds_bytes(P), stream, Q,
                     X.cell_counts, X.slots, X.cells, X.qscratch, X.qnode_scratch, X.qscratch_per_fl,
                     X.qkeys, X.qcounts, X.err);
  rec(4);
  dim3 og((P.kp_per_frame + 3) / 4, batch);
  hipLaunchKernelGGL(orient_brief_kernel, og, dim3(256), 0, stream, Q, lp, X.blur, X.qkeys, X.qcounts, X.umax,
                     d_kps, d_desc, d_counts);
  rec(5);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

size_t quadtree_lds_bytes(const ExtractParams& P) {
  auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t MN = P.maxnodes, SN = P.sortn;
  size_t b = 0;
  b += r16(8 * SN);
  b += 2 * r16(sizeof(QNode) * MN);
  b += 4 * r16(4 * MN);
  b += r16(16 * MN);
  b += 2 * r16(4 * (MN + 1));
  b += 2 * r16(4 * MN);
  b += r16(4 * (P.max_cells_level + 1));
  b += 2 * r16(64);
  b += r16(4ull * P.kcap_lds);
  b += r16(2ull * P.kcap_lds);
  return b;
}

}  // namespace orbx
