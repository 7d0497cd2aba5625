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
// One launch per level (each level depends on the previous). A 256-thread
// block produces a 16-row x 256-column output tile: the source rows/columns
// the tile touches are staged in LDS with 16-byte loads, then each thread
// computes a 4x4 output block from LDS and writes 4 x 32-bit stores.
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
          D0 = r0[s] * a0v[q] + r0[s + 1] * a1v[q];
          D1 = r1[s] * a0v[q] + r1[s + 1] * a1v[q];
        } else {
          D0 = r0[s] * 2048;
          D1 = r1[s] * 2048;
        }
        const int b0 = (short)(yt.y & 0xFFFF), b1 = (short)(yt.y >> 16);
        v[q] = sat_u8((D0 * b0 + D1 * b1 + (1 << 21)) >> 22);
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

int launch_pyramid(const ExtractParams& P, const LevelPtrs& lp, const int2* rtab, int batch, hipStream_t s) {
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
