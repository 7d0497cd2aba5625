// orbx_blur.hip — GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101)
// (src/ORBextractor.cc:1735-1749), OpenCV 3.x 8U fixed point: kernel taps
// round(256*g) = [18,34,49,55,49,34,18] (sum 257) applied along rows then
// columns, result (acc + 2^15) >> 16 (the 8U smooth-symmetric branch of
// createSeparableLinearFilter). The blurred levels feed the rBRIEF tests.
#include "orbx_device.cuh"

namespace orbx {

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
  const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int f = wg / gridDim.x, tid = threadIdx.x;
  int t = wg % gridDim.x, l = 0;
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

int launch_blur(const ExtractParams& P, const LevelPtrs& lp, uint8_t* blur, int batch, hipStream_t s) {
  int tiles = 0;
  for (int l = 0; l < P.L; ++l)
    tiles += ((P.lv[l].w + kBlurTW - 1) / kBlurTW) * ((P.lv[l].h + kBlurTH - 1) / kBlurTH);
  hipLaunchKernelGGL(blur_kernel, dim3(tiles, batch), dim3(256), 0, s, P, lp, blur);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
