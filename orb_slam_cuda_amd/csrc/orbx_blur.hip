// orbx_blur.hip — GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101)
// (src/ORBextractor.cc:1735-1749), OpenCV 3.x 8U fixed point: kernel taps
// round(256*g) = [18,34,49,55,49,34,18] (sum 257) applied along rows then
// columns, result (acc + 2^15) >> 16 (the 8U smooth-symmetric branch of
// createSeparableLinearFilter). The blurred levels feed the rBRIEF tests.
#include "orbx_device.cuh"

namespace orbx {

// Separable 7-tap fixed-point Gaussian, BORDER_REFLECT_101 at the level edges.
// Tile = 128 x 48 outputs per 256-thread block (alone 64 rows was best of
// 16..80, 1.1x halo rows; in the pipelined step 48 rows, 22.5 instead of 29 KB
// of LDS, gave +0.5-1 % over six interleaved pairs). The input tile (+3 halo, 16-B
// aligned: columns [x0-16, x0+144)) is staged with 16-byte loads (byte loads
// with reflection only where a chunk leaves the image).
//   row pass:    v_dot4_u32_u8 of a pixel dword with a tap dword: 10 dot4 per
//                4 outputs (sums <= 257*255 = 65535 fit u16); the sums of two
//                vertically adjacent rows are packed into one dword,
//   column pass: v_dot2_u32_u16 of such a row pair with a tap pair: 4 dot2
//                per output, then (acc + 2^15) >> 16.
#ifndef ORBX_BLUR_TH
#define ORBX_BLUR_TH 48
#endif
#ifndef ORBX_BLUR_TW
#define ORBX_BLUR_TW 128
#endif
// small tiles for launches that would not fill the chip with the large ones
// (a single frame: 272 tiles of 128 x 48 for 256 CUs, ~1000 of 64 x 32)
constexpr int kBlurTWs = 64, kBlurTHs = 32;

typedef unsigned short us2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t dot4(uint32_t px, uint32_t taps, uint32_t acc) {
  return __builtin_amdgcn_udot4(px, taps, acc, false);
}
__device__ __forceinline__ uint32_t dot2(uint32_t pair, uint32_t taps, uint32_t acc) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(us2_t, pair), __builtin_bit_cast(us2_t, taps), acc, false);
}

template <int kBlurTW, int kBlurTH>
__global__ __launch_bounds__(256) void blur_kernel(ExtractParams P, LevelPtrs lp, const int2* __restrict__ rtab,
                                                   int tiles, int ntiles, unsigned magic, uint8_t* __restrict__ blur) {
  constexpr int kBlurInW = kBlurTW + 32;
  constexpr int kBlurPairs = (kBlurTH + 6 + 1) / 2;  // staged row pairs (19 for 48-row tiles)
  __shared__ __attribute__((aligned(16))) uint8_t in[kBlurPairs * 2][kBlurInW];
  __shared__ __attribute__((aligned(16))) uint32_t tmp[kBlurPairs][kBlurTW];  // {row 2p, row 2p+1} u16 sums
  const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  // the frame by a multiply-high (exact for every id of the plan's batch,
  // checked at plan time), the tile's level and origin by one table load: no
  // division and no level search before the tile's first address
  const int f = magic ? (int)__umulhi((unsigned)wg, magic) : wg / ntiles, tid = threadIdx.x;
  const int e = rtab[tiles + wg - f * ntiles].x;
  const int l = e & 15, x0 = (e >> 4) & 0xFFF, y0 = e >> 16;
  const LevelGeom& g = P.lv[l];
  const int W = g.w, H = g.h;
  const uint8_t* S = lp.base[l] + f * lp.fstride[l];
  const int pitch = lp.pitch[l];
  // stage rows y0-3 .. y0+TH+2, columns x0-16 .. x0+TW+15
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int kChunks = kBlurInW / 16, kItems = (kBlurTH + 6) * kChunks, kPer = (kItems + 255) / 256;
  if (lp.aligned16[l]) {
    // every chunk is a 16-byte load from inside its (row-reflected) source
    // row: chunks left of column 0 or past ceil16(W) load a clamped chunk of
    // the row instead (a chunk holding a column < W never needs the clamp:
    // W <= pitch, both multiples of 16 apart from W). The 3 columns each side
    // of the level that BORDER_REFLECT_101 supplies are written afterwards
    // from the staged columns, on edge tiles only.
    // last chunk start: inside ceil16(W) (level 0 is the caller's frame, whose
    // rows orbx_extract_batch only promises readable that far, orbx_c.h)
    const int xmax = min(pitch, (W + 15) & ~15) - 16;
    u32x4 v[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = min(tid + 256 * q, kItems - 1);
      const int r = i / kChunks, ch = i - r * kChunks;
      const int gy = reflect101(min(max(y0 + r - 3, -(H - 1)), 2 * H - 2), H);
      const int gx = min(max(x0 - 16 + ch * 16, 0), xmax);
      v[q] = *(const u32x4*)(S + (long long)gy * pitch + gx);
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = min(tid + 256 * q, kItems - 1);
      const int r = i / kChunks, ch = i - r * kChunks;
      *(u32x4*)&in[r][ch * 16] = v[q];
    }
    const bool left = x0 == 0, right = x0 + kBlurTW + 3 > W;
    if (left || right) {
      __syncthreads();
      // column x < 0 -> -x, x >= W -> 2W - 2 - x (staged column = x - x0 + 16)
      for (int i = tid; i < (kBlurTH + 6) * 6; i += 256) {
        const int r = i / 6, kk = i - r * 6;
        int x = kk < 3 ? -1 - kk : W + kk - 3;
        if ((kk < 3 && !left) || (kk >= 3 && !right) || x - x0 + 16 >= kBlurInW) continue;
        in[r][x - x0 + 16] = in[r][reflect101(x, W) - x0 + 16];
      }
    }
  } else {
    // unaligned levels: chunks that leave the image are rewritten from byte
    // loads with reflection after the aligned chunks are stored
    u32x4 v[kPer];
    bool direct[kPer];
    int gys[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = min(tid + 256 * q, kItems - 1);
      const int r = i / kChunks, ch = i - r * kChunks;
      gys[q] = reflect101(min(max(y0 + r - 3, -(H - 1)), 2 * H - 2), H);
      const int gx = x0 - 16 + ch * 16;
      const uint8_t* src = S + (long long)gys[q] * pitch + gx;
      direct[q] = gx >= 0 && gx + 16 <= W && (((uintptr_t)src) & 15) == 0;
      v[q] = *(const u32x4*)(direct[q] ? src : S);
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = min(tid + 256 * q, kItems - 1);
      const int r = i / kChunks, ch = i - r * kChunks;
      *(u32x4*)&in[r][ch * 16] = v[q];
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      if (direct[q]) continue;
      const int i = min(tid + 256 * q, kItems - 1);
      const int r = i / kChunks, ch = i - r * kChunks;
      const int gx = x0 - 16 + ch * 16;
      const uint8_t* src = S + (long long)gys[q] * pitch;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int xx = min(max(gx + k, -(W - 1)), 2 * W - 2);
        in[r][ch * 16 + k] = src[reflect101(xx, W)];
      }
    }
  }
  __syncthreads();
  const int* k = P.gauss;
  // tap dwords of the row pass: output x reads staged bytes [x+13, x+20)
  // from dwords A = [x+12, x+16), B = [x+16, x+20), C = [x+20, x+24)
  const uint32_t kA0 = (k[0] << 8) | (k[1] << 16) | (k[2] << 24), kB0 = k[3] | (k[4] << 8) | (k[5] << 16) | (k[6] << 24);
  const uint32_t kA1 = (k[0] << 16) | (k[1] << 24), kB1 = k[2] | (k[3] << 8) | (k[4] << 16) | (k[5] << 24), kC1 = k[6];
  const uint32_t kA2 = k[0] << 24, kB2 = k[1] | (k[2] << 8) | (k[3] << 16) | (k[4] << 24), kC2 = k[5] | (k[6] << 8);
  const uint32_t kB3 = k[0] | (k[1] << 8) | (k[2] << 16) | (k[3] << 24), kC3 = k[4] | (k[5] << 8) | (k[6] << 16);
  // row pass: item = (row pair, 4 columns)
  for (int i = tid; i < kBlurPairs * (kBlurTW / 4); i += 256) {
    const int pr = i / (kBlurTW / 4), x = (i - pr * (kBlurTW / 4)) * 4;
    uint32_t o[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t* row = (const uint32_t*)in[2 * pr + h];
      const uint32_t A = row[(x + 12) >> 2], B = row[(x + 16) >> 2], C = row[(x + 20) >> 2];
      o[h][0] = dot4(B, kB0, dot4(A, kA0, 0));
      o[h][1] = dot4(C, kC1, dot4(B, kB1, dot4(A, kA1, 0)));
      o[h][2] = dot4(C, kC2, dot4(B, kB2, dot4(A, kA2, 0)));
      o[h][3] = dot4(C, kC3, dot4(B, kB3, 0));
    }
    *(uint4*)&tmp[pr][x] = make_uint4(o[0][0] | (o[1][0] << 16), o[0][1] | (o[1][1] << 16),
                                      o[0][2] | (o[1][2] << 16), o[0][3] | (o[1][3] << 16));
  }
  __syncthreads();
  // column pass: thread -> 2 output rows (o, o+1) x 4 columns, reading row pairs o/2 .. o/2+3
  const uint32_t t01 = k[0] | (k[1] << 16), t23 = k[2] | (k[3] << 16), t45 = k[4] | (k[5] << 16), t6 = k[6];
  const uint32_t u0 = k[0] << 16, u12 = k[1] | (k[2] << 16), u34 = k[3] | (k[4] << 16), u56 = k[5] | (k[6] << 16);
  uint8_t* D = blur + g.off + f * g.plane;
  for (int i = tid; i < (kBlurTH / 2) * (kBlurTW / 4); i += 256) {
    const int rp = i / (kBlurTW / 4), cx = (i - rp * (kBlurTW / 4)) * 4;
    const uint4 q0 = *(const uint4*)&tmp[rp][cx], q1 = *(const uint4*)&tmp[rp + 1][cx];
    const uint4 q2 = *(const uint4*)&tmp[rp + 2][cx], q3 = *(const uint4*)&tmp[rp + 3][cx];
    const uint32_t P0[4] = {q0.x, q0.y, q0.z, q0.w}, P1[4] = {q1.x, q1.y, q1.z, q1.w};
    const uint32_t P2[4] = {q2.x, q2.y, q2.z, q2.w}, P3[4] = {q3.x, q3.y, q3.z, q3.w};
    int va[4], vb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t a = dot2(P3[q], t6, dot2(P2[q], t45, dot2(P1[q], t23, dot2(P0[q], t01, 1u << 15))));
      const uint32_t b = dot2(P3[q], u56, dot2(P2[q], u34, dot2(P1[q], u12, dot2(P0[q], u0, 1u << 15))));
      va[q] = min((int)(a >> 16), 255);
      vb[q] = min((int)(b >> 16), 255);
    }
    const uint32_t pa = pack4_u8(va[0], va[1], va[2], va[3]), pb = pack4_u8(vb[0], vb[1], vb[2], vb[3]);
    const int x = x0 + cx;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int y = y0 + 2 * rp + h;
      if (y >= H) break;
      const uint32_t packed = h ? pb : pa;
      uint8_t* dst = D + (long long)y * g.pitch + x;
      if (x + 4 <= W) {
        *(uint32_t*)dst = packed;
      } else {
        for (int q = 0; q < 4 && x + q < W; ++q) dst[q] = (uint8_t)(packed >> (8 * q));
      }
    }
  }
}

void blur_tile_dims(int small, int* tw, int* th) {
  *tw = small ? kBlurTWs : ORBX_BLUR_TW;
  *th = small ? kBlurTHs : ORBX_BLUR_TH;
}

int launch_blur(const ExtractParams& P, const LevelPtrs& lp, const int2* rtab, uint8_t* blur, int batch,
                hipStream_t s) {
  static const int cus = [] {
    int dev = 0, n = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n;
  }();
  // the large tiles once they give every CU two workgroups
  if ((long long)P.blur_ntiles[0] * batch >= 2ll * cus)
    hipLaunchKernelGGL((blur_kernel<ORBX_BLUR_TW, ORBX_BLUR_TH>), dim3(P.blur_ntiles[0], batch), dim3(256), 0, s, P,
                       lp, rtab, P.blur_tiles[0], P.blur_ntiles[0], P.blur_magic[0], blur);
  else
    hipLaunchKernelGGL((blur_kernel<kBlurTWs, kBlurTHs>), dim3(P.blur_ntiles[1], batch), dim3(256), 0, s, P, lp,
                       rtab, P.blur_tiles[1], P.blur_ntiles[1], P.blur_magic[1], blur);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
