// orbx_device.cuh — device helpers shared by the extractor kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "orbx_internal.h"
#include "orbx_wave.cuh"

namespace orbx {

__device__ __forceinline__ int sat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// Pack four saturated bytes into one dword. The empty asm stops the backend
// from fusing (ashr, clamp, pack) pairs into v_ashr_pk_u8_i32: hipcc (ROCm
// 7.2, gfx950) then ORs the other two bytes into that register as if its
// upper half were zero, which it is not (corrupted bytes 2-3 of every packed
// pyramid store until this barrier went in; tests/test_gpu_extract.py).
__device__ __forceinline__ uint32_t pack4_u8(int a, int b, int c, int d) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}

// BORDER_REFLECT_101 (cv::borderInterpolate) for p in [-(len-1), 2*len-2].
__device__ __forceinline__ int reflect101(int p, int len) {
  if (p < 0) p = -p;
  if (p >= len) p = 2 * len - 2 - p;
  return p;
}
__device__ __forceinline__ int reflect101_clamped(int p, int len) {
  return reflect101(min(max(p, -(len - 1)), 2 * len - 2), len);
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// XCD-aware workgroup order. Workgroups are dealt round-robin over the 8
// XCDs (each with its own L2), so consecutive linear ids land on different
// L2s and neighbouring tiles' shared halo lines are fetched once per XCD.
// This bijection hands each XCD a contiguous run of logical tiles instead
// (q = n/8, r = n%8; MI355X_MICROARCH.md "Workgroup dispatch"). Speed only:
// any placement is correct.
__device__ __forceinline__ int xcd_remap(int orig, int n) {
  const int q = n >> 3, r = n & 7, x = orig & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (orig >> 3);
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// cv::fastAtan2 (OpenCV 3.x polynomial), float arithmetic without contraction.
__device__ __forceinline__ float fast_atan2_dev(float y, float x) {
  const float p1 = __fmul_rn(0.9997878412794807f, (float)(180 / M_PI));
  const float p3 = __fmul_rn(-0.3258083974640975f, (float)(180 / M_PI));
  const float p5 = __fmul_rn(0.1555786518463281f, (float)(180 / M_PI));
  const float p7 = __fmul_rn(-0.04432655554792128f, (float)(180 / M_PI));
  const float eps = (float)2.220446049250313e-16;  // (float)DBL_EPSILON
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = __fdiv_rn(ay, __fadd_rn(ax, eps));
    c2 = __fmul_rn(c, c);
    a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
  } else {
    c = __fdiv_rn(ax, __fadd_rn(ay, eps));
    c2 = __fmul_rn(c, c);
    a = __fsub_rn(90.f,
                  __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1),
                            c));
  }
  if (x < 0) a = __fsub_rn(180.f, a);
  if (y < 0) a = __fsub_rn(360.f, a);
  return a;
}

// Workgroup barrier that orders LDS only. __syncthreads() is a workgroup
// release/acquire fence on all memory: on gfx950 it first waits for every
// outstanding global store of the thread (s_waitcnt vmcnt(0)), which stalls a
// kernel that streams results to HBM between LDS phases. Use this one where
// no thread reads global data another thread of the workgroup wrote.
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Exclusive scan of a[0..n) in LDS by NT threads; returns the total.
// LDS_ONLY: the barriers order LDS only (lds_sync).
template <int NT, bool LDS_ONLY = false>
__device__ int block_scan_excl(int* a, int n, int* s_tmp) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = (n + NT - 1) / NT;
  const int b = min(tid * per, n), e = min(b + per, n);
  int sum = 0;
  for (int i = b; i < e; ++i) sum += a[i];
  const int x = wave_incl_scan_dpp(sum);
  if (lane == 63) s_tmp[w] = x;
  if (LDS_ONLY) lds_sync(); else __syncthreads();
  int wpre = 0, total = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
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
  if (LDS_ONLY) lds_sync(); else __syncthreads();
  return total;
}

// Host launchers of the stage kernels (one translation unit each).
int launch_pyramid(const ExtractParams& P, const LevelPtrs& lp, const int2* rtab, int batch, hipStream_t s);
int launch_blur(const ExtractParams& P, const LevelPtrs& lp, const int2* rtab, uint8_t* blur, int batch, hipStream_t s);
int launch_fast(const ExtractParams& P, const LevelPtrs& lp, const CellGeom* cells, uint32_t* slots,
                int* cell_counts, int batch, hipStream_t s);
int launch_quadtree(const ExtractParams& P, const ExtractBuffers& X, int batch, hipStream_t s);
int launch_orient_brief(const ExtractParams& P, const LevelPtrs& lp, const ExtractBuffers& X, orbx_kp* kps,
                        uint8_t* desc, int* counts, int batch, hipStream_t s);
size_t quadtree_lds_bytes(const ExtractParams& P);
size_t pyr_band_lds_bytes(const ExtractParams& P);
const void* pyr_band_kernel_ptr();
size_t fast_lds_bytes(const ExtractParams& P);
const void* quadtree_kernel_ptr(const ExtractParams& P);

}  // namespace orbx
