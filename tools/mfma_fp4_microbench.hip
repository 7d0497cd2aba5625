// Issue rate of v_mfma_scale_f32_32x32x64_f8f6f4 (e2m1 operands) vs
// v_mfma_f32_32x32x16_bf16: independent accumulator chains, operands in
// registers, every SIMD busy. Prints ns per MFMA per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_fp4_microbench.hip -o /tmp/mfma_mb
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
template <int MODE>
__global__ __launch_bounds__(256) void mb(float* out, int iters, int seed) {
  v8i a = {seed + (int)threadIdx.x, 2, 3, 4, 0, 0, 0, 0}, b = {5, seed, 7, 8, 0, 0, 0, 0};
  v8bf ab, bb;
  for (int i = 0; i < 8; ++i) { ab[i] = (__bf16)(float)(threadIdx.x + i); bb[i] = (__bf16)(float)(seed + i); }
  v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {
      c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, 4, 4, 0, 127, 0, 127);
      c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c1, 4, 4, 0, 127, 0, 127);
      c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c2, 4, 4, 0, 127, 0, 127);
      c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c3, 4, 4, 0, 127, 0, 127);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, c3, 0, 0, 0);
    }
  }
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  if (s == 12345.f) out[threadIdx.x] = s;
}
int main() {
  float* out;
  hipMalloc(&out, 4096);
  const int iters = 4096, wgs = 256 * 8;  // 8 waves per CU... 4 waves per WG x 2048 WGs
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(mb<0>, dim3(wgs), dim3(256), 0, 0, out, iters, 1);
      else hipLaunchKernelGGL(mb<1>, dim3(wgs), dim3(256), 0, 0, out, iters, 1);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double mfma_per_simd = (double)wgs * 4 * iters * 4 / 1024.0;
      if (rep) printf("%s: %.3f ms, %.2f ns per MFMA per SIMD (%.1f cycles at 2.4 GHz)\n",
                      mode == 0 ? "fp4 scaled 32x32x64" : "bf16 32x32x16", ms, ms * 1e6 / mfma_per_simd,
                      ms * 1e6 / mfma_per_simd * 2.4);
    }
  }
  return 0;
}
