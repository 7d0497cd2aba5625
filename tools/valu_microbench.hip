#include <hip/hip_runtime.h>
#include <cstdio>
// Microbenchmark: wave-instruction throughput of the Hamming inner loop's
// instruction mix (xor + bcnt) on all CUs, 8 waves per SIMD.
__device__ __forceinline__ int bcnt_acc(unsigned x, int acc) { int r; asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc)); return r; }
template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned* out, int iters) {
  unsigned a0 = threadIdx.x * 2654435761u, a1 = a0 ^ 0x12345678, a2 = a0 * 3, a3 = a0 + 7, a4 = a0 ^ 0xdead, a5 = a0 - 1, a6 = a0 * 5, a7 = ~a0;
  int d = 0, b = 256, c = 256;
  for (int i = 0; i < iters; ++i) {
    unsigned s = (unsigned)i * 0x9E3779B9u;
    if (MODE == 0) {
      d = bcnt_acc(a0 ^ s, d); d = bcnt_acc(a1 ^ s, d); d = bcnt_acc(a2 ^ s, d); d = bcnt_acc(a3 ^ s, d);
      d = bcnt_acc(a4 ^ s, d); d = bcnt_acc(a5 ^ s, d); d = bcnt_acc(a6 ^ s, d); d = bcnt_acc(a7 ^ s, d);
    } else if (MODE == 2) {  // xor only
      a0 ^= s; a1 ^= a0; a2 ^= a1; a3 ^= a2; a4 ^= a3; a5 ^= a4; a6 ^= a5; a7 ^= a6;
      a0 ^= a7; a1 ^= s; a2 ^= a0; a3 ^= a1; a4 ^= a2; a5 ^= a3; a6 ^= a4; a7 ^= a5;
    } else if (MODE == 3) {  // bcnt only
      d = bcnt_acc(a0, d); d = bcnt_acc(a1, d); d = bcnt_acc(a2, d); d = bcnt_acc(a3, d);
      d = bcnt_acc(a4, d); d = bcnt_acc(a5, d); d = bcnt_acc(a6, d); d = bcnt_acc(a7, d);
      a0 += d; a1 += d; a2 += d; a3 += d; a4 += d; a5 += d; a6 += d; a7 += d;
    } else {
      int e0 = bcnt_acc(a0 ^ s, 0), e1 = bcnt_acc(a1 ^ s, 0), e2 = bcnt_acc(a2 ^ s, 0), e3 = bcnt_acc(a3 ^ s, 0);
      e0 = bcnt_acc(a4 ^ s, e0); e1 = bcnt_acc(a5 ^ s, e1); e2 = bcnt_acc(a6 ^ s, e2); e3 = bcnt_acc(a7 ^ s, e3);
      d += e0 + e1 + e2 + e3;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = d + a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
int main() {
  unsigned* o; hipMalloc(&o, 8192 * 64 * 4);
  const int iters = 20000;
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(2048), dim3(256), 0, 0, o, iters);
      else if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(2048), dim3(256), 0, 0, o, iters);
      else if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(2048), dim3(256), 0, 0, o, iters);
      else hipLaunchKernelGGL(k<3>, dim3(2048), dim3(256), 0, 0, o, iters);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      double instrs = 8192.0 * iters * 16;  // xor + bcnt
      printf("mode %d (%s): %.3f ms, %.3f T wave-instr/s (16 counted per iteration)\n", mode,
             mode == 0 ? "xor+bcnt chain" : mode == 1 ? "xor+bcnt 4 chains" : mode == 2 ? "xor" : "bcnt+add",
             ms, instrs / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
