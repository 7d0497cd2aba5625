// orbx_sincosf.h — glibc's single-precision sinf/cosf, restated bit-exactly.
//
// computeOrbDescriptor (src/ORBextractor.cc:199-200) rotates the BRIEF
// pattern with a = (float)cos(angle), b = (float)sin(angle) on a float
// argument, i.e. glibc cosf/sinf. Those are not correctly rounded: over
// [0, 2pi) they differ from (float)cos((double)x) on ~1.5M inputs, and a
// 1-ulp difference can move a cvRound of a rotated pattern point. This is
// the algorithm glibc 2.35 runs on x86-64 CPUs with FMA (the FMA ifunc
// variant of the optimized-routines sinf/cosf; aarch64 builds contract the
// same expressions into FMAs): double-precision reduction by pi/2 and short
// polynomials, every FMA single-rounded. Coefficients are those of glibc's
// __sincosf_table. Valid for |x| < 120 (extraction only passes [0, 2pi)).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace orbx {

struct SinCosfTable {
  double sign[4];
  double hpi_inv, hpi;
  double c0, c1, s1, c2, s2, c3, s3, c4;
};

__host__ __device__ inline const SinCosfTable& sincosf_table(int k) {
  // {sign[4], hpi_inv = 2^24 * 2/pi, hpi = pi/2, c0, c1, s1, c2, s2, c3, s3, c4}
  static constexpr SinCosfTable T[2] = {
      {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1.0p+0, -0x1.ffffffd0c621cp-2,
       -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10,
       -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
      {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -0x1.0p+0, 0x1.ffffffd0c621cp-2,
       -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10,
       -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16}};
  return T[k];
}

// fused multiply-add, one rounding (v_fma_f64 on the device, fma() on a host)
__host__ __device__ inline double sincosf_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// sin polynomial: x + x^3 s1 + x^5 (s2 + x^2 s3)
__host__ __device__ inline float sincosf_sinpoly(const SinCosfTable& p, double x, double x2) {
  const double x3 = x2 * x;
  const double x5 = x2 * x3;
  const double s = sincosf_fma(x3, p.s1, x);
  return (float)sincosf_fma(sincosf_fma(x2, p.s3, p.s2), x5, s);
}
// cos polynomial: c0 + x^2 c1 + x^4 c2 + x^6 (c3 + x^2 c4)
__host__ __device__ inline float sincosf_cospoly(const SinCosfTable& p, double x2) {
  const double x4 = x2 * x2;
  const double a = sincosf_fma(x2, p.c1, p.c0);
  const double b = sincosf_fma(x2, p.c4, p.c3);
  const double x6 = x2 * x4;
  const double c = sincosf_fma(x4, p.c2, a);
  return (float)sincosf_fma(b, x6, c);
}

__host__ __device__ inline void glibc_sincosf(float y, float* sn, float* cs) {
  uint32_t u;
  __builtin_memcpy(&u, &y, 4);
  const uint32_t top12 = (u >> 20) & 0x7ff;
  const double x = y;
  if (top12 < 0x3f4) {  // |y| < 0.75 (glibc's abstop12(y) < abstop12(pi/4))
    if (top12 <= 0x397) {  // |y| < 2^-12
      *sn = y;
      *cs = 1.0f;
      return;
    }
    const double x2 = x * x;
    *sn = sincosf_sinpoly(sincosf_table(0), x, x2);
    *cs = sincosf_cospoly(sincosf_table(0), x2);
    return;
  }
  const SinCosfTable& t0 = sincosf_table(0);
  const double r = x * t0.hpi_inv;
  const int n = ((int)r + 0x800000) >> 24;                // round(x * 2/pi)
  const double xr = sincosf_fma(-(double)n, t0.hpi, x);   // x - n*pi/2, one rounding
  const double x2 = xr * xr;
  const SinCosfTable& p = sincosf_table((n & 2) ? 1 : 0);
  const double xs = xr * t0.sign[n & 3];
  if (n & 1) {
    *sn = sincosf_cospoly(p, x2);
    *cs = sincosf_sinpoly(p, xs, x2);
  } else {
    *sn = sincosf_sinpoly(p, xs, x2);
    *cs = sincosf_cospoly(p, x2);
  }
}

}  // namespace orbx
