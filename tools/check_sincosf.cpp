// Exhaustive check of the glibc sinf/cosf restatement (orbx_sincosf.h)
// against the host's glibc over every float in [lo, hi) (default [0, 2pi)).
// Build: hipcc -O2 -I orb_slam_cuda_amd/csrc tools/check_sincosf.cpp -o /tmp/check_sincosf
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "orbx_sincosf.h"

int main(int argc, char** argv) {
  float lo = argc > 1 ? strtof(argv[1], nullptr) : 0.0f;
  float hi = argc > 2 ? strtof(argv[2], nullptr) : 6.2831855f;
  long long n = 0, bad = 0;
  for (float x = lo; x < hi; x = nextafterf(x, 1e30f)) {
    float s, c;
    orbx::glibc_sincosf(x, &s, &c);
    const float gs = sinf(x), gc = cosf(x);
    if (memcmp(&s, &gs, 4) || memcmp(&c, &gc, 4)) {
      if (bad < 10) printf("mismatch x=%a sin %a/%a cos %a/%a\n", x, s, gs, c, gc);
      ++bad;
    }
    ++n;
  }
  printf("checked %lld floats in [%g, %g): %lld mismatches\n", n, lo, hi, bad);
  return bad != 0;
}
