// orbx_wave.cuh — wave64 reductions and scans on DPP (no LDS round trips).
//
// __shfl_xor / __shfl_up lower to ds_bpermute_b32 (an LDS-pipe instruction
// with LDS latency); the serial loops of the matchers run one reduction per
// query, so these use DPP row operations instead: quad_perm, row_half_mirror
// and row_mirror inside 16-lane rows, then row_bcast:15 / row_bcast:31
// across rows (GFX9-family DPP, available on gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <climits>

namespace orbx {

// popcount of the bits of m below this lane
__device__ __forceinline__ int mbcnt64(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int dpp_i(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, 0xf, false);
}

constexpr int kDppQuad1032 = 0xB1;  // quad_perm:[1,0,3,2]
constexpr int kDppQuad2301 = 0x4E;  // quad_perm:[2,3,0,1]
constexpr int kDppHalfMirror = 0x141;
constexpr int kDppMirror = 0x140;
constexpr int kDppBcast15 = 0x142;
constexpr int kDppBcast31 = 0x143;
constexpr int kDppShr1 = 0x111, kDppShr2 = 0x112, kDppShr4 = 0x114, kDppShr8 = 0x118;

// wave-uniform min of v over all 64 lanes (every lane must be active)
__device__ __forceinline__ int wave_min_dpp(int v) {
  v = min(v, dpp_i<kDppQuad1032>(INT_MAX, v));
  v = min(v, dpp_i<kDppQuad2301>(INT_MAX, v));
  v = min(v, dpp_i<kDppHalfMirror>(INT_MAX, v));
  v = min(v, dpp_i<kDppMirror>(INT_MAX, v));
  v = min(v, dpp_i<kDppBcast15, 0xa>(INT_MAX, v));
  v = min(v, dpp_i<kDppBcast31, 0xc>(INT_MAX, v));
  return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ int wave_sum_dpp(int v) {
  v += dpp_i<kDppQuad1032>(0, v);
  v += dpp_i<kDppQuad2301>(0, v);
  v += dpp_i<kDppHalfMirror>(0, v);
  v += dpp_i<kDppMirror>(0, v);
  v += dpp_i<kDppBcast15, 0xa>(0, v);
  v += dpp_i<kDppBcast31, 0xc>(0, v);
  return __builtin_amdgcn_readlane(v, 63);
}

// inclusive prefix sum over lanes 0..63 (every lane must be active)
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
  v += dpp_i<kDppShr1>(0, v);
  v += dpp_i<kDppShr2>(0, v);
  v += dpp_i<kDppShr4>(0, v);
  v += dpp_i<kDppShr8>(0, v);
  v += dpp_i<kDppBcast15, 0xa>(0, v);
  v += dpp_i<kDppBcast31, 0xc>(0, v);
  return v;
}

}  // namespace orbx
