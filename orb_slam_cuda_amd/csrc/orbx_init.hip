// orbx_init.hip — ORBmatcher::SearchForInitialization on the GPU
// (src/ORBmatcher.cc:405-520 + Frame::AssignFeaturesToGrid / GetFeaturesInArea
// / PosInGrid src/Frame.cc:229-244, 326-391), three launches per batch of
// (F1, F2) pairs.
//
// The reference visits F1's octave-0 keypoints i1 in order. Each takes the
// best / second Hamming distance over F2's octave-0 keypoints in its 2r x 2r
// window (cells column by column, index order inside a cell), skipping every
// i2 whose vMatchedDistance (the distance of the latest earlier query that
// accepted it) is <= the current distance; accepting steals i2 from its
// previous owner. Every query's outcome is a function of the earlier
// outcomes: a triangular system whose unique fixed point is the sequential
// result.
//
// Two facts make the window search a per-query, order-free computation:
//  * the reference's candidate order is (cell column-major, then index), the
//    same for every query, so a candidate's tie-break rank is the key
//    (cell, o2) (o2 = its rank among F2's octave-0 keypoints, index
//    order), and a query's "best, first on ties" and "second" are the two
//    smallest (distance, rank) keys among its UNBLOCKED candidates;
//  * large distances decide nothing: acceptance needs best <= TH_LOW = 50, so
//    any best2 with nnratio x best2 > 50 passes the ratio test whatever its
//    exact value, and vMatchedDistance values are accepted distances (<= 50),
//    so blocking is the same at any distance above 50. With D = 2^dbits - 1
//    the smallest such that nnratio x D > 50 (dbits 6 for the reference's 0.9,
//    7 for 0.7, up to 9 = exact), keys are
//    min(distance, D) << (32 - dbits) | cell << (20 - dbits) | o2: 32 bits,
//    o2 < 2^(20 - dbits) (16384 at 0.9).
//
//   1. search_init_prep_kernel (a workgroup per pair): F2's octave-0
//      keypoints ranked (o2) and bucketed by grid column into a column-sorted
//      record array (x, y, key base, cell row) + descriptors; F1's octave-0
//      queries listed in index order. A window's cell columns are one
//      contiguous run of records, its cell rows a test.
//   2. search_init_query_kernel (8 lanes per query, several workgroups per
//      pair): each query's candidate count and its 8 smallest keys over its
//      window's records. There are no candidate lists, so nothing can
//      overflow.
//   3. search_init_resolve_kernel (a workgroup per pair): Jacobi rounds, every
//      query re-deciding from the previous round's accepted outcomes (per-o2
//      claim lists) by walking its 8 keys; a query whose keys run out (fewer
//      than 2 unblocked of 8, more than 8 candidates) is rescanned by a whole
//      wave over its window. A round without change is the fixed point; past
//      kInitMaxRounds one wave runs the sequential greedy. Then the latest
//      acceptor keeps each i2, rotation consistency (ComputeThreeMaxima), the
//      outputs and the vbPrevMatched update.
#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orbx_device.cuh"
#include "orbx_wave.cuh"

namespace orbx {

constexpr int kInitGridCols = 64, kInitGridRows = 48;  // FRAME_GRID_COLS / ROWS include/Frame.h:37-38
constexpr int kInitHisto = 30;                         // HISTO_LENGTH
constexpr int kInitThLow = 50;                         // TH_LOW
constexpr int kInitMaxRounds = 48;
constexpr int kInitK = 8;       // smallest keys kept per query (a rescan when fewer than 2 of them are unblocked)
constexpr int kInitQLanes = 8;  // lanes per query in the key pass (a DPP half-row)
// 512: a prep workgroup waits for 8 free wave slots beside the extraction
// streams instead of 16 (pipelined search_init stage 0.13-0.14 -> 0.113-0.115
// ms per 64 pairs, frames/s equal within the run-to-run spread, tools/init_ab3.sh)
#ifndef ORBX_INIT_PREP_THREADS
#define ORBX_INIT_PREP_THREADS 512
#endif
#ifndef ORBX_INIT_RESOLVE_THREADS
#define ORBX_INIT_RESOLVE_THREADS 512
#endif
constexpr int kInitPrepThreads = ORBX_INIT_PREP_THREADS;
constexpr int kInitQueryThreads = 256;
constexpr int kInitResolveThreads = ORBX_INIT_RESOLVE_THREADS;
constexpr int kInitKeyRegs = 2;  // queries per resolve thread whose keys are held in registers
constexpr uint32_t kKeyNone = 0xFFFFFFFFu;

#define LDSP __attribute__((address_space(3)))

// Per-pair workspace, ints: [0..64] column starts (64 = records in the grid),
// [66] queries, [67] octave-0 F2 keypoints; then, for K = kp_pitch: records
// (4K: x, y, key base, cell row), descriptors (8K), o2 -> i2 (K), query -> i1
// (K), keys (kInitK K), candidate counts (K). The two K-int tables are padded
// to Kp = K rounded up to 4 ints, so `keys` stays 16-byte aligned (dwordx4)
// for any (odd) pitch.
struct InitWs {
  int* hdr;
  uint4* rec;
  uint4* desc;  // two per record
  int* o2map;
  int* qi;
  uint4* keys;
  int* qcnt;
};
__device__ __forceinline__ InitWs init_ws(int* base, int K) {
  InitWs w;
  w.hdr = base;
  int* p = base + 68;
  w.rec = (uint4*)p;
  p += 4 * (size_t)K;
  w.desc = (uint4*)p;
  p += 8 * (size_t)K;
  const size_t Kp = ((size_t)K + 3) & ~(size_t)3;
  w.o2map = p;
  p += Kp;
  w.qi = p;
  p += Kp;
  w.keys = (uint4*)p;
  p += (size_t)kInitK * K;
  w.qcnt = p;
  return w;
}

size_t init_ws_bytes_per_pair(int kp_pitch) {
  const size_t Kp = ((size_t)kp_pitch + 3) & ~(size_t)3;
  return ((68 + (size_t)kp_pitch * (4 + 8 + kInitK + 1) + 2 * Kp) * 4 + 255) & ~(size_t)255;
}

// Frame::PosInGrid: round() of a float, half away from zero
__device__ __forceinline__ bool init_pos_in_grid(float x, float y, const InitParams& P, int* px, int* py) {
  *px = (int)roundf(__fmul_rn(__fsub_rn(x, P.minX), P.invW));
  *py = (int)roundf(__fmul_rn(__fsub_rn(y, P.minY), P.invH));
  return !(*px < 0 || *px >= kInitGridCols || *py < 0 || *py >= kInitGridRows);
}

// GetFeaturesInArea's cell window (src/Frame.cc:330-346); false when empty
__device__ __forceinline__ bool init_window(float x, float y, const InitParams& P, int& cx0, int& cx1, int& cy0,
                                           int& cy1) {
  const float r = P.r;
  cx0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(x, P.minX), r), P.invW)));
  if (cx0 >= kInitGridCols) return false;
  cx1 = min(kInitGridCols - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(x, P.minX), r), P.invW)));
  if (cx1 < 0) return false;
  cy0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(y, P.minY), r), P.invH)));
  if (cy0 >= kInitGridRows) return false;
  cy1 = min(kInitGridRows - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(y, P.minY), r), P.invH)));
  if (cy1 < 0) return false;
  return true;
}

// GetFeaturesInArea's per-keypoint test inside the window's columns: cell row
// and |dx|, |dy| < r (:350-364)
__device__ __forceinline__ bool init_in_window(const uint4& rc, float x, float y, int cy0, int cy1, float r) {
  const int py = (int)rc.w;
  return py >= cy0 && py <= cy1 && fabsf(__fsub_rn(__uint_as_float(rc.x), x)) < r &&
         fabsf(__fsub_rn(__uint_as_float(rc.y), y)) < r;
}

__device__ __forceinline__ int init_hamming(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ int lds_atomic_add(LDSP int* p, int v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the query's window centre: vbPrevMatched, or F1's own keypoint when prev is
// null (Tracking::MonocularInitialization's initial vbPrevMatched, src/Tracking.cc:645-647)
__device__ __forceinline__ void init_centre(const orbx_kp* kp1, const float* prev, int i1, float& x, float& y) {
  if (prev) {
    x = prev[2 * i1];
    y = prev[2 * i1 + 1];
  } else {
    x = kp1[i1].x;
    y = kp1[i1].y;
  }
}

// ---------------------------------------------------------------- 1. prep
// Ordered compaction: this thread's rank among the workgroup's flagged threads
// (thread order, after the *run flagged before); adds the total to *run.
__device__ __forceinline__ int init_block_rank(bool z, LDSP int* s_w, int* run) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t m = __ballot(z);
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  if (lane == 0) s_w[wv] = __popcll(m);
  __syncthreads();
  int before = *run, tot = 0;
#pragma unroll
  for (int w = 0; w < kInitPrepThreads / 64; ++w) {
    const int c = s_w[w];
    if (w < wv) before += c;
    tot += c;
  }
  __syncthreads();
  *run += tot;
  return before + __popcll(m & lt);
}

__global__ __launch_bounds__(kInitPrepThreads) void search_init_prep_kernel(
    InitParams P, const orbx_kp* __restrict__ kp1_all, const int* __restrict__ n1_all,
    const orbx_kp* __restrict__ kp2_all, const uint8_t* __restrict__ desc2_all, const int* __restrict__ n2_all,
    int* __restrict__ ws_all, int* __restrict__ matches_all) {
  __shared__ int s_col_[kInitGridCols + 1];
  __shared__ int s_w_[kInitPrepThreads / 64];
  LDSP int* s_col = (LDSP int*)s_col_;
  LDSP int* s_w = (LDSP int*)s_w_;
  const int pr = blockIdx.x, tid = threadIdx.x, K = P.kp_pitch;
  const int n1 = n1_all[pr], n2 = n2_all[pr];
  const orbx_kp* kp1 = kp1_all + (size_t)pr * K;
  const orbx_kp* kp2 = kp2_all + (size_t)pr * K;
  const uint8_t* desc2 = desc2_all + (size_t)pr * K * 32;
  InitWs w = init_ws(ws_all + (size_t)pr * P.ws_ints, K);
  int* m12_out = matches_all + (size_t)pr * K;
  for (int c = tid; c <= kInitGridCols; c += kInitPrepThreads) s_col[c] = 0;
  // every output starts unmatched (vnMatches12 = -1, :408)
  for (int i = tid; i < n1; i += kInitPrepThreads) m12_out[i] = -1;
  __syncthreads();
  // F2's octave-0 keypoints (GetFeaturesInArea(.., 0, 0)): rank o2 in index
  // order, column histogram of those in the grid (AssignFeaturesToGrid); the
  // rank inside the column (any order: the keys carry the tie-break) waits in qi
  int n0 = 0;
  for (int i0 = 0; i0 < n2; i0 += kInitPrepThreads) {
    const int i = i0 + tid;
    const bool z = i < n2 && kp2[i].octave == 0;
    const int o2 = init_block_rank(z, s_w, &n0);
    if (z) {
      w.o2map[o2] = i;
      int px, py;
      w.qi[o2] = init_pos_in_grid(kp2[i].x, kp2[i].y, P, &px, &py) ? (px << 16 | lds_atomic_add(&s_col[px], 1)) : -1;
    }
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the 64 column counts
    const int c = s_col[tid];
    const int x = wave_incl_scan_dpp(c);
    s_col[tid] = x - c;
    if (tid == 63) s_col[kInitGridCols] = x;
  }
  __syncthreads();
  for (int o2 = tid; o2 < n0; o2 += kInitPrepThreads) {
    const int t = w.qi[o2];
    if (t < 0) continue;
    const int i2 = w.o2map[o2];
    const orbx_kp k = kp2[i2];
    int px, py;
    init_pos_in_grid(k.x, k.y, P, &px, &py);
    const int s = s_col[t >> 16] + (t & 0xFFFF);
    w.rec[s] = make_uint4(__float_as_uint(k.x), __float_as_uint(k.y),
                          (uint32_t)((px * kInitGridRows + py) << P.obits | o2), (uint32_t)py);
    const uint4* d = (const uint4*)(desc2 + (size_t)i2 * 32);
    w.desc[2 * s] = d[0];
    w.desc[2 * s + 1] = d[1];
  }
  __syncthreads();  // the parked column ranks are read above before the query list overwrites qi
  // F1's octave-0 queries in index order (level1 > 0 is skipped, :424-428)
  int nq = 0;
  for (int i0 = 0; i0 < n1; i0 += kInitPrepThreads) {
    const int i = i0 + tid;
    const bool z = i < n1 && kp1[i].octave == 0;
    const int q = init_block_rank(z, s_w, &nq);
    if (z) w.qi[q] = i;
  }
  for (int c = tid; c <= kInitGridCols; c += kInitPrepThreads) w.hdr[c] = s_col[c];
  if (tid == 0) {
    w.hdr[66] = nq;
    w.hdr[67] = n0;
  }
}

// ---------------------------------------------------------------- 2. keys
// sorted insertion of k into the ascending kInitK-list t
__device__ __forceinline__ void topk_insert(uint32_t (&t)[kInitK], uint32_t k) {
#pragma unroll
  for (int j = 0; j < kInitK; ++j) {
    const uint32_t lo = min(t[j], k);
    k = max(t[j], k);
    t[j] = lo;
  }
}
// the kInitK smallest of two ascending lists, ascending: the elementwise
// minimum against the reversed other list is bitonic, then a bitonic sort
__device__ __forceinline__ void topk_merge(uint32_t (&t)[kInitK], const uint32_t (&o)[kInitK]) {
#pragma unroll
  for (int j = 0; j < kInitK; ++j) t[j] = min(t[j], o[kInitK - 1 - j]);
#pragma unroll
  for (int d = kInitK / 2; d >= 1; d >>= 1)
#pragma unroll
    for (int j = 0; j < kInitK; ++j)
      if ((j & d) == 0) {
        const uint32_t lo = min(t[j], t[j + d]), hi = max(t[j], t[j + d]);
        t[j] = lo;
        t[j + d] = hi;
      }
}
template <int CTRL>
__device__ __forceinline__ void topk_merge_dpp(uint32_t (&t)[kInitK]) {
  uint32_t o[kInitK];
#pragma unroll
  for (int j = 0; j < kInitK; ++j) o[j] = (uint32_t)dpp_i<CTRL>(0, (int)t[j]);
  topk_merge(t, o);
}

__global__ __launch_bounds__(kInitQueryThreads) void search_init_query_kernel(
    InitParams P, const orbx_kp* __restrict__ kp1_all, const uint8_t* __restrict__ desc1_all,
    const float* __restrict__ prev_all, int* __restrict__ ws_all) {
  const int pr = blockIdx.y, tid = threadIdx.x, K = P.kp_pitch;
  InitWs w = init_ws(ws_all + (size_t)pr * P.ws_ints, K);
  const int nq = w.hdr[66];
  const orbx_kp* kp1 = kp1_all + (size_t)pr * K;
  const uint8_t* desc1 = desc1_all + (size_t)pr * K * 32;
  const float* prev = prev_all ? prev_all + (size_t)pr * K * 2 : nullptr;
  const int l = tid & (kInitQLanes - 1);
  constexpr int kQPerWg = kInitQueryThreads / kInitQLanes;
  for (int qb = blockIdx.x * kQPerWg; qb < nq; qb += gridDim.x * kQPerWg) {
    const int q = qb + tid / kInitQLanes;
    uint32_t t[kInitK];
#pragma unroll
    for (int j = 0; j < kInitK; ++j) t[j] = kKeyNone;
    int cnt = 0;
    int cx0, cx1, cy0, cy1;
    float x = 0.f, y = 0.f;
    int i1 = 0;
    if (q < nq) {
      i1 = w.qi[q];
      init_centre(kp1, prev, i1, x, y);
    }
    if (q < nq && init_window(x, y, P, cx0, cx1, cy0, cy1)) {  // uniform across the query's 8 lanes
      const int s1 = w.hdr[cx1 + 1];
      const uint4* qd = (const uint4*)(desc1 + (size_t)i1 * 32);
      const uint4 a0 = qd[0], a1 = qd[1];
      // two records per lane and step, both loads issued before either is used
      for (int s = w.hdr[cx0] + l; s < s1; s += 2 * kInitQLanes) {
        const int s2 = min(s + kInitQLanes, s1 - 1);
        const uint4 rc = w.rec[s], rc2 = w.rec[s2];
        const uint4 b0 = w.desc[2 * s], b1 = w.desc[2 * s + 1];
        const uint4 c0 = w.desc[2 * s2], c1 = w.desc[2 * s2 + 1];
        if (init_in_window(rc, x, y, cy0, cy1, P.r)) {
          const uint32_t d = (uint32_t)min(init_hamming(a0, a1, b0, b1), P.dclamp);
          topk_insert(t, d << P.dshift | rc.z);
          ++cnt;
        }
        if (s + kInitQLanes < s1 && init_in_window(rc2, x, y, cy0, cy1, P.r)) {
          const uint32_t d = (uint32_t)min(init_hamming(a0, a1, c0, c1), P.dclamp);
          topk_insert(t, d << P.dshift | rc2.z);
          ++cnt;
        }
      }
    }
    // the query's 8 lanes merge their lists (quad_perm 1032, 2301, then the
    // other quad of the half-row by row_half_mirror) and sum their counts
    topk_merge_dpp<kDppQuad1032>(t);
    topk_merge_dpp<kDppQuad2301>(t);
    topk_merge_dpp<kDppHalfMirror>(t);
    cnt += dpp_i<kDppQuad1032>(0, cnt);
    cnt += dpp_i<kDppQuad2301>(0, cnt);
    cnt += dpp_i<kDppHalfMirror>(0, cnt);
    if (q < nq && l < kInitK / 4) {  // the first kInitK / 4 lanes store a uint4 each
      uint32_t v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = t[j];
#pragma unroll
        for (int u = 1; u < kInitK / 4; ++u)
          if (l == u) v[j] = t[4 * u + j];
      }
      w.keys[(size_t)q * (kInitK / 4) + l] = make_uint4(v[0], v[1], v[2], v[3]);
      if (l == 0) w.qcnt[q] = cnt;
    }
  }
}

// ---------------------------------------------------------------- 3. resolve
__device__ __forceinline__ void load_keys(const InitWs& w, int q, uint32_t (&key)[kInitK]) {
#pragma unroll
  for (int u = 0; u < kInitK / 4; ++u) {
    const uint4 kk = w.keys[(size_t)q * (kInitK / 4) + u];
    key[4 * u] = kk.x;
    key[4 * u + 1] = kk.y;
    key[4 * u + 2] = kk.z;
    key[4 * u + 3] = kk.w;
  }
}

// vMatchedDistance[o2] at query q's turn: the smallest distance of an earlier
// query's claim on o2 in the snapshot (INT_MAX if none)
__device__ __forceinline__ int init_claim_md(const LDSP int* head, const LDSP int* nxt, int o2, int q) {
  int md = INT_MAX;
  for (int hd = head[o2]; hd >= 0;) {
    const int x = nxt[hd];
    if (hd < q) md = min(md, x & 511);
    hd = (x >> 9) - 1;
  }
  return md;
}

// One query's decision from its two smallest unblocked keys (:447-471): -1, or
// o2 << 9 | bestDist
__device__ __forceinline__ int init_decide(uint32_t k1, uint32_t k2, const InitParams& P) {
  if (k1 == kKeyNone) return -1;
  const int best = (int)(k1 >> P.dshift);
  const float best2 = k2 == kKeyNone ? (float)INT_MAX : (float)(int)(k2 >> P.dshift);
  const bool ok = best <= kInitThLow && (float)best < __fmul_rn(best2, P.nnratio);
  return ok ? (int)((k1 & P.omask) << 9) | best : -1;
}

// unsigned wave minimum from two signed 16-bit-half minima (every lane active)
__device__ __forceinline__ uint32_t wave_umin(uint32_t v) {
  const int hi = wave_min_dpp((int)(v >> 16));
  const int lo = wave_min_dpp((int)((v >> 16) == (uint32_t)hi ? (v & 0xFFFF) : 0xFFFFu));
  return (uint32_t)hi << 16 | (uint32_t)lo;
}

// A whole wave's scan of query q's window when its keys ran out: the decision
// from the two smallest unblocked keys (wave minima; keys are unique).
// blocked(o2, d): an earlier query's claim blocks candidate o2 at distance d.
template <typename Blocked>
__device__ int init_rescan_wave(const InitParams& P, const InitWs& w, const orbx_kp* kp1, const uint8_t* desc1,
                                const float* prev, int q, Blocked blocked) {
  const int lane = threadIdx.x & 63;
  const int i1 = w.qi[q];
  float x, y;
  init_centre(kp1, prev, i1, x, y);
  int cx0, cx1, cy0, cy1;
  if (!init_window(x, y, P, cx0, cx1, cy0, cy1)) return -1;
  const uint4* qd = (const uint4*)(desc1 + (size_t)i1 * 32);
  const uint4 a0 = qd[0], a1 = qd[1];
  uint32_t k1 = kKeyNone, k2 = kKeyNone;
  const int s1 = w.hdr[cx1 + 1];
  for (int s = w.hdr[cx0] + lane; s < s1; s += 64) {
    const uint4 rc = w.rec[s];
    if (!init_in_window(rc, x, y, cy0, cy1, P.r)) continue;
    const int d = min(init_hamming(a0, a1, w.desc[2 * s], w.desc[2 * s + 1]), P.dclamp);
    if (blocked((int)(rc.z & P.omask), d)) continue;
    const uint32_t key = (uint32_t)d << P.dshift | rc.z;
    k2 = min(k2, max(k1, key));
    k1 = min(k1, key);
  }
  const uint32_t b1 = wave_umin(k1);
  const uint32_t b2 = wave_umin(k1 == b1 ? k2 : k1);
  return init_decide(b1, b2, P);
}

__global__ __launch_bounds__(kInitResolveThreads) void search_init_resolve_kernel(
    InitParams P, const orbx_kp* __restrict__ kp1_all, const uint8_t* __restrict__ desc1_all,
    const orbx_kp* __restrict__ kp2_all, float* __restrict__ prev_all, int* __restrict__ ws_all,
    int* __restrict__ matches_all, int* __restrict__ nmatches) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NT = kInitResolveThreads;
  const int pr = blockIdx.x, tid = threadIdx.x, K = P.kp_pitch;
  const int lane = tid & 63, wv = tid >> 6;
  InitWs w = init_ws(ws_all + (size_t)pr * P.ws_ints, K);
  const orbx_kp* kp1 = kp1_all + (size_t)pr * K;
  const orbx_kp* kp2 = kp2_all + (size_t)pr * K;
  const uint8_t* desc1 = desc1_all + (size_t)pr * K * 32;
  float* prev = prev_all ? prev_all + (size_t)pr * K * 2 : nullptr;
  int* m12_out = matches_all + (size_t)pr * K;
  const int nq = w.hdr[66], n0 = w.hdr[67];
  // LDS: res[K] (per query: -1 or o2 << 9 | distance), head[K] (per o2: latest
  // claimer of the snapshot; later vMatchedDistance / the keeper), nxt[K] (per
  // query: (next claimer + 1) << 9 | its distance; later the rotHist entry),
  // queue[K] (rescans; later vnMatches21), var[32], hist[32]
  const long long t0 = P.prof ? (long long)__builtin_amdgcn_s_memtime() : 0;
  auto stamp = [&](int k) {
    if (P.prof && tid == 0) P.prof[pr * 16 + k] = (long long)__builtin_amdgcn_s_memtime() - t0;
  };
  LDSP int* res = (LDSP int*)smem;
  LDSP int* head = res + K;
  LDSP int* nxt = head + K;
  LDSP int* queue = nxt + K;
  LDSP int* var = queue + K;
  LDSP int* hist = var + 32;
  if (tid < 32) {
    var[tid] = 0;
    hist[tid] = 0;
  }
  for (int i = tid; i < nq; i += NT) res[i] = -1;
  for (int i = tid; i < n0; i += NT) head[i] = -1;
  // the keys of this thread's first queries stay in registers over the rounds
  uint32_t kreg[kInitKeyRegs][kInitK];
  int creg[kInitKeyRegs];
#pragma unroll
  for (int j = 0; j < kInitKeyRegs; ++j) {
    const int q = min(tid + j * NT, max(nq - 1, 0));
    load_keys(w, q, kreg[j]);
    creg[j] = w.qcnt[q];
  }
  __syncthreads();
  if (tid == 0) var[6] = 1;  // changed
  __syncthreads();
  stamp(1);
  bool converged = false;
  int rounds = 0;
  for (int round = 0; round < kInitMaxRounds; ++round) {
    if (var[6] == 0) {
      converged = true;
      break;
    }
    ++rounds;
    __syncthreads();
    if (tid == 0) {
      var[6] = 0;
      var[7] = 0;  // rescan queue length
    }
    __syncthreads();
    int changed = 0;
    auto visit = [&](int q, const uint32_t* key, int qc) {
      uint32_t k1 = kKeyNone, k2 = kKeyNone;
      int found = 0;
#pragma unroll
      for (int u = 0; u < kInitK; ++u) {
        if (found == 2 || key[u] == kKeyNone) continue;
        const int d = (int)(key[u] >> P.dshift), o2 = (int)(key[u] & P.omask);
        if (init_claim_md(head, nxt, o2, q) <= d) continue;  // (:444-445)
        if (found == 0) k1 = key[u];
        else k2 = key[u];
        ++found;
      }
      if (found < 2 && qc > kInitK) {
        queue[lds_atomic_add(&var[7], 1)] = q;  // keys ran out: a wave rescans the window
        return;
      }
      const int r = init_decide(k1, k2, P);
      if (res[q] != r) {
        res[q] = r;
        changed = 1;
      }
    };
    // the register-held queries with compile-time indices (no dynamic
    // register indexing, which would go through scratch), then the rest
#pragma unroll
    for (int j = 0; j < kInitKeyRegs; ++j)
      if (tid + j * NT < nq) visit(tid + j * NT, kreg[j], creg[j]);
    for (int q = tid + kInitKeyRegs * NT; q < nq; q += NT) {
      uint32_t key[kInitK];
      load_keys(w, q, key);
      visit(q, key, w.qcnt[q]);
    }
    __syncthreads();
    const int nrs = var[7];
    if (P.prof && tid == 0) P.prof[pr * 16 + 9] += nrs;
    for (int j = wv; j < nrs; j += NT / 64) {
      const int q = queue[j];
      const int r = init_rescan_wave(P, w, kp1, desc1, prev, q,
                                     [&](int o2, int d) { return init_claim_md(head, nxt, o2, q) <= d; });
      if (lane == 0 && res[q] != r) {
        res[q] = r;
        changed = 1;
      }
    }
    if (changed) var[6] = 1;
    __syncthreads();
    // snapshot of this round's outcomes as per-o2 claim lists
    for (int i = tid; i < n0; i += NT) head[i] = -1;
    __syncthreads();
    for (int q = tid; q < nq; q += NT) {
      const int r = res[q];
      if (r >= 0)
        nxt[q] = ((__hip_atomic_exchange(&head[r >> 9], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) + 1) << 9) |
                 (r & 511);
    }
    __syncthreads();
  }
  stamp(2);
  if (P.prof && tid == 0) P.prof[pr * 16 + 8] = rounds + (converged ? 0 : 1000);
  LDSP int* src = nxt;  // per query: the o2 its acceptance entered into rotHist, then its bin
  if (converged) {
    // the latest accepting query keeps each o2 (earlier ones were stolen
    // from, :463-467); every accepted query entered rotHist (:469-470)
    for (int i = tid; i < n0; i += NT) head[i] = -1;
    __syncthreads();
    for (int q = tid; q < nq; q += NT) {
      const int r = res[q];
      if (r >= 0) __hip_atomic_fetch_max(&head[r >> 9], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    int kept = 0;
    for (int q = tid; q < nq; q += NT) {
      const int r = res[q];
      const int b = r >= 0 ? (r >> 9) : -1;
      const bool keep = r >= 0 && head[b] == q;
      src[q] = b;
      res[q] = keep ? b : -1;  // res becomes vnMatches12 (as o2)
      kept += keep ? 1 : 0;
    }
    kept = wave_sum_dpp(kept);
    if (lane == 0 && kept) lds_atomic_add(&var[0], kept);
    __syncthreads();
  } else {
    // ---- sequential greedy in query order (one wave; pathological chains only)
    LDSP int* md = head;    // per o2: vMatchedDistance
    LDSP int* m21 = queue;  // per o2: vnMatches21
    for (int i = tid; i < n0; i += NT) {
      md[i] = INT_MAX;
      m21[i] = -1;
    }
    for (int q = tid; q < nq; q += NT) {
      res[q] = -1;
      src[q] = -1;
    }
    __syncthreads();
    if (wv == 0) {
      int nm = 0;
      for (int q = 0; q < nq; ++q) {
        uint32_t key[kInitK];
        load_keys(w, q, key);
        uint32_t k1 = kKeyNone, k2 = kKeyNone;
        int found = 0;
        for (int j = 0; j < kInitK && found < 2; ++j) {
          if (key[j] == kKeyNone) break;
          const int d = (int)(key[j] >> P.dshift), o2 = (int)(key[j] & P.omask);
          if (md[o2] <= d) continue;
          if (found == 0) k1 = key[j];
          else k2 = key[j];
          ++found;
        }
        const int r = (found < 2 && w.qcnt[q] > kInitK)
                          ? init_rescan_wave(P, w, kp1, desc1, prev, q, [&](int o2, int d) { return md[o2] <= d; })
                          : init_decide(k1, k2, P);
        if (r >= 0 && lane == 0) {
          const int b = r >> 9;
          if (m21[b] >= 0) {  // steal (:463-467)
            res[m21[b]] = -1;
            nm--;
          }
          res[q] = b;
          m21[b] = q;
          md[b] = r & 511;
          nm++;
          src[q] = b;
        }
        // lane 0's LDS stores before every lane's next reads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      if (lane == 0) var[0] = nm;
    }
    __syncthreads();
  }
  stamp(3);
  // Rotation consistency (:473-512, ComputeThreeMaxima :1601-1642)
  const float factor = 1.0f / kInitHisto;
  if (P.check_ori) {
    for (int q = tid; q < nq; q += NT) {
      const int j = src[q];
      int bin = -1;
      if (j >= 0) {
        float rot = __fsub_rn(kp1[w.qi[q]].angle, kp2[w.o2map[j]].angle);
        if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
        bin = (int)roundf(__fmul_rn(rot, factor));
        if (bin == kInitHisto) bin = 0;
        lds_atomic_add(&hist[bin], 1);
      }
      src[q] = bin;
    }
    __syncthreads();
    if (tid < 64) {
      // ComputeThreeMaxima's sequential scan (strict >, first index wins) is a
      // stable top-3 of the positive bins by (count desc, index asc): three wave
      // maxima of (count << 8 | 255 - bin), each excluding the previous winner
      int key = tid < kInitHisto && hist[tid] > 0 ? (hist[tid] << 8) | (255 - tid) : 0;
      int top[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        top[k] = INT_MAX - wave_min_dpp(INT_MAX - key);
        if (key == top[k]) key = 0;
      }
      if (tid == 0) {
        const int max1 = top[0] >> 8, max2 = top[1] >> 8, max3 = top[2] >> 8;
        int ind1 = max1 ? 255 - (top[0] & 255) : -1, ind2 = max2 ? 255 - (top[1] & 255) : -1,
            ind3 = max3 ? 255 - (top[2] & 255) : -1;
        if (max2 < __fmul_rn(0.1f, (float)max1)) {
          ind2 = -1;
          ind3 = -1;
        } else if (max3 < __fmul_rn(0.1f, (float)max1)) {
          ind3 = -1;
        }
        var[1] = ind1;
        var[2] = ind2;
        var[3] = ind3;
      }
    }
    __syncthreads();
    const int ind1 = var[1], ind2 = var[2], ind3 = var[3];
    int rej = 0;
    for (int q = tid; q < nq; q += NT) {
      const int b = src[q];
      if (b < 0 || b == ind1 || b == ind2 || b == ind3) continue;
      if (res[q] >= 0) {
        res[q] = -1;
        ++rej;
      }
    }
    rej = wave_sum_dpp(rej);
    if (lane == 0 && rej) lds_atomic_add(&var[0], -rej);
    __syncthreads();
  }
  // outputs: vnMatches12 of the matched queries (the prep kernel wrote -1 for
  // every i1) and their vbPrevMatched (:515-517)
  for (int q = tid; q < nq; q += NT) {
    const int b = res[q];
    if (b < 0) continue;
    const int i1 = w.qi[q], i2 = w.o2map[b];
    m12_out[i1] = i2;
    if (prev) {
      prev[2 * i1] = kp2[i2].x;
      prev[2 * i1 + 1] = kp2[i2].y;
    }
  }
  if (tid == 0) nmatches[pr] = var[0];
  stamp(4);
}

static size_t init_resolve_lds_bytes(int kp_pitch) { return (size_t)kp_pitch * 16 + 256; }

static int init_dbits(float nnratio) {
  int dbits = 6;
  while (dbits < 9 && !((float)((1 << dbits) - 1) * nnratio > (float)kInitThLow)) ++dbits;
  return dbits;
}

// The largest kp_pitch launch_search_init accepts at this nnratio: o2 must fit
// the key's 20 - dbits bits, the resolve kernel's tables one workgroup's LDS.
int search_init_max_pitch(float nnratio) {
  const int by_key = 1 << (20 - init_dbits(nnratio));
  const int by_lds = (int)((kInitLdsBudget - 256) / 16);
  return std::min(by_key, by_lds);
}

int launch_search_init(const InitParams& P0, const orbx_kp* kp1, const uint8_t* desc1, const int* n1,
                       const orbx_kp* kp2, const uint8_t* desc2, const int* n2, float* prev, int* ws,
                       int* matches12, int* nmatches, int pairs, void* stream) {
  InitParams P = P0;
  // the key layout for this ratio: the fewest distance bits whose clamp value
  // still passes the ratio test for every acceptable best (see the header)
  const int dbits = init_dbits(P.nnratio);
  P.dshift = 32 - dbits;
  P.obits = 20 - dbits;
  P.omask = (1u << P.obits) - 1;
  P.dclamp = (1 << dbits) - 1;
  // o2 must fit its key field; the resolve kernel's four per-keypoint LDS
  // tables must fit one workgroup's LDS
  if (P.kp_pitch < 1 || P.kp_pitch > (1 << P.obits) || init_resolve_lds_bytes(P.kp_pitch) > kInitLdsBudget)
    return ORBX_ECAPACITY;
  P.ws_ints = (long long)(init_ws_bytes_per_pair(P.kp_pitch) / 4);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(search_init_prep_kernel, dim3(pairs), dim3(kInitPrepThreads), 0, s, P, kp1, n1, kp2, desc2, n2, ws,
                     matches12);
  // query workgroups per pair: 32 queries each, up to 16 (a KITTI pair's ~430
  // octave-0 queries in one pass), grid-strided beyond
  const int qblocks = std::max(1, std::min(16, (P.kp_pitch + 31) / 32));
  hipLaunchKernelGGL(search_init_query_kernel, dim3(qblocks, pairs), dim3(kInitQueryThreads), 0, s, P, kp1, desc1,
                     prev, ws);
  const size_t lds = init_resolve_lds_bytes(P.kp_pitch);
  if (raise_lds_limit((const void*)search_init_resolve_kernel, lds)) return ORBX_EDEVICE;
  // ORBX_INIT_PROF=1 (diagnostics): the resolve kernel's phase clocks, averaged
  // over the pairs and printed after the call (synchronises)
  static long long* prof = nullptr;
  static const bool do_prof = getenv("ORBX_INIT_PROF") && getenv("ORBX_INIT_PROF")[0] == '1';
  if (do_prof) {
    if (pairs > 4096) return ORBX_EINVAL;
    if (!prof && hipMalloc(&prof, (size_t)4096 * 16 * 8) != hipSuccess) return ORBX_EDEVICE;
    if (hipMemsetAsync(prof, 0, (size_t)pairs * 16 * 8, s) != hipSuccess) return ORBX_EDEVICE;
    P.prof = prof;
  }
  hipLaunchKernelGGL(search_init_resolve_kernel, dim3(pairs), dim3(kInitResolveThreads), lds, s, P, kp1, desc1, kp2,
                     prev, ws, matches12, nmatches);
  if (do_prof) {
    std::vector<long long> h((size_t)pairs * 16);
    if (hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(h.data(), prof, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
      return ORBX_EDEVICE;
    double a[16] = {0};
    for (int q = 0; q < pairs; ++q)
      for (int k = 0; k < 16; ++k) a[k] += (double)h[q * 16 + k] / pairs;
    fprintf(stderr, "search_init resolve (avg clocks from start): keys %.0f rounds %.0f keep %.0f rotation+out %.0f | "
            "rounds %.2f rescans %.2f\n", a[1], a[2], a[3], a[4], a[8], a[9]);
  }
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
