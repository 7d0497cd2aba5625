// orbx_init.hip — ORBmatcher::SearchForInitialization on the GPU
// (src/ORBmatcher.cc:405-520 + Frame::AssignFeaturesToGrid / GetFeaturesInArea
// / PosInGrid src/Frame.cc:229-244, 326-391), one workgroup per (F1, F2) pair.
//
// The reference visits F1's octave-0 keypoints i1 in order. Each takes the
// best / second Hamming distance over F2's octave-0 keypoints in its 2r x 2r
// window (visited cell column by column, index order inside a cell),
// skipping every i2 whose vMatchedDistance (the distance of the latest
// earlier query that accepted it) is <= the current distance; accepting
// steals i2 from its previous owner. Every query's outcome is a function of
// the earlier outcomes: a triangular system whose unique fixed point is the
// sequential result.
//
// Here one LANE serves one query in every phase (lane-per-query keeps the
// per-candidate work at a few scalar-like VALU ops and needs no cross-lane
// reductions):
//   0. counting sort of F2's octave-0 keypoints by grid cell (stable: index
//      order inside a cell), positions / indices / descriptors to LDS in
//      sorted order, so a window column is one contiguous run;
//   1. per query: candidate count (window test on positions);
//   2. per query: candidate list (index, distance) in reference order;
//   3. Jacobi rounds: every query recomputes its top-2 from the previous
//      round's accepted outcomes, honouring only claims of earlier queries
//      (per-i2 claim lists); a round without change is the fixed point. Past
//      kInitMaxRounds one lane runs the sequential greedy instead;
//   4. the latest acceptor keeps each i2, rotation consistency, outputs.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "orbx_device.cuh"
#include "orbx_wave.cuh"

namespace orbx {

constexpr int kInitGridCols = 64, kInitGridRows = 48;  // FRAME_GRID_COLS / ROWS include/Frame.h:37-38
constexpr int kInitCells = kInitGridCols * kInitGridRows;
constexpr int kInitHisto = 30;  // HISTO_LENGTH
constexpr int kInitThLow = 50;  // TH_LOW
constexpr int kInitMaxRounds = 48;
constexpr int kD0Stride = 9;
#ifndef ORBX_INIT_ROUND_LANES
#define ORBX_INIT_ROUND_LANES 4
#endif
constexpr int kRoundLanes = ORBX_INIT_ROUND_LANES;  // lanes per query in the Jacobi rounds
#ifndef ORBX_INIT_WIN_LANES
#define ORBX_INIT_WIN_LANES 4
#endif
constexpr int kWinLanes = ORBX_INIT_WIN_LANES;
constexpr uint32_t kInitVoid = 0xFFFFFFFFu;  // list slot of a window-cell keypoint outside the r-square  // lanes per query in the window count / list phases  // words per staged F2 descriptor: odd, so random rows spread over the LDS banks

#define LDSP __attribute__((address_space(3)))

size_t init_lds_fixed_bytes(int kp_pitch) {
  auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t K = (size_t)kp_pitch;
  return r16(4 * (kInitCells + 1)) + r16(4 * K) /* cof / head / md */ + r16(8 * K) /* pos / nxt */ +
         r16(4 * K) /* idx / m21 */ + r16(4 * (K + 1)) /* coff */ + r16(4 * K) /* qlist / res */ +
         r16(4 * K) /* src */ + r16(4 * K) /* queue */ + 3 * r16(128);
}

// Frame::PosInGrid: round() of a float, half away from zero
__device__ __forceinline__ bool init_pos_in_grid(float x, float y, const InitParams& P, int* c) {
  const int px = (int)roundf(__fmul_rn(__fsub_rn(x, P.minX), P.invW));
  const int py = (int)roundf(__fmul_rn(__fsub_rn(y, P.minY), P.invH));
  *c = px * kInitGridRows + py;
  return !(px < 0 || px >= kInitGridCols || py < 0 || py >= kInitGridRows);
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

__device__ __forceinline__ int init_hamming(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// DPP helpers over groups of G lanes (1, 2, 4, 8 or 16) inside a 16-lane row;
// every lane of a group must be active
template <int G>
__device__ __forceinline__ int group_incl_scan(int v) {
  if (G == 1) return v;
  const int lg = threadIdx.x & (G - 1);
  int t = dpp_i<kDppShr1>(0, v);
  v += lg >= 1 ? t : 0;
  if (G == 2) return v;
  t = dpp_i<kDppShr2>(0, v);
  v += lg >= 2 ? t : 0;
  if (G > 4) {
    t = dpp_i<kDppShr4>(0, v);
    v += lg >= 4 ? t : 0;
  }
  if (G > 8) {
    t = dpp_i<kDppShr8>(0, v);
    v += lg >= 8 ? t : 0;
  }
  return v;
}
template <int G>
__device__ __forceinline__ int group_sum(int v) {
  if (G == 1) return v;
  v += dpp_i<kDppQuad1032>(0, v);
  if (G == 2) return v;
  v += dpp_i<kDppQuad2301>(0, v);
  if (G > 4) v += dpp_i<kDppHalfMirror>(0, v);
  if (G > 8) v += dpp_i<kDppMirror>(0, v);
  return v;
}
// (k1, k2) = the two smallest keys of the row
template <int CTRL>
__device__ __forceinline__ void row_top2_step(uint32_t& k1, uint32_t& k2) {
  const uint32_t o1 = (uint32_t)dpp_i<CTRL>(0, (int)k1), o2 = (uint32_t)dpp_i<CTRL>(0, (int)k2);
  k2 = min(min(max(k1, o1), k2), o2);
  k1 = min(k1, o1);
}
template <int G = 16>
__device__ __forceinline__ void row_top2(uint32_t& k1, uint32_t& k2) {
  if (G == 1) return;
  row_top2_step<kDppQuad1032>(k1, k2);
  if (G == 2) return;
  row_top2_step<kDppQuad2301>(k1, k2);
  if (G > 4) row_top2_step<kDppHalfMirror>(k1, k2);
  if (G > 8) row_top2_step<kDppMirror>(k1, k2);
}

// vMatchedDistance[i2] at i1's turn: the smallest distance of an earlier
// query's claim on i2 in the snapshot (INT_MAX if none)
__device__ __forceinline__ int init_claim_md(const LDSP int* head, const LDSP int* nxt, int i2, int i1) {
  int md = INT_MAX;
  for (int hd = head[i2]; hd >= 0;) {
    const int x = nxt[hd];
    if (hd < i1) md = min(md, x & 511);
    hd = (x >> 9) - 1;
  }
  return md;
}

struct InitShared {
  LDSP int* cell;     // [kInitCells + 1] first sorted position of each cell
  LDSP int* cof;      // [K] cell of each F2 keypoint (sort), then head[i2] (rounds), md[i2] (fallback)
  LDSP float* pos;    // [2K] sorted positions x, y (phases 1-2), then nxt[i1] (rounds)
  LDSP int* idx;      // [K] sorted position -> i2 (phases 0-2), then m21[i2] (fallback)
  LDSP int* coff;     // [K + 1] candidate offsets per i1
  LDSP int* qlist;    // [K] octave-0 queries (phases 1-2), then res[i1] / vnMatches12
  LDSP int* src;      // [K] i2 accepted by i1 (rotHist entries), -1
  LDSP int* queue;    // [K] queries with candidates
  LDSP float* src_f;    // src viewed as query window x (phases 1-2)
  LDSP float* queue_f;  // queue viewed as query window y (phases 1-2)
  LDSP int* var;      // [32]
  LDSP int* hist;     // [32]
  LDSP int* tmp;      // [32]
  LDSP uint32_t* d0;  // [kD0Stride n0] sorted descriptors (when they fit)
  LDSP uint32_t* cand;  // candidate entries in LDS
};

__device__ __forceinline__ int lds_atomic_add(LDSP int* p, int v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Exclusive scan of a[0..n) in LDS (NT threads); returns the total.
template <int NT>
__device__ int init_scan(LDSP int* a, int n, LDSP int* s_tmp) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = (n + NT - 1) / NT;
  const int b = min(tid * per, n), e = min(b + per, n);
  int sum = 0;
  for (int i = b; i < e; ++i) sum += a[i];
  const int x = wave_incl_scan_dpp(sum);
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
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
  __syncthreads();
  return total;
}

// Phases 2-4 with the candidate list in one memory space (LDS or global), so
// each instantiation addresses a single known space.
__device__ __forceinline__ void init_stamp(const InitParams& P, int k) {
  if (P.prof && threadIdx.x == 0) P.prof[blockIdx.x * 16 + k] = (long long)__builtin_amdgcn_s_memtime();
}

template <typename CandPtr, bool DESC_LDS>
__device__ void init_solve(const InitParams& P, const InitShared& S, CandPtr cand, const orbx_kp* __restrict__ kp1,
                           const uint8_t* __restrict__ desc1, const uint8_t* __restrict__ desc2,
                           const float* __restrict__ prev, int n1, int n2, int nq0, int total) {
  const int tid = threadIdx.x;
  // ---- phase 2a: candidate lists in reference order: a 16-lane row per
  // query, a lane per window column; column c's entries follow the entries of
  // columns < c (row prefix sum), each (query slot << 16 | sorted position)
  for (int g = tid / kWinLanes; g < nq0; g += kInitThreads / kWinLanes) {
    const int l16 = tid & (kWinLanes - 1);
    const int i1 = S.qlist[g];
    const int off = S.coff[i1];
    if (off == S.coff[i1 + 1]) continue;  // group-uniform
    const float x = S.src_f[g], y = S.queue_f[g];
    int cx0, cx1, cy0, cy1;
    init_window(x, y, P, cx0, cx1, cy0, cy1);
    const int ncol = cx1 - cx0 + 1;
    int base = off;
    for (int c0 = 0; c0 < ncol; c0 += kWinLanes) {
      const int ci = c0 + l16;
      int pb = 0, pe = 0;
      if (ci < ncol) {
        const int ix = cx0 + ci;
        pb = S.cell[ix * kInitGridRows + cy0];
        pe = S.cell[ix * kInitGridRows + cy1 + 1];
      }
      const int own = pe - pb;
      int o = base + group_incl_scan<kWinLanes>(own) - own;
      // one slot per keypoint of the column's cells; those outside the
      // |dx|, |dy| < r square stay in the list as kInitVoid (skipped by every
      // later pass), so the list keeps the reference's candidate order
      for (int p = pb; p < pe; ++p) {
        const float qx = S.pos[2 * p], qy = S.pos[2 * p + 1];
        cand[o++] = fabsf(__fsub_rn(qx, x)) < P.r && fabsf(__fsub_rn(qy, y)) < P.r
                        ? ((uint32_t)g << 16) | (uint32_t)p
                        : kInitVoid;
      }
      base += group_sum<kWinLanes>(own);
    }
  }
  __syncthreads();
  init_stamp(P, 4);
  // the queries' descriptors to LDS (in the position array, free from here on)
  const bool qd_lds = nq0 * 8 <= 2 * P.kp_pitch;
  LDSP uint32_t* qd = (LDSP uint32_t*)S.pos;
  if (qd_lds) {
    for (int t = tid; t < 2 * nq0; t += kInitThreads) {
      const uint4 v = ((const uint4*)(desc1 + (size_t)S.qlist[t >> 1] * 32))[t & 1];
      LDSP uint32_t* w = qd + 4 * t;
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    }
    __syncthreads();
  }
  // ---- phase 2b: every candidate's Hamming distance, candidate-parallel;
  // the entry becomes (i2 | distance << 23)
  for (int c = tid; c < total; c += kInitThreads) {
    const uint32_t e = cand[c];
    if (e == kInitVoid) continue;
    const int g = (int)(e >> 16), p = (int)(e & 0xFFFF);
    uint4 a0, a1;
    if (qd_lds) {
      const LDSP uint32_t* w = qd + 8 * g;
      a0 = make_uint4(w[0], w[1], w[2], w[3]);
      a1 = make_uint4(w[4], w[5], w[6], w[7]);
    } else {
      const uint4* dq = (const uint4*)(desc1 + (size_t)S.qlist[g] * 32);
      a0 = dq[0];
      a1 = dq[1];
    }
    const int i2 = S.idx[p];
    uint4 b0, b1;
    if (DESC_LDS) {
      const LDSP uint32_t* w = S.d0 + kD0Stride * p;
      b0 = make_uint4(w[0], w[1], w[2], w[3]);
      b1 = make_uint4(w[4], w[5], w[6], w[7]);
    } else {
      const uint4* d2 = (const uint4*)(desc2 + (size_t)i2 * 32);
      b0 = d2[0];
      b1 = d2[1];
    }
    cand[c] = (uint32_t)i2 | ((uint32_t)init_hamming(a0, a1, b0, b1) << 23);
  }
  __syncthreads();
  init_stamp(P, 5);
  if (P.stop == 3) return;

  // ---- phase 3: Jacobi rounds over the queue of queries with candidates
  LDSP int* res = S.qlist;          // per i1: -1, or bestIdx2 << 9 | bestDist
  LDSP int* head = S.cof;           // per i2: latest claiming i1 of the snapshot, or -1
  LDSP int* nxt = (LDSP int*)S.pos;  // per i1: (next claimer + 1) << 9 | its distance
  for (int i = tid; i < n1; i += kInitThreads) res[i] = -1;
  for (int i = tid; i < n2; i += kInitThreads) head[i] = -1;
  if (tid == 0) {
    S.var[0] = 0;  // nmatches
    S.var[6] = 1;  // changed
    S.var[7] = 0;  // queue length
  }
  __syncthreads();
  for (int i = tid; i < n1; i += kInitThreads)
    if (S.coff[i + 1] > S.coff[i]) S.queue[lds_atomic_add(&S.var[7], 1)] = i;
  __syncthreads();
  const int nq = S.var[7];
  init_stamp(P, 6);
  bool converged = false;
  for (int round = 0; round < kInitMaxRounds; ++round) {
    if (S.var[6] == 0) {
      converged = true;
      if (P.prof && tid == 0) P.prof[blockIdx.x * 16 + 11] = round;
      break;
    }
    __syncthreads();
    if (tid == 0) S.var[6] = 0;
    __syncthreads();
    int changed = 0;
    {
      // a 16-lane row per query: lane l scans candidates c0 + l, c0 + l + 16, ...
      // keeping the two smallest (distance << 22 | position) keys; the row merge
      // gives the sequential scan's best (earliest on equal distances) and second
      // kRoundLanes lanes per query (a DPP row holds 16 / kRoundLanes queries)
      for (int g = tid / kRoundLanes; g < nq; g += kInitThreads / kRoundLanes) {
        const int l16 = tid & (kRoundLanes - 1);
        const int i1 = S.queue[g];
        const int c0 = S.coff[i1], c1 = S.coff[i1 + 1];
        uint32_t k1 = 0xFFFFFFFFu, k2 = 0xFFFFFFFFu;
        for (int c = c0 + l16; c < c1; c += kRoundLanes) {
          const uint32_t e = cand[c];
          if (e == kInitVoid) continue;
          const int i2 = (int)(e & 0x7FFFFF), dist = (int)(e >> 23);
          if (init_claim_md(head, nxt, i2, i1) <= dist) continue;  // (:444-445)
          const uint32_t key = ((uint32_t)dist << 22) | (uint32_t)(c - c0);
          k2 = min(k2, max(k1, key));
          k1 = min(k1, key);
        }
        row_top2<kRoundLanes>(k1, k2);
        const int best = k1 == 0xFFFFFFFFu ? INT_MAX : (int)(k1 >> 22);
        const int best2 = k2 == 0xFFFFFFFFu ? INT_MAX : (int)(k2 >> 22);
        const bool ok = best <= kInitThLow && (float)best < __fmul_rn((float)best2, P.nnratio);
        if (l16 == 0) {
          const int r = ok ? ((int)(cand[c0 + (k1 & 0x3FFFFF)] & 0x7FFFFF) << 9 | best) : -1;
          if (res[i1] != r) {
            res[i1] = r;
            changed = 1;
          }
        }
      }
    }
    if (changed) S.var[6] = 1;
    __syncthreads();
    const long long t_snap = P.prof ? (long long)__builtin_amdgcn_s_memtime() : 0;
    // snapshot of this round's outcomes as per-i2 claim lists
    for (int i = tid; i < n2; i += kInitThreads) head[i] = -1;
    __syncthreads();
    for (int qq = tid; qq < nq; qq += kInitThreads) {
      const int i1 = S.queue[qq];
      const int r = res[i1];
      if (r >= 0)
        nxt[i1] = ((__hip_atomic_exchange(&head[r >> 9], i1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) + 1)
                   << 9) |
                  (r & 511);
    }
    __syncthreads();
    if (P.prof && tid == 0) P.prof[blockIdx.x * 16 + 9] += (long long)__builtin_amdgcn_s_memtime() - t_snap;
  }
  init_stamp(P, 7);
  if (P.prof && tid == 0) P.prof[blockIdx.x * 16 + 12] = converged ? 1 : 0;
  if (converged) {
    // the latest accepting query keeps each i2 (earlier ones were stolen
    // from, :463-467); every accepted query entered rotHist (:469-470)
    for (int i = tid; i < n2; i += kInitThreads) head[i] = -1;
    __syncthreads();
    for (int qq = tid; qq < nq; qq += kInitThreads) {
      const int i1 = S.queue[qq];
      const int r = res[i1];
      if (r >= 0) __hip_atomic_fetch_max(&head[r >> 9], i1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    int kept = 0;
    for (int i = tid; i < n1; i += kInitThreads) {
      const int r = res[i];
      const int b = r >= 0 ? (r >> 9) : -1;
      const bool keep = r >= 0 && head[b] == i;
      S.src[i] = b;
      res[i] = keep ? b : -1;  // res becomes vnMatches12
      kept += keep ? 1 : 0;
    }
    kept = wave_sum_dpp(kept);
    if ((tid & 63) == 0 && kept) lds_atomic_add(&S.var[0], kept);
    __syncthreads();
    return;
  }
  // ---- sequential greedy in i1 order (one lane; pathological chains only)
  LDSP int* md = S.cof;
  LDSP int* m21 = S.idx;
  LDSP int* m12 = res;
  for (int i = tid; i < n2; i += kInitThreads) {
    md[i] = INT_MAX;
    m21[i] = -1;
  }
  for (int i = tid; i < n1; i += kInitThreads) {
    m12[i] = -1;
    S.src[i] = -1;
  }
  __syncthreads();
  if (tid == 0) {
    int nm = 0;
    for (int i1 = 0; i1 < n1; ++i1) {
      const int c1 = S.coff[i1 + 1];
      int best = INT_MAX, best2 = INT_MAX, bidx = -1;
      for (int c = S.coff[i1]; c < c1; ++c) {
        const uint32_t e = cand[c];
        if (e == kInitVoid) continue;
        const int i2 = (int)(e & 0x7FFFFF), dist = (int)(e >> 23);
        if (md[i2] <= dist) continue;
        if (dist < best) {
          best2 = best;
          best = dist;
          bidx = i2;
        } else if (dist < best2) {
          best2 = dist;
        }
      }
      if (best <= kInitThLow && (float)best < __fmul_rn((float)best2, P.nnratio)) {
        if (m21[bidx] >= 0) {  // steal (:463-467)
          m12[m21[bidx]] = -1;
          nm--;
        }
        m12[i1] = bidx;
        m21[bidx] = i1;
        md[bidx] = best;
        nm++;
        S.src[i1] = bidx;
      }
    }
    S.var[0] = nm;
  }
  __syncthreads();
}

// Rotation consistency (src/ORBmatcher.cc:473-512, ComputeThreeMaxima
// :1601-1642) and the outputs: vnMatches12 and the vbPrevMatched update
// (:515-517). src[i1] = the i2 every accepting query entered into rotHist
// (-1 if none), m12 = vnMatches12 after the steals, var[0] = the match count;
// hist[0..30) zeroed.
template <int NT>
__device__ void init_finish(const InitParams& P, LDSP int* src, LDSP int* m12, LDSP int* hist, LDSP int* var,
                            const orbx_kp* __restrict__ kp1, const orbx_kp* __restrict__ kp2, int n1, float* prev,
                            int* m12_out, int* nmatches_out) {
  const int tid = threadIdx.x;
  const float factor = 1.0f / kInitHisto;
  if (P.check_ori) {
    for (int i = tid; i < n1; i += NT) {
      const int j = src[i];
      int bin = -1;
      if (j >= 0) {
        float rot = __fsub_rn(kp1[i].angle, kp2[j].angle);
        if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
        bin = (int)roundf(__fmul_rn(rot, factor));
        if (bin == kInitHisto) bin = 0;
        lds_atomic_add(&hist[bin], 1);
      }
      src[i] = bin;
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
    for (int i = tid; i < n1; i += NT) {
      const int b = src[i];
      if (b < 0 || b == ind1 || b == ind2 || b == ind3) continue;
      if (m12[i] >= 0) {
        m12[i] = -1;
        ++rej;
      }
    }
    rej = wave_sum_dpp(rej);
    if ((tid & 63) == 0 && rej) lds_atomic_add(&var[0], -rej);
    __syncthreads();
  }
  for (int i = tid; i < n1; i += NT) {
    const int j = m12[i];
    m12_out[i] = j;
    if (prev && j >= 0) {
      prev[2 * i] = kp2[j].x;
      prev[2 * i + 1] = kp2[j].y;
    }
  }
  if (tid == 0) *nmatches_out = var[0];
}

// Frame::AssignFeaturesToGrid for F2's octave-0 keypoints (the only ones
// GetFeaturesInArea(.., 0, 0) returns), as a counting sort by cell, stable in
// index order: cell[c] = first sorted position of cell c (column-major cells,
// so a window column is one run), pos / idx in sorted order. slot / members
// are scratch of n2 entries. Returns n0; no trailing barrier.
template <int NT>
__device__ int init_build_grid(const InitParams& P, const orbx_kp* __restrict__ kp2, int n2, LDSP int* cell,
                               LDSP int* cof, LDSP float* pos, LDSP int* idx, LDSP int* slot, LDSP int* members,
                               LDSP int* tmp) {
  const int tid = threadIdx.x;
  for (int c = tid; c <= kInitCells; c += NT) cell[c] = 0;
  __syncthreads();
  for (int i = tid; i < n2; i += NT) {
    const orbx_kp k = kp2[i];
    int c = -1;
    if (!(k.octave == 0 && init_pos_in_grid(k.x, k.y, P, &c))) c = -1;
    cof[i] = c;
    if (c >= 0) slot[i] = lds_atomic_add(&cell[c], 1);
  }
  __syncthreads();
  const int n0 = init_scan<NT>(cell, kInitCells + 1, tmp);
  for (int i = tid; i < n2; i += NT) {
    const int c = cof[i];
    if (c >= 0) members[cell[c] + slot[i]] = i;
  }
  __syncthreads();
  // stable placement: rank inside the cell = members with a smaller index
  // (cells hold a handful of octave-0 keypoints)
  for (int i = tid; i < n2; i += NT) {
    const int c = cof[i];
    if (c < 0) continue;
    const int b = cell[c], e = cell[c + 1];
    int p = b;
    for (int q = b; q < e; ++q) p += members[q] < i ? 1 : 0;
    const orbx_kp k = kp2[i];
    pos[2 * p] = k.x;
    pos[2 * p + 1] = k.y;
    idx[p] = i;
  }
  return n0;
}

__global__ __launch_bounds__(kInitThreads) void search_init_kernel(
    InitParams P, const orbx_kp* __restrict__ kp1_all, const uint8_t* __restrict__ desc1_all,
    const int* __restrict__ n1_all, const orbx_kp* __restrict__ kp2_all, const uint8_t* __restrict__ desc2_all,
    const int* __restrict__ n2_all, float* __restrict__ prev_all, uint32_t* __restrict__ cand_all,
    int* __restrict__ matches_all, int* __restrict__ nmatches, int* err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int pr = blockIdx.x, tid = threadIdx.x;
  const int n1 = n1_all[pr], n2 = n2_all[pr], K = P.kp_pitch;
  const orbx_kp* kp1 = kp1_all + (size_t)pr * K;
  const orbx_kp* kp2 = kp2_all + (size_t)pr * K;
  const uint8_t* desc1 = desc1_all + (size_t)pr * K * 32;
  const uint8_t* desc2 = desc2_all + (size_t)pr * K * 32;
  // prev_all == nullptr: windows centred on F1's own keypoints (the initial
  // mvbPrevMatched of Tracking::MonocularInitialization, src/Tracking.cc:645-647)
  float* prev = prev_all ? prev_all + (size_t)pr * K * 2 : nullptr;
  int* m12_out = matches_all + (size_t)pr * K;

  LDSP unsigned char* sp = (LDSP unsigned char*)smem;
  auto take = [&](size_t bytes) {
    LDSP unsigned char* r = sp;
    sp += (bytes + 15) & ~(size_t)15;
    return r;
  };
  InitShared S;
  S.cell = (LDSP int*)take(4ull * (kInitCells + 1));
  S.cof = (LDSP int*)take(4ull * K);
  S.pos = (LDSP float*)take(8ull * K);
  S.idx = (LDSP int*)take(4ull * K);
  S.coff = (LDSP int*)take(4ull * (K + 1));
  S.qlist = (LDSP int*)take(4ull * K);
  S.src = (LDSP int*)take(4ull * K);
  S.queue = (LDSP int*)take(4ull * K);
  S.src_f = (LDSP float*)S.src;
  S.queue_f = (LDSP float*)S.queue;
  S.var = (LDSP int*)take(128);
  S.hist = (LDSP int*)take(128);
  S.tmp = (LDSP int*)take(128);
  LDSP uint32_t* tail = (LDSP uint32_t*)sp;  // P.cand_lds entries: descriptors, then candidates

  init_stamp(P, 0);
  if (tid < 32) {
    S.hist[tid] = 0;
    S.var[tid] = 0;
  }
  // F2's descriptors are staged after the list sizes are known (the tail goes
  // to the candidate lists first, then to the descriptors)
  const int n0 = init_build_grid<kInitThreads>(P, kp2, n2, S.cell, S.cof, S.pos, S.idx, S.src, S.queue, S.tmp);
  // F1's octave-0 queries, compacted in index order
  for (int i = tid; i <= n1; i += kInitThreads) S.coff[i] = 0;
  __syncthreads();
  init_stamp(P, 1);
  if (P.stop == 1) return;
  {
    const int lane = tid & 63;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int i0 = (tid >> 6) * 64; i0 < n1; i0 += kInitThreads) {
      const int i = i0 + lane;
      const bool z = i < n1 && kp1[i].octave == 0;
      const uint64_t mz = __ballot(z);
      int base = 0;
      if (lane == 0 && mz) base = lds_atomic_add(&S.var[5], __popcll(mz));
      base = __builtin_amdgcn_readlane(base, 0);
      if (z) S.qlist[base + __popcll(mz & lt)] = i;
    }
  }
  __syncthreads();
  const int nq0 = S.var[5];
  // window centres of the queries (vbPrevMatched, or the keypoints) to LDS
  LDSP float* qx = (LDSP float*)S.src;    // free until phase 3
  LDSP float* qy = (LDSP float*)S.queue;  // free until phase 3
  for (int g = tid; g < nq0; g += kInitThreads) {
    const int i1 = S.qlist[g];
    qx[g] = prev ? prev[2 * i1] : kp1[i1].x;
    qy[g] = prev ? prev[2 * i1 + 1] : kp1[i1].y;
  }
  __syncthreads();
  init_stamp(P, 2);
  // ---- phase 1: list slots per query = the keypoints of its window's cells
  // (Frame::GetFeaturesInArea(x, y, r, 0, 0) before the |dx|, |dy| < r test:
  // a column's cells are one run of sorted positions, so no position is read
  // here); kWinLanes lanes per query, a lane per window column
  for (int g = tid / kWinLanes; g < nq0; g += kInitThreads / kWinLanes) {
    const int l16 = tid & (kWinLanes - 1);
    const int i1 = S.qlist[g];
    const float x = qx[g], y = qy[g];
    int cx0, cx1, cy0, cy1, cnt = 0;
    const int ncol = init_window(x, y, P, cx0, cx1, cy0, cy1) ? cx1 - cx0 + 1 : 0;
    for (int ci = l16; ci < ncol; ci += kWinLanes) {
      const int ix = cx0 + ci;
      cnt += S.cell[ix * kInitGridRows + cy1 + 1] - S.cell[ix * kInitGridRows + cy0];
    }
    cnt = group_sum<kWinLanes>(cnt);
    if (l16 == 0) S.coff[i1] = cnt;
  }
  __syncthreads();
  const int total = init_scan<kInitThreads>(S.coff, n1 + 1, S.tmp);
  init_stamp(P, 3);
  if (P.prof && tid == 0) P.prof[blockIdx.x * 16 + 13] = total;
  if (P.stop == 2) return;
  if (total > P.cand_lds && total > P.cand_cap) {
    // overflow is reported (status bit 8, the largest list total in err[1]),
    // never truncated: the pair gets no matches rather than stale outputs of
    // an earlier call; the host entry point grows its workspace and re-runs
    for (int i = tid; i < min(n1, K); i += kInitThreads) m12_out[i] = -1;
    if (tid == 0) {
      atomicOr(err, 8);
      atomicMax(err + 1, total);
      nmatches[pr] = 0;
    }
    return;
  }
  // tail layout: [candidate lists (if they fit) | F2 descriptors (if they fit)]
  const bool cand_in_lds = total <= P.cand_lds;
  const int d0_at = cand_in_lds ? ((total + 15) & ~15) : 0;
  const bool d0_lds = d0_at + kD0Stride * n0 <= P.cand_lds;
  S.cand = tail;
  S.d0 = tail + d0_at;
  if (d0_lds) {
    for (int t = tid; t < 2 * n0; t += kInitThreads) {
      const int p = t >> 1, h = t & 1;
      const uint4 u = ((const uint4*)(desc2 + (size_t)S.idx[p] * 32))[h];
      LDSP uint32_t* w = S.d0 + kD0Stride * p + 4 * h;
      w[0] = u.x; w[1] = u.y; w[2] = u.z; w[3] = u.w;
    }
  }
  if (cand_in_lds) {
    if (d0_lds)
      init_solve<LDSP uint32_t*, true>(P, S, S.cand, kp1, desc1, desc2, prev, n1, n2, nq0, total);
    else
      init_solve<LDSP uint32_t*, false>(P, S, S.cand, kp1, desc1, desc2, prev, n1, n2, nq0, total);
  } else {
    uint32_t* c = cand_all + (size_t)pr * P.cand_cap;
    if (d0_lds)
      init_solve<uint32_t*, true>(P, S, c, kp1, desc1, desc2, prev, n1, n2, nq0, total);
    else
      init_solve<uint32_t*, false>(P, S, c, kp1, desc1, desc2, prev, n1, n2, nq0, total);
  }
  if (P.stop == 3) return;
  init_finish<kInitThreads>(P, S.src, S.qlist, S.hist, S.var, kp1, kp2, n1, prev, m12_out, nmatches + pr);
  init_stamp(P, 8);
}

int launch_search_init(const InitParams& P0, const orbx_kp* kp1, const uint8_t* desc1, const int* n1,
                       const orbx_kp* kp2, const uint8_t* desc2, const int* n2, float* prev, uint32_t* cand,
                       int* matches12, int* nmatches, int* err, int pairs, void* stream) {
  InitParams P = P0;
  const size_t fixed = init_lds_fixed_bytes(P.kp_pitch);
  // query slots and sorted positions are 16-bit fields of the candidate entries;
  // the per-keypoint tables must leave LDS room for candidates
  if (P.kp_pitch > 65535 || fixed + 4096 > kInitLdsBudget) return ORBX_ECAPACITY;
  // LDS request: the whole CU by default; ORBX_INIT_LDS_KB caps it (candidates and
  // F2's descriptors then spill to global memory) so a workgroup can start on a CU
  // that extraction workgroups still partly occupy
  static const int cap_kb = getenv("ORBX_INIT_LDS_KB") ? atoi(getenv("ORBX_INIT_LDS_KB")) : 0;
  const size_t budget = cap_kb > 0 ? std::min(kInitLdsBudget, std::max(fixed + 64, (size_t)cap_kb * 1024)) : kInitLdsBudget;
  P.cand_lds = (int)((budget - fixed) / 4) & ~15;
  if (raise_lds_limit((const void*)search_init_kernel, kInitLdsBudget)) return ORBX_EDEVICE;
  const size_t lds = fixed + (size_t)P.cand_lds * 4;
  hipLaunchKernelGGL(search_init_kernel, dim3(pairs), dim3(kInitThreads), lds, (hipStream_t)stream, P, kp1, desc1, n1,
                     kp2, desc2, n2, prev, cand, matches12, nmatches, err);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
