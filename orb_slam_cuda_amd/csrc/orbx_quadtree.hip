// orbx_quadtree.hip — DistributeOctTree (src/ORBextractor.cc:889-1120).
//
// The reference keeps the quadtree as a std::list<ExtractorNode>: nIni root
// columns; then rounds that split every multi-key node in list order,
// pushing the non-empty children n1..n4 to the FRONT of the list and erasing
// the parent, until the list holds >= N nodes or a round changes nothing;
// once the next full round would overshoot N it switches to splitting the
// previous round's children in (size, heap-address) descending order, again
// stopping as soon as the list reaches N. Each node finally keeps its
// max-response key (first in key order on ties).
//
// Data-parallel restatement (one workgroup per frame x level): the list is a
// node table indexed by list position. A round is "split a prefix of the
// candidate sequence": candidates = nodes with > 1 key, taken in list order
// (breadth rounds) or sorted by (size desc, creation desc) (sorted rounds;
// creation order stands in for the reference's heap-pointer tie-break, the
// same rule the oracle uses); the prefix ends where the running list size
// reaches N. The new list is [children of the split nodes, last split first,
// each as n4 n3 n2 n1] followed by the untouched nodes in their old order,
// which is exactly what the reference's push_front/erase sequence produces.
//
// Sorted-key path (qt_sorted_path, the default): a node's box never depends
// on the data — the roots are nIni columns of width hX (:894-914), a child is
// a half of its parent by DivideNode's ceil halves (:833-834) — so the
// quadrant a key falls in at every depth is a function of its coordinates
// alone. The plan tabulates that path per column and per row (x codes carry
// the root index), a key's code is xs[x] | ys[y], and keys counted into bins
// of their depth-Dh code prefix (Dh = 4..6, 4096 or 8192 bins) and scattered
// by the bins' prefix sum leave every node of depth <= Dh a contiguous range
// of the binned keys whose size and four child ranges are five prefix-sum
// reads. The rounds then move node records only: no key is re-homed, no
// child count is accumulated. One wave runs them without barriers (the rest
// of the workgroup joins for the sorted rounds' candidate ranking); the kept
// key of a node is the max over its range of (score, first original index).
// A node deeper than Dh that must be split, or a level with more keys than
// the workgroup holds in registers, falls back to the legacy rounds.
//
// Legacy path (qt_legacy): keys never move, each key carries its node index;
// lean rounds (node tables that fit 16-bit packing, < 65536 keys) and generic
// rounds (ORBX_QT_GENERIC=1 forces them for tests). DESIGN.md section 6 has
// the barrier counts and timings of both.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orbx_device.cuh"

namespace orbx {

// the first bytes of the quadtree's LDS hold the sorted path's round state;
// the legacy layout starts after them, so a fallback never overwrites what a
// slower wave is still reading
constexpr int kQtHeader = 256;
constexpr int kQtKpt = 8;  // sorted path: keys per thread (kept in registers from the gather to the scatter)
constexpr int kQtBig = 128;  // sorted rounds: candidates of size >= 64 ranked among themselves up to this many

struct QNode {
  int16_t x0, y0, x1, y1;
};

__device__ __forceinline__ void halves(const QNode& nd, int* mx, int* my) {
  // DivideNode: halfX = ceil((UR.x-UL.x)/2) in float (src/ORBextractor.cc:833-834)
  *mx = nd.x0 + (int)ceilf(__fdiv_rn((float)(nd.x1 - nd.x0), 2.f));
  *my = nd.y0 + (int)ceilf(__fdiv_rn((float)(nd.y1 - nd.y0), 2.f));
}

__device__ __forceinline__ int quadrant(const QNode& nd, int kx, int ky) {
  int mx, my;
  halves(nd, &mx, &my);
  return (kx >= mx ? 1 : 0) + (ky >= my ? 2 : 0);  // 0=n1 1=n2 2=n3 3=n4
}

__device__ __forceinline__ QNode child_box(const QNode& nd, int q) {
  int mx, my;
  halves(nd, &mx, &my);
  QNode c;
  c.x0 = (q & 1) ? mx : nd.x0;
  c.x1 = (q & 1) ? nd.x1 : mx;
  c.y0 = (q & 2) ? my : nd.y0;
  c.y1 = (q & 2) ? nd.y1 : my;
  return c;
}

__device__ __forceinline__ int nonempty(int4 c) { return (c.x > 0) + (c.y > 0) + (c.z > 0) + (c.w > 0); }

#ifndef ORBX_QT_MINW
#define ORBX_QT_MINW 1
#endif

// ---------------------------------------------------------------- sorted-key path
//
// Node record (int2): x = b | e << 16 (its range of binned keys), y = prefix
// | depth << 13 | creation << 16 (prefix: root index and depth quadrant
// digits, R + 2 depth <= 13 bits). A node's four child ranges are read from
// the bins' prefix sum when a round needs them (children of a node at depth
// Dh are not tabulated: such a node with > 1 key sends the level to the
// legacy rounds before any round would read them).
namespace qts {
__device__ __forceinline__ int rb(int2 r) { return r.x & 0xFFFF; }
__device__ __forceinline__ int re(int2 r) { return (int)((uint32_t)r.x >> 16); }
__device__ __forceinline__ int rcnt(int2 r) { return re(r) - rb(r); }
__device__ __forceinline__ int rpre(int2 r) { return r.y & 0x1FFF; }
__device__ __forceinline__ int rdepth(int2 r) { return (r.y >> 13) & 7; }
__device__ __forceinline__ int rseq(int2 r) { return (int)((uint32_t)r.y >> 16); }
__device__ __forceinline__ int2 mkrec(int b, int e, int pre, int d, int seq) {
  return make_int2(b | (e << 16), pre | (d << 13) | (seq << 16));
}
// compiler-level ordering of one wave's LDS accesses: a wave's LDS
// operations execute in order, so lanes of one wave exchange data through LDS
// without a barrier as long as the compiler keeps program order
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ int wave_max_dpp(int v) { return INT_MAX - wave_min_dpp(INT_MAX - v); }
enum { V_TRANK = 10, V_BIG = 12 };  // header ints: PROF ranking clocks, large-size candidate counts (two)
enum { ST_DONE = 2, ST_FALLBACK = 3 };
}  // namespace qts

template <int NT>
struct QtSortedLds {
  int* coff;
  uint32_t *xs, *S32, *bkey;
  uint16_t* bidx;  // the keys' cells after the count scan; in register mode the binned keys' original indices
  int* nodeof;     // spill mode, after the gather: per bin the kept node that holds it (aliases bidx)
  int2 *recA, *recB;
  int *rank, *spos;
  uint32_t* candk;
  int* candn;
  int* s_wave;
  int* part;     // block scans: two alternating buffers of 4 x 16 wave partials, then two of 16 wave maxima
  uint32_t* bm;  // sorted rounds: two alternating [64 sizes][bmw] bitmaps of candidate indices
  int* gw;       // ... per wave: candidates of size > s, s < 64
  uint32_t* bigk;  // ... keys of the candidates of size >= 64 (kQtBig)
  int bmw;       // words per bitmap row (maxnodes / 32)
  size_t fixed, bytes;
  // the key region last: register mode bidx + bkey (6 B per key, NT x kQtKpt
  // keys), spill mode bidx for qt_ownmax keys, then the bins' node map
  __host__ __device__ static size_t region(const ExtractParams& P) {
    const size_t a = 6ull * NT * kQtKpt, b = 2ull * P.qt_ownmax, c = 4ull * P.qt_nbmax;
    return a > b ? (a > c ? a : c) : (b > c ? b : c);
  }
  __host__ __device__ QtSortedLds(const ExtractParams& P, unsigned char* base) {
    unsigned char* p = base + kQtHeader;
    auto take = [&](size_t b) { unsigned char* r = p; p += (b + 15) & ~(size_t)15; return r; };
    const size_t MN = P.maxnodes;
    coff = (int*)take(4ull * (P.max_cells_level + 1));
    xs = (uint32_t*)take(4ull * P.qt_tabmax);
    S32 = (uint32_t*)take(4ull * (P.qt_nbmax / 2 + 1));
    recA = (int2*)take(8 * MN);
    recB = (int2*)take(8 * MN);
    rank = (int*)take(4 * MN);
    spos = (int*)take(4 * MN);
    candk = (uint32_t*)take(4 * MN);
    candn = (int*)take(4 * MN);
    s_wave = (int*)take(4 * 64);
    part = (int*)take(4 * (2 * 64 + 2 * 16));
    bmw = (int)((MN + 31) / 32);
    bm = (uint32_t*)take(4ull * 2 * 64 * bmw);
    gw = (int*)take(4ull * NT);
    bigk = (uint32_t*)take(4ull * kQtBig);
    fixed = (size_t)(p - base);
    unsigned char* kb = take(region(P));
    bidx = (uint16_t*)kb;
    bkey = (uint32_t*)(kb + 2ull * NT * kQtKpt);
    nodeof = (int*)kb;
    bytes = (size_t)(p - base);
  }
};

// The sorted-key DistributeOctTree of one (frame, level). Returns false,
// uniformly and before writing any output, when the level needs the legacy
// rounds (more keys than NT x kQtKpt, or a node deeper than Dh to split).
template <int NT, bool PROF>
__device__ __forceinline__ bool qt_sorted_path(const ExtractParams& P, const int* __restrict__ cell_counts,
                               const uint32_t* __restrict__ slots, const CellGeom* __restrict__ cells,
                               const uint32_t* __restrict__ qtab, uint32_t* __restrict__ qscratch,
                               uint32_t* __restrict__ qkeys, int* __restrict__ qcounts, int* __restrict__ qties,
                               int* err, int* dbg, unsigned char* smem, const unsigned long long t_begin) {
  using namespace qts;
  constexpr int NW = NT / 64;
  constexpr int kIt = 2;  // nodes (and candidate ranks) per thread: the plan keeps maxnodes <= 2 NT
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int l = blockIdx.x, f = blockIdx.y;
  const LevelGeom& g = P.lv[l];
  const int ncells = g.ncells, N = g.N, nIni = g.nIni;
  const int tw = g.qt_dims & 0xFFFF, th = (int)((uint32_t)g.qt_dims >> 16);
  const int shB = g.qt_bits & 0xFF, Dh = (g.qt_bits >> 8) & 0xFF, NB = 1 << ((g.qt_bits >> 16) & 0xFF);
  QtSortedLds<NT> M(P, smem);
  int* s_var = (int*)smem;
  const uint32_t* ys = M.xs + tw;
  const uint16_t* S = (const uint16_t*)M.S32;
  unsigned long long t_scan = 0, t_own = 0, t_gather = 0, t_bins = 0, t_scatter = 0, t_rounds = 0;

  // ---- cell counts and the level's code tables (loads in flight
  // together); bins cleared. A thread takes the cells [cb, ce) (one at KITTI
  // sizes). (Touching each cell's first slot lines here, so that the gather
  // would hit L2, was measured: the untargeted lines cost more bandwidth than
  // the gather's round trip)
  const int stride = g.slot_stride;
  const uint32_t* fslots = slots + (long long)f * P.slots_per_frame + g.slot0;
  const int cper = (ncells + NT - 1) / NT, cb = min(tid * cper, ncells), ce = min(cb + cper, ncells);
  {
    const int* cntp = cell_counts + (long long)f * P.ncells_total + g.cell0;
    const uint32_t* tab = qtab + g.qt_tab;
    const int nt = tw + th;
    for (int c = cb; c < ce; ++c) M.coff[c] = cntp[c];
    for (int i0 = 0; i0 < nt; i0 += 4 * NT) {
      uint32_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i0 + u * NT + tid < nt ? tab[i0 + u * NT + tid] : 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + u * NT + tid < nt) M.xs[i0 + u * NT + tid] = v[u];
    }
    for (int i = tid; i <= NB / 2; i += NT) M.S32[i] = 0u;
    for (int i = tid; i < 2 * 64 * M.bmw; i += NT) M.bm[i] = 0u;
    if (tid < 4) s_var[V_TRANK + tid] = 0;  // V_TRANK, -, V_BIG (two)
  }
  // ---- exclusive scan of the counts; the scan's write-back also lists each
  // key's cell (cells row-major, FAST order inside: the reference's key order)
  int K;
  {
    int sum = 0;
    for (int c = cb; c < ce; ++c) sum += M.coff[c];
    const int x = wave_incl_scan_dpp(sum);
    if (lane == 63) M.s_wave[wv] = x;
    lds_sync();
    int run = x - sum;
    K = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int v = M.s_wave[i];
      if (i < wv) run += v;
      K += v;
    }
    if (K <= P.qt_ownmax)
      for (int c = cb; c < ce; ++c) {
        const int n = M.coff[c];
        M.coff[c] = run;
        for (int i = 0; i < n; ++i) M.bidx[run + i] = (uint16_t)c;
        run += n;
      }
  }
  if (PROF) t_scan = __builtin_amdgcn_s_memtime();
  if (K > P.qt_ownmax) return false;  // uniform: every thread holds K
  // register mode: a thread's keys stay in registers from the gather to the
  // scatter; spill mode (more keys): the keys go to a compact global copy
  // (this level's slot range of qscratch), the bins are counted but not
  // scattered, and each key finds its kept node through a per-bin node map
  const bool spill = K > NT * kQtKpt;
  uint32_t* cs = qscratch + (long long)f * P.slots_per_frame + g.slot0;
  lds_sync();
  if (PROF) t_own = __builtin_amdgcn_s_memtime();

  // ---- gather (one memory round trip for all keys), code, bin, rank in bin.
  // Branch-free: keys past K read key K - 1's slot and are dropped later.
  uint32_t kv[kQtKpt];
  int kb[kQtKpt], kr[kQtKpt];
  if (spill) {
    for (int k0 = 0; k0 < K; k0 += 4 * NT) {
      uint32_t kk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kc = min(k0 + u * NT + tid, K - 1), c = M.bidx[kc];
        kk[u] = fslots[c * stride + kc - M.coff[c]];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u * NT + tid;
        if (k < K) {
          const int bn = (int)((M.xs[min(key_x(kk[u]), tw - 1)] | ys[min(key_y(kk[u]), th - 1)]) >> shB);
          atomicAdd(&M.S32[bn >> 1], 1u << ((bn & 1) << 4));
          cs[k] = kk[u];
        }
      }
    }
  } else if (K > 0) {
    int sl[kQtKpt];
#pragma unroll
    for (int u = 0; u < kQtKpt; ++u) {
      if (u * NT >= K) break;  // wave-uniform
      const int k = min(tid + u * NT, K - 1), c = M.bidx[k];
      sl[u] = c * stride + k - M.coff[c];
    }
#pragma unroll
    for (int u = 0; u < kQtKpt; ++u) {
      if (u * NT >= K) break;
      kv[u] = fslots[sl[u]];
    }
#pragma unroll
    for (int u = 0; u < kQtKpt; ++u) {
      if (u * NT >= K) break;
      kb[u] = (int)((M.xs[min(key_x(kv[u]), tw - 1)] | ys[min(key_y(kv[u]), th - 1)]) >> shB);
    }
#pragma unroll
    for (int u = 0; u < kQtKpt; ++u) {
      if (u * NT >= K) break;
      kr[u] = 0;
      if (tid + u * NT < K) {
        const uint32_t sh = (uint32_t)(kb[u] & 1) << 4;
        kr[u] = (int)((atomicAdd(&M.S32[kb[u] >> 1], 1u << sh) >> sh) & 0xFFFFu);
      }
    }
  }
  lds_sync();
  if (PROF) t_gather = __builtin_amdgcn_s_memtime();

  // ---- exclusive prefix sum of the bins (u16 pairs, in place); S[NB] = K
  {
    const int per = (NB >> 1) / NT;  // 2 .. 8 (the plan keeps NB >= 2 NT)
    uint32_t w[8];
    int sum = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < per) {
        w[i] = M.S32[tid * per + i];
        sum += (int)(w[i] & 0xFFFFu) + (int)(w[i] >> 16);
      }
    const int x = wave_incl_scan_dpp(sum);
    if (lane == 63) M.s_wave[16 + wv] = x;
    lds_sync();
    int run = x - sum;
#pragma unroll
    for (int i = 0; i < NW; ++i)
      if (i < wv) run += M.s_wave[16 + i];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < per) {
        const int lo = (int)(w[i] & 0xFFFFu), hi = (int)(w[i] >> 16);
        M.S32[tid * per + i] = (uint32_t)run | ((uint32_t)(run + lo) << 16);
        run += lo + hi;
      }
    if (tid == NT - 1) M.S32[NB >> 1] = (uint32_t)run;
    lds_sync();
  }
  if (PROF) t_bins = __builtin_amdgcn_s_memtime();

  // ---- scatter: every depth <= Dh node is now a contiguous range of bkey
#pragma unroll
  for (int u = 0; u < kQtKpt; ++u) {
    if (spill || u * NT >= K) break;  // wave-uniform
    const int k = tid + u * NT;
    if (k < K) {
      const int pos = (int)S[kb[u]] + kr[u];
      M.bkey[pos] = kv[u];
      M.bidx[pos] = (uint16_t)k;
    }
  }
  lds_sync();
  if (PROF) t_scatter = __builtin_amdgcn_s_memtime();

  // ---- the rounds, on the whole workgroup: a thread holds up to kIt
  // consecutive nodes of the list (and up to kIt consecutive candidate
  // ranks) in registers; every thread keeps the round state (size, m, T, the
  // candidate count) from block-level scans, so the waves agree without a
  // leader. The new list is written in place of the other node table.
  int2* nA = M.recA;
  int2* nB = M.recB;
  int pb = 0;  // partial-sum buffer of the next block scan (two, alternating)
  // exclusive prefix over the workgroup's threads of NV values, and totals;
  // one barrier
  auto bscan = [&](auto& v, auto& excl, auto& tot) {
    constexpr int NV = sizeof(v) / sizeof(v[0]);
    int x[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) x[k] = wave_incl_scan_dpp(v[k]);
    int* part = M.part + pb * 64;
    pb ^= 1;
    if (lane == 63)
#pragma unroll
      for (int k = 0; k < NV; ++k) part[k * 16 + wv] = x[k];
    lds_sync();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      int pre = 0, t = 0;
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const int p = part[k * 16 + i];
        if (i < wv) pre += p;
        t += p;
      }
      excl[k] = pre + x[k] - v[k];
      tot[k] = t;
    }
  };
  // the four child ranges of a node: bounds B[0..4] (B[0] = b, B[4] = e)
  auto bounds = [&](int2 r, int* B) {
    const int d = rdepth(r), pre = rpre(r);
    const int sh = 2 * max(Dh - d - 1, 0);
    const bool tab = rcnt(r) > 1 && d < Dh;
    B[0] = rb(r);
    B[4] = re(r);
    B[1] = S[tab ? ((pre << 2) | 1) << sh : 0];
    B[2] = S[tab ? ((pre << 2) | 2) << sh : 0];
    B[3] = S[tab ? ((pre << 2) | 3) << sh : 0];
    if (!tab) B[1] = B[2] = B[3] = B[4];
  };
  auto nonempty5 = [](const int* B) { return (B[1] > B[0]) + (B[2] > B[1]) + (B[3] > B[2]) + (B[4] > B[3]); };
  auto multi5 = [](const int* B) { return (B[1] > B[0] + 1) + (B[2] > B[1] + 1) + (B[3] > B[2] + 1) + (B[4] > B[3] + 1); };
  // children of split node (record r, bounds B, split rank j) at list
  // positions base, base + 1, ... as n4 n3 n2 n1 (creation j * 4 + q); its
  // multi-key children are listed as the next round's candidates from *cpos
  // on in creation order, so the candidate list is sorted by creation
  auto place_split = [&](int2 r, const int* B, int j, int base, int* cpos) {
    const int d = rdepth(r), pre = rpre(r);
    int c[4], p[4], k[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = B[q + 1] - B[q];
    p[3] = base;
#pragma unroll
    for (int q = 2; q >= 0; --q) p[q] = p[q + 1] + (c[q + 1] > 0);
    k[0] = *cpos;
#pragma unroll
    for (int q = 1; q < 4; ++q) k[q] = k[q - 1] + (c[q - 1] > 1);
    *cpos = k[3] + (c[3] > 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (c[q] > 0) {
        nB[p[q]] = mkrec(B[q], B[q + 1], (pre << 2) | q, d + 1, j * 4 + q);
        M.rank[p[q]] = -1;
      }
      if (c[q] > 1) {
        M.candk[k[q]] = ((uint32_t)c[q] << 16) | (uint32_t)(j * 4 + q);
        M.candn[k[q]] = p[q];
      }
    }
  };

  // roots: nIni columns (src/ORBextractor.cc:903-936), empty ones erased,
  // and the first breadth round over them folded in when it splits every
  // multi-key root (it does unless N is about nIni): every wave computes
  // them on its lanes (lane = root column), wave 0 writes them
  bool sorted = false, finished = false;
  int state = ST_DONE, rounds = 0, srounds = 0, tie_ev = 0, tie_nodes = 0, tie_keys = 0, ncand = 0, pbm = 0;
  int size;
  {
    int B[5] = {0, 0, 0, 0, 0};
    if (lane < nIni) {
      B[0] = S[lane << (2 * Dh)];
      B[4] = S[(lane + 1) << (2 * Dh)];
    }
    const int2 r = mkrec(B[0], B[4], lane, 0, 0);
    bounds(r, B);
    const uint64_t mk = __ballot(B[4] > B[0]);
    const int size0 = __popcll(mk), pos = mbcnt64(mk);
    const int v = rcnt(r) > 1 ? ((nonempty5(B) - 1) << 16) | 1 : 0, nm = v ? multi5(B) : 0;
    const int x = wave_incl_scan_dpp(v), cx = wave_incl_scan_dpp(nm);
    const int tot = __builtin_amdgcn_readlane(x, 63), nnext = __builtin_amdgcn_readlane(cx, 63);
    const int last = wave_max_dpp(v ? (lane << 2) | (nonempty5(B) - 1) : -1);
    const int Ctot = tot & 0xFFFF, Etot = (int)((uint32_t)tot >> 16);
    if (Ctot > 0 && size0 + Etot - (last & 3) < N) {
      const int m = Ctot, T = Etot + Ctot, run = x - v, E = (int)((uint32_t)run >> 16), C = run & 0xFFFF;
      int cpos = cx - nm;
      if (wv == 0 && B[4] > B[0]) {
        if (v) {
          place_split(r, B, C, T - (E + C + nonempty5(B)), &cpos);
        } else {
          nB[T + pos - min(C, m)] = r;
          M.rank[T + pos - min(C, m)] = -1;
        }
      }
      {
        int2* t = nA;
        nA = nB;
        nB = t;
      }
      size = T + (size0 - m);
      ncand = nnext;
      rounds = 1;
      finished = size >= N || size == size0;
      sorted = !finished && size + 3 * nnext > N;
    } else {
      size = size0;
      if (wv == 0 && B[4] > B[0]) {
        nA[pos] = r;
        M.rank[pos] = -1;
      }
    }
  }
  unsigned long long pr_b = 0, pr_s = 0;  // PROF: clocks of the breadth rounds, of the sorted rounds
  lds_sync();
  while (!finished) {
    const unsigned long long tr0 = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
    const bool was_sorted = sorted;
    if (rounds == 64) {
      if (tid == 0) atomicOr(err, 2);
      break;
    }
    const int per = (size + NT - 1) / NT;  // <= kIt (the plan keeps maxnodes <= kIt NT)
    const int nb = min(tid * per, size), ne = min(nb + per, size);
    int m = 0, T = 0, nnext = 0;
    if (!sorted) {
      // breadth round: packed scan value per node, candidates-before (low
      // half) and sum of (children - 1) over them (high half); split nodes
      // are the candidates with size + E < N, a prefix of them
      int2 r[kIt];
      int B[kIt][5];
      int v[kIt];
      // one scan: the packed values, the multi-key children and the deep
      // candidates as if every candidate were split, and (max) the last
      // candidate's children - 1. Every round but a breadth phase's last one
      // splits all its candidates, and that is decided from the totals alone
      // (size + E of the last candidate < N); the cut-off round takes a
      // second scan
      int s3[3] = {0, 0, 0}, last = -1;
#pragma unroll
      for (int i = 0; i < kIt; ++i) {
        if (i >= per) break;  // wave-uniform
        r[i] = nb + i < ne ? nA[nb + i] : make_int2(0, 0);
        bounds(r[i], B[i]);
        v[i] = rcnt(r[i]) > 1 ? ((nonempty5(B[i]) - 1) << 16) | 1 : 0;
        s3[0] += v[i];
        if (v[i]) {
          s3[1] += multi5(B[i]);
          s3[2] += rdepth(r[i]) >= Dh;  // its children are not in the bins
          last = ((nb + i) << 2) | (nonempty5(B[i]) - 1);
        }
      }
      int ex3[3], tot3[3];
      const int lmax = wave_max_dpp(last);
      if (lane == 63) M.part[128 + pb * 16 + wv] = lmax;
      const int pbl = pb;
      bscan(s3, ex3, tot3);
      int lastall = -1;
#pragma unroll
      for (int i = 0; i < NW; ++i) lastall = max(lastall, M.part[128 + pbl * 16 + i]);
      const int Ctot = tot3[0] & 0xFFFF, Etot = (int)((uint32_t)tot3[0] >> 16);
      int rn[kIt];
      int cpos = 0;
      if (Ctot == 0 || size + Etot - (lastall & 3) < N) {
        // a full round: every candidate splits
        if (tot3[2]) {  // a node to split below the bins' depth: the legacy rounds take the level
          state = ST_FALLBACK;
          break;
        }
        nnext = tot3[1];
        m = Ctot;
        T = Etot + Ctot;
        cpos = ex3[1];
        int run = ex3[0];
#pragma unroll
        for (int i = 0; i < kIt; ++i) {
          if (i >= per) break;  // wave-uniform
          rn[i] = run;
          run += v[i];
          if (!v[i]) v[i] = -1;  // kept
        }
      } else {
        // the cut-off round: split decisions; totals: candidates of the next
        // round (and this thread's first slot), splits, children of the
        // split nodes, deep
        int run = ex3[0];
        int s4[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < kIt; ++i) {
          if (i >= per) break;  // wave-uniform
          rn[i] = run;
          if (v[i] && size + (int)((uint32_t)run >> 16) < N) {
            s4[0] += multi5(B[i]);
            s4[1] += 1;
            s4[2] += nonempty5(B[i]);
            s4[3] |= rdepth(r[i]) >= Dh;
          } else {
            v[i] = -v[i] - 1;  // kept (the scan value is still needed below)
          }
          run += v[i] >= 0 ? v[i] : -v[i] - 1;
        }
        int ex4[4], tot4[4];
        bscan(s4, ex4, tot4);
        nnext = tot4[0];
        m = tot4[1];
        T = tot4[2];
        if (tot4[3]) {
          state = ST_FALLBACK;
          break;
        }
        cpos = ex4[0];
      }
#pragma unroll
      for (int i = 0; i < kIt; ++i) {
        if (i >= per) break;  // wave-uniform
        const int n = nb + i;
        if (n < ne) {
          const int E = (int)((uint32_t)rn[i] >> 16), C = rn[i] & 0xFFFF;
          if (v[i] >= 0) {
            place_split(r[i], B[i], C, T - (E + C + nonempty5(B[i])), &cpos);
          } else {
            const int pos = T + n - min(C, m);
            nB[pos] = r[i];
            M.rank[pos] = -1;
          }
        }
      }
    } else {
      // sorted round: the candidates (every multi-key node, all children of
      // the last round, listed in creation order) by (size, creation)
      // descending. rank = #(larger size) + #(same size, later creation): a
      // bitmap of candidate indices per size (sizes < 64), the group sizes'
      // suffix sums per wave, popcounts above the candidate's own bit
      ++srounds;
      const unsigned long long t0 = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
      const int bmw = M.bmw;
      uint32_t* BM = M.bm + pbm * 64 * bmw;
      uint32_t* BMo = M.bm + (pbm ^ 1) * 64 * bmw;
      int* nbig = s_var + V_BIG + pbm;
      for (int c = tid; c < ncand; c += NT) {
        const uint32_t key = M.candk[c];
        const int cnt = (int)(key >> 16);
        if (cnt < 64) {
          atomicOr(&BM[cnt * bmw + (c >> 5)], 1u << (c & 31));
        } else {
          const int bi = atomicAdd(nbig, 1);  // sizes >= 64: few, ranked among themselves
          if (bi < kQtBig) M.bigk[bi] = key;
        }
      }
      for (int i = tid; i < 64 * bmw; i += NT) BMo[i] = 0u;  // the last sorted round's bitmaps
      if (tid == 0) s_var[V_BIG + (pbm ^ 1)] = 0;
      lds_sync();
      const int nw32 = (ncand + 31) >> 5;
      {
        int gsz = 0;
        for (int w = 0; w < nw32; ++w) gsz += __popc(BM[lane * bmw + w]);
        const int all = wave_sum_dpp(gsz), pre = wave_incl_scan_dpp(gsz);
        M.gw[wv * 64 + lane] = *nbig + all - pre;  // candidates of size > lane
        wave_fence();
      }
      for (int c = tid; c < ncand; c += NT) {
        const uint32_t key = M.candk[c];
        const int cnt = (int)(key >> 16);
        int r = 0;
        if (cnt < 64) {
          const uint32_t* row = BM + cnt * bmw;
          const int w0 = c >> 5;
          r = M.gw[wv * 64 + cnt] + __popc(row[w0] & ((c & 31) == 31 ? 0u : ~0u << ((c & 31) + 1)));
          for (int w = w0 + 1; w < nw32; ++w) r += __popc(row[w]);
        } else if (*nbig <= kQtBig) {
          for (int j = 0; j < *nbig; ++j) r += M.bigk[j] > key ? 1 : 0;
        } else {
          for (int j = 0; j < ncand; ++j) r += M.candk[j] > key ? 1 : 0;
        }
        const int n = M.candn[c];
        M.spos[r] = n;
        M.rank[n] = r;
      }
      pbm ^= 1;
      lds_sync();
      if (PROF && tid == 0) s_var[V_TRANK] += (int)(__builtin_amdgcn_s_memtime() - t0);
      // a thread's consecutive ranks [cb, ce)
      const int cper = (ncand + NT - 1) / NT;
      const int cb = min(tid * cper, ncand), ce = min(cb + cper, ncand);
      int2 r[kIt];
      int B[kIt][5];
      int s1[1] = {0};
#pragma unroll
      for (int i = 0; i < kIt; ++i) {
        if (i >= cper) break;  // wave-uniform
        r[i] = cb + i < ce ? nA[M.spos[cb + i]] : make_int2(0, 0);
        bounds(r[i], B[i]);
        s1[0] += cb + i < ce ? nonempty5(B[i]) - 1 : 0;
      }
      int ex1[1], tot1[1];
      bscan(s1, ex1, tot1);
      int run = ex1[0], rn[kIt];
      int s4[4] = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < kIt; ++i) {
        if (i >= cper) break;  // wave-uniform
        rn[i] = run;
        if (cb + i < ce) {
          if (size + run < N) {
            s4[0] += multi5(B[i]);
            s4[1] += 1;
            s4[2] += nonempty5(B[i]);
            s4[3] |= rdepth(r[i]) >= Dh;
          }
          run += nonempty5(B[i]) - 1;
        }
      }
      int ex4[4], tot4[4];
      bscan(s4, ex4, tot4);
      nnext = tot4[0];
      m = tot4[1];
      T = tot4[2];
      if (tot4[3]) {
        state = ST_FALLBACK;
        break;
      }
      int cpos = ex4[0];
      // tie-straddle exposure: the cut-off at N fell
      // inside a group of equal-size candidates; and the kept nodes' order
      int s3[3] = {0, 0, 0};
      const bool straddle = m > 0 && m < ncand && rcnt(nA[M.spos[m - 1]]) == rcnt(nA[M.spos[m]]);
      if (straddle) {
        const int sz = rcnt(nA[M.spos[m - 1]]);
#pragma unroll
        for (int i = 0; i < kIt; ++i)
          if (cb + i < ce && rcnt(r[i]) == sz) {
            s3[0] += 1;
            s3[1] += cb + i < m ? nonempty5(B[i]) : 1;
          }
      }
      bool kp[kIt] = {};
      int2 k2[kIt];
#pragma unroll
      for (int i = 0; i < kIt; ++i) {
        if (i >= per) break;  // wave-uniform
        const int n = nb + i;
        const int j = n < ne ? M.rank[n] : 0;
        kp[i] = n < ne && !(j >= 0 && j < m);
        k2[i] = n < ne ? nA[n] : make_int2(0, 0);
        s3[2] += kp[i];
      }
      int ex3[3], tot3[3];
      bscan(s3, ex3, tot3);
      if (straddle) {
        tie_ev += 1;
        tie_nodes += tot3[0];
        tie_keys += tot3[1];
      }
      // children blocks of the split ranks, then the kept nodes in list order
#pragma unroll
      for (int i = 0; i < kIt; ++i) {
        if (i >= cper) break;  // wave-uniform
        const int j = cb + i;
        if (j < ce && j < m) place_split(r[i], B[i], j, T - (rn[i] + j + nonempty5(B[i])), &cpos);
      }
      int kpos = T + ex3[2];
#pragma unroll
      for (int i = 0; i < kIt; ++i)
        if (i < per && kp[i]) {
          nB[kpos] = k2[i];
          M.rank[kpos] = -1;
          ++kpos;
        }
    }
    const int newSize = T + (size - m);
    // finish when the list reached N or a round changed nothing (src/ORBextractor.cc:1026, 1091)
    const bool finish = newSize >= N || newSize == size;
    ++rounds;
    {
      int2* t = nA;
      nA = nB;
      nB = t;
    }
    size = newSize;
    ncand = nnext;
    lds_sync();
    if (PROF) (was_sorted ? pr_s : pr_b) += __builtin_amdgcn_s_memtime() - tr0;
    if (finish) break;
    // the breadth phase ends once one more full round would overshoot N (:1030);
    // nnext = the new list's multi-key nodes (nToExpand)
    if (!sorted && newSize + 3 * nnext > N) sorted = true;
  }
  if (PROF) t_rounds = __builtin_amdgcn_s_memtime();
  if (state == ST_FALLBACK) return false;  // uniform


  // ---- keep the best key per node: max FAST score, first original index on ties
  const int2* fin = nA;
  uint32_t* out = qkeys + (long long)f * P.kp_per_frame + g.kbase;
  if (spill) {
    // every bin holding keys lies in exactly one kept node: mark each node at
    // its first bin, fill forward (max scan of (bin + 1) << 16 | node), then
    // every key takes the max of (score, first index) into its node
    __syncthreads();  // the compact keys (global) of the gather, written by other threads
    int* nodeof = M.nodeof;
    int* best = M.rank;
    for (int i = tid; i < NB; i += NT) nodeof[i] = 0;
    for (int n = tid; n < size; n += NT) best[n] = 0;
    lds_sync();
    for (int n = tid; n < size; n += NT) {
      const int2 r = fin[n];
      const int lo = rpre(r) << (2 * (Dh - rdepth(r)));
      nodeof[lo] = ((lo + 1) << 16) | n;
    }
    lds_sync();
    {
      const int per = NB / NT;  // 4 .. 16
      int w[16], mx = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (i < per) {
          w[i] = nodeof[tid * per + i];
          mx = max(mx, w[i]);
        }
      int x = mx;  // inclusive max over the lanes
      x = max(x, dpp_i<kDppShr1>(0, x));
      x = max(x, dpp_i<kDppShr2>(0, x));
      x = max(x, dpp_i<kDppShr4>(0, x));
      x = max(x, dpp_i<kDppShr8>(0, x));
      x = max(x, dpp_i<kDppBcast15, 0xa>(0, x));
      x = max(x, dpp_i<kDppBcast31, 0xc>(0, x));
      if (lane == 63) M.s_wave[32 + wv] = x;
      const int prev = __shfl_up(x, 1);  // this lane's carry: the lanes before it
      lds_sync();
      int run = lane ? prev : 0;
#pragma unroll
      for (int i = 0; i < NW; ++i)
        if (i < wv) run = max(run, M.s_wave[32 + i]);
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (i < per) {
          run = max(run, w[i]);
          nodeof[tid * per + i] = run;
        }
    }
    lds_sync();
    for (int k0 = 0; k0 < K; k0 += 4 * NT) {
      uint32_t kk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) kk[u] = cs[min(k0 + u * NT + tid, K - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u * NT + tid;
        if (k < K) {
          const int bn = (int)((M.xs[min(key_x(kk[u]), tw - 1)] | ys[min(key_y(kk[u]), th - 1)]) >> shB);
          const int n = nodeof[bn] & 0xFFFF;
          atomicMax(&best[n], ((key_score(kk[u]) + 1) << 16) | (0xFFFF - k));
        }
      }
    }
    lds_sync();
    for (int n = tid; n < size && n < g.kcap; n += NT) {
      const int v = best[n];
      if (!v) atomicOr(err, 8);  // a node without keys: a broken list
      else out[n] = cs[0xFFFF - (v & 0xFFFF)];
    }
  }
  for (int n = tid; n < size && n < g.kcap && !spill; n += NT) {
    const int2 r = fin[n];
    const int b = rb(r), e = re(r);
    if (e <= b) {
      atomicOr(err, 8);  // a node without keys: a broken list, reported instead of read past the keys
      continue;
    }
    uint32_t best = ((M.bkey[b] >> 24) << 16) | (0xFFFFu - M.bidx[b]);
    int bi = b;
    for (int i = b + 1; i < e; ++i) {
      const uint32_t v = ((M.bkey[i] >> 24) << 16) | (0xFFFFu - M.bidx[i]);
      if (v > best) {
        best = v;
        bi = i;
      }
    }
    out[n] = M.bkey[bi];
  }
  if (tid == 0) {
    qcounts[f * P.L + l] = min(size, g.kcap);
    int* qt = qties + ((long long)f * P.L + l) * 4;
    qt[0] = tie_ev;
    qt[1] = tie_nodes;
    qt[2] = tie_keys;
    qt[3] = 1;  // orbx_get_quadtree_paths: the sorted-key path
    if (size > g.kcap) atomicOr(err, 4);
  }
  if (PROF && tid == 0) {  // diagnostics only (ORBX_QT_PROF=1)
    int* d = dbg + (blockIdx.y * gridDim.x + blockIdx.x) * 8;
    d[0] = (int)(t_rounds - t_begin);
    d[1] = (int)(__builtin_amdgcn_s_memtime() - t_begin);
    d[2] = rounds;
    d[3] = srounds;
    d[4] = K;
    d[5] = size;
    d[6] = (int)(t_scan - t_begin);
    d[7] = (int)(t_gather - t_begin);
    int* dp = dbg + gridDim.x * gridDim.y * 8 + (blockIdx.y * gridDim.x + blockIdx.x) * 8;
    dp[0] = (int)(t_own - t_begin);
    dp[1] = (int)(t_bins - t_begin);
    dp[2] = (int)(t_scatter - t_begin);
    dp[3] = s_var[V_TRANK];
    dp[4] = -1;  // marks the sorted path
    dp[5] = (int)pr_b;
    dp[6] = (int)pr_s;
    dp[7] = 0;
  }
  return true;
}

template <int NT, bool PROF>
__device__ __forceinline__ void qt_legacy(const ExtractParams& P, const int* __restrict__ cell_counts, const uint32_t* __restrict__ slots,
                          const CellGeom* __restrict__ cells, uint32_t* __restrict__ qscratch,
                          uint16_t* __restrict__ qnscratch, uint32_t* __restrict__ qkeys, int* __restrict__ qcounts,
                          int* __restrict__ qties, int* err, int* dbg, unsigned char* smem,
                          const unsigned long long t_begin) {
  int dbg_rounds = 0, dbg_sorted = 0;
  // phase clocks (ORBX_QT_PROF): scalars, not an array, so nothing lands in scratch
  unsigned long long dbg_p0 = 0, dbg_p1 = 0, dbg_p2 = 0, dbg_p3 = 0, dbg_p4 = 0, dbg_t = 0, dbg_init = 0, dbg_i1 = 0,
                     dbg_i2 = 0;
  auto ph = [&](int k) {
    if (!PROF) return;
    const unsigned long long t = __builtin_amdgcn_s_memtime(), d = t - dbg_t;
    if (k == 0) dbg_p0 += d;
    else if (k == 1) dbg_p1 += d;
    else if (k == 2) dbg_p2 += d;
    else if (k == 3) dbg_p3 += d;
    else if (k == 4) dbg_p4 += d;
    dbg_t = t;
  };
  const int l = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
  const LevelGeom& g = P.lv[l];
  const int MN = P.maxnodes, SN = P.sortn;
  unsigned char* p = smem + kQtHeader;
  auto take = [&](size_t bytes) { unsigned char* r = p; p += (bytes + 15) & ~(size_t)15; return r; };
  unsigned long long* s_sort = (unsigned long long*)take(8ull * SN);  // also best-key-per-node
  QNode* nodeA = (QNode*)take(sizeof(QNode) * MN);
  QNode* nodeB = (QNode*)take(sizeof(QNode) * MN);
  int* nkA = (int*)take(4ull * MN);
  int* nkB = (int*)take(4ull * MN);
  int* seqA = (int*)take(4ull * MN);
  int* seqB = (int*)take(4ull * MN);
  int4* cc = (int4*)take(16ull * MN);  // child key counts, then child list positions
  int* tA = (int*)take(4ull * (MN + 1));
  int* tB = (int*)take(4ull * (MN + 1));
  int* rank = (int*)take(4ull * MN);   // processing rank of a split node, or -1
  int* ord = (int*)take(4ull * MN);    // processing rank -> node
  int* coff = (int*)take(4ull * (P.max_cells_level + 1));
  int* s_soff = (int*)take(4ull * (P.max_cells_level + 1));  // cell slot offsets
  int2* s_mid = (int2*)take(8ull * MN);  // halves() of every node of this round
  int4* cc2 = (int4*)take(16ull * MN);    // register-resident rounds: next list's child counts
  int2* s_mid2 = (int2*)take(8ull * MN);  // ... and its halves()
  int* s_wave = (int*)take(512);          // ... per-wave partials (scan totals, counts, sums; 16 each)
  int* s_tmp = (int*)take(64);
  int* s_var = (int*)take(64);
  uint32_t* candk = (uint32_t*)take(4ull * MN);  // lean sorted rounds: candidates' sort keys ...
  int* candn = (int*)take(4ull * MN);            // ... and their nodes
  uint32_t* lkeys = (uint32_t*)take(4ull * P.kcap_lds);
  uint16_t* lnode = (uint16_t*)take(2ull * P.kcap_lds);

  // ---- the level's FAST keys in reference order (cells row-major, FAST order inside)
  const int* cntp = cell_counts + (long long)f * P.ncells_total + g.cell0;
  // cell counts and slot offsets are independent loads: one memory latency
  for (int c = tid; c < g.ncells; c += NT) {
    const int cnt = cntp[c], so = cells[g.cell0 + c].slot_off;
    coff[c] = cnt;
    s_soff[c] = so;
  }
  __syncthreads();
  const int K = block_scan_excl<NT>(coff, g.ncells, s_tmp);
  const unsigned long long t_scan = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
  uint32_t* keys = lkeys;
  uint16_t* knode = lnode;
  if (K > P.kcap_lds) {  // too many for LDS: same algorithm on an L2-resident scratch copy
    keys = qscratch + (long long)f * P.slots_per_frame + g.slot0;
    knode = qnscratch + (long long)f * P.slots_per_frame + g.slot0;
  }
  const uint32_t* fslots = slots + (long long)f * P.slots_per_frame;
  {
    // gather the K keys: cell c's keys (slot_off(c) .. + count) go to coff[c] ..
    if (tid == 0) coff[g.ncells] = K;
    __syncthreads();
    // per cell: its keys are one contiguous slot run; the first eight are
    // loaded together (most cells hold fewer), the rest in groups of four
    for (int c = tid; c < g.ncells; c += NT) {
      const int b = coff[c], n = coff[c + 1] - b;
      const uint32_t* src = fslots + s_soff[c];
      uint32_t v8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v8[i] = i < n ? src[i] : 0u;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (i < n) keys[b + i] = v8[i];
      int i = 8;
      for (; i + 4 <= n; i += 4) {
        const uint32_t v0 = src[i], v1 = src[i + 1], v2 = src[i + 2], v3 = src[i + 3];
        keys[b + i] = v0;
        keys[b + i + 1] = v1;
        keys[b + i + 2] = v2;
        keys[b + i + 3] = v3;
      }
      for (; i < n; ++i) keys[b + i] = src[i];
    }
  }
  const unsigned long long t_gather = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
  // ---- root nodes: nIni columns of width hX (src/ORBextractor.cc:894-936)
  const int nIni = g.nIni;
  int* rootCnt = tA;  // nIni <= MN
  for (int i = tid; i < nIni; i += NT) rootCnt[i] = 0;
  __syncthreads();
  // the non-empty roots in column order (one lane: nIni is a handful);
  // rootCnt[i] becomes the root's list position, -1 if empty (erased)
  auto build_roots = [&](bool reg) {
    if (tid != 0) return;
    int n = 0;
    for (int i = 0; i < nIni; ++i) {
      const int c = rootCnt[i];
      if (c > 0) {
        QNode nd;
        nd.x0 = (int16_t)(int)__fmul_rn(g.hX, (float)i);
        nd.x1 = (int16_t)(int)__fmul_rn(g.hX, (float)(i + 1));
        nd.y0 = 0;
        nd.y1 = (int16_t)g.boxH;
        nodeA[n] = nd;
        nkA[n] = c;
        seqA[n] = 0;
        if (reg) {
          int mx, my;
          halves(nd, &mx, &my);
          s_mid[n] = make_int2(mx, my);
          cc[n] = make_int4(0, 0, 0, 0);
        }
        rootCnt[i] = n++;
      } else {
        rootCnt[i] = -1;
      }
    }
    s_var[0] = n;  // list size
    s_var[1] = 0;  // sorted-phase flag
    s_var[6] = s_var[7] = s_var[8] = 0;  // tie-straddle events / group nodes / kept keys
    s_var[10] = 0;  // lean sorted rounds' candidate count
  };
  const int N = g.N;
  uint32_t* out = qkeys + (long long)f * P.kp_per_frame + g.kbase;
  auto write_tail = [&](int size, unsigned long long t_rounds) {
    if (tid == 0) {
      qcounts[f * P.L + l] = min(size, g.kcap);
      int* qt = qties + ((long long)f * P.L + l) * 4;
      qt[0] = s_var[6];
      qt[1] = s_var[7];
      qt[2] = s_var[8];
      qt[3] = 0;
      if (size > g.kcap) atomicOr(err, 4);
    }
    if (PROF && tid == 0) {  // diagnostics only (ORBX_QT_PROF=1)
      int* d = dbg + (blockIdx.y * gridDim.x + blockIdx.x) * 8;
      d[0] = (int)(t_rounds - t_begin);
      d[1] = (int)(__builtin_amdgcn_s_memtime() - t_begin);
      d[2] = dbg_rounds;
      d[3] = dbg_sorted;
      d[4] = K;
      d[5] = size;
      d[6] = (int)(t_scan - t_begin);
      d[7] = (int)(t_gather - t_begin);
      int* dp = dbg + gridDim.x * gridDim.y * 8 + (blockIdx.y * gridDim.x + blockIdx.x) * 8;
      dp[0] = (int)dbg_p0;
      dp[1] = (int)dbg_p1;
      dp[2] = (int)dbg_p2;
      dp[3] = (int)dbg_p3;
      dp[4] = (int)dbg_p4;
      dp[5] = (int)dbg_init;  // lean rounds: roots counted, roots built, first child counts done
      dp[6] = (int)dbg_i1;
      dp[7] = (int)dbg_i2;
    }
  };
  if (P.qt_lean && K < 65536) {  // sort keys pack a node's key count in 16 bits
    // ---- lean rounds. A key's node and its quadrant in that node are one
    // packed 16-bit entry (node << 2 | q); the next round's child counts are
    // added while the keys are re-homed, and the node-order scan runs over
    // per-thread chunks of the list with per-wave partials: four barriers
    // per breadth round (the generic path below takes nine). Key passes take
    // four keys per thread at a time so that their LDS latencies overlap.
    const int lane = tid & 63, wv = tid >> 6;
    constexpr int NW = NT / 64;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    uint32_t* s_key = (uint32_t*)ord;  // sorted rounds: size << 16 | creation per node
    for (int k0 = tid; k0 < K; k0 += 4 * NT) {
      uint32_t kk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) kk[u] = k0 + u * NT < K ? keys[k0 + u * NT] : 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + u * NT < K) {
          const int r = (int)__fdiv_rn((float)key_x(kk[u]), g.hX);  // vpIniNodes[kp.pt.x/hX]
          knode[k0 + u * NT] = (uint16_t)r;
          atomicAdd(&rootCnt[r], 1);
        }
      }
    }
    __syncthreads();
    if (PROF) dbg_i1 = __builtin_amdgcn_s_memtime() - t_begin;
    build_roots(true);
    __syncthreads();
    if (PROF) dbg_i2 = __builtin_amdgcn_s_memtime() - t_begin;
    QNode* nA = nodeA;
    QNode* nB = nodeB;
    int* kA = nkA;
    int* kB = nkB;
    int* qA = seqA;
    int* qB = seqB;
    int4* cA = cc;
    int4* cB = cc2;
    int2* mA = s_mid;
    int2* mB = s_mid2;
    // first child counts: a key counts into its node's quadrant if the node holds > 1 key
    for (int k0 = tid; k0 < K; k0 += 4 * NT) {
      uint32_t kk[4];
      int n[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool in = k0 + u * NT < K;
        kk[u] = in ? keys[k0 + u * NT] : 0u;
        n[u] = in ? knode[k0 + u * NT] : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) n[u] = rootCnt[n[u]];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + u * NT < K) {
          const int2 md = mA[n[u]];
          const int q = (key_x(kk[u]) >= md.x ? 1 : 0) + (key_y(kk[u]) >= md.y ? 2 : 0);
          if (kA[n[u]] > 1) atomicAdd(((int*)&cA[n[u]]) + q, 1);
          knode[k0 + u * NT] = (uint16_t)((n[u] << 2) | q);
        }
      }
    }
    int size = s_var[0];
    bool sorted_phase = false;
    lds_sync();
    if (PROF) dbg_init = __builtin_amdgcn_s_memtime() - t_begin;
    for (int round = 0; round < 64; ++round) {
      ph(-1);
      dbg_sorted += sorted_phase;
      const int per = (size + NT - 1) / NT;
      const int nb = min(tid * per, size), ne = min(nb + per, size);
      int expand = 0;
      // the next list: a kept node moves to pos; a split node's non-empty
      // children take base, base + 1, ... as n4 n3 n2 n1 (creation order
      // j * 4 + q), and cA[n] becomes their positions
      auto place_kept = [&](int n, int pos) {
        nB[pos] = nA[n];
        kB[pos] = kA[n];
        qB[pos] = qA[n];
        mB[pos] = mA[n];
        cB[pos] = make_int4(0, 0, 0, 0);
        // the re-homing reads a key's new node at cA[n][q] whether its node
        // was split (the child's position, place_split) or kept (here, all four)
        cA[n] = make_int4(pos, pos, pos, pos);
      };
      auto place_split = [&](int n, int j, int base) {
        const int4 c = cA[n];
        const QNode nd = nA[n];
        const int2 md = mA[n];
        const int cnts[4] = {c.x, c.y, c.z, c.w};
        int pos4[4];
        int after = 0;
#pragma unroll
        for (int q = 3; q >= 0; --q) {
          pos4[q] = -1;
          if (cnts[q] > 0) {
            const int pos = base + after++;
            QNode cb;
            cb.x0 = (q & 1) ? md.x : nd.x0;
            cb.x1 = (q & 1) ? nd.x1 : md.x;
            cb.y0 = (q & 2) ? md.y : nd.y0;
            cb.y1 = (q & 2) ? nd.y1 : md.y;
            int mx, my;
            halves(cb, &mx, &my);
            nB[pos] = cb;
            kB[pos] = cnts[q];
            qB[pos] = j * 4 + q;
            mB[pos] = make_int2(mx, my);
            cB[pos] = make_int4(0, 0, 0, 0);
            expand += cnts[q] > 1;
            pos4[q] = pos;
          }
        }
        cA[n] = make_int4(pos4[0], pos4[1], pos4[2], pos4[3]);
      };
      int m = 0, T = 0;
      if (!sorted_phase) {
        // breadth round (see the generic path): packed scan value per node,
        // candidates-before (low half) and sum of (children - 1) over them (high half)
        int sum = 0;
        for (int n = nb; n < ne; ++n) {
          const int v = kA[n] > 1 ? ((nonempty(cA[n]) - 1) << 16) | 1 : 0;
          tA[n] = v;
          sum += v;
        }
        const int x = wave_incl_scan_dpp(sum);
        if (lane == 63) s_wave[wv] = x;
        lds_sync();
        int run = x - sum;
#pragma unroll
        for (int i = 0; i < NW; ++i)
          if (i < wv) run += s_wave[i];
        int splits = 0, tmax = 0;
        for (int n = nb; n < ne; ++n) {
          const int v = tA[n], E = run >> 16, C = run & 0xFFFF;
          int j = -1;
          if (v && size + E < N) {
            j = C;
            ++splits;
            tmax = max(tmax, E + C + nonempty(cA[n]));
          }
          rank[n] = j;
          tA[n] = run;
          run += v;
        }
        splits = wave_sum_dpp(splits);
        tmax = INT_MAX - wave_min_dpp(INT_MAX - tmax);
        if (lane == 0) {
          s_wave[16 + wv] = splits;
          s_wave[32 + wv] = tmax;
        }
        lds_sync();
#pragma unroll
        for (int i = 0; i < NW; ++i) {
          m += s_wave[16 + i];
          T = max(T, s_wave[32 + i]);
        }
        ph(1);
        for (int n = nb; n < ne; ++n) {
          const int j = rank[n], v = tA[n];
          if (j < 0) place_kept(n, T + n - min(v & 0xFFFF, m));
          else place_split(n, j, T - ((v >> 16) + (v & 0xFFFF) + nonempty(cA[n])));
        }
      } else {
        // sorted round: the candidates (nodes with > 1 key; after a round
        // that did not finish, all of them children of that round) by (size,
        // creation) descending. s_key, filled while the keys were re-homed,
        // holds size << 16 | creation, distinct among the candidates, 0 for
        // the others; each candidate counts the larger keys.
        int* s_pos = (int*)s_sort;  // sorted rank -> node
        // the candidates and their keys were listed (in no particular order)
        // when the keys were written: a candidate's rank counts the larger
        // keys among the candidates only
        const int ncand = s_var[10];
        for (int c = tid; c < ncand; c += NT) {
          const uint32_t ki = candk[c];
          int r = 0, j = 0;
          for (; j + 16 <= ncand; j += 16) {  // sixteen broadcast keys in flight
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = *(const u32x4*)(candk + j + 4 * u);
#pragma unroll
            for (int u = 0; u < 4; ++u)
              r += (v[u].x > ki ? 1 : 0) + (v[u].y > ki ? 1 : 0) + (v[u].z > ki ? 1 : 0) + (v[u].w > ki ? 1 : 0);
          }
          for (; j < ncand; ++j) r += candk[j] > ki ? 1 : 0;
          const int i = candn[c];
          s_pos[r] = i;
          tA[r] = nonempty(cA[i]) - 1;
          rank[i] = r;
        }
        for (int i = tid; i < size; i += NT)
          if (!s_key[i]) rank[i] = -1;
        lds_sync();
        if (tid == 0) s_var[10] = 0;  // every thread has read the count (the next list's candidates count afresh)
        // split ranks: the prefix of ranks j with size + E_j < N, E_j = sum
        // of (children - 1) over the ranks before j (per-thread rank chunks)
        const int cper = (ncand + NT - 1) / NT;
        const int cb = min(tid * cper, ncand), ce = min(cb + cper, ncand);
        int csum = 0;
        for (int j = cb; j < ce; ++j) csum += tA[j];
        const int cx = wave_incl_scan_dpp(csum);
        if (lane == 63) s_wave[wv] = cx;
        lds_sync();
        int run = cx - csum;
#pragma unroll
        for (int i = 0; i < NW; ++i)
          if (i < wv) run += s_wave[i];
        int splits = 0, tsum = 0;
        for (int j = cb; j < ce; ++j) {
          const int v = tA[j];
          if (size + run < N) {
            ++splits;
            tsum += v + 1;
          }
          tA[j] = run;
          run += v;
        }
        splits = wave_sum_dpp(splits);
        tsum = wave_sum_dpp(tsum);
        if (lane == 0) {
          s_wave[32 + wv] = splits;
          s_wave[64 + wv] = tsum;
        }
        lds_sync();
#pragma unroll
        for (int i = 0; i < NW; ++i) {
          m += s_wave[32 + i];
          T += s_wave[64 + i];  // children block: the split ranks' children
        }
        ph(4);
        // tie-straddle exposure (generic path)
        if (m > 0 && m < ncand && (s_key[s_pos[m - 1]] >> 16) == (s_key[s_pos[m]] >> 16)) {
          const uint32_t sz = s_key[s_pos[m - 1]] >> 16;
          // (uniform branch) per-thread counts, one atomic per wave and counter:
          // the group's nodes all hit the same two counters
          int g7 = 0, g8 = 0;
          for (int j = tid; j < ncand; j += NT) {
            const int n = s_pos[j];
            if ((s_key[n] >> 16) == sz) {
              g7 += 1;
              g8 += j < m ? nonempty(cA[n]) : 1;
            }
          }
          g7 = wave_sum_dpp(g7);
          g8 = wave_sum_dpp(g8);
          if (lane == 0 && g7) {
            atomicAdd(&s_var[7], g7);
            atomicAdd(&s_var[8], g8);
          }
          if (tid == 0) s_var[6] += 1;
        }
        // kept nodes keep their list order after the children block
        int kept = 0;
        for (int n = nb; n < ne; ++n) kept += (rank[n] >= 0 && rank[n] < m) ? 0 : 1;
        const int kx = wave_incl_scan_dpp(kept);
        if (lane == 63) s_wave[80 + wv] = kx;
        lds_sync();
        int kpos = T + kx - kept;
#pragma unroll
        for (int i = 0; i < NW; ++i)
          if (i < wv) kpos += s_wave[80 + i];
        for (int n = nb; n < ne; ++n) {
          const int j = rank[n];
          if (j >= 0 && j < m) place_split(n, j, T - (tA[j] + j + nonempty(cA[n])));
          else place_kept(n, kpos++);
        }
      }
      expand = wave_sum_dpp(expand);
      if (lane == 0) s_wave[48 + wv] = expand;
      lds_sync();
      ph(2);
      int nExp = 0;
#pragma unroll
      for (int i = 0; i < NW; ++i) nExp += s_wave[48 + i];
      const int newSize = T + (size - m);
      // finish when the list reached N or a round changed nothing (src/ORBextractor.cc:1011, 1093)
      const bool finish = newSize >= N || newSize == size;
      // re-home the keys, counting them into the next list's children
      for (int k0 = tid; k0 < K; k0 += 4 * NT) {
        uint32_t kk[4];
        int pk[4], nn[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool in = k0 + u * NT < K;
          kk[u] = in ? keys[k0 + u * NT] : 0u;
          pk[u] = in ? knode[k0 + u * NT] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) nn[u] = ((const int*)cA)[pk[u]];  // pk = node << 2 | quadrant
        if (!finish) {
          int2 md[4];
          int big[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            big[u] = kB[nn[u]];
            md[u] = mB[nn[u]];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (k0 + u * NT < K) {
              const int q = (key_x(kk[u]) >= md[u].x ? 1 : 0) + (key_y(kk[u]) >= md[u].y ? 2 : 0);
              if (big[u] > 1) atomicAdd(((int*)&cB[nn[u]]) + q, 1);
              knode[k0 + u * NT] = (uint16_t)((nn[u] << 2) | q);
            }
          }
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (k0 + u * NT < K) knode[k0 + u * NT] = (uint16_t)(nn[u] << 2);
        }
      }
      // the breadth phase ends once one more full round would overshoot N (:1015)
      if (!finish && !sorted_phase && newSize + 3 * nExp > N) sorted_phase = true;
      if (!finish && sorted_phase)  // the next round's sort keys (the new list is kB, qB) and its candidate list
        for (int i = tid; i < newSize; i += NT) {
          const uint32_t key = kB[i] > 1 ? ((uint32_t)kB[i] << 16) | (uint32_t)qB[i] : 0u;
          s_key[i] = key;
          if (key) {
            const int c = atomicAdd(&s_var[10], 1);
            candk[c] = key;
            candn[c] = i;
          }
        }
      size = newSize;
      {
        QNode* t0 = nA; nA = nB; nB = t0;
        int* t1 = kA; kA = kB; kB = t1;
        int* t2 = qA; qA = qB; qB = t2;
        int4* t3 = cA; cA = cB; cB = t3;
        int2* t4 = mA; mA = mB; mB = t4;
      }
      lds_sync();
      ph(3);
      dbg_rounds++;
      if (finish) break;
      if (round == 63 && tid == 0) atomicOr(err, 2);
    }
    const unsigned long long t_rounds = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
    // ---- keep the best key per node: max FAST score, first in key order
    for (int n = tid; n < size; n += NT) s_sort[n] = 0;
    lds_sync();
    for (int k = tid; k < K; k += NT)
      atomicMax(&s_sort[knode[k] >> 2],
                ((unsigned long long)key_score(keys[k]) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)k));
    lds_sync();
    for (int n = tid; n < size && n < g.kcap; n += NT) {
      const unsigned long long b = s_sort[n];
      if (b) out[n] = keys[0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull)];
      else atomicOr(err, 8);  // a node without keys: a broken list, reported instead of read past the keys
    }
    write_tail(size, t_rounds);
    return;
  }
  for (int k = tid; k < K; k += NT) {
    const int r = (int)__fdiv_rn((float)key_x(keys[k]), g.hX);  // vpIniNodes[kp.pt.x/hX]
    knode[k] = (uint16_t)r;
    atomicAdd(&rootCnt[r], 1);
  }
  __syncthreads();
  build_roots(false);
  __syncthreads();
  for (int k = tid; k < K; k += NT) knode[k] = (uint16_t)rootCnt[knode[k]];
  __syncthreads();

  // node tables ping-pong between rounds (A = this round's list, B = the next)
  QNode* nA = nodeA;
  QNode* nB = nodeB;
  int* kA = nkA;
  int* kB = nkB;
  int* qA = seqA;
  int* qB = seqB;
  for (int round = 0; round < 64; ++round) {
    const int size = s_var[0];
    const bool sorted_phase = s_var[1] != 0;
    ph(-1);
    // child key counts of every splittable node
    for (int n = tid; n < size; n += NT) {
      cc[n] = make_int4(0, 0, 0, 0);
      int mx, my;
      halves(nA[n], &mx, &my);
      s_mid[n] = make_int2(mx, my);
    }
    if (tid == 0) {
      s_var[2] = 0;  // nodes split this round
      s_var[4] = 0;  // split children that hold > 1 key
      s_var[5] = 0;  // T: list positions taken by the children block
    }
    __syncthreads();
    for (int k0 = tid; k0 < K; k0 += 4 * NT) {  // four keys in flight per thread
      int n[4], q[4];
      uint32_t kk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u * NT;
        n[u] = k < K ? knode[k] : 0;
        kk[u] = k < K ? keys[k] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int2 m = s_mid[n[u]];
        q[u] = (k0 + u * NT < K && kA[n[u]] > 1)
                   ? (key_x(kk[u]) >= m.x ? 1 : 0) + (key_y(kk[u]) >= m.y ? 2 : 0)
                   : -1;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (q[u] >= 0) atomicAdd(((int*)&cc[n[u]]) + q[u], 1);
    }
    __syncthreads();
    ph(0);
    // After the order step every node has rank[n] (processing rank of a split
    // node, -1 if kept); the table step writes the next list and leaves in
    // tB[n] the new position of a kept node and in cc[n] those of a split
    // node's children. Children block: rank j lands at T - (E_j + C_j), E_j =
    // children of the ranks before j (last split first).
    if (!sorted_phase) {
      // breadth round: candidates = nodes with > 1 key in list order; one
      // packed scan gives per node C = candidates before it (low half) and
      // E' = sum of (children - 1) over them (high half). The split nodes are
      // the candidates with size + E' < N, a prefix of them, so for split node
      // n: rank = C, E_rank = E' + C; for a kept node: position T + n - min(C, m).
      for (int n = tid; n < size; n += NT)
        tA[n] = kA[n] > 1 ? ((nonempty(cc[n]) - 1) << 16) | 1 : 0;
      __syncthreads();
      block_scan_excl<NT>(tA, size, s_tmp);
      for (int n = tid; n < size; n += NT) {
        const int v = tA[n], E = v >> 16, C = v & 0xFFFF;
        if (kA[n] > 1 && size + E < N) {
          rank[n] = C;
          atomicAdd(&s_var[2], 1);
          atomicMax(&s_var[5], E + C + nonempty(cc[n]));
        } else {
          rank[n] = -1;
        }
      }
      __syncthreads();
      ph(1);
      const int m = s_var[2], T = s_var[5];
      for (int n = tid; n < size; n += NT) {
        const int j = rank[n], v = tA[n];
        if (j < 0) {
          const int pos = T + n - min(v & 0xFFFF, m);
          nB[pos] = nA[n];
          kB[pos] = kA[n];
          qB[pos] = qA[n];
          tB[n] = pos;
        } else {
          const int4 c = cc[n];
          const int cnts[4] = {c.x, c.y, c.z, c.w};
          const int base = T - ((v >> 16) + (v & 0xFFFF) + nonempty(c));
          int pos4[4];
          int after = 0, expand = 0;
#pragma unroll
          for (int q = 3; q >= 0; --q) {
            if (cnts[q] > 0) {
              pos4[q] = base + after++;
              nB[pos4[q]] = child_box(nA[n], q);
              kB[pos4[q]] = cnts[q];
              qB[pos4[q]] = j * 4 + q;  // creation order: split rank, then n1..n4
              expand += cnts[q] > 1;
            } else {
              pos4[q] = -1;
            }
          }
          cc[n] = make_int4(pos4[0], pos4[1], pos4[2], pos4[3]);
          if (expand) atomicAdd(&s_var[4], expand);
        }
      }
    } else {
      // descending order of the candidates by (size, creation): each candidate
      // counts the larger keys (keys are distinct), no sorting network
      unsigned long long* s_key = (unsigned long long*)nB;  // free until the table step
      for (int i = tid; i < size; i += NT) {
        s_key[i] = kA[i] > 1
                       ? ((unsigned long long)kA[i] << 40) | ((unsigned long long)qA[i] << 16) | (unsigned long long)i
                       : 0ull;
        s_sort[i] = 0;
        rank[i] = -1;
      }
      if (tid == 0) s_var[3] = 0;
      __syncthreads();
      for (int i = tid; i < size; i += NT) {
        const unsigned long long ki = s_key[i];
        if (ki) {
          int r = 0, j = 0;
          for (; j + 8 <= size; j += 8) {  // eight broadcast reads in flight
            unsigned long long v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = s_key[j + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) r += v[u] > ki ? 1 : 0;
          }
          for (; j < size; ++j) r += s_key[j] > ki ? 1 : 0;
          s_sort[r] = ki;
        }
      }
      __syncthreads();
      for (int j = tid; j < size; j += NT) {
        const unsigned long long key = s_sort[j];
        tA[j] = key ? nonempty(cc[(int)(key & 0xFFFF)]) - 1 : 0;
        if (key) atomicAdd(&s_var[3], 1);
      }
      __syncthreads();
      const int ncand = s_var[3];
      block_scan_excl<NT>(tA, ncand, s_tmp);
      for (int j = tid; j < ncand; j += NT) {
        if (size + tA[j] < N) {
          const int n = (int)(s_sort[j] & 0xFFFF);
          rank[n] = j;
          ord[j] = n;
          atomicAdd(&s_var[2], 1);
        }
      }
      __syncthreads();
      ph(4);
      const int m = s_var[2];
      // tie-straddle exposure: the cut-off at N fell inside a
      // group of equal-size candidates, so the creation-order stand-in for
      // the reference's heap-pointer order (src/ORBextractor.cc:1041) picked
      // which of them were split; count the group and the kept keys it yields
      if (m > 0 && m < ncand && (s_sort[m - 1] >> 40) == (s_sort[m] >> 40)) {
        const unsigned long long sz = s_sort[m - 1] >> 40;
        for (int j = tid; j < ncand; j += NT) {
          const unsigned long long key = s_sort[j];
          if ((key >> 40) == sz) {
            atomicAdd(&s_var[7], 1);
            atomicAdd(&s_var[8], j < m ? nonempty(cc[(int)(key & 0xFFFF)]) : 1);
          }
        }
        if (tid == 0) s_var[6] += 1;
      }
      for (int j = tid; j < m; j += NT) tA[j] = nonempty(cc[ord[j]]);
      __syncthreads();
      const int T = block_scan_excl<NT>(tA, m, s_tmp);
      for (int n = tid; n < size; n += NT) tB[n] = rank[n] < 0 ? 1 : 0;
      __syncthreads();
      block_scan_excl<NT>(tB, size, s_tmp);
      if (tid == 0) s_var[5] = T;
      for (int n = tid; n < size; n += NT) {
        const int j = rank[n];
        if (j < 0) {
          const int pos = T + tB[n];
          nB[pos] = nA[n];
          kB[pos] = kA[n];
          qB[pos] = qA[n];
          tB[n] = pos;
        } else {
          const int4 c = cc[n];
          const int cnts[4] = {c.x, c.y, c.z, c.w};
          const int base = T - (tA[j] + nonempty(c));
          int pos4[4];
          int after = 0, expand = 0;
#pragma unroll
          for (int q = 3; q >= 0; --q) {
            if (cnts[q] > 0) {
              pos4[q] = base + after++;
              nB[pos4[q]] = child_box(nA[n], q);
              kB[pos4[q]] = cnts[q];
              qB[pos4[q]] = j * 4 + q;
              expand += cnts[q] > 1;
            } else {
              pos4[q] = -1;
            }
          }
          cc[n] = make_int4(pos4[0], pos4[1], pos4[2], pos4[3]);
          if (expand) atomicAdd(&s_var[4], expand);
        }
      }
    }
    __syncthreads();
    ph(2);
    const int m = s_var[2], T = s_var[5];
    const int newSize = T + (size - m);
    // re-home the keys
    for (int k0 = tid; k0 < K; k0 += 4 * NT) {  // four keys in flight per thread
      int n[4], j[4], nn[4];
      uint32_t kk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u * NT;
        n[u] = k < K ? knode[k] : 0;
        kk[u] = k < K ? keys[k] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) j[u] = rank[n[u]];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (j[u] < 0) {
          nn[u] = tB[n[u]];
        } else {
          const int2 mm = s_mid[n[u]];
          nn[u] = ((const int*)&cc[n[u]])[(key_x(kk[u]) >= mm.x ? 1 : 0) + (key_y(kk[u]) >= mm.y ? 2 : 0)];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u * NT;
        if (k < K) knode[k] = (uint16_t)nn[u];
      }
    }
    // finish when the list reached N or a round changed nothing (src/ORBextractor.cc:1011, 1093);
    // the breadth phase ends once one more full round would overshoot N (:1015)
    const bool finish = newSize >= N || newSize == size;
    const int nExp = s_var[4];
    __syncthreads();
    if (tid == 0) {
      if (!finish && !sorted_phase && newSize + 3 * nExp > N) s_var[1] = 1;
      s_var[0] = newSize;
    }
    {  // the next list becomes this one
      QNode* t0 = nA; nA = nB; nB = t0;
      int* t1 = kA; kA = kB; kB = t1;
      int* t2 = qA; qA = qB; qB = t2;
    }
    __syncthreads();
    ph(3);
    dbg_rounds++;
    dbg_sorted += sorted_phase;
    if (finish) break;
    if (round == 63 && tid == 0) atomicOr(err, 2);
  }
  const unsigned long long t_rounds = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
  // ---- keep the best key per node: max FAST score, first in node (= original) order
  const int size = s_var[0];
  for (int n = tid; n < size; n += NT) s_sort[n] = 0;
  __syncthreads();
  for (int k = tid; k < K; k += NT) {
    const unsigned long long v =
        ((unsigned long long)key_score(keys[k]) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)k);
    atomicMax(&s_sort[knode[k]], v);
  }
  __syncthreads();
  for (int n = tid; n < size && n < g.kcap; n += NT) {
    const unsigned long long b = s_sort[n];
    if (b) out[n] = keys[0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull)];
    else atomicOr(err, 8);  // a node without keys: a broken list, reported instead of read past the keys
  }
  write_tail(size, t_rounds);
}

template <int NT, bool PROF>
__global__ __launch_bounds__(NT, ORBX_QT_MINW) void quadtree_kernel(ExtractParams P, const int* __restrict__ cell_counts,
                                                                   const uint32_t* __restrict__ slots,
                                                                   const CellGeom* __restrict__ cells,
                                                                   const uint32_t* __restrict__ qtab,
                                                                   uint32_t* __restrict__ qscratch,
                                                                   uint16_t* __restrict__ qnscratch,
                                                                   uint32_t* __restrict__ qkeys,
                                                                   int* __restrict__ qcounts, int* __restrict__ qties,
                                                                   int* err, int* dbg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned long long t_begin = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
  if (P.qt_sorted && P.lv[blockIdx.x].qt_tab >= 0 &&
      qt_sorted_path<NT, PROF>(P, cell_counts, slots, cells, qtab, qscratch, qkeys, qcounts, qties, err, dbg, smem,
                               t_begin))
    return;
  qt_legacy<NT, PROF>(P, cell_counts, slots, cells, qscratch, qnscratch, qkeys, qcounts, qties, err, dbg, smem, t_begin);
}

size_t quadtree_legacy_lds_bytes(const ExtractParams& P) {
  auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t MN = P.maxnodes, SN = P.sortn;
  return kQtHeader + r16(8 * SN) + 2 * r16(sizeof(QNode) * MN) + 4 * r16(4 * MN) + r16(16 * MN) +
         2 * r16(4 * (MN + 1)) + 2 * r16(4 * MN) + 2 * r16(4 * (P.max_cells_level + 1)) + r16(8 * MN) +
         r16(16 * MN) + r16(8 * MN) + 512 + 2 * r16(64) + 2 * r16(4 * MN) + r16(4ull * P.kcap_lds) +
         r16(2ull * P.kcap_lds);
}

size_t quadtree_sorted_lds_bytes(const ExtractParams& P, int big) {
  return big ? QtSortedLds<1024>(P, nullptr).bytes : QtSortedLds<kQtThreads>(P, nullptr).bytes;
}
// the sorted path's largest spill-mode key count for an LDS budget (0: the
// register mode's region does not fit)
int quadtree_sorted_ownmax(const ExtractParams& P, int big, size_t budget) {
  const size_t fixed = big ? QtSortedLds<1024>(P, nullptr).fixed : QtSortedLds<kQtThreads>(P, nullptr).fixed;
  const size_t nt = big ? 1024 : kQtThreads;
  const size_t need = std::max<size_t>(6 * nt * kQtKpt, 4ull * P.qt_nbmax) + 16;
  if (fixed + need > budget) return 0;
  return (int)std::min<size_t>(32767, std::max<size_t>(nt * kQtKpt, (budget - fixed - 16) / 2) & ~(size_t)7);
}

size_t quadtree_lds_bytes(const ExtractParams& P) {
  const size_t a = quadtree_legacy_lds_bytes(P);
  return P.qt_sorted ? std::max(a, quadtree_sorted_lds_bytes(P, P.qt_big)) : a;
}

template <bool PROF>
static const void* qt_kernel_ptr(const ExtractParams& P) {
  return P.qt_big ? (const void*)quadtree_kernel<1024, PROF> : (const void*)quadtree_kernel<kQtThreads, PROF>;
}
const void* quadtree_kernel_ptr(const ExtractParams& P) { return qt_kernel_ptr<false>(P); }

int launch_quadtree(const ExtractParams& P, const ExtractBuffers& X, int batch, hipStream_t s) {
  static int* dbg = nullptr;  // diagnostics only: per-(frame, level) cycles and rounds (ORBX_QT_PROF=1)
  static const bool prof = getenv("ORBX_QT_PROF") && getenv("ORBX_QT_PROF")[0] == '1';
  const int nwg = P.L * batch;
  const uint32_t* qtab = (const uint32_t*)X.rtab;
  const size_t lds = quadtree_lds_bytes(P);
  if (prof) {
    (void)hipFuncSetAttribute(qt_kernel_ptr<true>(P), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (!dbg) (void)hipMalloc(&dbg, (size_t)4096 * 96);
    if (nwg > 4096) return ORBX_EINVAL;
  }
#define QT_LAUNCH(NT_, PROF_)                                                                                     \
  hipLaunchKernelGGL((quadtree_kernel<NT_, PROF_>), dim3(P.L, batch), dim3(NT_), lds, s, P, X.cell_counts,        \
                     X.slots, X.cells, qtab, X.qscratch, X.qnode_scratch, X.qkeys, X.qcounts, X.qties, X.err, dbg)
  if (P.qt_big) {
    if (prof) QT_LAUNCH(1024, true);
    else QT_LAUNCH(1024, false);
  } else {
    if (prof) QT_LAUNCH(kQtThreads, true);
    else QT_LAUNCH(kQtThreads, false);
  }
#undef QT_LAUNCH
  if (prof) {
    std::vector<int> h((size_t)nwg * 24);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), dbg, h.size() * 4, hipMemcpyDeviceToHost);
    for (int l = 0; l < P.L; ++l) {
      double a[8] = {0}, q[8] = {0}, z[8] = {0};
      int mx = 0, nsorted = 0;
      for (int f = 0; f < batch; ++f) {
        for (int k = 0; k < 8; ++k) {
          a[k] += h[(f * P.L + l) * 8 + k];
          q[k] += h[(size_t)nwg * 8 + (f * P.L + l) * 8 + k];
          z[k] += h[(size_t)nwg * 16 + (f * P.L + l) * 8 + k];
        }
        mx = std::max(mx, h[(f * P.L + l) * 8 + 1]);
        nsorted += h[(size_t)nwg * 8 + (f * P.L + l) * 8 + 4] == -1;
      }
      for (int k = 0; k < 8; ++k) a[k] /= batch, q[k] /= batch, z[k] /= batch;
      if (nsorted == batch)
        fprintf(stderr,
                "quadtree L%d [sorted]: avg cycles rounds %.0f total %.0f (max %d) rounds %.1f sorted %.1f K %.0f out %.0f"
                " | scan %.0f own %.0f gather %.0f bins %.0f scatter %.0f | breadth rounds %.0f sorted rounds %.0f"
                " (ranking %.0f)\n",
                l, a[0], a[1], mx, a[2], a[3], a[4], a[5], a[6], q[0], a[7], q[1], q[2], q[5], q[6], q[3]);
      else
        fprintf(stderr,
                "quadtree L%d [legacy %d/%d]: avg cycles rounds %.0f total %.0f (max %d) rounds %.1f sorted %.1f K %.0f out %.0f"
                " | scan %.0f gather %.0f roots %.0f built %.0f init %.0f | count %.0f order %.0f sortorder %.0f table %.0f"
                " rehome %.0f\n",
                l, batch - nsorted, batch, a[0], a[1], mx, a[2], a[3], a[4], a[5], a[6], a[7], q[6], q[7], q[5], q[0],
                q[1], q[4], q[2], q[3]);
    }
  }
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
