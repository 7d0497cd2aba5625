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
// Data-parallel restatement (one 512-thread workgroup per frame x level):
// the list is a node table indexed by list position; keys never move, each
// key carries its node index. A round is "split a prefix of the candidate
// sequence": candidates = nodes with > 1 key, taken in list order (breadth
// rounds) or sorted by (size desc, creation desc) (sorted rounds; creation
// order stands in for the reference's heap-pointer tie-break, the same rule
// the oracle uses); the prefix ends where the running list size reaches N.
// The new list is [children of the split nodes, last split first, each as
// n4 n3 n2 n1] followed by the untouched nodes in their old order, which is
// exactly what the reference's push_front/erase sequence produces.
//
// Two implementations of the rounds share the key gather and the output:
// the lean rounds (every plan whose node table fits 16-bit packing and
// levels with < 65536 keys) and the generic rounds (the fallback, and the
// round-1 form, ORBX_QT_GENERIC=1 forces it for tests). DESIGN.md section 6
// has the barrier counts and timings of both.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orbx_device.cuh"

namespace orbx {

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
// kQtThreads: 512 (every plan whose node tables leave room for two blocks per
// CU) or 1024 (large levels, whose blocks take a CU each and whose key passes
// then run on twice the lanes)
template <int kQtThreads>
__global__ __launch_bounds__(kQtThreads, ORBX_QT_MINW) void quadtree_kernel(ExtractParams P, const int* __restrict__ cell_counts,
                                                              const uint32_t* __restrict__ slots,
                                                              const CellGeom* __restrict__ cells,
                                                              uint32_t* __restrict__ qscratch,
                                                              uint16_t* __restrict__ qnscratch,
                                                              uint32_t* __restrict__ qkeys,
                                                              int* __restrict__ qcounts, int* __restrict__ qties,
                                                              int* err, int* dbg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned long long t_begin = __builtin_amdgcn_s_memtime();
  int dbg_rounds = 0, dbg_sorted = 0;
  // phase clocks (ORBX_QT_PROF): scalars, not an array, so nothing lands in scratch
  unsigned long long dbg_p0 = 0, dbg_p1 = 0, dbg_p2 = 0, dbg_p3 = 0, dbg_p4 = 0, dbg_t = 0, dbg_init = 0, dbg_i1 = 0,
                     dbg_i2 = 0;
  auto ph = [&](int k) {
    if (!dbg) return;
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
  unsigned char* p = smem;
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
  for (int c = tid; c < g.ncells; c += kQtThreads) {
    const int cnt = cntp[c], so = cells[g.cell0 + c].slot_off;
    coff[c] = cnt;
    s_soff[c] = so;
  }
  __syncthreads();
  const int K = block_scan_excl<kQtThreads>(coff, g.ncells, s_tmp);
  const unsigned long long t_scan = __builtin_amdgcn_s_memtime();
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
    for (int c = tid; c < g.ncells; c += kQtThreads) {
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
  const unsigned long long t_gather = __builtin_amdgcn_s_memtime();
  // ---- root nodes: nIni columns of width hX (src/ORBextractor.cc:894-936)
  const int nIni = g.nIni;
  int* rootCnt = tA;  // nIni <= MN
  for (int i = tid; i < nIni; i += kQtThreads) rootCnt[i] = 0;
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
    if (dbg && tid == 0) {  // diagnostics only (ORBX_QT_PROF=1)
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
    constexpr int NW = kQtThreads / 64;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    uint32_t* s_key = (uint32_t*)ord;  // sorted rounds: size << 16 | creation per node
    for (int k0 = tid; k0 < K; k0 += 4 * kQtThreads) {
      uint32_t kk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) kk[u] = k0 + u * kQtThreads < K ? keys[k0 + u * kQtThreads] : 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + u * kQtThreads < K) {
          const int r = (int)__fdiv_rn((float)key_x(kk[u]), g.hX);  // vpIniNodes[kp.pt.x/hX]
          knode[k0 + u * kQtThreads] = (uint16_t)r;
          atomicAdd(&rootCnt[r], 1);
        }
      }
    }
    __syncthreads();
    if (dbg) dbg_i1 = __builtin_amdgcn_s_memtime() - t_begin;
    build_roots(true);
    __syncthreads();
    if (dbg) dbg_i2 = __builtin_amdgcn_s_memtime() - t_begin;
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
    for (int k0 = tid; k0 < K; k0 += 4 * kQtThreads) {
      uint32_t kk[4];
      int n[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool in = k0 + u * kQtThreads < K;
        kk[u] = in ? keys[k0 + u * kQtThreads] : 0u;
        n[u] = in ? knode[k0 + u * kQtThreads] : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) n[u] = rootCnt[n[u]];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + u * kQtThreads < K) {
          const int2 md = mA[n[u]];
          const int q = (key_x(kk[u]) >= md.x ? 1 : 0) + (key_y(kk[u]) >= md.y ? 2 : 0);
          if (kA[n[u]] > 1) atomicAdd(((int*)&cA[n[u]]) + q, 1);
          knode[k0 + u * kQtThreads] = (uint16_t)((n[u] << 2) | q);
        }
      }
    }
    int size = s_var[0];
    bool sorted_phase = false;
    lds_sync();
    if (dbg) dbg_init = __builtin_amdgcn_s_memtime() - t_begin;
    for (int round = 0; round < 64; ++round) {
      ph(-1);
      dbg_sorted += sorted_phase;
      const int per = (size + kQtThreads - 1) / kQtThreads;
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
        for (int c = tid; c < ncand; c += kQtThreads) {
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
        for (int i = tid; i < size; i += kQtThreads)
          if (!s_key[i]) rank[i] = -1;
        lds_sync();
        if (tid == 0) s_var[10] = 0;  // every thread has read the count (the next list's candidates count afresh)
        // split ranks: the prefix of ranks j with size + E_j < N, E_j = sum
        // of (children - 1) over the ranks before j (per-thread rank chunks)
        const int cper = (ncand + kQtThreads - 1) / kQtThreads;
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
          for (int j = tid; j < ncand; j += kQtThreads) {
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
      for (int k0 = tid; k0 < K; k0 += 4 * kQtThreads) {
        uint32_t kk[4];
        int pk[4], nn[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool in = k0 + u * kQtThreads < K;
          kk[u] = in ? keys[k0 + u * kQtThreads] : 0u;
          pk[u] = in ? knode[k0 + u * kQtThreads] : 0;
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
            if (k0 + u * kQtThreads < K) {
              const int q = (key_x(kk[u]) >= md[u].x ? 1 : 0) + (key_y(kk[u]) >= md[u].y ? 2 : 0);
              if (big[u] > 1) atomicAdd(((int*)&cB[nn[u]]) + q, 1);
              knode[k0 + u * kQtThreads] = (uint16_t)((nn[u] << 2) | q);
            }
          }
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (k0 + u * kQtThreads < K) knode[k0 + u * kQtThreads] = (uint16_t)(nn[u] << 2);
        }
      }
      // the breadth phase ends once one more full round would overshoot N (:1015)
      if (!finish && !sorted_phase && newSize + 3 * nExp > N) sorted_phase = true;
      if (!finish && sorted_phase)  // the next round's sort keys (the new list is kB, qB) and its candidate list
        for (int i = tid; i < newSize; i += kQtThreads) {
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
    const unsigned long long t_rounds = __builtin_amdgcn_s_memtime();
    // ---- keep the best key per node: max FAST score, first in key order
    for (int n = tid; n < size; n += kQtThreads) s_sort[n] = 0;
    lds_sync();
    for (int k = tid; k < K; k += kQtThreads)
      atomicMax(&s_sort[knode[k] >> 2],
                ((unsigned long long)key_score(keys[k]) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)k));
    lds_sync();
    for (int n = tid; n < size && n < g.kcap; n += kQtThreads) {
      const unsigned long long b = s_sort[n];
      if (b) out[n] = keys[0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull)];
      else atomicOr(err, 8);  // a node without keys: a broken list, reported instead of read past the keys
    }
    write_tail(size, t_rounds);
    return;
  }
  for (int k = tid; k < K; k += kQtThreads) {
    const int r = (int)__fdiv_rn((float)key_x(keys[k]), g.hX);  // vpIniNodes[kp.pt.x/hX]
    knode[k] = (uint16_t)r;
    atomicAdd(&rootCnt[r], 1);
  }
  __syncthreads();
  build_roots(false);
  __syncthreads();
  for (int k = tid; k < K; k += kQtThreads) knode[k] = (uint16_t)rootCnt[knode[k]];
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
    for (int n = tid; n < size; n += kQtThreads) {
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
    for (int k0 = tid; k0 < K; k0 += 4 * kQtThreads) {  // four keys in flight per thread
      int n[4], q[4];
      uint32_t kk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u * kQtThreads;
        n[u] = k < K ? knode[k] : 0;
        kk[u] = k < K ? keys[k] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int2 m = s_mid[n[u]];
        q[u] = (k0 + u * kQtThreads < K && kA[n[u]] > 1)
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
      for (int n = tid; n < size; n += kQtThreads)
        tA[n] = kA[n] > 1 ? ((nonempty(cc[n]) - 1) << 16) | 1 : 0;
      __syncthreads();
      block_scan_excl<kQtThreads>(tA, size, s_tmp);
      for (int n = tid; n < size; n += kQtThreads) {
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
      for (int n = tid; n < size; n += kQtThreads) {
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
      for (int i = tid; i < size; i += kQtThreads) {
        s_key[i] = kA[i] > 1
                       ? ((unsigned long long)kA[i] << 40) | ((unsigned long long)qA[i] << 16) | (unsigned long long)i
                       : 0ull;
        s_sort[i] = 0;
        rank[i] = -1;
      }
      if (tid == 0) s_var[3] = 0;
      __syncthreads();
      for (int i = tid; i < size; i += kQtThreads) {
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
      for (int j = tid; j < size; j += kQtThreads) {
        const unsigned long long key = s_sort[j];
        tA[j] = key ? nonempty(cc[(int)(key & 0xFFFF)]) - 1 : 0;
        if (key) atomicAdd(&s_var[3], 1);
      }
      __syncthreads();
      const int ncand = s_var[3];
      block_scan_excl<kQtThreads>(tA, ncand, s_tmp);
      for (int j = tid; j < ncand; j += kQtThreads) {
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
        for (int j = tid; j < ncand; j += kQtThreads) {
          const unsigned long long key = s_sort[j];
          if ((key >> 40) == sz) {
            atomicAdd(&s_var[7], 1);
            atomicAdd(&s_var[8], j < m ? nonempty(cc[(int)(key & 0xFFFF)]) : 1);
          }
        }
        if (tid == 0) s_var[6] += 1;
      }
      for (int j = tid; j < m; j += kQtThreads) tA[j] = nonempty(cc[ord[j]]);
      __syncthreads();
      const int T = block_scan_excl<kQtThreads>(tA, m, s_tmp);
      for (int n = tid; n < size; n += kQtThreads) tB[n] = rank[n] < 0 ? 1 : 0;
      __syncthreads();
      block_scan_excl<kQtThreads>(tB, size, s_tmp);
      if (tid == 0) s_var[5] = T;
      for (int n = tid; n < size; n += kQtThreads) {
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
    for (int k0 = tid; k0 < K; k0 += 4 * kQtThreads) {  // four keys in flight per thread
      int n[4], j[4], nn[4];
      uint32_t kk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u * kQtThreads;
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
        const int k = k0 + u * kQtThreads;
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
  const unsigned long long t_rounds = __builtin_amdgcn_s_memtime();
  // ---- keep the best key per node: max FAST score, first in node (= original) order
  const int size = s_var[0];
  for (int n = tid; n < size; n += kQtThreads) s_sort[n] = 0;
  __syncthreads();
  for (int k = tid; k < K; k += kQtThreads) {
    const unsigned long long v =
        ((unsigned long long)key_score(keys[k]) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)k);
    atomicMax(&s_sort[knode[k]], v);
  }
  __syncthreads();
  for (int n = tid; n < size && n < g.kcap; n += kQtThreads) {
    const unsigned long long b = s_sort[n];
    if (b) out[n] = keys[0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull)];
    else atomicOr(err, 8);  // a node without keys: a broken list, reported instead of read past the keys
  }
  write_tail(size, t_rounds);
}

size_t quadtree_lds_bytes(const ExtractParams& P) {
  auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t MN = P.maxnodes, SN = P.sortn;
  return r16(8 * SN) + 2 * r16(sizeof(QNode) * MN) + 4 * r16(4 * MN) + r16(16 * MN) + 2 * r16(4 * (MN + 1)) +
         2 * r16(4 * MN) + 2 * r16(4 * (P.max_cells_level + 1)) + r16(8 * MN) + r16(16 * MN) + r16(8 * MN) + 512 +
         2 * r16(64) + 2 * r16(4 * MN) +
         r16(4ull * P.kcap_lds) + r16(2ull * P.kcap_lds);
}

const void* quadtree_kernel_ptr(int big) {
  return big ? (const void*)quadtree_kernel<1024> : (const void*)quadtree_kernel<kQtThreads>;
}

int launch_quadtree(const ExtractParams& P, const ExtractBuffers& X, int batch, hipStream_t s) {
  static int* dbg = nullptr;  // diagnostics only: per-(frame, level) cycles and rounds (ORBX_QT_PROF=1)
  static const bool prof = getenv("ORBX_QT_PROF") && getenv("ORBX_QT_PROF")[0] == '1';
  const int nwg = P.L * batch;
  if (prof && !dbg) (void)hipMalloc(&dbg, (size_t)nwg * 64);
  if (P.qt_big)
    hipLaunchKernelGGL(quadtree_kernel<1024>, dim3(P.L, batch), dim3(1024), quadtree_lds_bytes(P), s, P,
                       X.cell_counts, X.slots, X.cells, X.qscratch, X.qnode_scratch, X.qkeys, X.qcounts, X.qties, X.err,
                       prof ? dbg : nullptr);
  else
    hipLaunchKernelGGL(quadtree_kernel<kQtThreads>, dim3(P.L, batch), dim3(kQtThreads), quadtree_lds_bytes(P), s, P,
                       X.cell_counts, X.slots, X.cells, X.qscratch, X.qnode_scratch, X.qkeys, X.qcounts, X.qties, X.err,
                       prof ? dbg : nullptr);
  if (prof) {
    std::vector<int> h((size_t)nwg * 16);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), dbg, h.size() * 4, hipMemcpyDeviceToHost);
    for (int l = 0; l < P.L; ++l) {
      double a[6] = {0};
      int mx = 0;
      for (int f = 0; f < batch; ++f)
        for (int k = 0; k < 6; ++k) {
          a[k] += h[(f * P.L + l) * 8 + k];
          if (k == 1) mx = std::max(mx, h[(f * P.L + l) * 8 + 1]);
        }
      double q[8] = {0};
      for (int f = 0; f < batch; ++f)
        for (int k = 0; k < 8; ++k) q[k] += h[(size_t)nwg * 8 + (f * P.L + l) * 8 + k];
      double sc = 0, ga = 0;
      for (int f = 0; f < batch; ++f) {
        sc += h[(f * P.L + l) * 8 + 6];
        ga += h[(f * P.L + l) * 8 + 7];
      }
      fprintf(stderr, "quadtree L%d: avg cycles rounds %.0f total %.0f (max %d) rounds %.1f sorted %.1f K %.0f out %.0f"
              " | scan %.0f gather %.0f roots %.0f built %.0f init %.0f | count %.0f order %.0f sortorder %.0f table %.0f"
              " rehome %.0f\n",
              l, a[0] / batch, a[1] / batch, mx, a[2] / batch, a[3] / batch, a[4] / batch, a[5] / batch,
              sc / batch, ga / batch, q[6] / batch, q[7] / batch, q[5] / batch, q[0] / batch, q[1] / batch, q[4] / batch, q[2] / batch, q[3] / batch);
    }
  }
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
