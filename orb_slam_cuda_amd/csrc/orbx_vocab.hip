// orbx_vocab.hip — DBoW2 vocabulary transform on the GPU (Frame::ComputeBoW).
//
// Reference: Frame::ComputeBoW (src/Frame.cc:394-401) calls
// TemplatedVocabulary::transform(descriptors, mBowVec, mFeatVec, 4)
// (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1192), which walks every
// descriptor down the vocabulary tree (:1214-1256: at each level the child with
// the smallest Hamming distance, first one on ties, until a node without
// children), adds the leaf's weight to the BowVector (std::map word -> value,
// BowVector.cpp:34-58) and the feature index to the FeatureVector entry of its
// ancestor at level L - levelsup (FeatureVector.cpp:31-45), then normalises
// the BowVector (BowVector.cpp:62-84) as the scoring type requires.
//
// Device layout: the tree is renumbered breadth-first so the children of a
// node are contiguous: child[n] = {first, count}; desc[n] = 32 B; word[n],
// weight[n] (double), orig[n] = the node's id in the vocabulary file (the
// NodeId the FeatureVector carries).
//
// Kernels:
//   voc_descend_kernel<GL>  GL lanes per descriptor (8 when k <= 16, else 32):
//                           at each level lane c takes child c (c += GL), the
//                           (dist << 16 | c) minimum over the group picks the
//                           child; one 32-byte gather per lane per level.
//   voc_assemble_kernel     one workgroup per frame: bitonic sort of
//                           (node << 32 | i) and (word << 32 | i) keys in LDS,
//                           run heads by a block scan, each word's value summed
//                           in feature order by the run's first thread, the
//                           norm summed in ascending word order by one thread
//                           (the order std::map iterates), so every double
//                           rounds as in the reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "orbx_device.cuh"
#include "orbx_internal.h"

namespace orbx {

struct VocDev {
  const int2* child;
  const uint4* desc;
  const uint32_t* word;
  const double* weight;
  const uint32_t* orig;
};

template <int GL>
__global__ __launch_bounds__(256) void voc_descend_kernel(VocDev V, const uint8_t* __restrict__ desc, size_t pitch,
                                                          const int* __restrict__ d_n, int frames, int cap,
                                                          int nid_level,
                                                          uint32_t* __restrict__ word_out,
                                                          uint32_t* __restrict__ nid_out,
                                                          double* __restrict__ w_out) {
  const int sub = threadIdx.x % GL;
  const long long gid = ((long long)blockIdx.x * 256 + threadIdx.x) / GL;
  const int f = (int)(gid / cap), i = (int)(gid % cap);
  if (f >= frames) return;
  const int n = d_n[f];
  if (i >= n) return;  // uniform over the group
  const uint4* q = (const uint4*)(desc + (size_t)f * pitch + (size_t)i * 32);
  const uint4 q0 = q[0], q1 = q[1];
  int node = 0, level = 0;
  uint32_t nid = 0;
  bool nid_set = nid_level <= 0;
  // group minimum on DPP (quad, half-row, row) for GL <= 16, no LDS round trip
  auto group_min = [](int v) {
    if (GL <= 16) {
      v = min(v, dpp_i<kDppQuad1032>(INT_MAX, v));
      v = min(v, dpp_i<kDppQuad2301>(INT_MAX, v));
      if (GL > 4) v = min(v, dpp_i<kDppHalfMirror>(INT_MAX, v));
      if (GL > 8) v = min(v, dpp_i<kDppMirror>(INT_MAX, v));
    } else {
#pragma unroll
      for (int o = GL / 2; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, GL));
    }
    return v;
  };
  // each candidate's own {first child, count} is loaded beside its descriptor,
  // and the winner's handed over by two more group minima, so a level costs
  // one dependent global round trip instead of two
  int2 cf = V.child[0];
  while (cf.y != 0) {  // isLeaf(): no children
    ++level;
    int mine = INT_MAX;
    int2 mcf = make_int2(0, 0);
    for (int c = sub; c < cf.y; c += GL) {
      const uint4 a = V.desc[2 * (cf.x + c)], b = V.desc[2 * (cf.x + c) + 1];
      const int2 nc = V.child[cf.x + c];
      const int d = __popc(a.x ^ q0.x) + __popc(a.y ^ q0.y) + __popc(a.z ^ q0.z) + __popc(a.w ^ q0.w) +
                    __popc(b.x ^ q1.x) + __popc(b.y ^ q1.y) + __popc(b.z ^ q1.z) + __popc(b.w ^ q1.w);
      const int key = (d << 16) | c;
      if (key < mine) {
        mine = key;
        mcf = nc;
      }
    }
    const int best = group_min(mine);  // keys are distinct: exactly one lane holds the winner
    node = cf.x + (best & 0xFFFF);
    const bool win = mine == best;
    cf = make_int2(group_min(win ? mcf.x : INT_MAX), group_min(win ? mcf.y : INT_MAX));
    if (level == nid_level) {
      nid = V.orig[node];
      nid_set = true;
    }
  }
  if (!nid_set) nid = V.orig[node];  // a leaf above level L - levelsup (see oracle/orb_vocab.cpp)
  if (sub == 0) {
    const size_t o = (size_t)f * cap + i;
    word_out[o] = V.word[node];
    nid_out[o] = nid;
    w_out[o] = V.weight[node];
  }
}

constexpr int kAsThreads = 512;

// ascending bitonic sort of S (power of two) 64-bit keys in LDS
__device__ void bitonic_sort64(uint64_t* s, int S) {
  for (int k = 2; k <= S; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < S / 2; t += kAsThreads) {
        const int i = 2 * t - (t & (j - 1));  // lower index of the pair
        const int l = i + j;
        const uint64_t a = s[i], b = s[l];
        const bool up = (i & k) == 0;
        if ((a > b) == up) {
          s[i] = b;
          s[l] = a;
        }
      }
      __syncthreads();
    }
  }
}

// The same sort for S = 4 * kAsThreads keys held in registers, 4 per thread
// (thread t: keys 4t .. 4t+3): partners 1 or 2 apart are in the thread,
// partners 4 .. 128 apart in the same wave (64-bit lane exchange), and only
// the stages 256 .. S/2 apart go through LDS with a barrier (6 of the 66 for
// S = 2048, instead of a barrier per stage).
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ void bitonic_sort64_reg(uint64_t* s) {
  constexpr int S = 4 * kAsThreads;
  const int t = threadIdx.x;
  uint64_t v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = s[4 * t + q];
  for (int k = 2; k <= S; k <<= 1) {
    int j = k >> 1;
    if (j >= 4 * 64) {  // partners in other waves: through LDS
#pragma unroll
      for (int q = 0; q < 4; ++q) s[4 * t + q] = v[q];
      __syncthreads();
      for (; j >= 4 * 64; j >>= 1) {
        for (int u = t; u < S / 2; u += kAsThreads) {
          const int i = 2 * u - (u & (j - 1));
          const int l = i + j;
          const uint64_t a = s[i], b = s[l];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            s[i] = b;
            s[l] = a;
          }
        }
        __syncthreads();
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = s[4 * t + q];
    }
    for (; j >= 4; j >>= 1) {  // partner thread t ^ (j / 4), same wave
      const bool lower = (t & (j >> 2)) == 0, up = ((4 * t) & k) == 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint64_t b = shfl_xor64(v[q], j >> 2);
        v[q] = (up == lower) ? (v[q] < b ? v[q] : b) : (v[q] < b ? b : v[q]);
      }
    }
    for (; j >= 1; j >>= 1) {  // partner in the thread
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q & j) continue;
        const bool up = ((4 * t + q) & k) == 0;
        const uint64_t a = v[q], b = v[q | j];
        const bool sw = (a > b) == up;
        v[q] = sw ? b : a;
        v[q | j] = sw ? a : b;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) s[4 * t + q] = v[q];
  __syncthreads();
}

// run heads of the sorted valid keys (high 32 bits change): returns the number
// of runs; s_head[t] = run index of a head, -1 otherwise. Keys == ~0 are invalid
// and sorted last.
__device__ int mark_runs(const uint64_t* s, int S, int* s_head, int* s_tmp) {
  const int tid = threadIdx.x;
  const int per = S / kAsThreads > 0 ? S / kAsThreads : 1;
  const int b = min(tid * per, S), e = min(b + per, S);
  int cnt = 0;
  for (int t = b; t < e; ++t) {
    const bool h = s[t] != ~0ull && (t == 0 || (s[t] >> 32) != (s[t - 1] >> 32));
    cnt += h;
  }
  const int lane = tid & 63, w = tid >> 6;
  const int x = wave_incl_scan_dpp(cnt);
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  int pre = 0, tot = 0;
  for (int i = 0; i < kAsThreads / 64; ++i) {
    if (i < w) pre += s_tmp[i];
    tot += s_tmp[i];
  }
  int r = pre + x - cnt;
  for (int t = b; t < e; ++t) {
    const bool h = s[t] != ~0ull && (t == 0 || (s[t] >> 32) != (s[t - 1] >> 32));
    s_head[t] = h ? r++ : -1;
  }
  __syncthreads();
  return tot;
}

__global__ __launch_bounds__(kAsThreads) void voc_assemble_kernel(
    int cap, int S, const int* __restrict__ d_n, const uint32_t* __restrict__ word, const uint32_t* __restrict__ nid,
    const double* __restrict__ w, int tf, int must, int l2, int nwords, uint32_t* __restrict__ bow_words,
    double* __restrict__ bow_values, int* __restrict__ bow_n, uint32_t* __restrict__ fv_nodes,
    int* __restrict__ fv_off, int* __restrict__ fv_idx, int* __restrict__ fv_n, int stop) {
  extern __shared__ __attribute__((aligned(16))) uint64_t s_key[];  // [S]
  int* s_head = (int*)(s_key + S);                                   // [S]
  __shared__ int s_tmp[kAsThreads / 64];
  __shared__ int s_m;
  __shared__ double s_norm;
  const int f = blockIdx.x, tid = threadIdx.x;
  const int n = nwords > 0 ? d_n[f] : 0;  // if(empty()) return (:1131-1134)
  const size_t base = (size_t)f * cap;

  // blockIdx.y = 0: the FeatureVector, 1: the BowVector (independent halves,
  // each in its own workgroup so that the two run side by side)
  if (blockIdx.y == 0) {
    // ---- FeatureVector: (node, feature) ascending = std::map order, push_back order
    if (tid == 0) s_m = 0;
    for (int i = tid; i < S; i += kAsThreads)
      s_key[i] = (i < n && w[base + i] > 0) ? ((uint64_t)nid[base + i] << 32) | (uint32_t)i : ~0ull;
    __syncthreads();
    if (S == 4 * kAsThreads) bitonic_sort64_reg(s_key); else bitonic_sort64(s_key, S);
    int runs = mark_runs(s_key, S, s_head, s_tmp);
    for (int t = tid; t < S; t += kAsThreads) {
      const uint64_t k = s_key[t];
      if (k == ~0ull) {
        if (t == 0 || s_key[t - 1] != ~0ull) s_m = t;  // number of valid features
        continue;
      }
      fv_idx[base + t] = (int)(uint32_t)k;
      const int r = s_head[t];
      if (r >= 0) {
        fv_nodes[base + r] = (uint32_t)(k >> 32);
        fv_off[(size_t)f * (cap + 1) + r] = t;
      }
    }
    __syncthreads();
    const int m = (s_key[S - 1] != ~0ull) ? S : s_m;
    if (tid == 0) {
      fv_off[(size_t)f * (cap + 1) + runs] = m;
      fv_n[f] = runs;
    }
    __syncthreads();
    return;
  }
  if (stop == 2) return;  // diagnostics (ORBX_VOC_STOP=2): FeatureVector only

  // ---- BowVector: (word, feature) ascending; value = weights added in feature order
  for (int i = tid; i < S; i += kAsThreads)
    s_key[i] = (i < n && w[base + i] > 0) ? ((uint64_t)word[base + i] << 32) | (uint32_t)i : ~0ull;
  __syncthreads();
  if (S == 4 * kAsThreads) bitonic_sort64_reg(s_key); else bitonic_sort64(s_key, S);
  const int runs = mark_runs(s_key, S, s_head, s_tmp);
  double* s_val = (double*)s_key;  // values overwrite the keys after they are read below
  double v_mine[16];  // S <= 8192 = 16 keys per thread
  int r_mine[16], nm = 0;
  for (int t = tid; t < S; t += kAsThreads) {
    const int r = s_head[t];
    if (r < 0) continue;
    const uint64_t k0 = s_key[t];
    double v = w[base + (uint32_t)k0];
    if (tf)  // addWeight: += in insertion (feature) order
      for (int u = t + 1; u < S && s_key[u] != ~0ull && (s_key[u] >> 32) == (k0 >> 32); ++u)
        v += w[base + (uint32_t)s_key[u]];
    // (IDF / BINARY: addIfNotExist keeps the first feature's weight)
    bow_words[base + r] = (uint32_t)(k0 >> 32);
    v_mine[nm] = v;
    r_mine[nm++] = r;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q)
    if (q < nm) s_val[r_mine[q]] = v_mine[q];
  __syncthreads();
  if (tf && runs > 0 && !must) {
    const double nd = (double)runs;
    for (int r = tid; r < runs; r += kAsThreads) s_val[r] /= nd;
    __syncthreads();
  }
  if (stop == 3) return;  // diagnostics (ORBX_VOC_STOP=3): no normalisation
  if (must) {
    if (tid == 0) {
      double norm = 0.0;
      if (!l2)
        for (int r = 0; r < runs; ++r) norm += fabs(s_val[r]);
      else {
        for (int r = 0; r < runs; ++r) norm += s_val[r] * s_val[r];
        norm = sqrt(norm);
      }
      s_norm = norm;
    }
    __syncthreads();
    const double norm = s_norm;
    if (norm > 0.0)
      for (int r = tid; r < runs; r += kAsThreads) s_val[r] /= norm;
    __syncthreads();
  }
  for (int r = tid; r < runs; r += kAsThreads) bow_values[base + r] = s_val[r];
  if (tid == 0) bow_n[f] = runs;
}

}  // namespace orbx

// ============================================================ C ABI (vocabulary)
using namespace orbx;

namespace {
thread_local std::string g_verr;
int vfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_verr = buf;
  return code;
}
}  // namespace

#define VHIP(expr)                                                                             \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return vfail(ORBX_EDEVICE, "%s: %s", #expr, hipGetErrorString(e_));  \
  } while (0)

struct orbv_vocabulary {
  int device = 0, k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0, n_words = 0, max_children = 0;
  int2* child = nullptr;
  uint4* desc = nullptr;
  uint32_t* word = nullptr;
  double* weight = nullptr;
  uint32_t* orig = nullptr;
  // per-feature workspace and staging of the synchronous entry point
  void* ws = nullptr;
  size_t ws_bytes = 0;
  hipStream_t stream = nullptr;
};

static int ws_reserve(orbv_vocabulary* v, size_t bytes) {
  if (v->ws_bytes >= bytes) return ORBX_OK;
  if (v->ws) (void)hipFree(v->ws);
  v->ws = nullptr;
  v->ws_bytes = 0;
  VHIP(hipMalloc(&v->ws, bytes));
  v->ws_bytes = bytes;
  return ORBX_OK;
}

extern "C" {

const char* orbv_last_error(void) { return g_verr.c_str(); }

int orbv_destroy(orbv_handle v) {
  if (!v) return ORBX_OK;
  (void)hipSetDevice(v->device);
  if (v->stream) (void)hipStreamSynchronize(v->stream);
  for (void* p : {(void*)v->child, (void*)v->desc, (void*)v->word, (void*)v->weight, (void*)v->orig, v->ws})
    if (p) (void)hipFree(p);
  if (v->stream) (void)hipStreamDestroy(v->stream);
  delete v;
  return ORBX_OK;
}

int orbv_create(int k, int L, int scoring, int weighting, int n_nodes, const int* parent, const uint8_t* is_leaf,
                const uint8_t* desc, const double* weight, int device, orbv_handle* out) {
  if (!out || n_nodes < 1 || (n_nodes > 1 && (!parent || !is_leaf || !desc || !weight)))
    return vfail(ORBX_EINVAL, "bad argument");
  if (k < 0 || L < 1 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3)
    return vfail(ORBX_EINVAL, "bad vocabulary header (k %d, L %d, scoring %d, weighting %d)", k, L, scoring,
                 weighting);
  // children in file order (loadFromTextFile :1389-1390); node 0 is the root
  std::vector<std::vector<int>> ch(n_nodes);
  for (int i = 1; i < n_nodes; ++i) {
    if (parent[i] < 0 || parent[i] >= i) return vfail(ORBX_EINVAL, "node %d: parent %d is not an earlier node", i, parent[i]);
    ch[parent[i]].push_back(i);
  }
  // breadth-first renumbering: the children of a node get consecutive ids
  std::vector<int> order{0}, newid(n_nodes, 0);
  order.reserve(n_nodes);
  for (size_t h = 0; h < order.size(); ++h)
    for (int c : ch[order[h]]) {
      newid[c] = (int)order.size();
      order.push_back(c);
    }
  std::vector<int2> hchild(n_nodes);
  std::vector<uint8_t> hdesc((size_t)n_nodes * 32, 0);
  std::vector<uint32_t> hword(n_nodes, 0), horig(n_nodes);
  std::vector<double> hweight(n_nodes, 0.0);
  std::vector<uint32_t> wid(n_nodes, 0);
  int nw = 0, maxc = 0;
  for (int i = 1; i < n_nodes; ++i)
    if (is_leaf[i]) wid[i] = (uint32_t)nw++;  // m_words in file order (:1405-1412)
  for (int j = 0; j < n_nodes; ++j) {
    const int o = order[j];
    hchild[j] = make_int2(ch[o].empty() ? 0 : newid[ch[o][0]], (int)ch[o].size());
    maxc = std::max(maxc, (int)ch[o].size());
    if (o > 0) {
      memcpy(&hdesc[(size_t)j * 32], desc + (size_t)o * 32, 32);
      hweight[j] = weight[o];
    }
    hword[j] = wid[o];  // Node(): word_id(0) for nodes that are not words
    horig[j] = (uint32_t)o;
  }
  if (maxc > 65535) return vfail(ORBX_EINVAL, "a node has more than 65535 children");
  if (hipSetDevice(device) != hipSuccess) return vfail(ORBX_EDEVICE, "no device %d", device);
  orbv_vocabulary* v = new orbv_vocabulary();
  v->device = device;
  v->k = k;
  v->L = L;
  v->scoring = scoring;
  v->weighting = weighting;
  v->n_nodes = n_nodes;
  v->n_words = nw;
  v->max_children = maxc;
  if (hipMalloc(&v->child, n_nodes * sizeof(int2)) != hipSuccess ||
      hipMalloc(&v->desc, (size_t)n_nodes * 32) != hipSuccess ||
      hipMalloc(&v->word, n_nodes * 4) != hipSuccess || hipMalloc(&v->weight, n_nodes * 8) != hipSuccess ||
      hipMalloc(&v->orig, n_nodes * 4) != hipSuccess) {
    orbv_destroy(v);
    return vfail(ORBX_ENOMEM, "vocabulary allocation failed (%d nodes)", n_nodes);
  }
  if (hipMemcpy(v->child, hchild.data(), n_nodes * sizeof(int2), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(v->desc, hdesc.data(), (size_t)n_nodes * 32, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(v->word, hword.data(), n_nodes * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(v->weight, hweight.data(), n_nodes * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(v->orig, horig.data(), n_nodes * 4, hipMemcpyHostToDevice) != hipSuccess) {
    orbv_destroy(v);
    return vfail(ORBX_EDEVICE, "vocabulary upload failed");
  }
  *out = v;
  return ORBX_OK;
}

int orbv_load_text(const char* path, int device, orbv_handle* out) {
  // TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1418)
  if (!path || !out) return vfail(ORBX_EINVAL, "bad argument");
  FILE* fp = fopen(path, "rb");
  if (!fp) return vfail(ORBX_EINVAL, "cannot open %s", path);
  std::vector<char> buf;
  {
    fseek(fp, 0, SEEK_END);
    const long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    buf.resize(sz > 0 ? (size_t)sz + 1 : 1);
    const size_t got = sz > 0 ? fread(buf.data(), 1, (size_t)sz, fp) : 0;
    buf[got] = 0;
  }
  fclose(fp);
  char* p = buf.data();
  auto line_end = [](char* s) {
    while (*s && *s != '\n') ++s;
    return s;
  };
  char* e = line_end(p);
  const char save = *e;
  *e = 0;
  int k = 0, L = 0, n1 = 0, n2 = 0;
  if (sscanf(p, "%d %d %d %d", &k, &L, &n1, &n2) != 4 || k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 ||
      n1 > 5 || n2 < 0 || n2 > 3)
    return vfail(ORBX_EINVAL, "%s: not a vocabulary text file (header)", path);
  *e = save;
  p = *e ? e + 1 : e;
  std::vector<int> parent{0};
  std::vector<uint8_t> leaf{0}, desc(32, 0);
  std::vector<double> weight{0.0};
  int lineno = 1;
  while (*p) {
    e = line_end(p);
    const char sv = *e;
    *e = 0;
    ++lineno;
    char* s = p;
    while (*s == ' ' || *s == '\t' || *s == '\r') ++s;
    if (*s) {  // lines without tokens are skipped (see oracle/orb_vocab.cpp)
      char* q = s;
      const long pid = strtol(q, &q, 10);
      const long isl = strtol(q, &q, 10);
      const int nid = (int)parent.size();
      if (pid < 0 || pid >= nid) return vfail(ORBX_EINVAL, "%s:%d: bad parent %ld", path, lineno, pid);
      parent.push_back((int)pid);
      leaf.push_back(isl > 0);
      for (int i = 0; i < 32; ++i) desc.push_back((uint8_t)strtol(q, &q, 10));  // FORB::fromString
      weight.push_back(strtod(q, &q));
    }
    *e = sv;
    p = *e ? e + 1 : e;
  }
  return orbv_create(k, L, n1, n2, (int)parent.size(), parent.data(), leaf.data(), desc.data(), weight.data(),
                     device, out);
}

int orbv_info(orbv_handle v, int* k, int* L, int* scoring, int* weighting, int* n_nodes, int* n_words) {
  if (!v) return vfail(ORBX_EINVAL, "null handle");
  if (k) *k = v->k;
  if (L) *L = v->L;
  if (scoring) *scoring = v->scoring;
  if (weighting) *weighting = v->weighting;
  if (n_nodes) *n_nodes = v->n_nodes;
  if (n_words) *n_words = v->n_words;
  return ORBX_OK;
}

int orbv_transform_batch(orbv_handle v, const uint8_t* d_desc, size_t desc_pitch, const int* d_n, int frames,
                         int cap, int levelsup, uint32_t* d_bow_words, double* d_bow_values, int* d_bow_n,
                         uint32_t* d_fv_nodes, int* d_fv_off, int* d_fv_idx, int* d_fv_n, uint32_t* d_word_ids,
                         uint32_t* d_node_ids, double* d_weights, void* stream) {
  if (!v || !d_desc || !d_n || frames < 1 || cap < 1 || !d_bow_words || !d_bow_values || !d_bow_n || !d_fv_nodes ||
      !d_fv_off || !d_fv_idx || !d_fv_n)
    return vfail(ORBX_EINVAL, "bad argument");
  if (cap > 8192) return vfail(ORBX_ECAPACITY, "cap %d > 8192 features per frame", cap);
  if (desc_pitch < (size_t)cap * 32 || (desc_pitch & 15)) return vfail(ORBX_EINVAL, "bad descriptor pitch");
  VHIP(hipSetDevice(v->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t nf = (size_t)frames * cap;
  if (!d_word_ids || !d_node_ids || !d_weights) {
    int rc;
    if ((rc = ws_reserve(v, nf * 16))) return rc;
    d_weights = (double*)v->ws;
    d_word_ids = (uint32_t*)(d_weights + nf);
    d_node_ids = d_word_ids + nf;
  }
  const VocDev V{v->child, v->desc, v->word, v->weight, v->orig};
  const int nid_level = v->L - levelsup;
  if (v->n_words > 0) {
    static const int gl_env = getenv("ORBX_VOC_GL") ? atoi(getenv("ORBX_VOC_GL")) : 0;  // A/B
    const long long groups = (long long)nf;
    if (v->max_children <= 16 && gl_env != 16 && gl_env != 4) {
      // 8 lanes per descriptor: k <= 16 children take one or two passes, and a
      // wave serves 8 descriptors instead of 4 (16 lanes left 6 of them idle at k = 10)
      hipLaunchKernelGGL(voc_descend_kernel<8>, dim3((unsigned)((groups * 8 + 255) / 256)), dim3(256), 0, st, V,
                         d_desc, desc_pitch, d_n, frames, cap, nid_level, d_word_ids, d_node_ids, d_weights);
    } else if (v->max_children <= 16 && gl_env == 4) {
      hipLaunchKernelGGL(voc_descend_kernel<4>, dim3((unsigned)((groups * 4 + 255) / 256)), dim3(256), 0, st, V,
                         d_desc, desc_pitch, d_n, frames, cap, nid_level, d_word_ids, d_node_ids, d_weights);
    } else if (v->max_children <= 16) {
      hipLaunchKernelGGL(voc_descend_kernel<16>, dim3((unsigned)((groups * 16 + 255) / 256)), dim3(256), 0, st, V,
                         d_desc, desc_pitch, d_n, frames, cap, nid_level, d_word_ids, d_node_ids, d_weights);
    } else {
      hipLaunchKernelGGL(voc_descend_kernel<32>, dim3((unsigned)((groups * 32 + 255) / 256)), dim3(256), 0, st, V,
                         d_desc, desc_pitch, d_n, frames, cap, nid_level, d_word_ids, d_node_ids, d_weights);
    }
    VHIP(hipGetLastError());
  }
  int voc_stop = 0;
#ifdef ORBX_DIAG  // diagnostics builds only: 1 = descend only, 2 = FeatureVector only, 3 = no normalisation
  if (const char* e = getenv("ORBX_VOC_STOP")) voc_stop = atoi(e);
#endif
  if (voc_stop == 1) return ORBX_OK;
  int S = 1;
  while (S < cap) S <<= 1;
  const size_t lds = (size_t)S * 12;
  if (raise_lds_limit((const void*)voc_assemble_kernel, lds))
    return vfail(ORBX_EDEVICE, "hipFuncSetAttribute(voc_assemble_kernel): %s", hipGetErrorString(hipGetLastError()));
  int l1 = v->scoring != 1;
  const int must = v->scoring != 5;
  const int tf = v->weighting == 0 || v->weighting == 1;
  hipLaunchKernelGGL(voc_assemble_kernel, dim3(frames, 2), dim3(kAsThreads), lds, st, cap, S, d_n, d_word_ids, d_node_ids,
                     d_weights, tf, must, !l1, v->n_words, d_bow_words, d_bow_values, d_bow_n, d_fv_nodes, d_fv_off,
                     d_fv_idx, d_fv_n,
                     voc_stop);
  VHIP(hipGetLastError());
  return ORBX_OK;
}

int orbv_transform(orbv_handle v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words, double* bow_values,
                   int* bow_n, uint32_t* fv_nodes, int* fv_off, int* fv_idx, int* fv_n, uint32_t* word_ids,
                   uint32_t* node_ids, double* weights) {
  if (!v || n < 0 || (n && !desc) || !bow_n || !fv_n || !fv_off || (n && (!bow_words || !bow_values || !fv_nodes || !fv_idx)))
    return vfail(ORBX_EINVAL, "bad argument");
  if (n > 8192) return vfail(ORBX_ECAPACITY, "more than 8192 features");
  VHIP(hipSetDevice(v->device));
  const int cap = std::max(n, 1);
  // staging: desc | n | bow words | bow values | fv nodes | fv off | fv idx | counts | per-feature
  const size_t dpitch = ((size_t)cap * 32 + 15) & ~(size_t)15;
  std::vector<size_t> sz = {dpitch, 16, (size_t)cap * 4, (size_t)cap * 8, (size_t)cap * 4, (size_t)(cap + 1) * 4,
                            (size_t)cap * 4, 16, (size_t)cap * 4, (size_t)cap * 4, (size_t)cap * 8};
  size_t tot = 0;
  std::vector<size_t> off;
  for (size_t s : sz) {
    off.push_back(tot);
    tot += (s + 255) & ~(size_t)255;
  }
  void* stage = nullptr;
  VHIP(hipMalloc(&stage, tot));
  uint8_t* b = (uint8_t*)stage;
  auto at = [&](int i) { return (void*)(b + off[i]); };
  if (!v->stream) VHIP(hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking));
  hipStream_t st = v->stream;
  int rc = ORBX_OK;
  do {
    if (n && hipMemcpyAsync(at(0), desc, (size_t)n * 32, hipMemcpyHostToDevice, st) != hipSuccess) { rc = vfail(ORBX_EDEVICE, "upload"); break; }
    if (hipMemcpyAsync(at(1), &n, 4, hipMemcpyHostToDevice, st) != hipSuccess) { rc = vfail(ORBX_EDEVICE, "upload"); break; }
    int* cnt = (int*)at(7);
    rc = orbv_transform_batch(v, (const uint8_t*)at(0), dpitch, (const int*)at(1), 1, cap, levelsup, (uint32_t*)at(2),
                              (double*)at(3), cnt, (uint32_t*)at(4), (int*)at(5), (int*)at(6), cnt + 1,
                              (uint32_t*)at(8), (uint32_t*)at(9), (double*)at(10), st);
    if (rc) break;
    int hc[2] = {0, 0};
    if (hipMemcpyAsync(hc, cnt, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) { rc = vfail(ORBX_EDEVICE, "transform failed"); break; }
    *bow_n = hc[0];
    *fv_n = hc[1];
    int nfeat = 0;
    if (hipMemcpyAsync(fv_off, at(5), (size_t)(hc[1] + 1) * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) { rc = vfail(ORBX_EDEVICE, "download"); break; }
    nfeat = fv_off[hc[1]];
    if ((hc[0] && (hipMemcpyAsync(bow_words, at(2), (size_t)hc[0] * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                   hipMemcpyAsync(bow_values, at(3), (size_t)hc[0] * 8, hipMemcpyDeviceToHost, st) != hipSuccess)) ||
        (hc[1] && hipMemcpyAsync(fv_nodes, at(4), (size_t)hc[1] * 4, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        (nfeat && hipMemcpyAsync(fv_idx, at(6), (size_t)nfeat * 4, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        (n && word_ids && hipMemcpyAsync(word_ids, at(8), (size_t)n * 4, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        (n && node_ids && hipMemcpyAsync(node_ids, at(9), (size_t)n * 4, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        (n && weights && hipMemcpyAsync(weights, at(10), (size_t)n * 8, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess) { rc = vfail(ORBX_EDEVICE, "download"); break; }
  } while (0);
  (void)hipFree(stage);
  return rc;
}

}  // extern "C"
