// orbx_host.hip — host plan + C ABI of the extractor (include/orbx_c.h).
//
// The constructor arithmetic of ORBextractor (src/ORBextractor.cc:496-560)
// and the per-level geometry of ComputePyramid / ComputeKeyPointsOctTree /
// DistributeOctTree are evaluated once per (config, frame size) on the host
// in the same float arithmetic as the reference, and shipped to the kernels
// as tables: resize coefficients, the FAST cell list with its slot ranges,
// quadtree roots. Everything per frame runs on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cfloat>
#include <cstdarg>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "orbx_internal.h"
#include "orbx_sincosf.h"

namespace orbx {

// Rectangle copy by the compute units (orbx_copy2d_kernel_async): a thread per
// 16-byte destination chunk, grid-strided; the source may be pinned host
// memory read over the link. A row's last chunk is clipped to its width.
__global__ __launch_bounds__(256) void copy2d_kernel(uint8_t* __restrict__ d, size_t dp, const uint8_t* __restrict__ s,
                                                     size_t sp, size_t w, size_t rows) {
  const size_t cpr = (w + 15) / 16, total = cpr * rows;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t r = i / cpr, c = (i - r * cpr) * 16;
    const uint8_t* src = s + r * sp + c;
    uint8_t* dst = d + r * dp + c;
    if (c + 16 <= w) {
      *(uint4*)dst = *(const uint4*)src;  // unaligned source rows: the memory path takes unaligned dwordx4
    } else {
      for (size_t k = 0; k < 16 && c + k < w; ++k) dst[k] = src[k];
    }
  }
}
size_t quadtree_lds_bytes(const ExtractParams& P);
size_t quadtree_legacy_lds_bytes(const ExtractParams& P);
size_t quadtree_sorted_lds_bytes(const ExtractParams& P, int big);
int quadtree_sorted_ownmax(const ExtractParams& P, int big, size_t budget);
extern const void* quadtree_kernel_ptr(const ExtractParams& P);
size_t pyr_band_lds_bytes(const ExtractParams& P);
void blur_tile_dims(int small, int* tw, int* th);
extern const void* pyr_band_kernel_ptr();
extern int pyr_band_occupancy(size_t lds);
}  // namespace orbx

using namespace orbx;

// offset of the descriptors in orbx_extract's output block (16-byte aligned
// for orient_brief's 16-byte stores)
static size_t out_desc_off(int cap_frame) { return (16 + (size_t)cap_frame * sizeof(orbx_kp) + 15) & ~(size_t)15; }

static thread_local std::string g_err;
static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define HIP_OK(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(ORBX_EDEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------ plan
namespace {

inline int cv_round(float v) { return (int)lrintf(v); }
inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
inline short sat_short(int v) { return (short)std::min(std::max(v, (int)SHRT_MIN), (int)SHRT_MAX); }

struct DeviceBuf {
  void* p = nullptr;
  size_t n = 0;
  ~DeviceBuf() { if (p) (void)hipFree(p); }
  int alloc(size_t bytes) {
    if (p) { (void)hipFree(p); p = nullptr; }
    n = bytes;
    if (!bytes) return ORBX_OK;
    if (hipMalloc(&p, bytes) != hipSuccess) return fail(ORBX_ENOMEM, "hipMalloc(%zu) failed", bytes);
    return ORBX_OK;
  }
  template <class T> T* as() const { return (T*)p; }
};

struct Plan {
  int W = 0, H = 0, B = 0;
  ExtractParams P{};
  std::vector<CellGeom> cells;
  std::vector<int2> rtab;
  DeviceBuf pyr, blur, rtab_d, cells_d, umax_d, slots, cell_counts, qkeys, qcounts, qties, qscratch, qnscratch,
      err;
};

}  // namespace

struct orbx_extractor {
  orbx_config cfg{};
  std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
  std::vector<int> nfeat;
  int umax[16];
  Plan plan;
  hipStream_t stream = nullptr;
  // staging for the synchronous API: device buffers, pinned host staging and
  // the captured H2D -> 5 kernels -> D2H chain of a one-frame call
  // orbx_extract's device output block, laid out as h_out so that one copy
  // brings back the count, the keypoints and the descriptors (out_desc_off)
  DeviceBuf d_in, d_out;
  void* h_in = nullptr;   // pinned: the image, rows at the device pitch
  void* h_out = nullptr;  // pinned: {count, status, -, -} + cap keypoints + (16-B aligned) cap descriptors
  size_t h_in_bytes = 0, h_out_bytes = 0;
  hipGraphExec_t graph = nullptr;
  int graph_w = 0, graph_h = 0;
  bool graph_hp = false;  // the graph holds the host-pyramid copy branch
  bool last_single = false;  // the last extraction was orbx_extract (outputs in d_out)
  bool last_empty = false;   // ... of an empty image (no outputs, src/ORBextractor.cc:1542-1543)
  int warm_w = 0, warm_h = 0;  // size of the last plain (uncaptured) call: capture from the next one
  int last_batch = 0;
  const uint8_t* last_frames = nullptr;
  size_t last_fpitch = 0, last_rstride = 0;
  bool timing = false;
  hipEvent_t ev[6] = {};
  void* user_ev[ORBX_STAGE_EVENTS] = {};
  bool has_user_ev = false;
  WsOrder ws;  // stream order of the plan buffers (pyramid, blur, slots, quadtree)
  // host pyramid (orbx_set_host_pyramid): orbx_extract also copies levels >= 1
  // of its frame into pinned memory, on a graph branch forked right after the
  // pyramid stage and joined at the end of the call (the copy overlaps FAST ..
  // BRIEF); level 0 is the pinned input staging itself
  bool host_pyr = false;
  bool host_pyr_valid = false;  // h_pyr holds the last orbx_extract's levels
  void* h_pyr = nullptr;
  size_t h_pyr_bytes = 0;
  long long h_pyr_off[kMaxLevels] = {};  // level l's offset in h_pyr (l >= 1)
  hipStream_t pstream = nullptr;         // the copy branch's stream (capture fork)
  hipEvent_t pev[2] = {};                // pyramid done, copy done
  // ORBX_EXTRACT_PROF=1 (diagnostics): orbx_extract's host phases per call
  // (s), their medians printed by orbx_destroy: staging copy, issue, wait, copy-out
  std::vector<float> prof_t[4];
  char order[6] = {};  // the stages' launch order (orbx_set_stage_order; default extract_stage_order())
  std::mutex mu;
};

WsOrder* orbx::extractor_ws(orbx_handle h) { return h ? &h->ws : nullptr; }

// ORBextractor::ORBextractor scalar tables (src/ORBextractor.cc:500-532) and
// umax (:540-555); the fork's scale override (:674-680) in mode F.
static void compute_scales(orbx_extractor* h) {
  const orbx_config& c = h->cfg;
  const int L = c.nlevels;
  h->scale.assign(L, 1.f);
  h->sigma2.assign(L, 1.f);
  for (int i = 1; i < L; i++) {
    h->scale[i] = h->scale[i - 1] * c.scale_factor;
    h->sigma2[i] = h->scale[i] * h->scale[i];
  }
  h->inv_scale.resize(L);
  h->inv_sigma2.resize(L);
  for (int i = 0; i < L; i++) {
    h->inv_scale[i] = 1.0f / h->scale[i];
    h->inv_sigma2[i] = 1.0f / h->sigma2[i];
  }
  h->nfeat.assign(L, 0);
  const float factor = 1.0f / c.scale_factor;
  float nDesired = c.nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)L));
  int sum = 0;
  for (int l = 0; l < L - 1; l++) {
    h->nfeat[l] = cv_round(nDesired);
    sum += h->nfeat[l];
    nDesired *= factor;
  }
  h->nfeat[L - 1] = std::max(c.nfeatures - sum, 0);
  const int HP = kHalfPatch;
  int v, v0;
  const int vmax = cv_floor(HP * sqrtf(2.f) / 2 + 1);
  const int vmin = (int)std::ceil(HP * sqrtf(2.f) / 2);
  const double hp2 = HP * HP;
  for (v = 0; v <= vmax; ++v) h->umax[v] = (int)lrint(sqrt(hp2 - v * v));
  for (v = HP, v0 = 0; v >= vmin; --v) {
    while (h->umax[v0] == h->umax[v0 + 1]) ++v0;
    h->umax[v] = v0;
    ++v0;
  }
  if (c.scale_mode == ORBX_SCALE_F) {
    for (int l = 0; l < L; ++l) {
      const unsigned vw = (unsigned)std::ceil(c.width * std::pow(0.8408964, l));
      h->scale[l] = ((float)c.width) / vw;
      h->inv_scale[l] = ((float)vw) / c.width;
    }
  }
}

// getGaussianKernel(7, 2, CV_32F) -> CV_32S x256 (the 8U smooth branch of
// createSeparableLinearFilter): [18, 34, 49, 55, 49, 34, 18].
static void gaussian7(int k[7]) {
  float cf[7];
  double sum = 0;
  for (int i = 0; i < 7; ++i) {
    const double x = i - 3.0;
    cf[i] = (float)std::exp(-0.5 / (2.0 * 2.0) * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 7; ++i) cf[i] = (float)(cf[i] * sum);
  for (int i = 0; i < 7; ++i) k[i] = cv_round(cf[i] * 256.f);
}

// OpenCV 3.x INTER_LINEAR coefficient tables from (sw,sh) to (dw,dh):
// x entries {sx, a0 | a1<<16}, y entries {sy0 | sy1<<16, b0 | b1<<16}.
static void resize_tables(int sw, int sh, int dw, int dh, std::vector<int2>& xt, std::vector<int2>& yt,
                          int* xmax_out, int* area2x) {
  const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
  const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
  const int isx = (int)lrint(scale_x), isy = (int)lrint(scale_y);
  const bool fast = std::fabs(scale_x - isx) < DBL_EPSILON && std::fabs(scale_y - isy) < DBL_EPSILON;
  *area2x = (fast && isx == 2 && isy == 2) ? 1 : 0;
  xt.resize(dw);
  yt.resize(dh);
  int xmax = dw;
  for (int dx = 0; dx < dw; ++dx) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = cv_floor(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= sw) {
      xmax = std::min(xmax, dx);
      if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
    }
    const int a0 = sat_short(cv_round((1.f - fx) * 2048)), a1 = sat_short(cv_round(fx * 2048));
    xt[dx] = make_int2(sx, (a0 & 0xFFFF) | (a1 << 16));
  }
  *xmax_out = xmax;
  auto clip = [](int x, int a, int b) { return x >= a ? (x < b ? x : b - 1) : a; };
  for (int dy = 0; dy < dh; ++dy) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = cv_floor(fy);
    fy -= sy;
    const int b0 = sat_short(cv_round((1.f - fy) * 2048)), b1 = sat_short(cv_round(fy * 2048));
    yt[dy] = make_int2(clip(sy, 0, sh) | (clip(sy + 1, 0, sh) << 16), (b0 & 0xFFFF) | (b1 << 16));
  }
}

// Row bands of the one-launch pyramid (orbx_pyramid.hip pyr_band_kernel).
// Bands of R rows partition the last level; walking down, a band's rows at
// level l start at the first source row of its first row at level l+1, and it
// OWNS (writes) the rows up to where the next band's start; it COMPUTES its
// own rows plus every source row its level-(l+1) rows read. Level 0 rows are
// only read. R shrinks until the two LDS row buffers fit; if even R = 1 does
// not, the per-level kernel is used.
// Column tiles split every band the same way (rows and columns are
// separable): tile c of the last level owns an even-aligned share of its
// columns; walking down, its columns at level l start at the first source
// column of its first column at level l+1 (rounded down to even, so that the
// owned ranges of every level start even and a 2-column store never straddles
// two tiles), and it computes every source column its level-(l+1) columns read.
// Per (tile, level) the table holds {comp_lo, comp_hi}, {own_lo, own_hi} and
// {LDS row pitch, LDS origin}: the column of LDS byte 0 (level 0, staged in
// 16-byte chunks: comp_lo rounded down to 16; else comp_lo).
struct PyrCols {
  int nct = 1;
  std::vector<int> lo, chi, ohi;  // [tile][level]
  int lpitch[kMaxLevels] = {};    // LDS row pitch per level (the widest tile)
};

static bool plan_pyr_cols(const ExtractParams& P, const std::vector<int2>& rtab, int nct, PyrCols& C) {
  const int L = P.L, WL = P.lv[L - 1].w;
  if (nct > 1 && WL / nct < 32) return false;  // tiles of >= 32 last-level columns
  C.nct = nct;
  C.lo.assign((size_t)nct * L, 0);
  C.chi.assign((size_t)nct * L, 0);
  C.ohi.assign((size_t)nct * L, 0);
  // source columns of output column x at level l (>= 1): sx and sx + 1 (xtab2
  // folds the 2x area case in as {2x, 0}); past the last column, the last one's
  auto src_lo_x = [&](int l, int x) { return rtab[P.lv[l].xtab2 + std::min(x, P.lv[l].w - 1)].x; };
  auto src_hi_x = [&](int l, int x) { return rtab[P.lv[l].xtab2 + std::min(x, P.lv[l].w - 1)].x + 1; };
  for (int c = 0; c < nct; ++c) {
    C.lo[c * L + L - 1] = c == 0 ? 0 : ((int)((long long)c * WL / nct) & ~1);
    C.chi[c * L + L - 1] = C.ohi[c * L + L - 1] = (c + 1 < nct ? ((int)((long long)(c + 1) * WL / nct) & ~1) : WL) - 1;
  }
  for (int l = L - 2; l >= 0; --l)
    for (int c = 0; c < nct; ++c) C.lo[c * L + l] = c == 0 ? 0 : (src_lo_x(l + 1, C.lo[c * L + l + 1]) & ~1);
  for (int l = L - 2; l >= 0; --l)
    for (int c = 0; c < nct; ++c) {
      const int own_hi = c + 1 < nct ? C.lo[(c + 1) * L + l] - 1 : P.lv[l].w - 1;
      if (own_hi < C.lo[c * L + l]) return false;  // a tile with no column of its own
      C.ohi[c * L + l] = own_hi;
      C.chi[c * L + l] = std::max(src_hi_x(l + 1, C.chi[c * L + l + 1]), l > 0 ? own_hi : 0);
    }
  for (int l = 0; l < L; ++l) {
    int p = 0;
    for (int c = 0; c < nct; ++c) {
      const int lo = C.lo[c * L + l], hi = C.chi[c * L + l];
      // level 0: 16-byte chunks from lo & ~15 up to column hi (the last sx + 1
      // read; past the image it reads an unstaged byte, weighted 0); other
      // levels: the 2-column runs of G = ceil(width / 8) groups end <= 6 past hi
      p = std::max(p, l == 0 ? ((hi - (lo & ~15) + 1 + 15) & ~15) : ((hi - lo + 1 + 8 + 15) & ~15));
    }
    // experiments: ORBX_PYR_PADMOD=m pads every LDS row pitch to m mod 128
    // (level 0 keeps its 16-byte rows: m rounded down to 16 there)
    if (const char* e = getenv("ORBX_PYR_PADMOD")) {
      const int m = (l == 0 ? atoi(e) & ~15 : atoi(e)) % 128, step = l == 0 ? 16 : 4;
      while (p % 128 != m) p += step;
    }
    C.lpitch[l] = p;
  }
  return true;
}

static void plan_band_pyramid(ExtractParams& P, std::vector<int2>& rtab) {
  P.pyr_fused = 0;
  const int L = P.L;
  if (L < 2) return;
  auto src_lo = [&](int l, int y) { return P.lv[l].area2x ? 2 * y : (rtab[P.lv[l].ytab + y].x & 0xFFFF); };
  auto src_hi = [&](int l, int y) { return P.lv[l].area2x ? 2 * y + 1 : (rtab[P.lv[l].ytab + y].x >> 16); };
  const int HL = P.lv[L - 1].h;
  // Candidate tilings: band heights R from a quarter of the last level down
  // to R0/3 (R0 = HL/18) x 1, 2 or 4 column tiles, within a CU's LDS (two
  // workgroups per CU up to budgets[0]). launch_pyramid picks one per launch
  // (pick_pyr_plan); up to 8 are kept (below).
  const size_t budgets[2] = {78 * 1024, 160 * 1024 - 1024};
  const int R0 = std::max(1, (HL + 17) / 18);
  struct Cand {
    int R, nb, nct;
    size_t need0, need1, ybytes;
    long long cost;
    std::vector<int> lo, chi, ohi;
    PyrCols cols;
  };
  std::vector<Cand> cands;
  PyrCols colplans[3];
  bool colok[3];
  for (int k = 0; k < 3; ++k) colok[k] = plan_pyr_cols(P, rtab, 1 << k, colplans[k]);
  // band heights from a quarter of the last level (4 bands: one workgroup
  // per CU for a 32-64-frame batch once tiled) down to R0 / 3
  const int Rmax = std::max(R0 + 5, (HL + 3) / 4);
  for (int R = Rmax; R >= std::max(1, R0 / 3); --R) {
    const int nb = (HL + R - 1) / R;
    if (!cands.empty() && cands.back().nb == nb) continue;  // same band count as a taller R
    std::vector<int> lo((size_t)nb * L), chi((size_t)nb * L), ohi((size_t)nb * L);
    for (int b = 0; b < nb; ++b) {
      lo[b * L + L - 1] = b * R;
      chi[b * L + L - 1] = ohi[b * L + L - 1] = std::min((b + 1) * R, HL) - 1;
    }
    for (int l = L - 2; l >= 0; --l)
      for (int b = 0; b < nb; ++b) lo[b * L + l] = b == 0 ? 0 : src_lo(l + 1, lo[b * L + l + 1]);
    for (int l = L - 2; l >= 0; --l)
      for (int b = 0; b < nb; ++b) {
        const int own_hi = b + 1 < nb ? lo[(b + 1) * L + l] - 1 : P.lv[l].h - 1;
        ohi[b * L + l] = own_hi;
        chi[b * L + l] = std::max(src_hi(l + 1, chi[b * L + l + 1]), l > 0 ? own_hi : 0);
      }
    size_t ybytes = 0;
    for (int b = 0; b < nb; ++b) {
      size_t s = 0;
      for (int l = 1; l < L; ++l) s += (size_t)(chi[b * L + l] - lo[b * L + l] + 1) * 8;
      ybytes = std::max(ybytes, s);
    }
    for (int k = 0; k < 3; ++k) {
      if (!colok[k]) continue;
      const PyrCols& C = colplans[k];
      size_t need[2] = {0, 0};
      for (int l = 0; l < L; ++l) {
        int rows = 0;
        for (int b = 0; b < nb; ++b) rows = std::max(rows, chi[b * L + l] - lo[b * L + l] + 1);
        need[l & 1] = std::max(need[l & 1], (size_t)rows * C.lpitch[l]);
      }
      need[0] = (need[0] + 15) & ~(size_t)15;
      need[1] = (need[1] + 15) & ~(size_t)15;
      if (need[0] + need[1] + ybytes + 16 > budgets[1]) continue;  // a CU's LDS (occupancy 1 above budgets[0])
      long long cost = 0;
      for (int b = 0; b < nb; ++b)
        for (int c = 0; c < C.nct; ++c) {
          long long s = 0;
          for (int l = 0; l < L; ++l)
            s += (long long)(chi[b * L + l] - lo[b * L + l] + 1) * (C.chi[c * L + l] - C.lo[c * L + l] + 1);
          cost = std::max(cost, s);
        }
      cands.push_back(Cand{R, nb, C.nct, need[0], need[1], ybytes, cost, lo, chi, ohi, C});
    }
  }
  if (cands.empty()) return;
  // the plans kept: the one-tile plans (band heights as before column tiles
  // existed; the default first: R0's or the nearest), then for small batches
  // the column-tiled plan that pick_pyr_plan would take in one round
  std::vector<int> keep;
  // experiments (tools/pyr_plans.py): ORBX_PYR_KEEP="nb:nct,nb:nct,..." keeps
  // exactly those candidates (up to 8, in that order)
  const char* ek = getenv("ORBX_PYR_KEEP");
  if (ek) {
    for (const char* p = ek; *p && keep.size() < 8;) {
      int nb = 0, nct = 0, used = 0;
      if (sscanf(p, "%d:%d%n", &nb, &nct, &used) != 2) break;
      for (int i = 0; i < (int)cands.size(); ++i)
        if (cands[i].nb == nb && cands[i].nct == nct) keep.push_back(i);
      p += used;
      if (*p == ',') ++p;
    }
  }
  if (keep.empty()) {
    // the default (R0's band height or the nearest, one tile), then what the
    // launch-time rule (pick_pyr_plan) takes for batches of 1 .. 64 and B on
    // a 256-CU chip (two workgroups per CU up to 78 KB of LDS, else one: the
    // occupancy API sets the real count afterwards), then one-tile plans near R0
    int def = -1;
    for (int i = 0; i < (int)cands.size(); ++i)
      if (cands[i].nct == 1 && cands[i].need0 + cands[i].need1 + cands[i].ybytes + 16 <= budgets[0] &&
          (def < 0 || std::abs(cands[i].nb - (HL + R0 - 1) / R0) < std::abs(cands[def].nb - (HL + R0 - 1) / R0)))
        def = i;
    if (def < 0) def = 0;
    keep.push_back(def);
    std::vector<ExtractParams::PyrPlan> sim(cands.size());
    for (size_t i = 0; i < cands.size(); ++i) {
      sim[i].nbands = cands[i].nb;
      sim[i].nct = cands[i].nct;
      sim[i].cost = (int)cands[i].cost;
      sim[i].occ = cands[i].need0 + cands[i].need1 + cands[i].ybytes + 16 <= budgets[0] ? 2 : 1;
    }
    const int batches[8] = {1, 2, 4, 8, 16, 32, 64, P.B};
    for (int bt : batches) {
      const int best = pick_pyr_plan(sim.data(), (int)sim.size(), bt, 256);
      if (keep.size() < 8 && std::find(keep.begin(), keep.end(), best) == keep.end()) keep.push_back(best);
    }
    for (int d = 1; keep.size() < 8 && d < (int)cands.size(); ++d)
      for (int i : {def - d, def + d})
        if (i >= 0 && i < (int)cands.size() && cands[i].nct == 1 && keep.size() < 8 &&
            std::find(keep.begin(), keep.end(), i) == keep.end())
          keep.push_back(i);
  }
  P.pyr_nplans = 0;
  for (int i : keep) {
    const Cand& c = cands[i];
    ExtractParams::PyrPlan& q = P.pyr_plan[P.pyr_nplans++];
    q.nbands = c.nb;
    q.nct = c.nct;
    q.lds_a = (int)c.need0;
    q.lds_b = (int)c.need1;
    q.lds_y = (int)c.ybytes;
    q.cost = (int)c.cost;
    q.occ = 0;
    q.bands = (int)rtab.size();
    for (int b = 0; b < c.nb; ++b)
      for (int l = 0; l < L; ++l) {
        rtab.push_back(make_int2(c.lo[b * L + l], c.chi[b * L + l]));
        rtab.push_back(make_int2(c.lo[b * L + l], c.ohi[b * L + l]));
      }
    q.ctiles = (int)rtab.size();
    const PyrCols& C = c.cols;
    for (int t = 0; t < C.nct; ++t)
      for (int l = 0; l < L; ++l) {
        const int lo = C.lo[t * L + l];
        rtab.push_back(make_int2(lo, C.chi[t * L + l]));
        rtab.push_back(make_int2(lo, C.ohi[t * L + l]));
        rtab.push_back(make_int2(C.lpitch[l], l == 0 ? (lo & ~15) : lo));
      }
  }
  P.pyr_fused = 1;
  select_pyr_plan(P, 0);  // the default; launch_pyramid picks per launch
}

// Path codes of the sorted-key quadtree (orbx_quadtree.hip): a node box of
// DistributeOctTree never depends on the data (roots: nIni columns of width
// hX, src/ORBextractor.cc:903-914; children: DivideNode's ceil halves,
// :833-834), so the quadrant of a key at every depth is a function of its x
// alone (x half) and of its y alone (y half). t = boxW x codes (root index in
// the top bits, x digit at even bits), then boxH y codes (y digit at odd
// bits), Dh digits each: xs[x] | ys[y] is the key's bin, its node at depth
// Dh. bits = 0 (code shift) | Dh << 8 | log2(bins) << 16; bins stay within
// 4096..8192 so that the bin scan keeps 2..8 words per thread.
static bool qt_code_tables(const LevelGeom& g, std::vector<uint32_t>& t, int* bits) {
  int R = 0;
  while ((1 << R) < g.nIni) ++R;
  if (R > 5 || g.boxW < 1 || g.boxH < 1 || g.boxW > 0xFFFF || g.boxH > 0xFFFF) return false;
  const int Dh = (13 - R) / 2;
  t.assign((size_t)g.boxW + g.boxH, 0u);
  for (int x = 0; x < g.boxW; ++x) {
    // vpIniNodes[kp.pt.x/hX] (:920); columns past the last root never hold keys
    const int r = std::min((int)((float)x / g.hX), g.nIni - 1);
    int a = (int)(g.hX * (float)r), c = (int)(g.hX * (float)(r + 1));
    uint32_t code = (uint32_t)r << (2 * Dh);
    for (int j = 0; j < Dh; ++j) {
      const int mid = a + (int)std::ceil((float)(c - a) / 2.f);
      const int bit = x >= mid;
      if (bit) a = mid; else c = mid;
      code |= (uint32_t)bit << (2 * (Dh - 1 - j));
    }
    t[x] = code;
  }
  for (int y = 0; y < g.boxH; ++y) {
    int a = 0, c = g.boxH;
    uint32_t code = 0;
    for (int j = 0; j < Dh; ++j) {
      const int mid = a + (int)std::ceil((float)(c - a) / 2.f);
      const int bit = y >= mid;
      if (bit) a = mid; else c = mid;
      code |= (uint32_t)bit << (2 * (Dh - 1 - j) + 1);
    }
    t[(size_t)g.boxW + y] = code;
  }
  *bits = (Dh << 8) | ((R + 2 * Dh) << 16);
  return true;
}

static int build_plan(orbx_extractor* h, int W, int Hh, int B) {
  Plan& pl = h->plan;
  const orbx_config& c = h->cfg;
  const int L = c.nlevels;
  ExtractParams P{};
  P.L = L;
  P.B = B;
  const int ini = std::min(std::max(c.ini_th_fast, 0), 255), mn = std::min(std::max(c.min_th_fast, 0), 255);
  P.t_ini = ini;
  P.t_min = mn;
  P.t_low = std::min(ini, mn);
  P.pattern_upstream = c.pattern_mode == ORBX_PATTERN_UPSTREAM;
  gaussian7(P.gauss);
  pl.cells.clear();
  pl.rtab.clear();
  long long lvl_off = 0;  // level planes [l][B][h][pitch], same offsets in pyramid and blur
  int slot = 0, kbase = 0, maxnodes = 0, maxcells = 0;
  for (int l = 0; l < L; ++l) {
    LevelGeom& g = P.lv[l];
    const float inv = h->inv_scale[l];
    g.w = cv_round((float)W * inv);
    g.h = cv_round((float)Hh * inv);
    if (g.w > kMaxLevelDim || g.h > kMaxLevelDim)
      return fail(ORBX_EINVAL, "level %d is %dx%d; at most %d px per side", l, g.w, g.h, kMaxLevelDim);
    g.pitch = (g.w + 63) & ~63;
    g.plane = (long long)g.h * g.pitch;
    // FAST grid (src/ORBextractor.cc:1133-1147)
    g.minBX = kEdgeThreshold - 3;
    g.minBY = g.minBX;
    g.maxBX = g.w - kEdgeThreshold + 3;
    g.maxBY = g.h - kEdgeThreshold + 3;
    const float width = (float)(g.maxBX - g.minBX), height = (float)(g.maxBY - g.minBY);
    g.nCols = (int)(width / kGridW);
    g.nRows = (int)(height / kGridW);
    if (g.nCols < 1 || g.nRows < 1)
      return fail(ORBX_EINVAL,
                  "level %d (%dx%d) is smaller than one %d-px FAST cell inside the %d-px border; "
                  "the reference divides by zero here (src/ORBextractor.cc:1144-1147)",
                  l, g.w, g.h, kGridW, kEdgeThreshold);
    g.wCell = (int)std::ceil(width / g.nCols);
    g.hCell = (int)std::ceil(height / g.nRows);
    if (g.wCell + 6 > kMaxRoi - 1 || g.hCell + 6 > kMaxRoi - 1)
      return fail(ORBX_EINVAL, "level %d cell %dx%d exceeds the ROI tile", l, g.wCell, g.hCell);
    g.cell0 = (int)pl.cells.size();
    g.slot0 = slot;
    for (int i = 0; i < g.nRows; i++) {
      const float iniY = g.minBY + i * g.hCell;
      float maxY = iniY + g.hCell + 6;
      const bool skipRow = iniY >= g.maxBY - 3;
      if (maxY > g.maxBY) maxY = g.maxBY;
      for (int j = 0; j < g.nCols; j++) {
        const float iniX = g.minBX + j * g.wCell;
        float maxX = iniX + g.wCell + 6;
        const bool skip = skipRow || iniX >= g.maxBX - 6;
        if (maxX > g.maxBX) maxX = g.maxBX;
        CellGeom cg{};
        cg.level = (int16_t)l;
        cg.c0 = (int16_t)(int)iniX;
        cg.r0 = (int16_t)(int)iniY;
        cg.c1 = (int16_t)(int)maxX;
        cg.r1 = (int16_t)(int)maxY;
        const int bw = cg.c1 - cg.c0 - 6, bh = cg.r1 - cg.r0 - 6;
        cg.cap = (skip || bw <= 0 || bh <= 0) ? 0 : (int16_t)(((bw + 1) / 2) * ((bh + 1) / 2));
        if (cg.cap) {
          P.fast_rh_max = std::max(P.fast_rh_max, cg.r1 - cg.r0);
          P.fast_bw_max = std::max(P.fast_bw_max, bw);
          P.fast_bh_max = std::max(P.fast_bh_max, bh);
        }
        cg.pitch = l == 0 ? 0 : g.pitch;
        cg.row_off = l == 0 ? cg.r0 : (int)(lvl_off + (long long)cg.r0 * g.pitch);
        cg.fstride = l == 0 ? 0 : (int)g.plane;
        cg.geo = (g.h - 1 - cg.r0) | (((g.w + 15) & ~15) << 16);
        pl.cells.push_back(cg);
      }
    }
    g.ncells = (int)pl.cells.size() - g.cell0;
    // slot ranges at one stride per level (the largest cell's NMS bound):
    // cell c's keys start at slot0 + c * stride, so the sorted quadtree
    // finds them without reading the cell records
    int stride = 1;
    for (int c = g.cell0; c < (int)pl.cells.size(); ++c) stride = std::max(stride, (int)pl.cells[c].cap);
    for (int c = g.cell0; c < (int)pl.cells.size(); ++c) pl.cells[c].slot_off = slot + (c - g.cell0) * stride;
    g.slot_stride = stride;
    slot += g.ncells * stride;
    g.nslots = slot - g.slot0;
    maxcells = std::max(maxcells, g.ncells);
    // DistributeOctTree (src/ORBextractor.cc:894-898)
    g.N = h->nfeat[l];
    g.boxW = g.maxBX - g.minBX;
    g.boxH = g.maxBY - g.minBY;
    g.nIni = (int)roundf(static_cast<float>(g.boxW) / g.boxH);
    if (g.nIni < 1) return fail(ORBX_EINVAL, "level %d: nIni = 0 (image taller than 1.5x its width)", l);
    g.hX = static_cast<float>(g.boxW) / g.nIni;
    g.kcap = std::max(g.N + 3, g.nIni);
    g.kbase = kbase;
    // levels start at multiples of kKpGroup slots, so an orient+BRIEF
    // workgroup's keypoints all sit in one level
    kbase += (g.kcap + kKpGroup - 1) / kKpGroup * kKpGroup;
    maxnodes = std::max(maxnodes, g.kcap + 4);
    g.scale = h->scale[l];
    g.size = (float)(int)(kPatchSize * h->scale[l]);
    g.off = lvl_off;
    lvl_off += (long long)B * g.plane;
    if (l >= 1) {
      std::vector<int2> xt, yt;
      resize_tables(P.lv[l - 1].w, P.lv[l - 1].h, g.w, g.h, xt, yt, &g.xmax, &g.area2x);
      // the pyramid kernel stages each 16 x 256 output tile's source footprint
      // in a 36 x 576 LDS tile (orbx_pyramid.hip): true for scaleFactor <= 2
      for (int x0 = 0; x0 < g.w; x0 += 256) {
        const int xe = std::min(x0 + 255, g.w - 1);
        const int lo = g.area2x ? 2 * x0 : xt[x0].x, hi = g.area2x ? 2 * xe + 1 : xt[xe].x + 1;
        if (hi - (lo & ~15) + 16 > 576)
          return fail(ORBX_EINVAL, "scaleFactor %g too large for the pyramid tile (max 2.0)", c.scale_factor);
      }
      for (int y0 = 0; y0 < g.h; y0 += 16) {
        const int ye = std::min(y0 + 15, g.h - 1);
        const int lo = g.area2x ? 2 * y0 : (yt[y0].x & 0xFFFF), hi = g.area2x ? 2 * ye + 1 : (yt[ye].x >> 16);
        if (hi - lo + 1 > 36)
          return fail(ORBX_EINVAL, "scaleFactor %g too large for the pyramid tile (max 2.0)", c.scale_factor);
      }
      g.xtab = (int)pl.rtab.size();
      pl.rtab.insert(pl.rtab.end(), xt.begin(), xt.end());
      g.ytab = (int)pl.rtab.size();
      pl.rtab.insert(pl.rtab.end(), yt.begin(), yt.end());
      // band-pyramid column table: columns at or past xmax replicate S[sx]
      // (x2048), the same as coefficients {2048, 0}
      g.xtab2 = (int)pl.rtab.size();
      for (int dx = 0; dx < g.w; ++dx) {
        int2 e = xt[dx];
        if (g.area2x) e = make_int2(2 * dx, 0);
        else if (dx >= g.xmax) e.y = 2048;
        pl.rtab.push_back(e);
      }
    }
  }
  // sorted-key quadtree: per level, the depth-Dh path code of every column
  // (root index on top) and of every row (orbx_quadtree.hip), two u32 per
  // int2 of the resize table
  P.qt_tabmax = 0;
  P.qt_nbmax = 0;
  for (int l = 0; l < L; ++l) {
    LevelGeom& g = P.lv[l];
    std::vector<uint32_t> t;
    int bits = 0;
    g.qt_tab = -1;
    if (qt_code_tables(g, t, &bits)) {
      g.qt_tab = (int)pl.rtab.size() * 2;
      g.qt_dims = g.boxW | (g.boxH << 16);
      g.qt_bits = bits;
      if (t.size() & 1) t.push_back(0u);
      for (size_t i = 0; i < t.size(); i += 2) pl.rtab.push_back(make_int2((int)t[i], (int)t[i + 1]));
      P.qt_tabmax = std::max(P.qt_tabmax, g.boxW + g.boxH);
      P.qt_nbmax = std::max(P.qt_nbmax, 1 << ((bits >> 16) & 0xFF));
    }
  }
  if (lvl_off > INT_MAX)  // FAST's cell records hold 32-bit plane offsets
    return fail(ORBX_EINVAL, "max_batch %d: the pyramid planes take %lld bytes, over 2 GiB", B, lvl_off);
  plan_band_pyramid(P, pl.rtab);
  for (int v = 0; v < 2; ++v) {
    // blur tiles, large and small, level-major, row-major inside a level (orbx_blur.hip)
    int tw = 0, th = 0;
    blur_tile_dims(v, &tw, &th);
    P.blur_tiles[v] = (int)pl.rtab.size();
    for (int l = 0; l < L; ++l)
      for (int y0 = 0; y0 < P.lv[l].h; y0 += th)
        for (int x0 = 0; x0 < P.lv[l].w; x0 += tw) pl.rtab.push_back(make_int2(l | (x0 << 4) | (y0 << 16), 0));
    P.blur_ntiles[v] = (int)pl.rtab.size() - P.blur_tiles[v];
    const unsigned long long d = (unsigned long long)P.blur_ntiles[v];
    P.blur_magic[v] = 0u;
    if (d > 1) {
      const unsigned long long m = ((1ull << 32) + d - 1) / d, e = m * d - (1ull << 32);
      if (d * (unsigned long long)B * e < (1ull << 32)) P.blur_magic[v] = (unsigned)m;
    }
  }
  if (maxnodes > 65000) return fail(ORBX_EINVAL, "nfeatures too large for the quadtree node table");
  P.slots_per_frame = slot;
  P.ncells_total = (int)pl.cells.size();
  {
    // FAST's frame index without a division: mulhi(id, m) with m = ceil(2^32 / d)
    // equals id / d while id * (m * d - 2^32) < 2^32 (ids < d * B)
    const unsigned long long d = (unsigned long long)P.ncells_total;
    P.ncells_magic = 0u;
    if (d > 1) {
      const unsigned long long m = ((1ull << 32) + d - 1) / d, e = m * d - (1ull << 32);
      if (d * (unsigned long long)B * e < (1ull << 32)) P.ncells_magic = (unsigned)m;
    }
  }
  P.kp_per_frame = kbase;
  P.maxnodes = maxnodes;
  int sn = 1;
  while (sn < maxnodes) sn <<= 1;
  P.sortn = sn;
  P.max_cells_level = maxcells;
  P.kcap_lds = 0;
  {
    const char* e = getenv("ORBX_QT_GENERIC");  // tests: the generic rounds on any plan
    P.qt_lean = maxnodes < 16384 && !(e && e[0] == '1');
    // the sorted-key path first (ORBX_QT_SORTED=0: the legacy rounds only, for A/B and tests)
    const char* so = getenv("ORBX_QT_SORTED");
    P.qt_sorted = P.qt_lean && P.qt_nbmax > 0 && !(so && so[0] == '0');
  }
  {
    // keep the LDS footprint at 80 KiB so two quadtree blocks fit one CU,
    // unless the node tables alone nearly fill that (large levels: 1920x1080
    // has 102 KB of them). Then a block takes a whole CU: 1024 threads (its
    // key passes, which set its time there, on twice the lanes) and 160 KiB,
    // the rest of it for keys
#ifndef ORBX_QT_LDS_KB
#define ORBX_QT_LDS_KB 80
#endif
    const size_t base = quadtree_legacy_lds_bytes(P);
    size_t small = ORBX_QT_LDS_KB * 1024, big = 160 * 1024 - 512;
    if (const char* e = getenv("ORBX_QT_LDS_KB")) small = (size_t)std::max(32, atoi(e)) * 1024;  // A/B: blocks per CU
    P.qt_big = base + 16 * 1024 > small ? 1 : 0;
    const size_t budget = P.qt_big ? big : small;
    P.kcap_lds = base < budget ? (int)((budget - base) / 6) & ~15 : 0;
    // the sorted path shares the block's LDS (its layout is the legacy one's
    // alternative, not an addition): on when it fits the same budget
    if (P.qt_sorted) {
      P.qt_ownmax = quadtree_sorted_ownmax(P, P.qt_big, budget);
      if (!P.qt_ownmax || quadtree_sorted_lds_bytes(P, P.qt_big) > budget) P.qt_sorted = 0;
    }
    // the sorted path's rounds hold two nodes per thread
    if (maxnodes > 2 * (P.qt_big ? 1024 : kQtThreads)) P.qt_sorted = 0;
    if (getenv("ORBX_PLAN_INFO"))  // diagnostics: the quadtree block's LDS per path
      fprintf(stderr,
              "plan %dx%d B %d: quadtree LDS legacy %zu sorted %zu (budget %zu) sorted %d big %d maxnodes %d "
              "nbmax %d tabmax %d ownmax %d\n",
              W, Hh, B, base, P.qt_nbmax ? quadtree_sorted_lds_bytes(P, P.qt_big) : (size_t)0, budget, P.qt_sorted,
              P.qt_big, maxnodes, P.qt_nbmax, P.qt_tabmax, P.qt_ownmax);
  }
  pl.P = P;
  pl.W = W;
  pl.H = Hh;
  pl.B = B;
  // device buffers (the pyramid's level-0 planes stay unused: level 0 is the caller's frames)
  int rc;
  if ((rc = pl.pyr.alloc((size_t)lvl_off))) return rc;
  if ((rc = pl.blur.alloc((size_t)lvl_off))) return rc;
  if ((rc = pl.rtab_d.alloc(std::max<size_t>(pl.rtab.size(), 1) * sizeof(int2)))) return rc;
  if ((rc = pl.cells_d.alloc(pl.cells.size() * sizeof(CellGeom)))) return rc;
  if ((rc = pl.umax_d.alloc(16 * sizeof(int)))) return rc;
  if ((rc = pl.slots.alloc((size_t)B * slot * 4 + 4 + 4 * 96))) return rc;  // + the quadtree's prefetch overrun
  if ((rc = pl.cell_counts.alloc((size_t)B * P.ncells_total * 4))) return rc;
  if ((rc = pl.qkeys.alloc((size_t)B * P.kp_per_frame * 4))) return rc;
  if ((rc = pl.qcounts.alloc((size_t)B * L * 4 + 4 * kMaxLevels))) return rc;  // orient_brief reads kMaxLevels counts per frame
  if ((rc = pl.qties.alloc((size_t)B * L * 16))) return rc;
  if ((rc = pl.qscratch.alloc((size_t)B * slot * 4 + 4))) return rc;
  if ((rc = pl.qnscratch.alloc((size_t)B * slot * 2 + 4))) return rc;
  if ((rc = pl.err.alloc(16))) return rc;
  HIP_OK(hipMemcpy(pl.rtab_d.p, pl.rtab.data(), pl.rtab.size() * sizeof(int2), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(pl.cells_d.p, pl.cells.data(), pl.cells.size() * sizeof(CellGeom), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(pl.umax_d.p, h->umax, 16 * sizeof(int), hipMemcpyHostToDevice));
  HIP_OK(hipMemset(pl.err.p, 0, 16));
  if (P.pyr_fused && getenv("ORBX_PYR_PROF") && getenv("ORBX_PYR_PROF")[0] == '1')
    for (int i = 0; i < P.pyr_nplans; ++i)
      fprintf(stderr, "pyr plan %d: %d bands x %d column tiles, lds %d + %d + %d, cost %d\n", i,
              P.pyr_plan[i].nbands, P.pyr_plan[i].nct, P.pyr_plan[i].lds_a, P.pyr_plan[i].lds_b, P.pyr_plan[i].lds_y,
              P.pyr_plan[i].cost);
  if (P.pyr_fused) {
    size_t mx = 0;
    for (int i = 0; i < P.pyr_nplans; ++i) {
      ExtractParams Q = P;
      select_pyr_plan(Q, i);
      mx = std::max(mx, pyr_band_lds_bytes(Q));
    }
    if (raise_lds_limit(pyr_band_kernel_ptr(), mx))
      return fail(ORBX_EDEVICE, "LDS limit of pyr_band_kernel: %s", hipGetErrorString(hipGetLastError()));
    for (int i = 0; i < P.pyr_nplans; ++i) {
      ExtractParams Q = P;
      select_pyr_plan(Q, i);
      pl.P.pyr_plan[i].occ = pyr_band_occupancy(pyr_band_lds_bytes(Q));
      if (getenv("ORBX_PYR_PROF") && getenv("ORBX_PYR_PROF")[0] == '1')
        fprintf(stderr, "pyr plan %d: %d workgroups per CU\n", i, pl.P.pyr_plan[i].occ);
    }
  }
  if (raise_lds_limit(quadtree_kernel_ptr(P), quadtree_lds_bytes(P)))
    return fail(ORBX_EDEVICE, "LDS limit of quadtree_kernel: %s", hipGetErrorString(hipGetLastError()));
  return ORBX_OK;
}

static ExtractBuffers buffers_of(const Plan& pl) {
  ExtractBuffers X;
  X.pyr = pl.pyr.as<uint8_t>();
  X.blur = pl.blur.as<uint8_t>();
  X.rtab = pl.rtab_d.as<int2>();
  X.cells = pl.cells_d.as<CellGeom>();
  X.umax = pl.umax_d.as<int>();
  X.slots = pl.slots.as<uint32_t>();
  X.cell_counts = pl.cell_counts.as<int>();
  X.qkeys = pl.qkeys.as<uint32_t>();
  X.qcounts = pl.qcounts.as<int>();
  X.qties = pl.qties.as<int>();
  X.qscratch = pl.qscratch.as<uint32_t>();
  X.qnode_scratch = pl.qnscratch.as<uint16_t>();
  X.qscratch_per_fl = 0;
  X.err = pl.err.as<int>();
  return X;
}

// The device pyramid (mvImagePyramid) of frames [frame0, frame0 + n) of the
// last extraction: level 0 is the caller's frames, levels >= 1 the plan's planes.
int orbx::extractor_pyramid(orbx_handle h, int frame0, int n, LevelPtrs* lp, int* w, int* hgt, float* scale,
                            float* inv_scale, int* L) {
  if (!h) return fail(ORBX_EINVAL, "null extractor handle");
  if (frame0 < 0 || n < 1 || frame0 + n > h->last_batch || !h->last_frames)
    return fail(ORBX_EINVAL, "frames [%d, %d) not in the extractor's last extraction (%d frames)", frame0,
                frame0 + n, h->last_batch);
  const ExtractParams& P = h->plan.P;
  const ExtractBuffers X = buffers_of(h->plan);
  *L = P.L;
  for (int l = 0; l < P.L; ++l) {
    const LevelGeom& g = P.lv[l];
    if (l == 0) {
      lp->base[0] = h->last_frames + (long long)frame0 * h->last_fpitch;
      lp->fstride[0] = (long long)h->last_fpitch;
      lp->pitch[0] = (int)h->last_rstride;
    } else {
      lp->base[l] = X.pyr + g.off + (long long)frame0 * g.plane;
      lp->fstride[l] = g.plane;
      lp->pitch[l] = g.pitch;
    }
    lp->aligned16[l] = 0;
    w[l] = g.w;
    hgt[l] = g.h;
    scale[l] = h->scale[l];
    inv_scale[l] = h->inv_scale[l];
  }
  return ORBX_OK;
}

int orbx::extractor_last_output(orbx_handle h, const int** d_count, const orbx_kp** d_kps, const uint8_t** d_desc,
                                int* cap) {
  if (!h) return fail(ORBX_EINVAL, "null extractor handle");
  if (h->last_empty) {  // an empty image: no keypoints
    *d_count = nullptr;
    *d_kps = nullptr;
    *d_desc = nullptr;
    *cap = 0;
    return ORBX_OK;
  }
  if (!h->last_single || !h->d_out.p)
    return fail(ORBX_EINVAL, "the extractor's last extraction was not an orbx_extract call");
  const int c = h->plan.P.kp_per_frame;
  uint8_t* d = h->d_out.as<uint8_t>();
  *d_count = (const int*)d;
  *d_kps = (const orbx_kp*)(d + 16);
  *d_desc = d + out_desc_off(c);
  *cap = c;
  return ORBX_OK;
}

// Dynamic-LDS limits are per kernel and device, shared by every handle of the
// process: only ever raise them (a handle with a smaller plan must not lower
// the limit a larger one launches with).
int orbx::raise_lds_limit(const void* fn, size_t bytes) {
  static std::mutex mu;
  static std::vector<std::pair<std::pair<const void*, int>, size_t>> set;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return ORBX_EDEVICE;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& e : set)
    if (e.first.first == fn && e.first.second == dev) {
      if (bytes <= e.second) return ORBX_OK;
      if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess)
        return ORBX_EDEVICE;
      e.second = bytes;
      return ORBX_OK;
    }
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess)
    return ORBX_EDEVICE;
  set.push_back({{fn, dev}, bytes});
  return ORBX_OK;
}

// ------------------------------------------------------------ C ABI
extern "C" {

const char* orbx_last_error(void) { return g_err.c_str(); }
#ifdef ORBX_DIAG
const char* orbx_version(void) { return "orbx 0.3 (gfx950, diag)"; }
#else
const char* orbx_version(void) { return "orbx 0.3 (gfx950)"; }
#endif

int orbx_create(const orbx_config* cfg, orbx_handle* out) {
  if (!cfg || !out) return fail(ORBX_EINVAL, "null argument");
  *out = nullptr;
  const orbx_config& c = *cfg;
  if (c.nlevels < 1 || c.nlevels > kMaxLevels) return fail(ORBX_EINVAL, "nlevels must be 1..%d", kMaxLevels);
  if (c.nfeatures < 0) return fail(ORBX_EINVAL, "nfeatures < 0");
  if (!(c.scale_factor > 1.0f)) return fail(ORBX_EINVAL, "scaleFactor must be > 1");
  // Camera.width/height absent from the yaml (the reference's mono KITTI /
  // EuRoC settings, src/Tracking.cc:124-133) arrive as 0: mode U's tables do
  // not depend on the size, so the plan waits for the first image; mode F's
  // scale override is computed from the width (src/ORBextractor.cc:674-680)
  const bool deferred = c.width == 0 && c.height == 0 && c.scale_mode == ORBX_SCALE_U;
  if (!deferred && (c.width <= 0 || c.height <= 0))
    return fail(ORBX_EINVAL, c.scale_mode == ORBX_SCALE_F && c.width == 0 && c.height == 0
                                 ? "scale mode F needs width/height (Camera.width/height)"
                                 : "width/height must be > 0, or both 0 in scale mode U (Camera.width/height)");
  if (c.max_batch < 1) return fail(ORBX_EINVAL, "max_batch must be >= 1");
  if (c.scale_mode != ORBX_SCALE_U && c.scale_mode != ORBX_SCALE_F) return fail(ORBX_EINVAL, "bad scale_mode");
  if (c.pattern_mode != ORBX_PATTERN_FORK && c.pattern_mode != ORBX_PATTERN_UPSTREAM)
    return fail(ORBX_EINVAL, "bad pattern_mode");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(ORBX_EDEVICE, "no HIP device");
  if (c.device < 0 || c.device >= ndev) return fail(ORBX_EINVAL, "device %d out of range", c.device);
  HIP_OK(hipSetDevice(c.device));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, c.device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(ORBX_EDEVICE, "device %d is %s; liborbx is built for gfx950 only", c.device, prop.gcnArchName);
  orbx_extractor* h = new orbx_extractor();
  h->cfg = c;
  memcpy(h->order, extract_stage_order(), 6);
  compute_scales(h);
  h->plan.B = c.max_batch;
  int rc = deferred ? ORBX_OK : build_plan(h, c.width, c.height, c.max_batch);
  if (rc) { delete h; return rc; }
  // h->stream (the synchronous API's stream) is created on first use: an idle
  // stream would still take one of the process's few hardware queues, and a
  // host that pipelines on its own streams wants those on distinct queues
  const char* t = getenv("ORBX_TIMING");
  h->timing = t && t[0] == '1';
  if (h->timing)
    for (auto& e : h->ev) (void)hipEventCreate(&e);
  *out = h;
  return ORBX_OK;
}

int orbx_destroy(orbx_handle h) {
  if (!h) return ORBX_OK;
  (void)hipSetDevice(h->cfg.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  if (h->ws.ev) (void)hipEventSynchronize(h->ws.ev);
  h->ws.release();
  if (h->graph) (void)hipGraphExecDestroy(h->graph);
  if (h->pstream) (void)hipStreamSynchronize(h->pstream);
  if (h->prof_t[0].size() > 20) {
    // medians over the calls after the first 20 (plan, capture, warm-up)
    double med[4];
    for (int k = 0; k < 4; ++k) {
      std::vector<float> v(h->prof_t[k].begin() + 20, h->prof_t[k].end());
      std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
      med[k] = v[v.size() / 2] * 1e6;
    }
    fprintf(stderr, "orbx_extract host phases, median of %zu calls (us): stage %.1f issue %.1f wait %.1f out %.1f\n",
            h->prof_t[0].size() - 20, med[0], med[1], med[2], med[3]);
  }
  if (h->h_in) (void)hipHostFree(h->h_in);
  if (h->h_out) (void)hipHostFree(h->h_out);
  if (h->h_pyr) (void)hipHostFree(h->h_pyr);
  for (auto& e : h->pev)
    if (e) (void)hipEventDestroy(e);
  if (h->pstream) (void)hipStreamDestroy(h->pstream);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return ORBX_OK;
}

int orbx_frame_capacity(orbx_handle h) { return h ? h->plan.P.kp_per_frame : 0; }

int orbx_extract_batch(orbx_handle h, const uint8_t* d_frames, int batch, size_t frame_pitch, size_t row_stride,
                       orbx_kp* d_kps, uint8_t* d_desc, int* d_counts, void* stream) {
  if (!h || !d_frames || !d_kps || !d_desc || !d_counts) return fail(ORBX_EINVAL, "null argument");
  if (batch < 1 || batch > h->plan.B) return fail(ORBX_EINVAL, "batch %d not in 1..max_batch(%d)", batch, h->plan.B);
  if (h->plan.W == 0)
    return fail(ORBX_EINVAL, "no frame size yet: the handle was created with width/height 0 and has seen no orbx_extract");
  if (row_stride < (size_t)h->plan.W) return fail(ORBX_EINVAL, "row_stride < width");
  // one call of a handle at a time: a synchronous orbx_extract in flight on
  // another thread holds the lock until its chain has finished (it records
  // no workspace event for a batch call to wait on)
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_OK(hipSetDevice(h->cfg.device));
  void** ev = h->has_user_ev ? h->user_ev : (h->timing ? (void**)h->ev : nullptr);
  h->has_user_ev = false;
  if (h->ws.before((hipStream_t)stream)) return fail(ORBX_EDEVICE, "stream wait on the handle's last use failed");
  const int rc = launch_extract(h->plan.P, buffers_of(h->plan), d_frames, batch, frame_pitch, row_stride, d_kps,
                                d_desc, d_counts, stream, ev, nullptr, nullptr, h->order);
  if (!rc && h->ws.after((hipStream_t)stream)) return fail(ORBX_EDEVICE, "event record failed");
  h->last_batch = batch;
  h->last_frames = d_frames;
  h->last_fpitch = frame_pitch;
  h->last_rstride = row_stride;
  h->host_pyr_valid = false;  // the pinned host pyramid is of an earlier orbx_extract
  h->last_single = false;
  h->last_empty = false;
  if (rc) return fail(rc, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
  return ORBX_OK;
}

// ORBextractor::operator() on one host image (the call Tracking makes per
// frame, src/Frame.cc:246-252 -> src/ORBextractor.cc:1538). The image is
// staged in a pinned buffer; the H2D copy, the five extraction launches and
// one D2H copy of {count, status, keypoints, descriptors} (full capacity, so
// no second round trip) run as one captured hipGraph replayed per call, and
// the call synchronises once. ORBX_EXTRACT_GRAPH=0 issues the same chain as
// plain stream operations (A/B); ORBX_TIMING=1 implies that path.
static int host_reserve(void** p, size_t* have, size_t need) {
  if (*have >= need) return ORBX_OK;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *have = 0;
  if (hipHostMalloc(p, need, hipHostMallocDefault) != hipSuccess) return fail(ORBX_ENOMEM, "hipHostMalloc(%zu)", need);
  *have = need;
  return ORBX_OK;
}


// Host-pyramid layout: frame 0's levels 1..L-1 packed at their device pitches.
// With max_batch 1 the device planes of levels >= 1 are one contiguous block
// (level-major [l][B][h][pitch]), so the copy is one linear D2H.
static size_t host_pyr_layout(orbx_extractor* h) {
  const ExtractParams& P = h->plan.P;
  size_t off = 0;
  for (int l = 1; l < P.L; ++l) {
    h->h_pyr_off[l] = (long long)off;
    off += (size_t)P.lv[l].plane;
  }
  return off;
}

static int issue_one_frame(orbx_extractor* h, size_t pitch, int hh, int cap_frame) {
  hipStream_t s = h->stream;
  const ExtractParams& P = h->plan.P;
  HIP_OK(hipMemcpyAsync(h->d_in.p, h->h_in, pitch * hh, hipMemcpyHostToDevice, s));
  uint8_t* d = h->d_out.as<uint8_t>();
  const size_t doff = out_desc_off(cap_frame);
  const bool hp = h->host_pyr && P.L > 1;
  const int rc = launch_extract(P, buffers_of(h->plan), h->d_in.as<uint8_t>(), 1, pitch * hh, pitch,
                                (orbx_kp*)(d + 16), d + doff, (int*)d, s, h->timing ? (void**)h->ev : nullptr,
                                hp ? (void*)h->pev[0] : nullptr, (int*)d + 1, h->order);
  if (rc) return fail(rc, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
  if (hp) {
    // fork: the pyramid levels go to pinned host memory beside FAST .. BRIEF
    HIP_OK(hipStreamWaitEvent(h->pstream, h->pev[0], 0));
    const uint8_t* pyr = h->plan.pyr.as<uint8_t>();
    uint8_t* hpyr = (uint8_t*)h->h_pyr;
    if (h->plan.B == 1) {
      const size_t bytes = (size_t)(P.lv[P.L - 1].off + P.lv[P.L - 1].plane - P.lv[1].off);
      HIP_OK(hipMemcpyAsync(hpyr, pyr + P.lv[1].off, bytes, hipMemcpyDeviceToHost, h->pstream));
    } else {
      for (int l = 1; l < P.L; ++l)
        HIP_OK(hipMemcpyAsync(hpyr + h->h_pyr_off[l], pyr + P.lv[l].off, (size_t)P.lv[l].plane,
                              hipMemcpyDeviceToHost, h->pstream));
    }
    HIP_OK(hipEventRecord(h->pev[1], h->pstream));
  }
  // count, status word (bytes 4..7 of the block's header, written there by
  // the last stage), keypoints and descriptors in one copy
  uint8_t* o = (uint8_t*)h->h_out;
  HIP_OK(hipMemcpyAsync(o, d, doff + (size_t)cap_frame * 32, hipMemcpyDeviceToHost, s));
  if (hp) HIP_OK(hipStreamWaitEvent(s, h->pev[1], 0));  // join
  return ORBX_OK;
}

// orbx_extract's halves. extract_submit: the image staged in the handle's
// pinned buffer and the call's chain (H2D, the five launches, one D2H of
// {count, status, keypoints, descriptors}) issued on its stream; the handle's
// lock is held, the image is not empty. extract_finish: after that stream was
// waited for, the outputs copied out of the pinned block.
// extract_submit = extract_prepare (plan and buffers for the image size),
// extract_stage (the copy into the pinned staging; no HIP call, so another
// thread may run it) and extract_issue (the chain on the handle's stream).
static int extract_prepare(orbx_extractor* h, const uint8_t* img, int w, int hh, size_t stride) {
  h->last_empty = false;
  if (!img || w < 0 || hh < 0 || stride < (size_t)w) return fail(ORBX_EINVAL, "bad image");
  HIP_OK(hipSetDevice(h->cfg.device));
  if (w != h->plan.W || hh != h->plan.H) {
    // the reference accepts any image size per call: re-plan for it (after
    // every launch that uses the current plan's buffers)
    if (h->ws.ev) (void)hipEventSynchronize(h->ws.ev);
    if (h->graph) (void)hipGraphExecDestroy(h->graph);
    h->graph = nullptr;
    const int rc = build_plan(h, w, hh, h->plan.B);
    if (rc) return rc;
    h->d_in.alloc(0);
  }
  const int cap_frame = h->plan.P.kp_per_frame;
  const size_t pitch = ((size_t)w + 63) & ~(size_t)63;
  const size_t out_bytes = out_desc_off(cap_frame) + (size_t)cap_frame * 32;
  int rc;
  auto drop_graph = [&]() {
    if (h->graph) (void)hipGraphExecDestroy(h->graph);
    h->graph = nullptr;
  };
  if (h->d_in.n < pitch * hh) {
    drop_graph();
    if ((rc = h->d_in.alloc(pitch * hh))) return rc;
  }
  if (h->d_out.n < out_bytes) {
    drop_graph();
    if ((rc = h->d_out.alloc(out_bytes))) return rc;
  }
  if (h->h_in_bytes < pitch * hh || h->h_out_bytes < out_bytes) drop_graph();
  if ((rc = host_reserve(&h->h_in, &h->h_in_bytes, pitch * hh)) ||
      (rc = host_reserve(&h->h_out, &h->h_out_bytes, out_bytes)))
    return rc;
  if (!h->stream) HIP_OK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  h->host_pyr_valid = false;
  if (h->graph && h->graph_hp != h->host_pyr) drop_graph();  // captured with / without the copy branch
  if (h->host_pyr) {
    const size_t pb = host_pyr_layout(h);
    if (h->h_pyr_bytes < pb) drop_graph();
    if ((rc = host_reserve(&h->h_pyr, &h->h_pyr_bytes, std::max<size_t>(pb, 64)))) return rc;
    if (!h->pstream) HIP_OK(hipStreamCreateWithFlags(&h->pstream, hipStreamNonBlocking));
    for (auto& e : h->pev)
      if (!e) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  return ORBX_OK;
}

static void extract_stage(orbx_extractor* h, const uint8_t* img, int w, int hh, size_t stride) {
  // the pinned staging buffer is free: every call waits for its chain before it returns
  // (plain stores: streaming ones that skip the destination's read-for-ownership
  // measured slower, 0.108 vs 0.100 ms per call: the copy engine then reads DRAM
  // instead of lines still in the host's caches)
  const size_t pitch = ((size_t)w + 63) & ~(size_t)63;
  if (stride == pitch) {
    memcpy(h->h_in, img, pitch * hh);
  } else {
    for (int y = 0; y < hh; ++y) memcpy((uint8_t*)h->h_in + (size_t)y * pitch, img + (size_t)y * stride, w);
  }
}

// mark: record the handle's workspace event after the chain (for work another
// stream orders after it: the stereo pair's left chain); the synchronous
// callers wait for the chain themselves, so later users find it finished
static int extract_issue(orbx_extractor* h, int w, int hh, bool mark) {
  const int cap_frame = h->plan.P.kp_per_frame;
  const size_t pitch = ((size_t)w + 63) & ~(size_t)63;
  int rc;
  auto drop_graph = [&]() {
    if (h->graph) (void)hipGraphExecDestroy(h->graph);
    h->graph = nullptr;
  };
  // the plan buffers may still be in use by a batch call on another stream
  if (h->ws.before_pending(h->stream)) return fail(ORBX_EDEVICE, "stream wait on the handle's last use failed");
  static const bool use_graph = !(getenv("ORBX_EXTRACT_GRAPH") && getenv("ORBX_EXTRACT_GRAPH")[0] == '0');
  // the first call of a size runs plain (one-time uploads and attribute
  // queries of the launchers happen outside any capture); later ones replay
  if (h->graph && (h->graph_w != w || h->graph_h != hh)) drop_graph();
  if (use_graph && !h->timing && (h->graph || (h->warm_w == w && h->warm_h == hh))) {
    if (!h->graph) {
      drop_graph();
      hipGraph_t g = nullptr;
      HIP_OK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
      rc = issue_one_frame(h, pitch, hh, cap_frame);
      const hipError_t ec = hipStreamEndCapture(h->stream, &g);
      if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
      }
      if (ec != hipSuccess) return fail(ORBX_EDEVICE, "hipStreamEndCapture: %s", hipGetErrorString(ec));
      const hipError_t ei = hipGraphInstantiate(&h->graph, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ei != hipSuccess) {
        h->graph = nullptr;
        return fail(ORBX_EDEVICE, "hipGraphInstantiate: %s", hipGetErrorString(ei));
      }
      h->graph_w = w;
      h->graph_h = hh;
      h->graph_hp = h->host_pyr;
    }
    HIP_OK(hipGraphLaunch(h->graph, h->stream));
  } else {
    if ((rc = issue_one_frame(h, pitch, hh, cap_frame))) return rc;
    h->warm_w = w;
    h->warm_h = hh;
  }
  if (mark && h->ws.after(h->stream)) return fail(ORBX_EDEVICE, "event record failed");
  h->last_batch = 1;
  h->last_single = true;
  h->last_frames = h->d_in.as<uint8_t>();
  h->last_fpitch = pitch * hh;
  h->last_rstride = pitch;
  return ORBX_OK;
}

static int extract_submit(orbx_extractor* h, const uint8_t* img, int w, int hh, size_t stride, double* t_staged) {
  const int rc = extract_prepare(h, img, w, hh, stride);
  if (rc) return rc;
  extract_stage(h, img, w, hh, stride);
  if (t_staged) *t_staged = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  return extract_issue(h, w, hh, false);
}

static int extract_finish(orbx_extractor* h, orbx_kp* kps, int cap, uint8_t* desc, int* n) {
  h->host_pyr_valid = h->host_pyr;
  const int cap_frame = h->plan.P.kp_per_frame;
  const int* head = (const int*)h->h_out;
  const int cnt = head[0], err = head[1];
  if (err) {
    // reported once, not on every later call: cleared in the handle's stream
    // order (after any batch call still using the plan, before the next one)
    if (h->ws.before(h->stream)) return fail(ORBX_EDEVICE, "stream wait on the handle's last use failed");
    HIP_OK(hipMemsetAsync(h->plan.err.p, 0, 16, h->stream));
    if (h->ws.after(h->stream)) return fail(ORBX_EDEVICE, "event record failed");
    HIP_OK(hipStreamSynchronize(h->stream));
    return fail(ORBX_ECAPACITY, "device error word 0x%x", err);
  }
  *n = cnt;
  if (cnt > cap) return fail(ORBX_ECAPACITY, "%d keypoints do not fit cap %d", cnt, cap);
  const uint8_t* o = (const uint8_t*)h->h_out + 16;
  if (kps) memcpy(kps, o, (size_t)cnt * sizeof(orbx_kp));
  if (desc) memcpy(desc, (const uint8_t*)h->h_out + out_desc_off(cap_frame), (size_t)cnt * 32);
  return ORBX_OK;
}

static void extract_empty(orbx_extractor* h) {
  // src/ORBextractor.cc:1542-1543: no outputs. Later readers of "the last
  // extraction" (the stereo matcher on the device outputs, the host pyramid)
  // see an empty one, as the reference's Frame sees empty mvKeysRight
  h->last_single = false;
  h->last_empty = true;
  h->host_pyr_valid = false;
  h->last_batch = 0;
}

int orbx_extract(orbx_handle h, const uint8_t* img, int w, int hh, size_t stride, orbx_kp* kps, int cap,
                 uint8_t* desc, int* n) {
  if (!h || !n) return fail(ORBX_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(h->mu);
  *n = 0;
  if (w == 0 || hh == 0) {
    extract_empty(h);
    return ORBX_OK;
  }
  static const bool prof = getenv("ORBX_EXTRACT_PROF") && getenv("ORBX_EXTRACT_PROF")[0] == '1';
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t0 = prof ? now() : 0;
  double t1 = 0;
  int rc = extract_submit(h, img, w, hh, stride, prof ? &t1 : nullptr);
  if (rc) return rc;
  const double t2 = prof ? now() : 0;
  HIP_OK(hipStreamSynchronize(h->stream));
  const double t3 = prof ? now() : 0;
  if ((rc = extract_finish(h, kps, cap, desc, n))) return rc;
  if (prof) {
    const double t4 = now();
    h->prof_t[0].push_back((float)(t1 - t0));
    h->prof_t[1].push_back((float)(t2 - t1));
    h->prof_t[2].push_back((float)(t3 - t2));
    h->prof_t[3].push_back((float)(t4 - t3));
  }
  return ORBX_OK;
}

int orbx_get_scales(orbx_handle h, float* s, float* is, float* s2, float* is2) {
  if (!h) return fail(ORBX_EINVAL, "null handle");
  const int L = h->cfg.nlevels;
  for (int l = 0; l < L; ++l) {
    if (s) s[l] = h->scale[l];
    if (is) is[l] = h->inv_scale[l];
    if (s2) s2[l] = h->sigma2[l];
    if (is2) is2[l] = h->inv_sigma2[l];
  }
  return ORBX_OK;
}

int orbx_get_levels_info(orbx_handle h, int* nlevels, int* lw, int* lh, int* nf) {
  if (!h) return fail(ORBX_EINVAL, "null handle");
  const ExtractParams& P = h->plan.P;
  const int L = h->cfg.nlevels;  // also before a deferred plan (sizes 0 until the first image)
  if (nlevels) *nlevels = L;
  for (int l = 0; l < L; ++l) {
    if (lw) lw[l] = P.L ? P.lv[l].w : 0;
    if (lh) lh[l] = P.L ? P.lv[l].h : 0;
    if (nf) nf[l] = h->nfeat[l];
  }
  return ORBX_OK;
}

// Synchronous reads of a handle's buffers wait for the handle's own last
// launch (its workspace event, recorded on whatever stream that launch used),
// never for the whole device: another handle's work (the other extractor of a
// stereo pair, on another thread) goes on. The copies run on the handle's stream.
static int handle_quiesce(orbx_extractor* h) {
  HIP_OK(hipSetDevice(h->cfg.device));
  if (h->ws.used) HIP_OK(hipEventSynchronize(h->ws.ev));
  if (!h->stream) HIP_OK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  return ORBX_OK;
}
static int handle_d2h(orbx_extractor* h, void* dst, const void* src, size_t bytes) {
  HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
  HIP_OK(hipStreamSynchronize(h->stream));
  return ORBX_OK;
}

int orbx_set_host_pyramid(orbx_handle h, int enable) {
  if (!h) return fail(ORBX_EINVAL, "null handle");
  std::lock_guard<std::mutex> lk(h->mu);
  h->host_pyr = enable != 0;
  h->host_pyr_valid = false;
  return ORBX_OK;
}

int orbx_get_host_pyramid(orbx_handle h, const uint8_t** levels, size_t* pitches, int cap_levels) {
  if (!h || !levels || !pitches) return fail(ORBX_EINVAL, "null argument");
  const ExtractParams& P = h->plan.P;
  if (cap_levels < P.L) return fail(ORBX_ECAPACITY, "%d levels do not fit %d entries", P.L, cap_levels);
  if (!h->host_pyr_valid)
    return fail(ORBX_EINVAL, "no host pyramid: enable it (orbx_set_host_pyramid) before an orbx_extract call");
  const size_t pitch0 = ((size_t)P.lv[0].w + 63) & ~(size_t)63;  // orbx_extract's staging pitch
  levels[0] = (const uint8_t*)h->h_in;
  pitches[0] = pitch0;
  for (int l = 1; l < P.L; ++l) {
    levels[l] = (const uint8_t*)h->h_pyr + h->h_pyr_off[l];
    pitches[l] = (size_t)P.lv[l].pitch;
  }
  return ORBX_OK;
}

int orbx_get_level(orbx_handle h, int frame, int level, int blurred, uint8_t* out, size_t out_stride) {
  if (!h || !out) return fail(ORBX_EINVAL, "null argument");
  const Plan& pl = h->plan;
  if (level < 0 || level >= pl.P.L || frame < 0 || frame >= h->last_batch)
    return fail(ORBX_EINVAL, "no such frame/level");
  const LevelGeom& g = pl.P.lv[level];
  if (h->host_pyr_valid && !blurred && frame == 0) {
    // the pinned copy orbx_extract already made
    const uint8_t* lv[kMaxLevels];
    size_t lp[kMaxLevels];
    if (int rc = orbx_get_host_pyramid(h, lv, lp, kMaxLevels)) return rc;
    for (int y = 0; y < g.h; ++y) memcpy(out + (size_t)y * out_stride, lv[level] + (size_t)y * lp[level], g.w);
    return ORBX_OK;
  }
  if (int rc = handle_quiesce(h)) return rc;
  const ExtractBuffers X = buffers_of(pl);
  const uint8_t* src;
  size_t spitch;
  if (blurred) {
    src = X.blur + g.off + (long long)frame * g.plane;
    spitch = g.pitch;
  } else if (level == 0) {
    src = h->last_frames + (long long)frame * h->last_fpitch;
    spitch = h->last_rstride;
  } else {
    src = X.pyr + g.off + (long long)frame * g.plane;
    spitch = g.pitch;
  }
  HIP_OK(hipMemcpy2DAsync(out, out_stride, src, spitch, g.w, g.h, hipMemcpyDeviceToHost, h->stream));
  HIP_OK(hipStreamSynchronize(h->stream));
  return ORBX_OK;
}

int orbx_get_fast_candidates(orbx_handle h, int frame, int level, orbx_kp* out, int cap, int* n) {
  if (!h || !n) return fail(ORBX_EINVAL, "null argument");
  const Plan& pl = h->plan;
  if (level < 0 || level >= pl.P.L || frame < 0 || frame >= h->last_batch)
    return fail(ORBX_EINVAL, "no such frame/level");
  if (int rc = handle_quiesce(h)) return rc;
  const LevelGeom& g = pl.P.lv[level];
  std::vector<int> cnt(g.ncells);
  std::vector<uint32_t> slots(std::max(g.nslots, 1));
  if (int rc = handle_d2h(h, cnt.data(), pl.cell_counts.as<int>() + (size_t)frame * pl.P.ncells_total + g.cell0,
                          g.ncells * 4))
    return rc;
  if (int rc = handle_d2h(h, slots.data(), pl.slots.as<uint32_t>() + (size_t)frame * pl.P.slots_per_frame + g.slot0,
                          (size_t)g.nslots * 4))
    return rc;
  int k = 0;
  for (int c = 0; c < g.ncells; ++c) {
    const CellGeom& cg = pl.cells[g.cell0 + c];
    for (int i = 0; i < cnt[c]; ++i, ++k) {
      if (k >= cap || !out) continue;
      const uint32_t key = slots[cg.slot_off - g.slot0 + i];
      orbx_kp kp{(float)key_x(key), (float)key_y(key), 7.f, -1.f, (float)key_score(key), 0, -1};
      out[k] = kp;
    }
  }
  *n = k;
  return k > cap ? fail(ORBX_ECAPACITY, "cap too small") : ORBX_OK;
}

int orbx_get_status(orbx_handle h, int reset, int* status) {
  if (!h || !status) return fail(ORBX_EINVAL, "null argument");
  if (int rc = handle_quiesce(h)) return rc;
  int e = 0;
  if (int rc = handle_d2h(h, &e, h->plan.err.p, 4)) return rc;
  // cleared on the handle's stream, ordered after the batches that set it
  if (reset && e) {
    HIP_OK(hipMemsetAsync(h->plan.err.p, 0, 16, h->stream));
    if (h->ws.after(h->stream)) return fail(ORBX_EDEVICE, "event record failed");
    HIP_OK(hipStreamSynchronize(h->stream));
  }
  *status = e;
  return ORBX_OK;
}


int orbx_get_quadtree_paths(orbx_handle h, int frame0, int nframes, int* out) {
  if (!h || !out) return fail(ORBX_EINVAL, "null argument");
  const Plan& pl = h->plan;
  if (frame0 < 0 || nframes < 1 || frame0 + nframes > h->last_batch)
    return fail(ORBX_EINVAL, "frames [%d, %d) not in the last extraction (%d frames)", frame0, frame0 + nframes,
                h->last_batch);
  if (int rc = handle_quiesce(h)) return rc;
  const int L = pl.P.L;
  std::vector<int> t((size_t)nframes * L * 4);
  if (int rc = handle_d2h(h, t.data(), pl.qties.as<int>() + (size_t)frame0 * L * 4, t.size() * 4)) return rc;
  for (size_t i = 0; i < (size_t)nframes * L; ++i) out[i] = t[i * 4 + 3];
  return ORBX_OK;
}

int orbx_get_tie_stats(orbx_handle h, int frame0, int nframes, int* out) {
  if (!h || !out) return fail(ORBX_EINVAL, "null argument");
  const Plan& pl = h->plan;
  if (frame0 < 0 || nframes < 1 || frame0 + nframes > h->last_batch)
    return fail(ORBX_EINVAL, "frames [%d, %d) not in the last extraction (%d frames)", frame0, frame0 + nframes,
                h->last_batch);
  if (int rc = handle_quiesce(h)) return rc;
  const int L = pl.P.L;
  std::vector<int> t((size_t)nframes * L * 4);
  if (int rc = handle_d2h(h, t.data(), pl.qties.as<int>() + (size_t)frame0 * L * 4, t.size() * 4)) return rc;
  for (size_t i = 0; i < (size_t)nframes * L; ++i)
    for (int k = 0; k < 3; ++k) out[i * 3 + k] = t[i * 4 + k];
  return ORBX_OK;
}

int orbx_get_stage_order(orbx_handle h, char* out) {
  if (!out) return fail(ORBX_EINVAL, "null argument");
  memcpy(out, h ? h->order : extract_stage_order(), 6);
  return ORBX_OK;
}

int orbx_set_stage_order(orbx_handle h, const char* order) {
  if (!h) return fail(ORBX_EINVAL, "null handle");
  if (!valid_stage_order(order))
    return fail(ORBX_EINVAL, "stage order must be 5 letters of p b f q o: p first, o last, f before q");
  std::lock_guard<std::mutex> lk(h->mu);
  if (memcmp(h->order, order, 5) == 0) return ORBX_OK;
  // the single-frame graph was captured with the old order (after the launches using it)
  if (h->ws.ev) (void)hipEventSynchronize(h->ws.ev);
  if (h->graph) (void)hipGraphExecDestroy(h->graph);
  h->graph = nullptr;
  memcpy(h->order, order, 6);
  return ORBX_OK;
}

int orbx_get_stage_times(orbx_handle h, float* ms, const char** names, int cap, int* n) {
  auto name_of = [](char c) -> const char* {
    switch (c) {
      case 'p': return "Pyramid/Resize";
      case 'b': return "Gaussian Blur";
      case 'f': return "FAST+Grid";
      case 'q': return "Make quadtree";
      default: return "Compute angle+ORB descriptor+scale";
    }
  };
  const char* order = h->order;
  if (!h || !n) return fail(ORBX_EINVAL, "null argument");
  *n = 0;
  if (!h->timing) return ORBX_OK;
  HIP_OK(hipEventSynchronize(h->ev[5]));
  for (int i = 0; i < 5 && i < cap; ++i) {
    float t = 0;
    HIP_OK(hipEventElapsedTime(&t, h->ev[i], h->ev[i + 1]));
    if (ms) ms[i] = t;
    if (names) names[i] = name_of(order[i]);
    *n = i + 1;
  }
  return ORBX_OK;
}

int orbx_set_stage_events(orbx_handle h, void** events) {
  if (!h || !events) return fail(ORBX_EINVAL, "null argument");
  for (int i = 0; i < ORBX_STAGE_EVENTS; ++i) h->user_ev[i] = events[i];
  h->has_user_ev = true;
  return ORBX_OK;
}

// ---------------------------------------------------------- plumbing
int orbx_device_count(int* n) {
  if (!n) return fail(ORBX_EINVAL, "null");
  HIP_OK(hipGetDeviceCount(n));
  return ORBX_OK;
}
int orbx_set_device(int d) { HIP_OK(hipSetDevice(d)); return ORBX_OK; }
int orbx_malloc(void** p, size_t b) { HIP_OK(hipMalloc(p, b)); return ORBX_OK; }
int orbx_free(void* p) { HIP_OK(hipFree(p)); return ORBX_OK; }
int orbx_memcpy_htod(void* d, const void* s, size_t b) { HIP_OK(hipMemcpy(d, s, b, hipMemcpyHostToDevice)); return ORBX_OK; }
int orbx_memcpy_dtoh(void* d, const void* s, size_t b) { HIP_OK(hipMemcpy(d, s, b, hipMemcpyDeviceToHost)); return ORBX_OK; }
int orbx_memset(void* d, int v, size_t b) { HIP_OK(hipMemset(d, v, b)); return ORBX_OK; }
int orbx_host_alloc(void** p, size_t b) { HIP_OK(hipHostMalloc(p, b, hipHostMallocDefault)); return ORBX_OK; }
int orbx_host_free(void* p) { HIP_OK(hipHostFree(p)); return ORBX_OK; }
int orbx_memcpy_htod_async(void* d, const void* s, size_t b, void* st) {
  HIP_OK(hipMemcpyAsync(d, s, b, hipMemcpyHostToDevice, (hipStream_t)st));
  return ORBX_OK;
}
int orbx_memcpy_dtoh_async(void* d, const void* s, size_t b, void* st) {
  HIP_OK(hipMemcpyAsync(d, s, b, hipMemcpyDeviceToHost, (hipStream_t)st));
  return ORBX_OK;
}
int orbx_memcpy2d_htod_async(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t rows, void* st) {
  if (!d || !s || w > dp || w > sp) return fail(ORBX_EINVAL, "bad 2D copy");
  if (!w || !rows) return ORBX_OK;
  HIP_OK(hipMemcpy2DAsync(d, dp, s, sp, w, rows, hipMemcpyHostToDevice, (hipStream_t)st));
  return ORBX_OK;
}
int orbx_copy2d_kernel_async(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t rows, int blocks,
                             void* st) {
  if (!d || !s || w > dp || w > sp || blocks < 1 || (dp & 15)) return fail(ORBX_EINVAL, "bad 2D copy");
  if (!w || !rows) return ORBX_OK;
  hipLaunchKernelGGL(orbx::copy2d_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)st, (uint8_t*)d, dp,
                     (const uint8_t*)s, sp, w, rows);
  return hipGetLastError() == hipSuccess ? ORBX_OK : fail(ORBX_EDEVICE, "copy kernel launch failed");
}
int orbx_memcpy_dtod_async(void* d, const void* s, size_t b, void* st) {
  HIP_OK(hipMemcpyAsync(d, s, b, hipMemcpyDeviceToDevice, (hipStream_t)st));
  return ORBX_OK;
}
int orbx_stream_create(void** s) { HIP_OK(hipStreamCreateWithFlags((hipStream_t*)s, hipStreamNonBlocking)); return ORBX_OK; }
int orbx_stream_create_priority(void** s, int high) {
  int least = 0, greatest = 0;
  HIP_OK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  HIP_OK(hipStreamCreateWithPriority((hipStream_t*)s, hipStreamNonBlocking, high ? greatest : least));
  return ORBX_OK;
}
int orbx_stream_create_cumask(void** s, const uint32_t* mask, int nwords) {
  if (!s || !mask || nwords < 1) return fail(ORBX_EINVAL, "bad argument");
  HIP_OK(hipExtStreamCreateWithCUMask((hipStream_t*)s, (uint32_t)nwords, mask));
  return ORBX_OK;
}
int orbx_stream_destroy(void* s) { HIP_OK(hipStreamDestroy((hipStream_t)s)); return ORBX_OK; }
int orbx_stream_synchronize(void* s) { HIP_OK(hipStreamSynchronize((hipStream_t)s)); return ORBX_OK; }
int orbx_event_create(void** e) { HIP_OK(hipEventCreate((hipEvent_t*)e)); return ORBX_OK; }
int orbx_event_destroy(void* e) { HIP_OK(hipEventDestroy((hipEvent_t)e)); return ORBX_OK; }
int orbx_event_record(void* e, void* s) { HIP_OK(hipEventRecord((hipEvent_t)e, (hipStream_t)s)); return ORBX_OK; }
int orbx_sincosf_glibc(const float* x, int n, float* s, float* c) {
  if (n < 0 || (n && (!x || !s || !c))) return fail(ORBX_EINVAL, "bad argument");
  for (int i = 0; i < n; ++i) glibc_sincosf(x[i], s + i, c + i);
  return ORBX_OK;
}
int orbx_stream_wait_event(void* s, void* e) {
  HIP_OK(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)e, 0));
  return ORBX_OK;
}
int orbx_event_elapsed_ms(void* a, void* b, float* ms) {
  HIP_OK(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b));
  return ORBX_OK;
}

}  // extern "C"

int orbx::copy_to_host_async(void* host_dst, const void* dev_src, size_t bytes, hipStream_t stream) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host_dst, 0) != hipSuccess) return fail(ORBX_EDEVICE, "hipHostGetDevicePointer failed");
  const int blocks = (int)std::min<size_t>(64, (bytes + 4095) / 4096);
  hipLaunchKernelGGL(orbx::copy2d_kernel, dim3(std::max(blocks, 1)), dim3(256), 0, stream, (uint8_t*)d, bytes,
                     (const uint8_t*)dev_src, bytes, bytes, (size_t)1);
  return hipGetLastError() == hipSuccess ? ORBX_OK : fail(ORBX_EDEVICE, "copy kernel launch failed");
}

// A process-wide helper thread for orbm_stereo_frame: it copies the right
// image into its handle's pinned staging while the calling thread stages and
// issues the left one, so the two copies take two host cores as the
// reference's two extraction threads do, without spawning threads per frame.
// One job at a time: a caller that finds it busy copies inline. The worker
// makes no HIP call. ORBX_STAGE_THREAD=0: both copies on the calling thread.
namespace {
class StageHelper {
 public:
  static StageHelper& get() {
    static StageHelper s;
    return s;
  }
  bool try_post(orbx_extractor* h, const uint8_t* img, int w, int hh, size_t stride) {
    if (busy_.test_and_set(std::memory_order_acquire)) return false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!th_.joinable()) th_ = std::thread([this] { loop(); });
      h_ = h;
      img_ = img;
      w_ = w;
      hh_ = hh;
      stride_ = stride;
      state_.store(1, std::memory_order_relaxed);
    }
    cv_.notify_one();
    return true;
  }
  void wait() {  // the posted copy is done (spin briefly, then yield)
    for (int i = 0; state_.load(std::memory_order_acquire) != 2; ++i) {
      if (i < 2000) __builtin_ia32_pause();
      else std::this_thread::yield();
    }
    state_.store(0, std::memory_order_relaxed);
    busy_.clear(std::memory_order_release);
  }
  ~StageHelper() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_one();
    if (th_.joinable()) th_.join();
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return quit_ || state_.load(std::memory_order_relaxed) == 1; });
      if (quit_) return;
      lk.unlock();
      extract_stage(h_, img_, w_, hh_, stride_);
      state_.store(2, std::memory_order_release);
      lk.lock();
    }
  }
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic_flag busy_ = ATOMIC_FLAG_INIT;
  std::atomic<int> state_{0};  // 0 idle, 1 posted, 2 done
  bool quit_ = false;
  orbx_extractor* h_ = nullptr;
  const uint8_t* img_ = nullptr;
  int w_ = 0, hh_ = 0;
  size_t stride_ = 0;
};
}  // namespace

int orbx::extract_pair(orbx_handle L, orbx_handle R, const uint8_t* imL, size_t strideL, const uint8_t* imR,
                       size_t strideR, int w, int hh, const std::function<int(hipStream_t)>& between,
                       orbx_kp* kpsL, int capL, uint8_t* descL, int* nL, orbx_kp* kpsR, int capR, uint8_t* descR,
                       int* nR, double* stamps) {
  auto stamp = [stamps](int i) {
    if (stamps) stamps[i] = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  if (!L || !R || !nL || !nR) return fail(ORBX_EINVAL, "null argument");
  if (L == R) return fail(ORBX_EINVAL, "left and right need two extractor handles");
  if (w <= 0 || hh <= 0) return fail(ORBX_EINVAL, "empty image");
  if (L->cfg.device != R->cfg.device) return fail(ORBX_EINVAL, "left and right extractors on different devices");
  std::unique_lock<std::mutex> lkL(L->mu, std::defer_lock), lkR(R->mu, std::defer_lock);
  std::lock(lkL, lkR);
  *nL = *nR = 0;
  // left first: its chain runs while the right image is staged
  int rc;
  if ((rc = extract_prepare(L, imL, w, hh, strideL)) || (rc = extract_prepare(R, imR, w, hh, strideR))) return rc;
  static const bool use_helper = !(getenv("ORBX_STAGE_THREAD") && getenv("ORBX_STAGE_THREAD")[0] == '0');
  const bool posted = use_helper && StageHelper::get().try_post(R, imR, w, hh, strideR);
  extract_stage(L, imL, w, hh, strideL);
  stamp(0);
  if ((rc = extract_issue(L, w, hh, true))) {
    if (posted) StageHelper::get().wait();
    return rc;
  }
  stamp(1);
  if (posted) StageHelper::get().wait();
  else extract_stage(R, imR, w, hh, strideR);
  stamp(2);
  if ((rc = extract_issue(R, w, hh, false))) return rc;
  stamp(3);
  const int rb = between(R->stream);
  stamp(4);
  // both streams: `between` may have failed before it ordered anything after the right chain
  HIP_OK(hipStreamSynchronize(L->stream));
  HIP_OK(hipStreamSynchronize(R->stream));
  stamp(5);
  if ((rc = extract_finish(L, kpsL, capL, descL, nL)) || (rc = extract_finish(R, kpsR, capR, descR, nR))) return rc;
  stamp(6);
  return rb;
}
