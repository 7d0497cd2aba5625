// orbx_internal.h — device/host shared layout of the MI355X ORB front-end.
//
// Memory layout in HBM (one extractor handle, B = max_batch frames):
//   level 0          : the caller's frames (read in place, never copied)
//   pyramid levels>=1: level-major planes  [l][B][h_l][pitch_l]   u8
//   blurred levels   : level-major planes  [l][B][h_l][pitch_l]   u8
//   FAST key slots   : [B][slots_per_frame]  u32 packed (x|y<<12|score<<24),
//                      one fixed slot range per grid cell (cap = NMS bound)
//   cell counts      : [B][ncells_total]     i32
//   quadtree keys    : [B][kp_per_frame]     u32 packed, level-major slots
//   quadtree counts  : [B][L]                i32
//   outputs          : caller's [B][cap] orbx_kp + [B][cap][32] u8 + [B] i32
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>

#include "../../include/orbx_c.h"

namespace orbx {

constexpr int kMaxLevels = 16;
constexpr int kEdgeThreshold = 19;      // EDGE_THRESHOLD  src/ORBextractor.cc:97
constexpr int kPatchSize = 31;          // PATCH_SIZE      src/ORBextractor.cc:95
constexpr int kHalfPatch = 15;          // HALF_PATCH_SIZE src/ORBextractor.cc:96
constexpr int kGridW = 30;              // W               src/ORBextractor.cc:1126
constexpr int kMaxRoi = 66;             // largest FAST cell ROI side (+6 halo)
constexpr int kMaxLevelDim = 4096;      // packed key coordinates are 12 bits
#ifndef ORBX_QT_THREADS
#define ORBX_QT_THREADS 512
#endif
constexpr int kQtThreads = ORBX_QT_THREADS;  // quadtree workgroup size

struct LevelGeom {
  int w, h, pitch;
  long long plane;   // bytes of one frame's plane (h * pitch)
  long long off;     // byte offset of this level's planes in the pyramid / blur buffers
  // INTER_LINEAR resize from level l-1 (l >= 1): offsets into the resize table
  int xtab, ytab, xmax, area2x;
  // FAST grid (ComputeKeyPointsOctTree src/ORBextractor.cc:1133-1147)
  int minBX, minBY, maxBX, maxBY;
  int nCols, nRows, wCell, hCell;
  int cell0, ncells;     // range in the cell table
  int slot0, nslots;     // key-slot range of this level inside a frame's slots
  int slot_stride;       // cell c of the level: slots slot0 + c * slot_stride .. (+ its cap)
  // DistributeOctTree (src/ORBextractor.cc:889-898)
  int N, nIni, boxW, boxH;
  float hX;
  int kcap, kbase;       // quadtree output slots of this level inside a frame
  float scale;           // mvScaleFactor[l]
  float size;            // (float)(int)(PATCH_SIZE * mvScaleFactor[l])
  int xtab2;             // band pyramid column table: {sx, a0 | a1 << 16}, replicate folded in
  // sorted-key quadtree (orbx_quadtree.hip): path-code tables of this level
  // in the resize table (u32 units: x codes, then y codes), their lengths
  // (tw | th << 16) and the code layout (bin shift | Dh << 8 | log2 bins << 16);
  // qt_tab < 0: the level's codes do not separate every position (legacy rounds)
  int qt_tab, qt_dims, qt_bits;
};

// keypoint slots per orient+BRIEF workgroup; every level's slot range starts
// at a multiple of it (orbx_host.hip plan)
constexpr int kKpGroup = 8;

struct CellGeom {
  int16_t c0, r0, c1, r1;  // ROI [c0,c1) x [r0,r1) in level coordinates
  int slot_off;            // first key slot (frame-relative)
  int16_t cap, level;      // slot capacity (0 = cell skipped by the reference)
  // FAST staging, precomputed at plan time so that a wave needs no
  // level-indexed parameter after its one record load (orbx_fast.hip).
  // Levels >= 1 live in the plan's pyramid buffer; level 0 is the caller's
  // frames, whose row stride the kernel applies (pitch == 0 marks level 0).
  int row_off;   // levels >= 1: byte offset of the ROI's row r0 in frame 0's plane (from the pyramid buffer); level 0: r0
  int pitch;     // levels >= 1: the level's row pitch; 0 for level 0
  int fstride;   // levels >= 1: bytes between two frames' planes
  int geo;       // (h - 1 - r0) | ceil16(w) << 16: the buffer range's rows below r0 and last readable column
};
static_assert(sizeof(CellGeom) == 32, "one 32-byte scalar load per FAST wave");

struct ExtractParams {
  int L, B;
  int t_low, t_ini, t_min;
  int slots_per_frame, ncells_total;
  unsigned ncells_magic;       // ceil(2^32 / ncells_total) when frame = mulhi(id, magic) is exact for every id of the plan's batch, else 0
  int kp_per_frame;            // == output capacity per frame
  int maxnodes, sortn;         // quadtree node-table size, bitonic size (pow2)
  int max_cells_level;         // largest ncells of any level
  int kcap_lds;                // quadtree keys kept in LDS up to this count
  int qt_lean;                 // quadtree: lean rounds (packed 16-bit key nodes, maxnodes < 16384), else the generic ones
  int qt_big;                  // quadtree: node tables past 64 KB of LDS: 1024-thread blocks, a whole CU's LDS each
  int qt_sorted;               // quadtree: the sorted-key path first (levels with code tables, K <= threads x 8, maxnodes <= 2 x threads)
  int qt_tabmax, qt_nbmax;     // largest code-table length (tw + th) and bin count of any level
  int qt_ownmax;               // sorted path: most keys of a level (spill mode past threads x 8: keys in global scratch)
  int fast_rh_max;             // largest FAST cell ROI height
  int fast_bw_max, fast_bh_max;  // largest FAST detection band
  int pattern_upstream;
  // band pyramid (orbx_pyramid.hip): one workgroup per (frame, band of rows, column tile)
  int pyr_fused;               // 0 = one launch per level instead
  int pyr_nbands;              // bands per frame
  int pyr_bands;               // int2 offset in the resize table: per (band, level) {comp_lo, comp_hi}, {own_lo, own_hi}
  int pyr_nct;                 // column tiles per band
  int pyr_ctiles;              // int2 offset: per (tile, level) {comp_lo, comp_hi}, {own_lo, own_hi}, {LDS pitch, LDS origin}
  int pyr_lds_a, pyr_lds_b;    // LDS bytes of the even-level and odd-level row buffers
  int pyr_lds_y;               // LDS bytes of the band's staged row coefficients
  // alternative tilings, one picked per launch (launch_pyramid): the
  // workgroup count nbands x nct x batch against the resident workgroups per CU
  struct PyrPlan {
    int nbands, nct, bands, ctiles, lds_a, lds_b, lds_y;
    int cost;  // largest per-tile pixel count over the levels (level 0 staged + computed rows x columns)
    int occ;   // resident workgroups per CU at this plan's LDS (occupancy API, set at plan time)
  } pyr_plan[8];
  int pyr_nplans;
  int gauss[7];                // 7-tap Gaussian fixed-point kernel (sum 257)
  // blur tiles (orbx_blur.hip), [0] large / [1] small: per frame,
  // blur_ntiles entries of the resize table from blur_tiles on, level | x0 << 4
  // | y0 << 16 each; the frame of a workgroup id by a multiply-high with
  // blur_magic when exact (else 0)
  int blur_tiles[2], blur_ntiles[2];
  unsigned blur_magic[2];
  LevelGeom lv[kMaxLevels];
  // single-frame calls: the device status word copied to status_dst by the
  // last stage (orient_brief_kernel), so the output block carries it and one
  // read-back serves both (null otherwise)
  const int* status_src;
  int* status_dst;
};

inline void select_pyr_plan(ExtractParams& P, int i) {
  const ExtractParams::PyrPlan& q = P.pyr_plan[i];
  P.pyr_nbands = q.nbands;
  P.pyr_bands = q.bands;
  P.pyr_nct = q.nct;
  P.pyr_ctiles = q.ctiles;
  P.pyr_lds_a = q.lds_a;
  P.pyr_lds_b = q.lds_b;
  P.pyr_lds_y = q.lds_y;
}

// Estimated launch time of a tiling: the largest tile's pixel count times
// the workgroups the busiest CU runs (wpc = ceil(workgroups / CUs)), less
// 13 % per co-resident one (occ per CU: LDS and registers). Measured on
// gfx950 (tools/pyr_plans.py, 32 KITTI frames alone): a CU's second resident
// band workgroup adds ~87 % of the first's time, a third ~80 %.
inline long long pyr_plan_time(long long cost, long long wgs, int cus, int occ) {
  const long long wpc = (wgs + cus - 1) / cus;
  const long long res = std::min<long long>(wpc, std::max(1, occ));
  return cost * (100 * wpc - 13 * (res - 1));
}

// The band plan for a launch of `batch` frames. The one-tile plans compete
// by (rounds of resident workgroups) x (largest tile's pixel count), the
// rule measured best over band heights for 32-frame launches; a column-tiled
// plan replaces that pick when pyr_plan_time puts it at least 15 % faster
// (the estimate's error on the measured plans: tools/pyr_plans.py). A single
// frame then spreads over many small tiles (KITTI: 53 bands x 4, one per
// CU), a 32-frame KITTI batch over 4 x 4 large ones (less halo recompute).
inline int pick_pyr_plan(const ExtractParams::PyrPlan* plans, int n, int batch, int cus) {
  int i1 = -1, i2 = -1;
  long long t1 = -1, t2 = -1;
  for (int i = 0; i < n; ++i) {
    const ExtractParams::PyrPlan& q = plans[i];
    const long long wgs = (long long)q.nbands * q.nct * batch;
    if (q.nct == 1) {
      const long long slots = (long long)cus * std::max(1, q.occ);
      const long long t = ((wgs + slots - 1) / slots) * (long long)q.cost;
      if (t1 < 0 || t < t1) i1 = i, t1 = t;
    }
    const long long t = pyr_plan_time(q.cost, wgs, cus, q.occ);
    if (t2 < 0 || t < t2) i2 = i, t2 = t;
  }
  if (i1 < 0) return i2 < 0 ? 0 : i2;
  const ExtractParams::PyrPlan& q1 = plans[i1];
  const long long t1m = pyr_plan_time(q1.cost, (long long)q1.nbands * batch, cus, q1.occ);
  return (plans[i2].nct > 1 && t2 * 115 < t1m * 100) ? i2 : i1;
}
inline int pick_pyr_plan(const ExtractParams& P, int batch, int cus) {
  return pick_pyr_plan(P.pyr_plan, P.pyr_nplans, batch, cus);
}

// Pointers to level data for one launch. Level 0 is the caller's frames.
struct LevelPtrs {
  const uint8_t* base[kMaxLevels];
  long long fstride[kMaxLevels];  // bytes between frames
  int pitch[kMaxLevels];          // bytes between rows
  int aligned16[kMaxLevels];      // base, pitch and frame stride all 16-byte aligned
};
// both travel as kernel arguments of every extraction kernel (4 KB limit)
static_assert(sizeof(ExtractParams) + sizeof(LevelPtrs) + 128 <= 4096, "kernel arguments over 4 KB");

__host__ __device__ inline uint32_t pack_key(int x, int y, int score) {
  return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)score << 24);
}
__host__ __device__ inline int key_x(uint32_t k) { return (int)(k & 0xFFFu); }
__host__ __device__ inline int key_y(uint32_t k) { return (int)((k >> 12) & 0xFFFu); }
__host__ __device__ inline int key_score(uint32_t k) { return (int)(k >> 24); }

// ------------------------------------------------------------ launchers
// (implemented in orbx_extract.hip; all asynchronous on `stream`)
struct ExtractBuffers {
  uint8_t* pyr;        // levels >= 1
  uint8_t* blur;       // all levels
  const int2* rtab;    // resize tables
  const CellGeom* cells;
  const int* umax;     // 16 ints
  uint32_t* slots;
  int* cell_counts;
  uint32_t* qkeys;
  int* qcounts;
  int* qties;          // [B][L][4] tie-straddle events, group nodes, kept keys (quadtree)
  uint32_t* qscratch;  // global fallback for quadtree keys (K > kcap_lds)
  uint16_t* qnode_scratch;
  long long qscratch_per_fl;  // entries per (frame, level)
  int* err;            // device error word
};

// orbx_extract.hip: the stages' default launch order, one letter each (p
// pyramid, b blur, f FAST, q quadtree, o orient+BRIEF), and the check of one
const char* extract_stage_order();
bool valid_stage_order(const char* order);
// pyr_event (optional): recorded on `stream` right after the pyramid stage, so
// a caller can fork work that only needs the pyramid (orbx_extract's host copy)
int launch_extract(const ExtractParams& P, const ExtractBuffers& X, const uint8_t* d_frames,
                   int batch, size_t frame_pitch, size_t row_stride, orbx_kp* d_kps,
                   uint8_t* d_desc, int* d_counts, void* stream, void** stage_events,
                   void* pyr_event = nullptr, int* status_dst = nullptr, const char* stage_order = nullptr);

// orbx_match.hip
int launch_hamming_top2(const uint8_t* A, size_t a_pitch, const int* nA, int a_cap,
                        const uint8_t* B, size_t b_pitch, const int* nB, int pairs, int* best_idx,
                        int* best, int* second, int* err, void* stream);


// orbx_stereo.hip — Frame::ComputeStereoMatches over a batch of rectified pairs.
// Pyramid pointers address pair 0; pair p's level l is at base[l] + p * fstride[l].
struct StereoParams {
  LevelPtrs pl, pr;
  int lw[kMaxLevels], lh[kMaxLevels];
  float scale[kMaxLevels], inv_scale[kMaxLevels];
  int L, nrows;        // levels; rows of level 0 (the row table's size)
  int kp_pitch, groups;
  int jobs_cap;        // SAD jobs a workgroup can hold: its share of left keypoints
  float mb, mbf;
  int stop;            // diagnostics: 1 = return after the row table, 2 = after the Hamming search
};
size_t stereo_lds_bytes(int nrows, int kp_pitch, int jobs_cap);
int launch_stereo(const StereoParams& P, const orbx_kp* kpL, const uint8_t* descL, const int* nL,
                  const orbx_kp* kpR, const uint8_t* descR, const int* nR, int pairs, float* uRight,
                  float* depth, int* sad, int* nkept, void* stream);
// orbx_init.hip — SearchForInitialization: prep, key and resolve launches per batch of pairs
struct InitParams {
  float minX, maxX, minY, maxY, invW, invH;  // F2 grid bounds
  float r;                                   // windowSize
  float nnratio;
  int check_ori;
  int kp_pitch;
  long long ws_ints;  // per-pair workspace stride in ints (set by the launcher)
  int dshift, obits, dclamp;  // key layout (set by the launcher from nnratio)
  uint32_t omask;
  long long* prof;  // diagnostics (ORBX_INIT_PROF=1): resolve-kernel phase clocks per pair, or null
};
constexpr size_t kInitLdsBudget = 160 * 1024 - 512;
size_t init_ws_bytes_per_pair(int kp_pitch);
int search_init_max_pitch(float nnratio);  // kp_pitch bound of launch_search_init at this ratio
int launch_search_init(const InitParams& P, const orbx_kp* kp1, const uint8_t* desc1, const int* n1,
                       const orbx_kp* kp2, const uint8_t* desc2, const int* n2, float* prev, int* ws,
                       int* matches12, int* nmatches, int pairs, void* stream);
// orbx_project.hip — SearchByProjection(Frame&, vector<MapPoint*>, th), one frame per workgroup
struct ProjParams {
  float minX, maxX, minY, maxY, invW, invH;  // Frame grid bounds, FRAME_GRID_COLS/ROWS over their extent
  float scale[kMaxLevels];                   // mvScaleFactors
  float th, nnratio;
  int kp_pitch, mp_pitch, has_uright;
  int max_rounds;                            // fixed-point rounds before the sequential pass
  long long* prof;                           // diagnostics: per-frame phase clocks, or null
};
size_t proj_lds_bytes(int kp_pitch);
int launch_search_proj(const ProjParams& P, const orbx_kp* kps, const uint8_t* desc, const int* n,
                       const float* uright, const uint8_t* blocked, const orbm_map_point_proj* mps,
                       const uint8_t* mpdesc, const int* nmp, int frames, int* out, int* nmatches, void* stream);
// orbx_project_pose.hip — the pose-projection SearchByProjection overloads, one frame per workgroup
struct PoseParams {
  int mode;                                  // ORBM_PROJ_LAST_FRAME / KEYFRAME / SIM3
  float minX, maxX, minY, maxY, invW, invH;  // grid bounds (image bounds of IsInImage / the u, v tests)
  float scale[kMaxLevels];                   // mvScaleFactors
  float pred_thr[kMaxLevels];                // PredictScale thresholds (orbm_predict_scale_thresholds)
  float inv_sigma2[kMaxLevels];              // mvInvLevelSigma2 (FUSE reprojection test)
  int L;                                     // mnScaleLevels
  float th;                                  // window factor
  int dist_th;                               // TH_HIGH / ORBdist / TH_LOW
  int check_ori;
  int kp_pitch, mp_pitch, has_uright;
  int max_rounds;                            // fixed-point rounds before the sequential pass
};
size_t pose_lds_bytes(int kp_pitch);
int launch_search_pose(const PoseParams& P, const orbx_kp* kps, const uint8_t* desc, const int* n,
                       const float* uright, const uint8_t* blocked, const orbm_pose* poses,
                       const orbm_map_point_world* mps, const uint8_t* mpdesc, const int* nmp, int frames, int* picks,
                       int* out, int* nmatches, void* stream);
// orbx_triangulate.hip — SearchForTriangulation, one keyframe pair per workgroup
struct TriSide {  // one side of the pairs; pitches of 0 share one keyframe across pairs
  const orbx_kp* kps;
  const uint8_t* desc;
  const float* uright;
  const uint8_t* has_mp;
  const int* n;
  const uint32_t* nodes;
  const int* off;  // node_pitch + 1 entries per pair
  const int* idx;
  const int* nn;
  int kp_pitch, node_pitch;
};
struct TriParams {
  float scale2[kMaxLevels], sigma2[kMaxLevels];  // pKF2->mvScaleFactors, mvLevelSigma2
  int only_stereo, check_ori, out_pitch;
};
int launch_search_tri(const TriParams& P, const TriSide& A, const TriSide& B, const orbm_tri_pair* pairs, int npairs,
                      int* matches12, int* nmatches, void* stream);
// Stream order of a handle's device workspace: a launch that uses it first
// waits for the last launch that used it (on whatever stream that was), so
// calls of one handle on different streams never overlap on its scratch.
struct WsOrder {
  hipEvent_t ev = nullptr;
  bool used = false;
  int before(hipStream_t s) {
    return used && hipStreamWaitEvent(s, ev, 0) != hipSuccess ? ORBX_EDEVICE : ORBX_OK;
  }
  // the same, but no wait when the last use has already finished (a
  // cross-stream wait is a barrier packet the next launch pays for); for the
  // synchronous entry points, which wait for their own work before returning
  // and so record no event after it
  int before_pending(hipStream_t s) {
    if (!used || hipEventQuery(ev) == hipSuccess) return ORBX_OK;
    return hipStreamWaitEvent(s, ev, 0) != hipSuccess ? ORBX_EDEVICE : ORBX_OK;
  }
  int after(hipStream_t s) {
    if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return ORBX_EDEVICE;
    if (hipEventRecord(ev, s) != hipSuccess) return ORBX_EDEVICE;
    used = true;
    return ORBX_OK;
  }
  void release() {
    if (ev) (void)hipEventDestroy(ev);
    ev = nullptr;
    used = false;
  }
};
// The streams a handle's status-word writers last ran on, each with an event
// recorded after its last such launch: a status poll waits for these events,
// not for the device (other handles' and threads' work goes on).
struct StreamMarks {
  static constexpr int kMax = 16;
  hipStream_t s[kMax] = {};
  hipEvent_t ev[kMax] = {};
  int n = 0;
  int mark(hipStream_t st) {
    int i = 0;
    while (i < n && s[i] != st) ++i;
    if (i == n) {
      if (n == kMax) {  // forget the oldest stream after waiting for it
        if (hipEventSynchronize(ev[0]) != hipSuccess) return ORBX_EDEVICE;
        hipEvent_t e0 = ev[0];
        for (int k = 1; k < n; ++k) { s[k - 1] = s[k]; ev[k - 1] = ev[k]; }
        ev[n - 1] = e0;
        i = n - 1;
      } else {
        if (!ev[i] && hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return ORBX_EDEVICE;
        ++n;
      }
      s[i] = st;
    }
    return hipEventRecord(ev[i], st) == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
  }
  int wait() {
    for (int i = 0; i < n; ++i)
      if (hipEventSynchronize(ev[i]) != hipSuccess) return ORBX_EDEVICE;
    return ORBX_OK;
  }
  void release() {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : ev) e = nullptr;
    n = 0;
  }
};
// orbx_host.hip: the workspace order of an extractor (its pyramid is read by
// the stereo matcher)
WsOrder* extractor_ws(orbx_handle h);
// orbx_host.hip: where the handle's last orbx_extract left its frame's
// outputs on the device (count, keypoints at a pitch of `cap`, descriptors);
// an empty image leaves cap = 0 and null pointers (no keypoints);
// ORBX_EINVAL when the last extraction was not an orbx_extract call
int extractor_last_output(orbx_handle h, const int** d_count, const orbx_kp** d_kps, const uint8_t** d_desc,
                          int* cap);
// orbx_host.hip: raise a kernel's dynamic-LDS limit on the current device to at
// least `bytes` (never lowers it; process-wide, thread-safe)
int raise_lds_limit(const void* fn, size_t bytes);
// orbx_host.hip: the pyramid of frames [frame0, frame0 + n) of an extractor's last extraction
int extractor_pyramid(orbx_handle h, int frame0, int n, LevelPtrs* lp, int* w, int* hgt, float* scale,
                      float* inv_scale, int* L);
// orbx_host.hip: `bytes` from device memory to pinned host memory by a copy
// kernel on `stream` (a blit launch, as a graph's memcpy node runs, instead of
// a copy-engine transfer and its start-up latency)
int copy_to_host_async(void* host_dst, const void* dev_src, size_t bytes, hipStream_t stream);
// orbx_host.hip: the stereo Frame's two extractions (src/Frame.cc:77-80) as two
// orbx_extract calls make them, from one thread and with one wait: left staged
// and launched on its handle's stream, right on its own (the two run
// concurrently), then `between(right's stream)` enqueues the work that reads
// both outputs on the device (ComputeStereoMatches; the left chain, started
// first, has normally finished by then, so its wait costs nothing on the
// critical path), then both streams are waited for and the outputs copied
// out. Two distinct handles, non-empty images of one size.
int extract_pair(orbx_handle L, orbx_handle R, const uint8_t* imL, size_t strideL, const uint8_t* imR,
                 size_t strideR, int w, int h, const std::function<int(hipStream_t)>& between, orbx_kp* kpsL,
                 int capL, uint8_t* descL, int* nL, orbx_kp* kpsR, int capR, uint8_t* descR, int* nR,
                 double* stamps = nullptr);  // diagnostics: host clock after each of its 7 phases

}  // namespace orbx
