/*
 * orbx_c.h — C ABI of the MI355X-native ORB front-end (liborbx.so).
 *
 * This is the drop-in boundary for ORB-SLAM2's ORBextractor / ORBmatcher hot
 * path (reference: falfab/orb_slam_cuda). Plain C types only; device memory
 * is addressed by plain pointers and HIP streams by `void*`.
 *
 * Entry points and the reference interface each one replaces:
 *   orbx_create            ORBextractor::ORBextractor(nfeatures, scaleFactor,
 *                          nlevels, iniThFAST, minThFAST, width, height)
 *                          include/ORBextractor.h:82-83, src/ORBextractor.cc:496-560
 *   orbx_destroy           ORBextractor::~ORBextractor  src/ORBextractor.cc:800
 *   orbx_extract           ORBextractor::operator()(image, mask, keypoints,
 *                          descriptors)  include/ORBextractor.h:90-92,
 *                          src/ORBextractor.cc:1538-1815 (CPU branch 1701-1809)
 *   orbx_extract_batch     same, B frames per call, device-resident in/out
 *                          (frame batching for MI355X; no reference equivalent)
 *   orbx_get_scales        GetScaleFactors / GetInverseScaleFactors /
 *                          GetScaleSigmaSquares / GetInverseScaleSigmaSquares
 *                          include/ORBextractor.h:94-114
 *   orbx_get_levels_info   GetLevels + per-level sizes / mnFeaturesPerLevel
 *   orbx_get_level         public mvImagePyramid[level]  include/ORBextractor.h:116
 *                          (read by Frame::ComputeStereoMatches src/Frame.cc:472,562,579)
 *   orbx_set_host_pyramid / orbx_get_host_pyramid  the same, filled by
 *                          orbx_extract itself into pinned memory (opt-in)
 *   orbm_descriptor_distance  ORBmatcher::DescriptorDistance
 *                          include/ORBmatcher.h:44, src/ORBmatcher.cc:1647-1663
 *   orbm_search_for_initialization  ORBmatcher::SearchForInitialization
 *                          include/ORBmatcher.h:69, src/ORBmatcher.cc:405-520
 *                          (+ Frame::AssignFeaturesToGrid/GetFeaturesInArea
 *                          src/Frame.cc:229-244,326-391)
 *   orbm_search_by_bow     ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...)
 *                          include/ORBmatcher.h:65, src/ORBmatcher.cc:159-288;
 *                          kf_vs_kf=1: SearchByBoW(KeyFrame*, KeyFrame*, ...)
 *                          include/ORBmatcher.h:66, src/ORBmatcher.cc:522-655
 *   orbm_hamming_top2      the best/second Hamming inner loop shared by every
 *                          matcher (dense, device-resident, batched)
 *   orbm_compute_stereo_matches  Frame::ComputeStereoMatches (mvuRight, mvDepth)
 *                          include/Frame.h:82, src/Frame.cc:465-639
 *   orbm_stereo_frame      the stereo Frame constructor's two ExtractORB
 *                          threads + ComputeStereoMatches, src/Frame.cc:77-89
 *   orbm_search_by_projection  ORBmatcher::SearchByProjection(Frame&,
 *                          const vector<MapPoint*>&, th)  include/ORBmatcher.h:48,
 *                          src/ORBmatcher.cc:45-126 (Tracking::SearchLocalPoints)
 *   orbm_search_by_projection_last_frame  ORBmatcher::SearchByProjection(
 *                          Frame& CurrentFrame, const Frame& LastFrame, th,
 *                          bMono)  include/ORBmatcher.h:52, src/ORBmatcher.cc:1328-1470
 *                          (Tracking::TrackWithMotionModel)
 *   orbm_search_by_projection_keyframe  ORBmatcher::SearchByProjection(
 *                          Frame&, KeyFrame*, const set<MapPoint*>&, th,
 *                          ORBdist)  include/ORBmatcher.h:56,
 *                          src/ORBmatcher.cc:1472-1599 (Tracking::Relocalization)
 *   orbm_search_by_projection_sim3  ORBmatcher::SearchByProjection(KeyFrame*,
 *                          cv::Mat Scw, const vector<MapPoint*>&,
 *                          vector<MapPoint*>&, th)  include/ORBmatcher.h:60,
 *                          src/ORBmatcher.cc:290-403 (LoopClosing::ComputeSim3)
 *   orbm_fuse / orbm_fuse_sim3  ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>,
 *                          th) / Fuse(KeyFrame*, Scw, vpPoints, th,
 *                          vpReplacePoint)  include/ORBmatcher.h:80,83,
 *                          src/ORBmatcher.cc:825-975, 977-1100 (matching part)
 *   orbm_search_by_sim3    ORBmatcher::SearchBySim3  include/ORBmatcher.h:77,
 *                          src/ORBmatcher.cc:1102-1326
 *   orbm_search_by_projection_pose_batch  all of the above, batched on device
 *   orbm_search_for_triangulation  ORBmatcher::SearchForTriangulation
 *                          include/ORBmatcher.h:72, src/ORBmatcher.cc:657-823
 *   orbv_load_text / orbv_create  ORBVocabulary::loadFromTextFile
 *                          (DBoW2 TemplatedVocabulary, include/ORBVocabulary.h:30,
 *                          Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1418)
 *   orbv_transform         Frame::ComputeBoW  src/Frame.cc:394-401 ->
 *                          TemplatedVocabulary::transform(features, BowVector,
 *                          FeatureVector, levelsup)  TemplatedVocabulary.h:1127-1256
 *
 * Error behaviour: every call returns ORBX_OK or a negative code; the
 * message of the last failure on the calling thread is orbx_last_error().
 * The C++ shim (include/orb_slam2/ORBextractor.h) turns codes into
 * std::runtime_error, as the reference's NVXIO_SAFE_CALL does
 * (nvxio/include/OVX/UtilityOVX.hpp:129-137).
 *
 * Threading: handles are independent and may be used concurrently from
 * different threads (the reference runs two extractors at once for stereo,
 * src/Frame.cc:77-80). One handle is not reentrant.
 */
#ifndef ORBX_C_H
#define ORBX_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBX_OK 0
#define ORBX_EINVAL (-1)    /* bad argument / unsupported configuration   */
#define ORBX_EDEVICE (-2)   /* HIP runtime error or no gfx950 device       */
#define ORBX_ECAPACITY (-3) /* caller buffer or internal capacity too small */
#define ORBX_ENOMEM (-4)    /* device allocation failed                    */

/* Binary-identical to cv::KeyPoint: pt.x, pt.y, size, angle, response
 * (float), octave, class_id (int) = 28 bytes. class_id is always -1. */
typedef struct orbx_kp {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} orbx_kp;

/* Parity-mode switches. */
#define ORBX_SCALE_U 0        /* level geometry from scaleFactor^l (default)   */
#define ORBX_SCALE_F 1        /* fork: VX ORB pyramid sizes override scales    */
#define ORBX_PATTERN_FORK 0   /* bit_pattern_31_[96] = VX_FAILURE-2 = -3 (default) */
#define ORBX_PATTERN_UPSTREAM 1 /* upstream ORB-SLAM2 table (-2)              */

typedef struct orbx_config {
  int nfeatures;      /* ORBextractor.nFeatures                  */
  float scale_factor; /* ORBextractor.scaleFactor                */
  int nlevels;        /* ORBextractor.nLevels (1..16)            */
  int ini_th_fast;    /* ORBextractor.iniThFAST                  */
  int min_th_fast;    /* ORBextractor.minThFAST                  */
  int width, height;  /* frame size (Camera.width / Camera.height); 0 x 0 in
                       * mode U = unknown until the first orbx_extract, as
                       * Tracking passes for the mono yamls that lack the keys
                       * (src/Tracking.cc:124-133): the plan is then built on
                       * the first image (mode F needs the size: EINVAL) */
  int device;         /* HIP device ordinal                       */
  int max_batch;      /* frames per orbx_extract_batch call (>=1); the
                       * pyramid planes of levels >= 1 of all max_batch
                       * frames must stay below 2 GiB (FAST's cell records
                       * hold 32-bit plane offsets): about 316 frames at
                       * 1920x1080 with 8 levels x 1.2, 39 at 4096x4096;
                       * orbx_create returns EINVAL past it */
  int scale_mode;     /* ORBX_SCALE_*                             */
  int pattern_mode;   /* ORBX_PATTERN_*                           */
  int reserved[5];    /* must be zero                             */
} orbx_config;

typedef struct orbx_extractor* orbx_handle;

const char* orbx_last_error(void);
const char* orbx_version(void);

int orbx_create(const orbx_config* cfg, orbx_handle* out);
int orbx_destroy(orbx_handle h);

/* Maximum keypoints one frame can produce (sizes per-frame output slots);
 * 0 while a handle created with width/height 0 has seen no image. */
int orbx_frame_capacity(orbx_handle h);

/* ORBextractor::operator(): host image in, host keypoints/descriptors out.
 * Synchronous. Empty image (w==0||h==0) -> *n = 0, ORBX_OK (reference
 * returns with outputs untouched, src/ORBextractor.cc:1542-1543). */
int orbx_extract(orbx_handle h, const uint8_t* img, int w, int h_, size_t stride,
                 orbx_kp* kps, int cap, uint8_t* desc, int* n);

/* Batched, device-resident, asynchronous on `stream` (hipStream_t; NULL =
 * the default stream).
 * d_frames: batch frames of (height x width) u8, row stride `row_stride`,
 * frame i at d_frames + i*frame_pitch. The kernels read each row in 16-byte
 * chunks: every row, the last row of the last frame included, must be
 * readable up to ceil16(width) bytes from its start (a 64-byte pitch, as
 * bench.py uses, always is). Outputs: frame i's keypoints at
 * d_kps + i*cap, descriptors at d_desc + i*cap*32, count in d_counts[i],
 * where cap = orbx_frame_capacity(h). Level-major order as the reference.
 * Calls on one handle from several threads are serialised by the handle's
 * lock (a synchronous orbx_extract holds it until its own work finished). */
int orbx_extract_batch(orbx_handle h, const uint8_t* d_frames, int batch,
                       size_t frame_pitch, size_t row_stride, orbx_kp* d_kps,
                       uint8_t* d_desc, int* d_counts, void* stream);

int orbx_get_scales(orbx_handle h, float* scale, float* inv_scale,
                    float* sigma2, float* inv_sigma2);
int orbx_get_levels_info(orbx_handle h, int* nlevels, int* level_w,
                         int* level_h, int* nfeatures_per_level);
/* Copy pyramid level `level` of frame `frame` of the last extraction to host
 * (mvImagePyramid). `blurred`=1 returns the 7x7 Gaussian-blurred level used
 * for the descriptors instead (stage probe). Waits for the handle's own last
 * launch only (not the device); served from the host pyramid below when that
 * holds the level. */
int orbx_get_level(orbx_handle h, int frame, int level, int blurred,
                   uint8_t* out, size_t out_stride);
/* Host pyramid: the reference's public mvImagePyramid (include/ORBextractor.h:116),
 * filled in place by ComputePyramid (src/ORBextractor.cc:1837-1863) and read
 * by Frame::ComputeStereoMatches (src/Frame.cc:472,562,579). With enable != 0
 * every later orbx_extract also leaves its frame's pyramid in handle-owned
 * pinned host memory: the levels >= 1 are copied on a branch of the call's
 * graph forked right after the pyramid kernel (the copy overlaps FAST ..
 * BRIEF), level 0 is the call's own pinned input staging. Off by default. */
int orbx_set_host_pyramid(orbx_handle h, int enable);
/* The host pyramid of the last orbx_extract: levels[l] / pitches[l] (bytes
 * between rows) for l < nlevels, valid until the next extraction on the
 * handle (as the reference's buffers are until its next operator() call).
 * ORBX_EINVAL when it is off or the last extraction was a batch call. */
int orbx_get_host_pyramid(orbx_handle h, const uint8_t** levels, size_t* pitches,
                          int cap_levels);
/* Stage probe: FAST + per-cell NMS candidates of (frame, level) of the last
 * extraction, in reference order, as keypoints (x,y relative to the border
 * box, response = FAST score). */
int orbx_get_fast_candidates(orbx_handle h, int frame, int level, orbx_kp* out,
                             int cap, int* n);
/* Quadtree tie-rule exposure of frames [frame0, frame0 +
 * nframes) of the last extraction: per (frame, level) three ints {events,
 * group nodes, kept keypoints}. DistributeOctTree's sorted rounds split nodes
 * in (size, heap-pointer) order (src/ORBextractor.cc:1041-1042) and stop at N;
 * an event is a cut-off inside a group of equal-size nodes, where the
 * reference's choice depends on its allocator and this library's on node
 * creation order (the oracle's rule). `kept keypoints` counts the outputs
 * that come from that group. Synchronous (waits for the device). */
int orbx_get_tie_stats(orbx_handle h, int frame0, int nframes, int* out);
/* Which DistributeOctTree implementation ran per (frame, level) of frames
 * [frame0, frame0 + nframes) of the last extraction: 1 = the sorted-key path
 * (node = contiguous range of keys binned by quadtree path code), 0 = the
 * legacy rounds (levels with more keys than the workgroup's registers hold,
 * a node to split below the bins' depth, or ORBX_QT_SORTED=0). Both give the
 * reference's output; this is a diagnostic for tests and profiles.
 * Synchronous (waits for the device). */
int orbx_get_quadtree_paths(orbx_handle h, int frame0, int nframes, int* out);
/* Device status word of the handle's kernels since the last call (0 = ok;
 * bit 1: quadtree round limit, bit 2: quadtree output over capacity, bit 3:
 * a quadtree node without keys, an internal invariant, never expected).
 * Waits for the device; `reset` != 0 clears it. orbx_extract checks and clears
 * it itself; batch callers (orbx_extract_batch) poll it here. */
int orbx_get_status(orbx_handle h, int reset, int* status);
/* The rBRIEF test table the kernels use (bit_pattern_31_,
 * src/ORBextractor.cc:236-494): 1024 ints in the reference's flat order
 * (test i = entries 4i..4i+3 = x0, y0, x1, y1), for pattern_mode
 * ORBX_PATTERN_FORK (entry 96 = VX_FAILURE-2 = -3, :261-262) or
 * ORBX_PATTERN_UPSTREAM (-2). Host only, no device needed. */
int orbx_get_pattern(int pattern_mode, int* out1024);
/* Per-stage device time (ms) of the last extraction, in launch order
 * (orbx_get_stage_order), stage names as the reference's GetTime labels
 * (src/ORBextractor.cc:1131,1331,1737,1753,1841). Filled only when the handle
 * was created with timing enabled (ORBX_TIMING=1 in the environment). */
int orbx_get_stage_times(orbx_handle h, float* ms, const char** names, int cap,
                         int* n);
/* The extraction stages' launch order of handle h (NULL: the default) as 5
 * letters + NUL into out[6]: p pyramid, b Gaussian blur, f FAST + grid, q
 * quadtree, o angle + descriptor (default "pfqbo", or ORBX_EXTRACT_ORDER).
 * Host only. */
int orbx_get_stage_order(orbx_handle h, char* out);
/* Set a handle's stage launch order for its later extractions: the pyramid
 * first, orient+BRIEF last, FAST before the quadtree ("pfqbo", "pbfqo",
 * "pfbqo"). Results do not depend on it; how the launches interleave with a
 * caller's other streams does (a pipeline that overlaps ComputeBoW and
 * SearchByBoW with the next extraction runs faster with "pbfqo", DESIGN.md
 * section 6). ORBX_EINVAL for any other string. */
int orbx_set_stage_order(orbx_handle h, const char* order);
/* Record caller-owned HIP events (ORBX_STAGE_EVENTS of them, hipEvent_t as
 * void*) between the stages of the NEXT orbx_extract_batch call on its
 * stream: ev[0] before the first stage, ev[i + 1] after the i-th stage
 * launched (orbx_get_stage_order). Lets a caller time every kernel of every
 * call without a host synchronisation. One-shot. */
#define ORBX_STAGE_EVENTS 6
int orbx_set_stage_events(orbx_handle h, void** events);

/* The descriptor rotation's sin/cos (src/ORBextractor.cc:199-200: glibc
 * sinf/cosf on a float argument) exactly as the kernels compute it, on the
 * host: s[i] = sinf(x[i]), c[i] = cosf(x[i]) for |x| < 120. For checking the
 * restatement against a host libm. */
int orbx_sincosf_glibc(const float* x, int n, float* s, float* c);

/* ------------------------------------------------------------- matcher */
typedef struct orbx_matcher* orbm_handle;

const char* orbm_last_error(void);

/* Workspace for batched matching of up to max_pairs frame pairs with up to
 * max_kps keypoints per frame. */
int orbm_create(int device, int max_pairs, int max_kps, orbm_handle* out);
int orbm_destroy(orbm_handle m);

/* Device status word of the matcher's batched kernels since the last call
 * (0 = ok; bit 16: orbm_hamming_top2 input over its limits, nA[p] > a_cap
 * or nB[p] > 65535, the excess rows / candidates were not searched; bit 32:
 * orbm_search_by_bow_batch saw a count above kp_pitch or a FeatureVector
 * index outside [0, n), which was skipped). SearchForInitialization keeps no
 * candidate lists (8 smallest keys per query) and never sets it. Waits for
 * the matcher's own launches that may set it (on whatever streams they ran),
 * not for the device; `reset` != 0 clears it. The synchronous entry points
 * check and clear it themselves.
 *
 * Device workspaces (candidate lists, stereo SAD, pose picks, SearchByBoW row
 * records and histograms) belong to the
 * handle: batched calls on different streams are ordered by the library
 * (each waits for the previous user of the workspace), so they never
 * overlap on it. The same holds for an extractor handle's plan buffers, and
 * orbm_compute_stereo_matches_batch orders itself after and before the two
 * extractors whose pyramids it reads. */
int orbm_get_status(orbm_handle m, int reset, int* status);

/* Hamming distance of two 32-byte descriptors (host, exact). */
int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Dense best/second search, device-resident, batched over `pairs`:
 * for pair p, A = d_A + p*a_pitch (nA[p] rows of 32 B), B likewise.
 * Outputs per query row (stride a_cap): best index (-1 if none), best
 * distance and second-best distance (256 when absent), with SearchByBoW's
 * sequential semantics (strict '<', first index wins ties). nB[p] <= 65535
 * (the candidate index shares a 32-bit key with the distance). */
int orbm_hamming_top2(orbm_handle m, const uint8_t* d_A, size_t a_pitch,
                      const int* d_nA, int a_cap, const uint8_t* d_B,
                      size_t b_pitch, const int* d_nB, int pairs,
                      int* d_best_idx, int* d_best, int* d_second, void* stream);

/* Frame-side inputs of SearchForInitialization: mvKeysUn (orbx_kp) and
 * descriptors, plus the image bounds Frame uses for its 64x48 grid
 * (mnMinX, mnMaxX, mnMinY, mnMaxY). */
typedef struct orbm_grid_bounds {
  float min_x, max_x, min_y, max_y;
} orbm_grid_bounds;

/* ORBmatcher::SearchForInitialization on host buffers (synchronous).
 * prev_xy: 2*n1 floats, vbPrevMatched, updated in place. matches12: n1.
 * n1 / n2 are not bounded by the matcher's max_kps: only octave-0 keypoints
 * take part (compacted on the host; up to the batch call's bound below per
 * frame: 10,192 at the reference's 0.9, 8192 at 0.7), and the kernels keep no candidate lists, so any
 * window density is matched, never refused for want of scratch. */
int orbm_search_for_initialization(orbm_handle m, const orbx_kp* kp1,
                                   const uint8_t* desc1, int n1,
                                   const orbx_kp* kp2, const uint8_t* desc2,
                                   int n2, orbm_grid_bounds bounds,
                                   float* prev_xy, int window, float nnratio,
                                   int check_ori, int* matches12,
                                   int* nmatches);

/* Batched device-resident variant: pair p matches frame F1 = (d_kp1 +
 * p*kp_pitch, d_desc1 + p*kp_pitch*32, d_n1[p]) against F2 likewise.
 * d_prev_xy: pairs x kp_pitch x 2 floats (in/out), or NULL to centre the
 * windows on F1's own keypoints (the initial mvbPrevMatched of
 * Tracking::MonocularInitialization, src/Tracking.cc:645-647; nothing is
 * written back then); d_matches12: pairs x kp_pitch; d_nmatches: pairs.
 * kp_pitch <= min(max_kps, 10,192, 2^(20 - dbits)); any window density is
 * matched (the kernels keep each query's 8 smallest keys, kInitK, not its
 * candidate list). 10,192 is the resolve kernel's LDS; dbits depends on
 * nnratio: distances are clamped to 2^dbits - 1 with the smallest dbits in
 * 6..9 for which nnratio * (2^dbits - 1) > 50, so the bound is 10,192 for
 * nnratio > 0.794, 8192 above 0.394, 4096 above 0.196 and 2048 below.
 * ECAPACITY's message names the bound that applied. */
int orbm_search_for_initialization_batch(
    orbm_handle m, const orbx_kp* d_kp1, const uint8_t* d_desc1,
    const int* d_n1, const orbx_kp* d_kp2, const uint8_t* d_desc2,
    const int* d_n2, int kp_pitch, int pairs, orbm_grid_bounds bounds,
    float* d_prev_xy, int window, float nnratio, int check_ori,
    int* d_matches12, int* d_nmatches, void* stream);

/* The MapPoint fields ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>,
 * th) reads (filled by Frame::isInFrustum, src/Frame.cc:277-324):
 * mTrackProjX/Y/XR, mTrackViewCos, mnTrackScaleLevel; track_in_view =
 * mbTrackInView && !isBad(); obs_positive = Observations() > 0. 24 bytes. */
typedef struct orbm_map_point_proj {
  float proj_x, proj_y, proj_xr, view_cos;
  int32_t predicted_level;
  uint8_t track_in_view, obs_positive, pad[2];
} orbm_map_point_proj;

/* SearchByProjection(Frame&, vpMapPoints, th) on host buffers (synchronous).
 * Frame: mvKeysUn (kps), mDescriptors, N; uright = mvuRight (NULL for a
 * monocular frame); bounds = mnMinX/MaxX/MinY/MaxY; scale = mvScaleFactors
 * (nlevels); blocked[idx] = mvpMapPoints[idx] && Observations() > 0 on entry.
 * Map points in vpMapPoints order with their descriptors (GetDescriptor()).
 * out[idx] = index into vpMapPoints of the point assigned to keypoint idx by
 * this call (the shim stores vpMapPoints[out[idx]] into mvpMapPoints[idx]),
 * -1 where the keypoint was not assigned. Up to 8192 map points. */
int orbm_search_by_projection(orbm_handle m, const orbx_kp* kps, const uint8_t* desc,
                              int n, const float* uright, orbm_grid_bounds bounds,
                              const float* scale, int nlevels, const uint8_t* blocked,
                              const orbm_map_point_proj* mps, const uint8_t* mpdesc,
                              int nmp, float th, float nnratio, int* out,
                              int* nmatches);

/* Batched device-resident variant: frame f's keypoints at d_kps + f*kp_pitch
 * (d_n[f] of them; descriptors, uright (or NULL), blocked and out likewise at
 * kp_pitch), its map points at d_mps + f*mp_pitch (d_nmp[f]; descriptors
 * likewise). All frames share the grid bounds and scale factors. */
int orbm_search_by_projection_batch(
    orbm_handle m, const orbx_kp* d_kps, const uint8_t* d_desc, const int* d_n,
    int kp_pitch, const float* d_uright, orbm_grid_bounds bounds,
    const float* scale, int nlevels, const uint8_t* d_blocked,
    const orbm_map_point_proj* d_mps, const uint8_t* d_mpdesc, const int* d_nmp,
    int mp_pitch, int frames, float th, float nnratio, int* d_out,
    int* d_nmatches, void* stream);

/* ---------------------------------------- pose-projection search overloads
 * The SearchByProjection overloads that project MapPoint world positions
 * with a pose inside the matcher. Frame/KeyFrame camera fields: fx, fy, cx,
 * cy, mb, mbf and rows 0..2 of mTcw, row-major (the Sim3 overload passes
 * Scw rows 0..2 here). */
typedef struct orbm_camera {
  float fx, fy, cx, cy, mb, mbf;
  float Tcw[12];
} orbm_camera;

/* A MapPoint as these overloads read it: GetWorldPos(), GetNormal() (Sim3
 * overload), mfMinDistance / mfMaxDistance (GetMin/MaxDistanceInvariance
 * scale them by 0.8f / 1.2f; PredictScale reads mfMaxDistance), the angle
 * and octave of the keypoint that holds the point in the source frame
 * (LastFrame.mvKeysUn[i].angle / mvKeys[i].octave; pKF->mvKeysUn[i].angle),
 * valid = the point is searched (LastFrame: pMP && !mvbOutlier[i]; KeyFrame:
 * pMP && !isBad() && !sAlreadyFound.count(pMP); Sim3: !isBad() && not in
 * vpMatched), obs_positive = Observations() > 0. 48 bytes. */
typedef struct orbm_map_point_world {
  float pos[3], normal[3];
  float min_distance, max_distance, angle;
  int32_t octave;
  uint8_t valid, obs_positive, pad[6];
} orbm_map_point_world;

#define ORBM_PROJ_LAST_FRAME 1 /* SearchByProjection  src/ORBmatcher.cc:1328-1470 */
#define ORBM_PROJ_KEYFRAME 2   /* SearchByProjection  src/ORBmatcher.cc:1472-1599 */
#define ORBM_PROJ_SIM3 3       /* SearchByProjection  src/ORBmatcher.cc:290-403   */
#define ORBM_PROJ_FUSE 4       /* Fuse(pKF, vpMapPoints, th)  :825-975            */
#define ORBM_PROJ_FUSE_SIM3 5  /* Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) :977-1100 */
#define ORBM_PROJ_SIM3_MATCH 6 /* SearchBySim3, one direction  :1102-1326       */

/* Per-frame projection prepared on the host from a camera (the scalar
 * cv::Mat work each overload does once per call): Rt = the 3x4 transform
 * applied to world points (Sim3: sRcw/scw | tcw/scw), Ow = -R^T t (camera
 * centre), level_mode (last-frame overload: 0 = levels lo-1..lo+1,
 * 1 = bForward: lo.., 2 = bBackward: 0..lo), Rt2 = the second transform of
 * SearchBySim3 (camera A to camera B: [sR21 | t21] or [sR12 | t12]).
 * 132 bytes. */
typedef struct orbm_pose {
  float Rt[12];
  float Ow[3];
  float fx, fy, cx, cy, mbf;
  int32_t level_mode;
  float Rt2[12];
} orbm_pose;

/* Fill *out for `mode` (LAST_FRAME, KEYFRAME, SIM3, FUSE, FUSE_SIM3; for
 * SIM3 and FUSE_SIM3 cam->Tcw = Scw). Tlw: LastFrame.mTcw rows 0..2
 * (ORBM_PROJ_LAST_FRAME only, else NULL); mono = bMono. Host only. */
int orbm_prepare_pose(int mode, const orbm_camera* cam, const float* Tlw, int mono,
                      orbm_pose* out);

/* The two directions of SearchBySim3 (src/ORBmatcher.cc:1114-1124):
 * out[0] projects pKF1's points into pKF2 (Rt = T1w, Rt2 = [sR21 | t21]),
 * out[1] pKF2's into pKF1 (Rt = T2w, Rt2 = [sR12 | t12]); both use cam1's
 * fx, fy, cx, cy as the reference does. R12 row-major 3x3. Host only. */
int orbm_prepare_sim3_match(const orbm_camera* cam1, const float* T1w, const float* T2w,
                            float s12, const float* R12, const float* t12, orbm_pose* out);

/* MapPoint::PredictScale(dist, Frame* or KeyFrame*) (src/MapPoint.cc:390-422)
 * as the kernels evaluate it: the level is the number of thresholds
 * thr[0..nlevels-2] the ratio mfMaxDistance/dist reaches, thr[k-1] = the
 * least float ratio with ceil(logf(ratio)/logf(scale_factor)) >= k, found
 * on the host with the host's logf. Host only. */
int orbm_predict_scale_thresholds(float scale_factor, int nlevels, float* thr);
int orbm_predict_scale(float max_distance, float dist, float scale_factor, int nlevels);

/* SearchByProjection(CurrentFrame, LastFrame, th, bMono), host buffers,
 * synchronous. Current frame as for orbm_search_by_projection (uright NULL
 * for monocular); blocked[i2] = mvpMapPoints[i2] && Observations() > 0 on
 * entry; cur = CurrentFrame camera and pose; Tlw = LastFrame.mTcw rows 0..2;
 * one map point record + descriptor per LastFrame keypoint. out[i2] = index
 * of the LastFrame keypoint whose point this call stored in
 * CurrentFrame.mvpMapPoints[i2]; -1 = not touched; -2 = stored and then
 * cleared (NULL) by the rotation consistency check. */
int orbm_search_by_projection_last_frame(
    orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n, const float* uright,
    orbm_grid_bounds bounds, const float* scale, int nlevels, const uint8_t* blocked,
    const orbm_camera* cur, const float* Tlw, const orbm_map_point_world* mps,
    const uint8_t* mpdesc, int nmp, float th, int mono, int check_ori, int* out,
    int* nmatches);

/* SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist):
 * has_mp[i2] = CurrentFrame.mvpMapPoints[i2] != NULL on entry; one record
 * per pKF->GetMapPointMatches() entry; scale_factor = mfScaleFactor (for
 * PredictScale). out as above. */
int orbm_search_by_projection_keyframe(
    orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n, orbm_grid_bounds bounds,
    const float* scale, int nlevels, float scale_factor, const uint8_t* has_mp,
    const orbm_camera* cur, const orbm_map_point_world* mps, const uint8_t* mpdesc, int nmp,
    float th, int orb_dist, int check_ori, int* out, int* nmatches);

/* SearchByProjection(pKF, Scw, vpPoints, vpMatched, th): pKF's keypoints,
 * grid bounds, mvScaleFactors and mfScaleFactor; kf->Tcw = Scw rows 0..2;
 * matched[idx] >= 0 where vpMatched[idx] is set on entry (NULL: none).
 * out[idx] = index into vpPoints stored in vpMatched[idx] by this call, -1
 * otherwise. */
int orbm_search_by_projection_sim3(
    orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n, orbm_grid_bounds bounds,
    const float* scale, int nlevels, float scale_factor, const orbm_camera* kf,
    const orbm_map_point_world* mps, const uint8_t* mpdesc, int nmp, int th,
    const int* matched, int* out, int* nmatches);

/* Fuse(pKF, vpMapPoints, th), the matching part (src/ORBmatcher.cc:825-930):
 * pKF's keypoints, descriptors, mvuRight (NULL = all monocular), grid bounds,
 * mvScaleFactors, mvInvLevelSigma2, mfScaleFactor, camera (fx, fy, cx, cy,
 * mbf, Tcw); one record per point (valid = pMP && !isBad() &&
 * !IsInKeyFrame(pKF)). out[i] = keypoint index the point fuses into
 * (bestDist <= TH_LOW), -1 otherwise; *nfused = their count. The caller
 * applies the reference's side effects in point order (:932-957: Replace
 * when the keypoint holds a MapPoint, else AddObservation + AddMapPoint),
 * re-checking isBad() at each point's turn. */
int orbm_fuse(orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n, const float* uright,
              orbm_grid_bounds bounds, const float* scale, const float* inv_sigma2, int nlevels,
              float scale_factor, const orbm_camera* kf, const orbm_map_point_world* mps,
              const uint8_t* mpdesc, int nmp, float th, int* out, int* nfused);

/* Fuse(pKF, Scw, vpPoints, th, vpReplacePoint), the matching part
 * (:977-1081): kf->Tcw = Scw rows 0..2; valid = !isBad() && not in
 * pKF->GetMapPoints(). out[i] = bestIdx (<= TH_LOW) or -1. The caller's
 * in-order tail (:1083-1097): GetMapPoint(bestIdx) ? vpReplacePoint[i] =
 * it (if !isBad()) : AddObservation + AddMapPoint. */
int orbm_fuse_sim3(orbm_handle m, const orbx_kp* kps, const uint8_t* desc, int n,
                   orbm_grid_bounds bounds, const float* scale, int nlevels, float scale_factor,
                   const orbm_camera* kf, const orbm_map_point_world* mps, const uint8_t* mpdesc,
                   int nmp, float th, int* out, int* nfused);

/* SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (:1102-1326).
 * Per keyframe: keypoints, descriptors, grid bounds, mvScaleFactors, Tcw
 * rows 0..2 and one record per keypoint for GetMapPointMatches() (valid =
 * pMP && !vbAlreadyMatched && !isBad()). cam1: pKF1's fx, fy, cx, cy.
 * match12[i1] = idx2 for every new mutual match (the shim stores
 * vpMapPoints2[idx2] into vpMatches12[i1]), -1 otherwise; *nfound. */
int orbm_search_by_sim3(orbm_handle m, const orbx_kp* kps1, const uint8_t* desc1, int n1,
                        orbm_grid_bounds bounds1, const float* T1w,
                        const orbm_map_point_world* mps1, const uint8_t* mpdesc1,
                        const orbx_kp* kps2, const uint8_t* desc2, int n2,
                        orbm_grid_bounds bounds2, const float* T2w,
                        const orbm_map_point_world* mps2, const uint8_t* mpdesc2,
                        const float* scale, int nlevels, float scale_factor,
                        const orbm_camera* cam1, float s12, const float* R12, const float* t12,
                        float th, int* match12, int* nfound);

/* Batched device-resident variant of every pose mode: frame f's keypoints
 * at d_kps + f*kp_pitch (d_n[f]; descriptors, d_uright (LAST_FRAME, FUSE,
 * or NULL) and d_blocked likewise), its points at d_mps + f*mp_pitch
 * (d_nmp[f]; descriptors likewise), d_poses[f] from orbm_prepare_pose /
 * orbm_prepare_sim3_match. d_blocked: the blocking state on entry of the
 * mode (LAST_FRAME: a point with observations; KEYFRAME: any point; SIM3:
 * vpMatched set; ignored by FUSE, FUSE_SIM3, SIM3_MATCH). dist_th: TH_HIGH
 * (100) / ORBdist / TH_LOW (50); th: the window factor. inv_sigma2
 * (FUSE): mvInvLevelSigma2, nlevels floats (host), else NULL. d_out: per keypoint at
 * kp_pitch (LAST_FRAME, KEYFRAME, SIM3) or per point at mp_pitch (FUSE,
 * FUSE_SIM3, SIM3_MATCH: the keypoint each point matched, -1). All frames
 * share grid bounds, scale factors and scale_factor. */
int orbm_search_by_projection_pose_batch(
    orbm_handle m, int mode, const orbx_kp* d_kps, const uint8_t* d_desc, const int* d_n,
    int kp_pitch, const float* d_uright, orbm_grid_bounds bounds, const float* scale,
    int nlevels, float scale_factor, const uint8_t* d_blocked, const orbm_pose* d_poses,
    const orbm_map_point_world* d_mps, const uint8_t* d_mpdesc, const int* d_nmp,
    int mp_pitch, int frames, float th, int dist_th, int check_ori,
    const float* inv_sigma2, int* d_out, int* d_nmatches, void* stream);

/* DBoW2::FeatureVector as CSR: nodes[k] ascending NodeIds; the feature
 * indices of node k are idx[off[k] .. off[k+1]). Each feature index appears
 * in at most one node (DBoW2 guarantees it; checked). */
typedef struct orbm_feature_vector {
  const uint32_t* nodes;
  const int* off;
  const int* idx;
  int n_nodes;
} orbm_feature_vector;

/* ORBmatcher::SearchByBoW on host buffers (synchronous).
 * A = KeyFrame (descriptors, mvKeysUn angles, MapPoint-valid mask = pMP &&
 * !pMP->isBad()). kf_vs_kf = 0: B = Frame (mp_validB ignored), out[nB] =
 * matched KF feature index per frame feature or -1 (vpMapPointMatches).
 * kf_vs_kf = 1: B = KeyFrame 2, out[nA] = idx2 or -1 (vpMatches12). */
int orbm_search_by_bow(orbm_handle m, const uint8_t* descA, const float* angleA,
                       const uint8_t* mp_validA, int nA,
                       orbm_feature_vector fvA, const uint8_t* descB,
                       const float* angleB, const uint8_t* mp_validB, int nB,
                       orbm_feature_vector fvB, float nnratio, int check_ori,
                       int kf_vs_kf, int* out, int* nmatches);

/* Batched device-resident SearchByBoW over `pairs` (A, B) pairs on `stream`,
 * one workgroup per pair (Tracking::TrackReferenceKeyFrame calls the KF-F
 * form once per frame, src/Tracking.cc:839-842; relocalisation once per
 * candidate, :1445). Pair p: keypoints (orbx_kp, angles read from them),
 * descriptors (32 B rows) and MapPoint masks at p*kp_pitch of each side
 * (d_mpA/d_mpB NULL = every feature has one; d_mpB is read for kf_vs_kf
 * only), counts d_nA[p]/d_nB[p]; FeatureVectors as CSR at p*node_pitch
 * (offsets at p*(node_pitch+1)), d_nnA[p]/d_nnB[p] nodes: exactly the layout
 * orbv_transform_batch writes (node_pitch = its cap). Output at p*kp_pitch:
 * kf_vs_kf = 0: out[iB] = matched A index or -1 (vpMapPointMatches);
 * kf_vs_kf = 1: out[iA] = matched B index or -1; d_nmatches[p]. */
int orbm_search_by_bow_batch(orbm_handle m, int pairs, int kp_pitch, int node_pitch,
                             const orbx_kp* d_kpA, const uint8_t* d_descA, const int* d_nA,
                             const uint8_t* d_mpA, const uint32_t* d_nodesA, const int* d_offA,
                             const int* d_idxA, const int* d_nnA, const orbx_kp* d_kpB,
                             const uint8_t* d_descB, const int* d_nB, const uint8_t* d_mpB,
                             const uint32_t* d_nodesB, const int* d_offB, const int* d_idxB,
                             const int* d_nnB, float nnratio, int check_ori, int kf_vs_kf,
                             int* d_out, int* d_nmatches, void* stream);

/* Frame::ComputeStereoMatches (src/Frame.cc:465-639) on host buffers
 * (synchronous). kpL/descL = mvKeys/mDescriptors of the left image, kpR/descR
 * = mvKeysRight/mDescriptorsRight; the SAD refinement reads mvImagePyramid of
 * the two extractors, i.e. the pyramid of frame 0 of each handle's last
 * extraction (`left` and `right` may be one handle only if it is re-run, as
 * each extraction replaces its pyramid). mb = baseline (m), mbf = baseline x
 * fx. Outputs uRight/depth (nL floats, -1 where no match: mvuRight, mvDepth)
 * and the number of kept matches. A block-match window reaching off the
 * pyramid level (an OpenCV range assertion in the reference) rejects that
 * keypoint. */
int orbm_compute_stereo_matches(orbm_handle m, orbx_handle left, orbx_handle right,
                                const orbx_kp* kpL, const uint8_t* descL, int nL,
                                const orbx_kp* kpR, const uint8_t* descR, int nR,
                                float mb, float mbf, float* uRight, float* depth,
                                int* nkept);
/* The same for the frames of the two handles' last orbx_extract calls, as the
 * stereo Frame constructor runs it right after its two extractions
 * (src/Frame.cc:77-89): keypoints and descriptors are read where those calls
 * left them on the device (no host-to-device copy). nL = the left call's
 * keypoint count (mvKeys.size()); outputs as above. ORBX_EINVAL when either
 * handle's last extraction was a batch call. An empty left or right image
 * (orbx_extract of 0 x 0) matches nothing: uRight = depth = -1, nkept = 0.
 * When the extractors' capacity passes the device path's limits (max_kps, or
 * the stereo kernel's LDS at very large nFeatures) the call copies both
 * extractions to the host and runs orbm_compute_stereo_matches on their
 * actual counts instead of failing. */
int orbm_compute_stereo_matches_last(orbm_handle m, orbx_handle left, orbx_handle right,
                                     float mb, float mbf, float* uRight, float* depth,
                                     int nL, int* nkept);
/* The stereo Frame constructor's extraction and matching steps
 * (src/Frame.cc:77-89: ExtractORB on threadLeft / threadRight, then
 * ComputeStereoMatches) from the calling thread with one device round trip.
 * Outputs equal orbx_extract(left, img_left ...), orbx_extract(right,
 * img_right ...) and orbm_compute_stereo_matches_last(m, left, right, mb, mbf,
 * uRight, depth, *n_left, nkept) made in that order; the two extraction chains
 * run concurrently on the handles' streams and the stereo kernel follows on
 * the device. Both images are w x h (their own row strides); uRight and depth
 * hold cap_left floats. `left` and `right` are two distinct handles. Empty
 * images (w or h 0) take the three calls' own path. */
int orbm_stereo_frame(orbm_handle m, orbx_handle left, orbx_handle right,
                      const uint8_t* img_left, size_t stride_left,
                      const uint8_t* img_right, size_t stride_right, int w, int h,
                      float mb, float mbf, orbx_kp* kps_left, int cap_left,
                      uint8_t* desc_left, int* n_left, orbx_kp* kps_right,
                      int cap_right, uint8_t* desc_right, int* n_right,
                      float* uRight, float* depth, int* nkept);

/* Batched device-resident variant: pair p = left frame (left_frame0 + p) of
 * `left`'s last orbx_extract_batch and right frame (right_frame0 + p) of
 * `right`'s (the same handle may hold both when one batch extracted left and
 * right frames together); keypoints/descriptors at d_kpL + p*kp_pitch,
 * d_descL + p*kp_pitch*32, d_nL[p] (right likewise). Outputs d_uRight /
 * d_depth: pairs x kp_pitch floats; d_nkept: pairs. Run it on the stream
 * that extracted (or after it) and before the next extraction on either
 * handle, which overwrites the pyramid. */
int orbm_compute_stereo_matches_batch(
    orbm_handle m, orbx_handle left, int left_frame0, orbx_handle right,
    int right_frame0, const orbx_kp* d_kpL, const uint8_t* d_descL,
    const int* d_nL, const orbx_kp* d_kpR, const uint8_t* d_descR,
    const int* d_nR, int kp_pitch, int pairs, float mb, float mbf,
    float* d_uRight, float* d_depth, int* d_nkept, void* stream);

/* ------------------------------------------------------ vocabulary (DBoW2) */
typedef struct orbv_vocabulary* orbv_handle;

const char* orbv_last_error(void);

/* TemplatedVocabulary::loadFromTextFile: header "k L scoring weighting", then
 * one line per node "parent isLeaf d0..d31 weight" (node ids in line order,
 * the root is node 0). Lines without tokens are skipped. The tree is kept on
 * `device`. */
int orbv_load_text(const char* path, int device, orbv_handle* out);

/* The same from arrays in file order (node 0 = root; parent[i] < i for i > 0;
 * is_leaf marks words, numbered in node order; desc n_nodes x 32 bytes;
 * weight per node). scoring: L1 0, L2 1, CHI_SQUARE 2, KL 3, BHATTACHARYYA 4,
 * DOT_PRODUCT 5; weighting: TF_IDF 0, TF 1, IDF 2, BINARY 3. */
int orbv_create(int k, int L, int scoring, int weighting, int n_nodes,
                const int* parent, const uint8_t* is_leaf, const uint8_t* desc,
                const double* weight, int device, orbv_handle* out);
int orbv_destroy(orbv_handle v);
int orbv_info(orbv_handle v, int* k, int* L, int* scoring, int* weighting,
              int* n_nodes, int* n_words);

/* transform(features, BowVector, FeatureVector, levelsup) on host buffers
 * (synchronous), n <= 8192 descriptors of 32 bytes. BowVector: bow_n words
 * ascending with their values (capacity n). FeatureVector as CSR: fv_n node
 * ids ascending (file node ids), fv_off[fv_n + 1], fv_idx feature indices
 * (capacity n each; fv_off capacity n + 1). word_ids / node_ids / weights:
 * optional per-feature outputs (NULL to skip). */
int orbv_transform(orbv_handle v, const uint8_t* desc, int n, int levelsup,
                   uint32_t* bow_words, double* bow_values, int* bow_n,
                   uint32_t* fv_nodes, int* fv_off, int* fv_idx, int* fv_n,
                   uint32_t* word_ids, uint32_t* node_ids, double* weights);

/* Batched device-resident variant: frame f's descriptors at d_desc +
 * f*desc_pitch, d_n[f] of them (<= cap <= 8192). Outputs per frame at pitch
 * cap (fv_off: cap + 1): d_bow_words/d_bow_values/d_bow_n,
 * d_fv_nodes/d_fv_off/d_fv_idx/d_fv_n; per-feature d_word_ids/d_node_ids/
 * d_weights (frames x cap) or all three NULL to use an internal workspace. */
int orbv_transform_batch(orbv_handle v, const uint8_t* d_desc, size_t desc_pitch,
                         const int* d_n, int frames, int cap, int levelsup,
                         uint32_t* d_bow_words, double* d_bow_values, int* d_bow_n,
                         uint32_t* d_fv_nodes, int* d_fv_off, int* d_fv_idx,
                         int* d_fv_n, uint32_t* d_word_ids, uint32_t* d_node_ids,
                         double* d_weights, void* stream);

/* ------------------------------------------------ SearchForTriangulation
 * Per pair: F12 (row-major 3x3, LocalMapping::ComputeF12) and the epipole
 * (ex, ey) of pKF1's camera centre in pKF2 (src/ORBmatcher.cc:664-670).
 * 44 bytes. */
typedef struct orbm_tri_pair {
  float F12[9];
  float ex, ey;
} orbm_tri_pair;

/* Fill *out from pKF1->GetCameraCenter() (cw1, 3 floats), pKF2's Tcw rows
 * 0..2 (T2w), pKF2's fx, fy, cx, cy (cam2) and F12. Host only. */
int orbm_prepare_triangulation(const float* cw1, const float* T2w, const float* cam2,
                               const float* F12, orbm_tri_pair* out);

/* SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
 * (src/ORBmatcher.cc:657-823), host buffers, synchronous. Per keyframe:
 * mvKeysUn, mDescriptors, mvuRight, has_mp[idx] = GetMapPoint(idx) != NULL,
 * mFeatVec (CSR). scale2 / sigma2: pKF2's mvScaleFactors / mvLevelSigma2.
 * matches12[idx1] = idx2 or -1 (vMatchedPairs = the pairs in idx1 order);
 * *nmatches = their count. */
int orbm_search_for_triangulation(
    orbm_handle m, const orbx_kp* kps1, const uint8_t* desc1, const float* uright1,
    const uint8_t* has_mp1, int n1, orbm_feature_vector fv1, const orbx_kp* kps2,
    const uint8_t* desc2, const float* uright2, const uint8_t* has_mp2, int n2,
    orbm_feature_vector fv2, const float* cw1, const float* T2w, const float* cam2,
    const float* scale2, const float* sigma2, int nlevels, const float* F12, int only_stereo,
    int check_ori, int* matches12, int* nmatches);

/* Batched device-resident variant: `pairs` keyframe pairs in one launch
 * (LocalMapping::CreateNewMapPoints: the new keyframe against each
 * neighbour). Side 1 arrays at kp_pitch1 / node_pitch1 per pair (0 and 0:
 * one pKF1 shared by every pair), side 2 at kp_pitch2 / node_pitch2.
 * d_off*: node_pitch + 1 ints per pair; d_nn*: node counts; d_n*: keypoint
 * counts. d_pairs from orbm_prepare_triangulation. scale2 / sigma2 are
 * host arrays shared by all pairs. d_matches12: pairs x out_pitch ints
 * (out_pitch >= n1); d_nmatches: pairs. */
int orbm_search_for_triangulation_batch(
    orbm_handle m, const orbx_kp* d_kps1, const uint8_t* d_desc1, const float* d_uright1,
    const uint8_t* d_has_mp1, const int* d_n1, const uint32_t* d_nodes1, const int* d_off1,
    const int* d_idx1, const int* d_nn1, int kp_pitch1, int node_pitch1,
    const orbx_kp* d_kps2, const uint8_t* d_desc2, const float* d_uright2,
    const uint8_t* d_has_mp2, const int* d_n2, const uint32_t* d_nodes2, const int* d_off2,
    const int* d_idx2, const int* d_nn2, int kp_pitch2, int node_pitch2,
    const orbm_tri_pair* d_pairs, const float* scale2, const float* sigma2, int nlevels,
    int pairs, int only_stereo, int check_ori, int* d_matches12, int out_pitch,
    int* d_nmatches, void* stream);

/* --------------------------------------------- device plumbing for hosts
 * Thin wrappers so a host without its own HIP binding (ctypes, cgo, JNI)
 * can stage buffers for the batched entry points. */
int orbx_device_count(int* n);
int orbx_set_device(int device);
int orbx_malloc(void** p, size_t bytes);
int orbx_free(void* p);
int orbx_memcpy_htod(void* dst, const void* src, size_t bytes);
int orbx_memcpy_dtoh(void* dst, const void* src, size_t bytes);
int orbx_memset(void* dst, int value, size_t bytes);
int orbx_memcpy_dtod_async(void* dst, const void* src, size_t bytes, void* stream);
/* Pinned (page-locked) host memory and asynchronous host<->device copies on
 * a stream: host-streamed input (frames uploaded per batch) and read-back. */
int orbx_host_alloc(void** p, size_t bytes);
int orbx_host_free(void* p);
int orbx_memcpy_htod_async(void* dst, const void* src, size_t bytes, void* stream);
int orbx_memcpy_dtoh_async(void* dst, const void* src, size_t bytes, void* stream);
/* Rows of `width` bytes from a host image with row stride `spitch` into device
 * rows of stride `dpitch` (the extractor's padded pitch), one DMA rectangle
 * copy: frames cross the link unpadded. */
int orbx_memcpy2d_htod_async(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                             size_t rows, void* stream);
/* The same rectangle copy done by a kernel of `blocks` 256-thread workgroups
 * reading pinned host memory (orbx_host_alloc) over the link directly, in
 * 16-byte loads, instead of by the DMA engines. */
int orbx_copy2d_kernel_async(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                             size_t rows, int blocks, void* stream);
int orbx_stream_create(void** stream);
/* A stream whose work the dispatcher prefers (high = 1) or defers (high = 0)
 * when both compete for compute units (hipStreamCreateWithPriority). */
int orbx_stream_create_priority(void** stream, int high);
/* A stream whose kernels run only on the compute units whose bits are set in
 * mask[0 .. nwords) (hipExtStreamCreateWithCUMask; bit i = CU i in the
 * runtime's order): partitions the chip between concurrent pipelines
 * (bench.py --match-cus). */
int orbx_stream_create_cumask(void** stream, const uint32_t* mask, int nwords);
int orbx_stream_destroy(void* stream);
int orbx_stream_synchronize(void* stream);
int orbx_event_create(void** ev);
int orbx_event_destroy(void* ev);
int orbx_event_record(void* ev, void* stream);
/* Make `stream` wait (on the device) for the work recorded in `ev`, so a
 * host can pipeline extraction and matching on two streams. */
int orbx_stream_wait_event(void* stream, void* ev);
int orbx_event_elapsed_ms(void* start, void* stop, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_C_H */
