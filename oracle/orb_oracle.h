/*
 * orb_oracle.h — C ABI of the CPU ORACLE (test infrastructure only).
 *
 * This library is a CPU restatement of the reference's ORB hot path
 * (falfab/orb_slam_cuda, CPU branch of ORBextractor::operator() and the
 * ORBmatcher searches). It exists ONLY to check the HIP product and to time
 * a CPU baseline: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it. The product library never links it.
 *
 * Parity status: the reference cannot be compiled here (it needs OpenCV,
 * VisionWorks and CUDA), and it ships no tests or golden
 * vectors for this path. The OpenCV primitives are restated from OpenCV 3.x
 * scalar semantics. => PARITY UNPINNED at the OpenCV
 * boundary; pinned only by the known-answer checks in tests/test_oracle.py
 * (umax, features-per-level, Hamming vs numpy on Examples/Monocular/map.yml).
 */
#pragma once
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Binary-identical to cv::KeyPoint (pt.x, pt.y, size, angle, response,
 * octave, class_id) = 28 bytes. */
typedef struct orc_kp {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} orc_kp;

typedef struct orc_config {
  int nfeatures;       /* ORBextractor.nFeatures                          */
  float scale_factor;  /* ORBextractor.scaleFactor                        */
  int nlevels;         /* ORBextractor.nLevels                            */
  int ini_th_fast;     /* ORBextractor.iniThFAST                          */
  int min_th_fast;     /* ORBextractor.minThFAST                          */
  int width, height;   /* Camera.width/height (fork ctor args)            */
  int scale_mode;      /* 0 = U (1.2^l geometry), 1 = F (VX ORB pyramid)  */
  int pattern_mode;    /* 0 = fork table (entry 96 = -3), 1 = upstream    */
} orc_config;

/* Per-level geometry the extractor derives in its constructor. */
int orc_level_info(const orc_config* cfg, int* level_w, int* level_h,
                   float* scale, float* inv_scale, float* sigma2,
                   float* inv_sigma2, int* nfeat_per_level, int* umax16);

/* Full ORBextractor::operator(): returns n keypoints (level-major order) and
 * n x 32 descriptor bytes. Returns 0, or -1 if cap is too small. */
int orc_extract(const orc_config* cfg, const uint8_t* img, int w, int h,
                size_t stride, orc_kp* kps, int cap, uint8_t* desc, int* n);

/* Stage probes (for stage-level parity tests). `out` receives level `level`
 * of the pyramid (w_l x h_l, packed) or its 7x7 Gaussian blur. */
int orc_pyramid_level(const orc_config* cfg, const uint8_t* img, int w, int h,
                      size_t stride, int level, uint8_t* out);
int orc_blur_level(const orc_config* cfg, const uint8_t* img, int w, int h,
                   size_t stride, int level, uint8_t* out);
/* FAST + per-cell NMS output of one level, in reference push order
 * (x,y relative to the border box, response = FAST score). */
int orc_fast_level(const orc_config* cfg, const uint8_t* img, int w, int h,
                   size_t stride, int level, orc_kp* kps, int cap, int* n);
/* Quadtree distribution of arbitrary keys (DistributeOctTree). */
int orc_distribute(const orc_kp* keys, int nkeys, int minX, int maxX,
                   int minY, int maxY, int N, orc_kp* out, int cap, int* n);

/* Tie-straddle exposure of the quadtree's creation-order tie rule (SURVEY.md
 * §8c): per level, the cut-offs at N that fell inside a group of equal-size
 * nodes (src/ORBextractor.cc:1041-1088), the nodes of that group and the kept
 * keypoints that came from them. */
int orc_extract_tie_stats(const orc_config* cfg, const uint8_t* img, int w, int h,
                          size_t stride, int* events, int* nodes, int* kps);
int orc_distribute_ties(const orc_kp* keys, int nkeys, int minX, int maxX, int minY,
                        int maxY, int N, int* events, int* nodes, int* kps);
/* Quadtree tie-rule study: orc_extract with the sorted
 * rounds' size ties broken by rule 0 = node creation order, later-created
 * first (the product's rule), 1 = the reference's real heap address with a
 * layout-identical ExtractorNode and its allocation sequence, 2 = creation
 * order, earlier-created first. */
int orc_extract_rule(const orc_config* cfg, int tie_rule, const uint8_t* img, int w,
                     int h, size_t stride, orc_kp* kps, int cap, uint8_t* desc, int* n);
/* Extracts nframes frames in sequence with rule_a (one extractor, as the
 * reference's Tracking thread does), then with rule_b, and reports per
 * (frame, level) whether the kept keypoint lists differ and how many
 * keypoint positions only one of them kept. */
int orc_tie_sequence(const orc_config* cfg, const uint8_t* frames, int nframes, int w,
                     int h, size_t stride, size_t frame_bytes, int rule_a, int rule_b,
                     int* differs, int* kept_diff);
/* The rBRIEF test table (bit_pattern_31_, src/ORBextractor.cc:236-494) the
 * oracle uses: 1024 entries, fork (0) or upstream (1) variant. */
void orc_pattern(int pattern_mode, signed char* out1024);

/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1647-1663). */
int orc_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Dense best/second Hamming search (SearchByBoW inner loop semantics:
 * strict '<', first index wins ties, distances start at 256). */
void orc_hamming_top2(const uint8_t* A, int nA, const uint8_t* B, int nB,
                      int* best_idx, int* best_dist, int* second_dist);

/* ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:405-520) over the
 * Frame grid (src/Frame.cc:229-244, 326-391). kp arrays are mvKeysUn.
 * prev_xy (2*n1 floats) is updated in place like vbPrevMatched. */
int orc_search_for_initialization(
    const orc_kp* kp1, const uint8_t* desc1, int n1,
    const orc_kp* kp2, const uint8_t* desc2, int n2,
    float min_x, float max_x, float min_y, float max_y,
    float* prev_xy, int window, float nnratio, int check_ori,
    int* matches12, int* nmatches);

/* ORBmatcher::SearchByBoW. FeatureVectors are CSR: fv_nodes[k] (ascending
 * NodeId), fv_off[k]..fv_off[k+1] index fv_idx. mp_valid = "MapPoint exists
 * and !isBad()". kf_vs_kf=0 -> (KeyFrame*, Frame&) variant (:159-288):
 * out[nB] = KF index matched to each frame feature or -1. kf_vs_kf=1 ->
 * (KeyFrame*, KeyFrame*) variant (:522-655): out[nA] = idx2 or -1. */
int orc_search_by_bow(
    const uint8_t* descA, const float* angleA, const uint8_t* mp_validA,
    int nA, const uint32_t* fvA_nodes, const int* fvA_off, const int* fvA_idx,
    int fvA_n,
    const uint8_t* descB, const float* angleB, const uint8_t* mp_validB,
    int nB, const uint32_t* fvB_nodes, const int* fvB_off, const int* fvB_idx,
    int fvB_n,
    float nnratio, int check_ori, int kf_vs_kf, int* out, int* nmatches);

/* Elementary OpenCV restatements, exported for unit tests. */
/* Frame::ComputeStereoMatches (src/Frame.cc:465-639) for a rectified pair.
 * Left/right keypoints + descriptors as extracted; the two image pyramids
 * per level (pointer, row stride; both images share level sizes level_w x
 * level_h); scale / inv_scale = mvScaleFactors / mvInvScaleFactors; mb =
 * baseline, mbf = baseline * fx. Writes mvuRight and mvDepth (nL floats,
 * -1 where no match survives). Returns the number of matches kept. */
int orc_compute_stereo_matches(const orc_kp* kpL, const uint8_t* descL, int nL,
                               const orc_kp* kpR, const uint8_t* descR, int nR,
                               const uint8_t* const* pyrL, const size_t* strideL,
                               const uint8_t* const* pyrR, const size_t* strideR,
                               const int* level_w, const int* level_h, int nlevels,
                               const float* scale, const float* inv_scale, float mb,
                               float mbf, float* uRight, float* depth);

float orc_fast_atan2(float y, float x);
/* The host libm's sinf/cosf (what computeOrbDescriptor calls, :199-200). */
void orc_sincosf(const float* x, int n, float* s, float* c);

/* DBoW2 vocabulary (orb_vocab.cpp). Nodes in file order, node 0 = root:
 * parent[n], leaf flag, 32-byte descriptor, weight. */
int orc_voc_load_text(const char* path, int* k, int* L, int* scoring, int* weighting, int* n_nodes, int cap,
                      int* parent, uint8_t* leaf, uint8_t* desc, double* weight);
int orc_voc_transform(int k, int L, int weighting, int scoring, int n_nodes, const int* parent, const uint8_t* leaf,
                      const uint8_t* node_desc, const double* node_weight, const uint8_t* desc, int n, int levelsup,
                      uint32_t* word_out, uint32_t* nid_out, double* w_out, uint32_t* bow_words,
                      double* bow_values, int* bow_n, uint32_t* fv_nodes, int* fv_off, int* fv_idx, int* fv_n);

/* MapPoint fields read by ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th):
 * mTrackProjX/Y/XR, mTrackViewCos, mnTrackScaleLevel, mbTrackInView && !isBad(),
 * Observations() > 0. */
typedef struct orc_map_point_proj {
  float proj_x, proj_y, proj_xr, view_cos;
  int32_t predicted_level;
  uint8_t track_in_view, obs_positive, pad[2];
} orc_map_point_proj;

int orc_search_by_projection(const orc_kp* kps, const uint8_t* desc, int n, const float* uright, float min_x,
                             float max_x, float min_y, float max_y, const float* scale, const uint8_t* blocked,
                             const orc_map_point_proj* mps, const uint8_t* mpdesc, int nmp, float th,
                             float mfNNratio, int* out, int* out_nmatches);

/* The overloads that project world points with a pose (src/ORBmatcher.cc:290-403,
 * 1328-1470, 1472-1599). Camera = Frame / KeyFrame fx, fy, cx, cy, mb, mbf and
 * rows 0..2 of mTcw (row-major 3x4; Scw for the Sim3 overload). */
typedef struct orc_camera {
  float fx, fy, cx, cy, mb, mbf;
  float Tcw[12];
} orc_camera;

/* A MapPoint as the pose overloads read it: GetWorldPos(), GetNormal(),
 * mfMinDistance / mfMaxDistance (the *DistanceInvariance getters scale them by
 * 0.8f / 1.2f), the angle and octave of the keypoint that holds it in the
 * source frame (LastFrame.mvKeysUn[i] / pKF->mvKeysUn[i]), valid = the point
 * is searched (LastFrame: pMP && !mvbOutlier[i]; KF: pMP && !isBad() && not
 * in sAlreadyFound; Sim3: !isBad() && not already found), obs_positive =
 * Observations() > 0. 48 bytes. */
typedef struct orc_map_point_world {
  float pos[3], normal[3];
  float min_distance, max_distance, angle;
  int32_t octave;
  uint8_t valid, obs_positive, pad[6];
} orc_map_point_world;

/* MapPoint::PredictScale(dist, Frame/KeyFrame*) (src/MapPoint.cc:390-422). */
int orc_predict_scale(float max_distance, float current_dist, float scale_factor, int nlevels);
/* The same on ratios = mfMaxDistance/currentDist directly (n of them). */
void orc_predict_scale_ratios(const float* ratio, int n, float scale_factor, int nlevels, int* out);

/* SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
 * (src/ORBmatcher.cc:1328-1470). Current frame: kps (mvKeysUn), desc, uright
 * (mvuRight or NULL), grid bounds, scale = mvScaleFactors, blocked[i2] =
 * mvpMapPoints[i2] && Observations() > 0 on entry. One map point record per
 * LastFrame keypoint (valid = pMP && !mvbOutlier). out[i2] = index of the
 * last-frame keypoint whose point this call stored in mvpMapPoints[i2], -1 =
 * untouched, -2 = stored and then cleared by the rotation check (NULL). */
int orc_search_by_projection_last_frame(const orc_kp* kps, const uint8_t* desc, int n, const float* uright,
                                        float min_x, float max_x, float min_y, float max_y, const float* scale,
                                        const uint8_t* blocked, const orc_camera* cur, const float* Tlw,
                                        const orc_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th,
                                        int bMono, int mbCheckOrientation, int* out, int* out_nmatches);

/* SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, sAlreadyFound, th,
 * ORBdist) (src/ORBmatcher.cc:1472-1599). has_mp[i2] = mvpMapPoints[i2] on
 * entry; one record per pKF->GetMapPointMatches() entry. out as above. */
int orc_search_by_projection_keyframe(const orc_kp* kps, const uint8_t* desc, int n, float min_x, float max_x,
                                      float min_y, float max_y, const float* scale, int nlevels,
                                      float scale_factor, const uint8_t* has_mp, const orc_camera* cur,
                                      const orc_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th,
                                      int ORBdist, int mbCheckOrientation, int* out, int* out_nmatches);

/* SearchByProjection(KeyFrame* pKF, Scw, vpPoints, vpMatched, th)
 * (src/ORBmatcher.cc:290-403). pKF's keypoints / grid; cam->Tcw = Scw rows
 * 0..2; matched[idx] >= 0 where vpMatched[idx] is set on entry. out[idx] =
 * index into vpPoints of the point stored by this call, -1 otherwise. */
int orc_search_by_projection_sim3(const orc_kp* kps, const uint8_t* desc, int n, float min_x, float max_x,
                                  float min_y, float max_y, const float* scale, int nlevels, float scale_factor,
                                  const orc_camera* kf, const orc_map_point_world* mps, const uint8_t* mpdesc,
                                  int nmp, int th, const int* matched, int* out, int* out_nmatches);

/* Fuse(pKF, vpMapPoints, th) (src/ORBmatcher.cc:825-975), the match part:
 * out[i] = bestIdx where point i (valid = pMP && !isBad() &&
 * !IsInKeyFrame(pKF) at call time) matches with bestDist <= TH_LOW, else -1.
 * uright = pKF->mvuRight; inv_sigma2 = mvInvLevelSigma2. The side effects
 * (Replace / AddObservation / AddMapPoint, :935-957) are the caller's.
 * Returns via *nfused the number of matched points. */
int orc_fuse(const orc_kp* kps, const uint8_t* desc, int n, const float* uright, float min_x, float max_x,
             float min_y, float max_y, const float* scale, const float* inv_sigma2, int nlevels, float scale_factor,
             const orc_camera* kf, const orc_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th, int* out,
             int* nfused);

/* Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:977-1100), the match part:
 * out[i] = bestIdx (bestDist <= TH_LOW) for valid points (!isBad() and not
 * in pKF->GetMapPoints()), else -1; kf->Tcw = Scw rows 0..2. */
int orc_fuse_sim3(const orc_kp* kps, const uint8_t* desc, int n, float min_x, float max_x, float min_y,
                  float max_y, const float* scale, int nlevels, float scale_factor, const orc_camera* kf,
                  const orc_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th, int* out, int* nfused);

/* SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (:1102-1326).
 * Per keyframe: keypoints, descriptors, grid bounds, mvScaleFactors, Tcw
 * rows 0..2, and one map point record per keypoint (valid = pMP &&
 * !vbAlreadyMatched && !isBad()). cam1 = pKF1's fx, fy, cx, cy (used for
 * both projections, as the reference does). match1[i1] = idx2 for the
 * new mutual matches (vpMatches12[i1] = vpMapPoints2[idx2]), else -1;
 * vnMatch1 / vnMatch2 (optional) receive the one-directional picks. */
int orc_search_by_sim3(const orc_kp* kps1, const uint8_t* desc1, int n1, const float* bounds1, const float* scale1,
                       const orc_kp* kps2, const uint8_t* desc2, int n2, const float* bounds2, const float* scale2,
                       int nlevels, float scale_factor, const orc_camera* cam1, const float* T1w, const float* T2w,
                       float s12, const float* R12, const float* t12, const orc_map_point_world* mps1,
                       const uint8_t* mpdesc1, const orc_map_point_world* mps2, const uint8_t* mpdesc2, float th,
                       int* match1, int* vnMatch1, int* vnMatch2, int* nfound);

/* SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
 * (:657-823, CheckDistEpipolarLine :140-157). Per keyframe: keypoints,
 * descriptors, mvuRight, has_mp (GetMapPoint(idx) != NULL), FeatureVector as
 * CSR. cw1 = pKF1->GetCameraCenter(); T2w = pKF2 Tcw rows 0..2; cam2 =
 * pKF2's fx, fy, cx, cy; scale2 / sigma2 = pKF2->mvScaleFactors /
 * mvLevelSigma2; F12 row-major 3x3. matches12[idx1] = idx2 or -1
 * (vMatchedPairs in idx1 order); returns the count via *nmatches. */
int orc_search_for_triangulation(const orc_kp* kps1, const uint8_t* desc1, const float* uright1,
                                 const uint8_t* has_mp1, int n1, const uint32_t* fv1_nodes, const int* fv1_off,
                                 const int* fv1_idx, int fv1_n, const orc_kp* kps2, const uint8_t* desc2,
                                 const float* uright2, const uint8_t* has_mp2, int n2, const uint32_t* fv2_nodes,
                                 const int* fv2_off, const int* fv2_idx, int fv2_n, const float* cw1,
                                 const float* T2w, const float* cam2, const float* scale2, const float* sigma2,
                                 const float* F12, int only_stereo, int check_ori, int* matches12, int* nmatches);

#ifdef __cplusplus
}
#endif
