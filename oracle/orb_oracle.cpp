/*
 * orb_oracle.cpp — CPU ORACLE for the ORB hot path. TEST INFRASTRUCTURE ONLY.
 *
 * A line-faithful CPU restatement of the reference's CPU branch
 * (built with DONT_USE_OPENVX, /root/reference/src/ORBextractor.cc:1701-1873)
 * and of ORBmatcher's SearchForInitialization / SearchByBoW, with the OpenCV
 * primitives those call restated from OpenCV 3.x scalar semantics because
 * OpenCV is not vendored in the reference.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py (cpu_baseline) load this.
 * PARITY UNPINNED at the OpenCV boundary (no reference test or fixture pins
 * resize/FAST/GaussianBlur/fastAtan2); see DESIGN.md "Oracle".
 *
 * Build: oracle/Makefile (g++ -O2 -ffp-contract=off, no fast-math).
 */
#include "orb_oracle.h"
#include "orb_pattern_tbl.h"

#include <algorithm>
#include <iterator>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <list>
#include <vector>

namespace {

typedef orc_kp KeyPoint;

// ---------------------------------------------------------------- OpenCV bits
// cvRound: round half to even (x86 cvtss2si under default MXCSR).
inline int cv_round(float v) { return (int)lrintf(v); }
inline int cv_round(double v) { return (int)lrint(v); }
// cvFloor / cvCeil as in OpenCV core/fast_math.hpp.
inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
inline int cv_ceil(double v) { int i = (int)v; return i + (i < v); }
inline short sat_short(int v) { return (short)std::min(std::max(v, (int)SHRT_MIN), (int)SHRT_MAX); }
inline uint8_t sat_u8(int v) { return (uint8_t)std::min(std::max(v, 0), 255); }

struct Mat8 {
  int w = 0, h = 0;
  std::vector<uint8_t> px;
  void alloc(int W, int H) { w = W; h = H; px.assign((size_t)W * H, 0); }
  uint8_t* row(int y) { return px.data() + (size_t)y * w; }
  const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
  uint8_t at(int y, int x) const { return px[(size_t)y * w + x]; }
};

// cv::fastAtan2, OpenCV 3.x core/src/mathfuncs_core.cpp (polynomial version).
const float atan2_p1 = 0.9997878412794807f * (float)(180 / M_PI);
const float atan2_p3 = -0.3258083974640975f * (float)(180 / M_PI);
const float atan2_p5 = 0.1555786518463281f * (float)(180 / M_PI);
const float atan2_p7 = -0.04432655554792128f * (float)(180 / M_PI);
float fast_atan2(float y, float x) {
  float ax = std::fabs(x), ay = std::fabs(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)DBL_EPSILON);
    c2 = c * c;
    a = (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
  } else {
    c = ax / (ay + (float)DBL_EPSILON);
    c2 = c * c;
    a = 90.f - (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// cv::resize(src, dst, Size(dw,dh), 0, 0, INTER_LINEAR) on CV_8UC1, OpenCV
// 3.x imgproc/src/resize.cpp scalar path: 11-bit fixed-point coefficients,
// HResizeLinear<uchar,int,short,2048> + VResizeLinear with FixedPtCast<22>.
// Includes the INTER_LINEAR -> INTER_AREA switch for an exact 2x downscale.
void resize_linear_u8(const Mat8& src, Mat8& dst, int dw, int dh) {
  dst.alloc(dw, dh);
  const double inv_scale_x = (double)dw / src.w, inv_scale_y = (double)dh / src.h;
  const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
  const int iscale_x = (int)lrint(scale_x), iscale_y = (int)lrint(scale_y);
  const bool is_area_fast = std::fabs(scale_x - iscale_x) < DBL_EPSILON &&
                            std::fabs(scale_y - iscale_y) < DBL_EPSILON;
  if (is_area_fast && iscale_x == 2 && iscale_y == 2) {
    // resizeAreaFast_ 2x2: (a+b+c+d+2)>>2
    for (int y = 0; y < dh; ++y) {
      const uint8_t* S = src.row(2 * y);
      const uint8_t* nS = src.row(std::min(2 * y + 1, src.h - 1));
      uint8_t* D = dst.row(y);
      for (int x = 0; x < dw; ++x) {
        int i = 2 * x;
        D[x] = (uint8_t)((S[i] + S[i + 1] + nS[i] + nS[i + 1] + 2) >> 2);
      }
    }
    return;
  }
  const int ONE = 2048;  // INTER_RESIZE_COEF_SCALE
  std::vector<int> xofs(dw);
  std::vector<short> ialpha(2 * dw);
  int xmax = dw;
  for (int dx = 0; dx < dw; ++dx) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = cv_floor(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= src.w) {
      xmax = std::min(xmax, dx);
      if (sx >= src.w - 1) { fx = 0; sx = src.w - 1; }
    }
    xofs[dx] = sx;
    ialpha[2 * dx] = sat_short(cv_round((1.f - fx) * ONE));
    ialpha[2 * dx + 1] = sat_short(cv_round(fx * ONE));
  }
  std::vector<int> rows0(dw), rows1(dw);
  auto hresize = [&](const uint8_t* S, int* D) {
    int dx = 0;
    for (; dx < xmax; ++dx) {
      int sx = xofs[dx];
      D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
    }
    for (; dx < dw; ++dx) D[dx] = S[xofs[dx]] * ONE;
  };
  auto clip = [](int x, int a, int b) { return x >= a ? (x < b ? x : b - 1) : a; };
  for (int dy = 0; dy < dh; ++dy) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = cv_floor(fy);
    fy -= sy;
    const int b0 = sat_short(cv_round((1.f - fy) * ONE));
    const int b1 = sat_short(cv_round(fy * ONE));
    hresize(src.row(clip(sy, 0, src.h)), rows0.data());
    hresize(src.row(clip(sy + 1, 0, src.h)), rows1.data());
    uint8_t* D = dst.row(dy);
    for (int x = 0; x < dw; ++x)
      D[x] = sat_u8((rows0[x] * b0 + rows1[x] * b1 + (1 << 21)) >> 22);
  }
}

// BORDER_REFLECT_101 index (cv::borderInterpolate).
inline int reflect101(int p, int len) {
  if (len == 1) return 0;
  while (p < 0 || p >= len) {
    if (p < 0) p = -p;
    if (p >= len) p = 2 * len - 2 - p;
  }
  return p;
}

// Gaussian kernel of getGaussianKernel(7, 2, CV_32F) converted to CV_32S with
// scale 256 (createSeparableLinearFilter 8U smooth-symmetric branch).
void gauss7_int(int k[7]) {
  const int n = 7;
  const double sigma = 2.0, scale2X = -0.5 / (sigma * sigma);
  float cf[7];
  double sum = 0;
  for (int i = 0; i < n; ++i) {
    double x = i - (n - 1) * 0.5;
    cf[i] = (float)std::exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < n; ++i) cf[i] = (float)(cf[i] * sum);
  for (int i = 0; i < n; ++i) k[i] = cv_round(cf[i] * 256.f);
}

// GaussianBlur(src, dst, Size(7,7), 2, 2, BORDER_REFLECT_101) on CV_8UC1:
// integer row pass, column pass sat_u8((acc + 2^15) >> 16).
void gaussian_blur7(const Mat8& src, Mat8& dst) {
  int k[7];
  gauss7_int(k);
  const int W = src.w, H = src.h;
  std::vector<int> tmp((size_t)W * H);
  for (int y = 0; y < H; ++y) {
    const uint8_t* S = src.row(y);
    for (int x = 0; x < W; ++x) {
      int acc = 0;
      for (int i = 0; i < 7; ++i) acc += k[i] * S[reflect101(x + i - 3, W)];
      tmp[(size_t)y * W + x] = acc;
    }
  }
  dst.alloc(W, H);
  for (int y = 0; y < H; ++y) {
    uint8_t* D = dst.row(y);
    for (int x = 0; x < W; ++x) {
      int acc = 0;
      for (int i = 0; i < 7; ++i) acc += k[i] * tmp[(size_t)reflect101(y + i - 3, H) * W + x];
      D[x] = sat_u8((acc + (1 << 15)) >> 16);
    }
  }
}

// ------------------------------------------------------------------- FAST
// cv::FAST(img, kps, threshold, nonmax=true, TYPE_9_16): OpenCV 3.x
// features2d/src/fast.cpp FAST_t<16> + cornerScore<16>, scalar path.
const int kRingX[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
const int kRingY[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

int corner_score16(const uint8_t* ptr, const int pixel[25], int threshold) {
  const int K = 8, N = K * 3 + 1;
  int k, v = ptr[0];
  short d[N];
  for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
  int a0 = threshold;
  for (k = 0; k < 16; k += 2) {
    int a = std::min((int)d[k + 1], (int)d[k + 2]);
    a = std::min(a, (int)d[k + 3]);
    if (a <= a0) continue;
    a = std::min(a, (int)d[k + 4]);
    a = std::min(a, (int)d[k + 5]);
    a = std::min(a, (int)d[k + 6]);
    a = std::min(a, (int)d[k + 7]);
    a = std::min(a, (int)d[k + 8]);
    a0 = std::max(a0, std::min(a, (int)d[k]));
    a0 = std::max(a0, std::min(a, (int)d[k + 9]));
  }
  int b0 = -a0;
  for (k = 0; k < 16; k += 2) {
    int b = std::max((int)d[k + 1], (int)d[k + 2]);
    b = std::max(b, (int)d[k + 3]);
    b = std::max(b, (int)d[k + 4]);
    b = std::max(b, (int)d[k + 5]);
    if (b >= b0) continue;
    b = std::max(b, (int)d[k + 6]);
    b = std::max(b, (int)d[k + 7]);
    b = std::max(b, (int)d[k + 8]);
    b0 = std::min(b0, std::max(b, (int)d[k]));
    b0 = std::min(b0, std::max(b, (int)d[k + 9]));
  }
  return -b0 - 1;
}

// FAST on the ROI [x0, x0+cols) x [y0, y0+rows) of `img`; keypoints are
// reported in ROI coordinates, row-major (the order FAST_t pushes them).
void fast_roi(const Mat8& img, int x0, int y0, int cols, int rows, int threshold,
              std::vector<KeyPoint>& out) {
  out.clear();
  if (rows < 7 || cols < 7) return;  // no candidate rows/cols in [3, n-3)
  const int K = 8, N = 16 + K + 1;
  threshold = std::min(std::max(threshold, 0), 255);
  const int step = img.w;
  int pixel[25];
  for (int k = 0; k < 16; ++k) pixel[k] = kRingX[k] + kRingY[k] * step;
  for (int k = 16; k < 25; ++k) pixel[k] = pixel[k - 16];
  uint8_t threshold_tab[512];
  for (int i = -255; i <= 255; i++)
    threshold_tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
  std::vector<uint8_t> buf(3 * (size_t)cols, 0);
  std::vector<int> cpbuf(3 * ((size_t)cols + 1), 0);
  uint8_t* bufp[3] = {buf.data(), buf.data() + cols, buf.data() + 2 * cols};
  int* cpb[3] = {cpbuf.data() + 1, cpbuf.data() + 1 + (cols + 1), cpbuf.data() + 1 + 2 * (cols + 1)};
  for (int i = 3; i < rows - 2; i++) {
    const uint8_t* ptr = img.row(y0 + i) + x0 + 3;
    uint8_t* curr = bufp[(i - 3) % 3];
    int* cornerpos = cpb[(i - 3) % 3];
    std::memset(curr, 0, cols);
    int ncorners = 0;
    if (i < rows - 3) {
      for (int j = 3; j < cols - 3; j++, ptr++) {
        int v = ptr[0];
        const uint8_t* tab = &threshold_tab[0] - v + 255;
        int d = tab[ptr[pixel[0]]] | tab[ptr[pixel[8]]];
        if (d == 0) continue;
        d &= tab[ptr[pixel[2]]] | tab[ptr[pixel[10]]];
        d &= tab[ptr[pixel[4]]] | tab[ptr[pixel[12]]];
        d &= tab[ptr[pixel[6]]] | tab[ptr[pixel[14]]];
        if (d == 0) continue;
        d &= tab[ptr[pixel[1]]] | tab[ptr[pixel[9]]];
        d &= tab[ptr[pixel[3]]] | tab[ptr[pixel[11]]];
        d &= tab[ptr[pixel[5]]] | tab[ptr[pixel[13]]];
        d &= tab[ptr[pixel[7]]] | tab[ptr[pixel[15]]];
        if (d & 1) {
          int vt = v - threshold, count = 0;
          for (int k = 0; k < N; k++) {
            int x = ptr[pixel[k]];
            if (x < vt) {
              if (++count > K) {
                cornerpos[ncorners++] = j;
                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                break;
              }
            } else {
              count = 0;
            }
          }
        }
        if (d & 2) {
          int vt = v + threshold, count = 0;
          for (int k = 0; k < N; k++) {
            int x = ptr[pixel[k]];
            if (x > vt) {
              if (++count > K) {
                cornerpos[ncorners++] = j;
                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                break;
              }
            } else {
              count = 0;
            }
          }
        }
      }
    }
    cornerpos[-1] = ncorners;
    if (i == 3) continue;
    const uint8_t* prev = bufp[(i - 4 + 3) % 3];
    const uint8_t* pprev = bufp[(i - 5 + 3) % 3];
    cornerpos = cpb[(i - 4 + 3) % 3];
    ncorners = cornerpos[-1];
    for (int k = 0; k < ncorners; k++) {
      int j = cornerpos[k];
      int score = prev[j];
      if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
          score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
          score > curr[j] && score > curr[j + 1]) {
        KeyPoint kp;
        kp.x = (float)j;
        kp.y = (float)(i - 1);
        kp.size = 7.f;
        kp.angle = -1.f;
        kp.response = (float)score;
        kp.octave = 0;
        kp.class_id = -1;
        out.push_back(kp);
      }
    }
  }
}

// ----------------------------------------------------------- extractor state
const int PATCH_SIZE = 31;
const int HALF_PATCH_SIZE = 15;
const int EDGE_THRESHOLD = 19;

// Exposure of the creation-order stand-in for the reference's heap-pointer
// tie-break: the sorted rounds split nodes in descending
// (size, pointer) order and stop as soon as the list reaches N (:1041-1088).
// When that cut-off falls inside a group of equal-size nodes, WHICH of them
// were split was decided by the tie rule. `events` counts such cut-offs (0 or
// 1 per call), `nodes` the nodes of the straddled group, `kps` the kept
// keypoints that come from them (the children of its split nodes plus one per
// unsplit node): the outputs another tie order could change.
struct TieStats {
  int events = 0, nodes = 0, kps = 0;
};

struct Extractor {
  orc_config cfg;
  std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
  std::vector<int> mnFeaturesPerLevel, umax;
  signed char tests[256][4];
  std::vector<Mat8> pyr;

  // ORBextractor::ORBextractor (src/ORBextractor.cc:496-560) incl. the fork's
  // buildGraph scale override (:640-680) when scale_mode == 1.
  explicit Extractor(const orc_config& c) : cfg(c) {
    const int nlevels = cfg.nlevels;
    const float scaleFactor = cfg.scale_factor;
    mvScaleFactor.resize(nlevels);
    mvLevelSigma2.resize(nlevels);
    mvScaleFactor[0] = 1.0f;
    mvLevelSigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
      mvScaleFactor[i] = mvScaleFactor[i - 1] * scaleFactor;
      mvLevelSigma2[i] = mvScaleFactor[i] * mvScaleFactor[i];
    }
    mvInvScaleFactor.resize(nlevels);
    mvInvLevelSigma2.resize(nlevels);
    for (int i = 0; i < nlevels; i++) {
      mvInvScaleFactor[i] = 1.0f / mvScaleFactor[i];
      mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
    }
    mnFeaturesPerLevel.resize(nlevels);
    float factor = 1.0f / scaleFactor;
    float nDesiredFeaturesPerScale =
        cfg.nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
    int sumFeatures = 0;
    for (int level = 0; level < nlevels - 1; level++) {
      mnFeaturesPerLevel[level] = cv_round(nDesiredFeaturesPerScale);
      sumFeatures += mnFeaturesPerLevel[level];
      nDesiredFeaturesPerScale *= factor;
    }
    mnFeaturesPerLevel[nlevels - 1] = std::max(cfg.nfeatures - sumFeatures, 0);

    std::memcpy(tests, kOracleBriefTests, sizeof(tests));
    if (cfg.pattern_mode == 1) tests[kOracleForkIndex / 4][kOracleForkIndex % 4] = kOracleUpstreamValue;

    umax.resize(HALF_PATCH_SIZE + 1);
    int v, v0, vmax = cv_floor(HALF_PATCH_SIZE * sqrt(2.f) / 2 + 1);
    int vmin = cv_ceil(HALF_PATCH_SIZE * sqrt(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (v = 0; v <= vmax; ++v) umax[v] = cv_round(sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
      while (umax[v0] == umax[v0 + 1]) ++v0;
      umax[v] = v0;
      ++v0;
    }
    if (cfg.scale_mode == 1) {
      // VX_SCALE_PYRAMID_ORB level widths, OpenVX ceil(w * 0.8408964^l).
      // VisionWorks' own rounding is unverifiable offline.
      for (int level = 0; level < nlevels; ++level) {
        unsigned v_width = (unsigned)std::ceil(cfg.width * std::pow(0.8408964, level));
        mvScaleFactor[level] = ((float)cfg.width) / v_width;
        mvInvScaleFactor[level] = ((float)v_width) / cfg.width;
      }
    }
  }

  void level_size(int level, int cols, int rows, int* w, int* h) const {
    float scale = mvInvScaleFactor[level];
    *w = cv_round((float)cols * scale);
    *h = cv_round((float)rows * scale);
  }

  // ComputePyramid (src/ORBextractor.cc:1837-1863): chained INTER_LINEAR.
  // The 19-px REFLECT_101 border is never read by extraction.
  void compute_pyramid(const Mat8& image) {
    pyr.assign(cfg.nlevels, Mat8());
    for (int level = 0; level < cfg.nlevels; ++level) {
      int w, h;
      level_size(level, image.w, image.h, &w, &h);
      if (level != 0)
        resize_linear_u8(pyr[level - 1], pyr[level], w, h);
      else
        pyr[0] = image;
    }
  }

  // FAST stage of ComputeKeyPointsOctTree (src/ORBextractor.cc:1128-1299).
  void fast_level(int level, std::vector<KeyPoint>& vToDistributeKeys, int* bx) const {
    const float W = 30;
    const Mat8& im = pyr[level];
    const int minBorderX = EDGE_THRESHOLD - 3;
    const int minBorderY = minBorderX;
    const int maxBorderX = im.w - EDGE_THRESHOLD + 3;
    const int maxBorderY = im.h - EDGE_THRESHOLD + 3;
    bx[0] = minBorderX; bx[1] = maxBorderX; bx[2] = minBorderY; bx[3] = maxBorderY;
    vToDistributeKeys.clear();
    vToDistributeKeys.reserve(cfg.nfeatures * 10);
    const float width = (maxBorderX - minBorderX);
    const float height = (maxBorderY - minBorderY);
    const int nCols = width / W;
    const int nRows = height / W;
    const int wCell = ceil(width / nCols);
    const int hCell = ceil(height / nRows);
    std::vector<KeyPoint> vKeysCell;
    for (int i = 0; i < nRows; i++) {
      const float iniY = minBorderY + i * hCell;
      float maxY = iniY + hCell + 6;
      if (iniY >= maxBorderY - 3) continue;
      if (maxY > maxBorderY) maxY = maxBorderY;
      for (int j = 0; j < nCols; j++) {
        const float iniX = minBorderX + j * wCell;
        float maxX = iniX + wCell + 6;
        if (iniX >= maxBorderX - 6) continue;
        if (maxX > maxBorderX) maxX = maxBorderX;
        const int r0 = (int)iniY, r1 = (int)maxY, c0 = (int)iniX, c1 = (int)maxX;
        fast_roi(im, c0, r0, c1 - c0, r1 - r0, cfg.ini_th_fast, vKeysCell);
        if (vKeysCell.empty())
          fast_roi(im, c0, r0, c1 - c0, r1 - r0, cfg.min_th_fast, vKeysCell);
        for (auto& kp : vKeysCell) {
          kp.x += j * wCell;
          kp.y += i * hCell;
          vToDistributeKeys.push_back(kp);
        }
      }
    }
  }

  void extract(const Mat8& image, std::vector<KeyPoint>& out, std::vector<uint8_t>& desc,
               std::vector<TieStats>* ties = nullptr);
  int tie_rule = 0;  // TieRule of the quadtree's sorted rounds (0 = the product's)
};

// --------------------------------------------------------------- quadtree
// ExtractorNode / DivideNode / DistributeOctTree (src/ORBextractor.cc:831-1120).
// The reference sorts pair<int, ExtractorNode*> (:1041), i.e. breaks size ties
// by heap address; the restatement breaks them by node creation sequence
// (`seq`), the documented stand-in shared with the HIP kernel.
struct ExtractorNode {
  std::vector<KeyPoint> vKeys;
  int ULx = 0, ULy = 0, URx = 0, URy = 0, BLx = 0, BLy = 0, BRx = 0, BRy = 0;
  std::list<ExtractorNode>::iterator lit;
  bool bNoMore = false;
  long seq = 0;
  void DivideNode(ExtractorNode& n1, ExtractorNode& n2, ExtractorNode& n3, ExtractorNode& n4) {
    const int halfX = ceil(static_cast<float>(URx - ULx) / 2);
    const int halfY = ceil(static_cast<float>(BRy - ULy) / 2);
    n1.ULx = ULx; n1.ULy = ULy;
    n1.URx = ULx + halfX; n1.URy = ULy;
    n1.BLx = ULx; n1.BLy = ULy + halfY;
    n1.BRx = ULx + halfX; n1.BRy = ULy + halfY;
    n1.vKeys.reserve(vKeys.size());
    n2.ULx = n1.URx; n2.ULy = n1.URy;
    n2.URx = URx; n2.URy = URy;
    n2.BLx = n1.BRx; n2.BLy = n1.BRy;
    n2.BRx = URx; n2.BRy = ULy + halfY;
    n2.vKeys.reserve(vKeys.size());
    n3.ULx = n1.BLx; n3.ULy = n1.BLy;
    n3.URx = n1.BRx; n3.URy = n1.BRy;
    n3.BLx = BLx; n3.BLy = BLy;
    n3.BRx = n1.BRx; n3.BRy = BLy;
    n3.vKeys.reserve(vKeys.size());
    n4.ULx = n3.URx; n4.ULy = n3.URy;
    n4.URx = n2.BRx; n4.URy = n2.BRy;
    n4.BLx = n3.BRx; n4.BLy = n3.BRy;
    n4.BRx = BRx; n4.BRy = BRy;
    n4.vKeys.reserve(vKeys.size());
    for (size_t i = 0; i < vKeys.size(); i++) {
      const KeyPoint& kp = vKeys[i];
      if (kp.x < n1.URx) {
        if (kp.y < n1.BRy) n1.vKeys.push_back(kp);
        else n3.vKeys.push_back(kp);
      } else if (kp.y < n1.BRy) {
        n2.vKeys.push_back(kp);
      } else {
        n4.vKeys.push_back(kp);
      }
    }
    if (n1.vKeys.size() == 1) n1.bNoMore = true;
    if (n2.vKeys.size() == 1) n2.bNoMore = true;
    if (n3.vKeys.size() == 1) n3.bNoMore = true;
    if (n4.vKeys.size() == 1) n4.bNoMore = true;
  }
};

struct SizeSeqNode {
  int size;
  long seq;
  ExtractorNode* node;
  bool operator<(const SizeSeqNode& o) const {
    return size != o.size ? size < o.size : seq < o.seq;
  }
};

// Tie rules of the sorted rounds (orc_config-independent; tie-rule study in
// orc_tie_sequence): 0 = creation order, later-created split first (the
// default shared with the HIP kernel); 1 = the reference's real heap address
// (distribute_oct_tree_ptr below); 2 = creation order, earlier-created first.
enum TieRule { kTieLaterFirst = 0, kTiePointer = 1, kTieEarlierFirst = 2 };

std::vector<KeyPoint> distribute_oct_tree(const std::vector<KeyPoint>& vToDistributeKeys,
                                          int minX, int maxX, int minY, int maxY, int N,
                                          TieStats* ties = nullptr, int tie_rule = kTieLaterFirst) {
  const int nIni = round(static_cast<float>(maxX - minX) / (maxY - minY));
  const float hX = static_cast<float>(maxX - minX) / nIni;
  long seq = 0;
  std::list<ExtractorNode> lNodes;
  std::vector<ExtractorNode*> vpIniNodes(nIni);
  for (int i = 0; i < nIni; i++) {
    ExtractorNode ni;
    ni.ULx = (int)(hX * static_cast<float>(i)); ni.ULy = 0;
    ni.URx = (int)(hX * static_cast<float>(i + 1)); ni.URy = 0;
    ni.BLx = ni.ULx; ni.BLy = maxY - minY;
    ni.BRx = ni.URx; ni.BRy = maxY - minY;
    ni.vKeys.reserve(vToDistributeKeys.size());
    ni.seq = seq++;
    lNodes.push_back(ni);
    vpIniNodes[i] = &lNodes.back();
  }
  for (size_t i = 0; i < vToDistributeKeys.size(); i++) {
    const KeyPoint& kp = vToDistributeKeys[i];
    vpIniNodes[(size_t)(kp.x / hX)]->vKeys.push_back(kp);
  }
  auto lit = lNodes.begin();
  while (lit != lNodes.end()) {
    if (lit->vKeys.size() == 1) {
      lit->bNoMore = true;
      lit++;
    } else if (lit->vKeys.empty()) {
      lit = lNodes.erase(lit);
    } else {
      lit++;
    }
  }
  bool bFinish = false;
  std::vector<SizeSeqNode> vSizeAndPointerToNode;
  vSizeAndPointerToNode.reserve(lNodes.size() * 4);
  auto push_child = [&](ExtractorNode& n, std::vector<SizeSeqNode>& v, int* nToExpand) {
    if (n.vKeys.size() > 0) {
      n.seq = seq++;
      lNodes.push_front(n);
      if (n.vKeys.size() > 1) {
        if (nToExpand) (*nToExpand)++;
        v.push_back({(int)n.vKeys.size(), lNodes.front().seq, &lNodes.front()});
        lNodes.front().lit = lNodes.begin();
      }
    }
  };
  while (!bFinish) {
    int prevSize = lNodes.size();
    lit = lNodes.begin();
    int nToExpand = 0;
    vSizeAndPointerToNode.clear();
    while (lit != lNodes.end()) {
      if ((int)lNodes.size() >= N) {
        bFinish = true;
        break;
      }
      if (lit->bNoMore) {
        lit++;
        continue;
      } else {
        ExtractorNode n1, n2, n3, n4;
        lit->DivideNode(n1, n2, n3, n4);
        push_child(n1, vSizeAndPointerToNode, &nToExpand);
        push_child(n2, vSizeAndPointerToNode, &nToExpand);
        push_child(n3, vSizeAndPointerToNode, &nToExpand);
        push_child(n4, vSizeAndPointerToNode, &nToExpand);
        lit = lNodes.erase(lit);
        continue;
      }
    }
    if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
      bFinish = true;
    } else if (((int)lNodes.size() + nToExpand * 3) > N) {
      while (!bFinish) {
        prevSize = lNodes.size();
        std::vector<SizeSeqNode> vPrevSizeAndPointerToNode = vSizeAndPointerToNode;
        vSizeAndPointerToNode.clear();
        std::sort(vPrevSizeAndPointerToNode.begin(), vPrevSizeAndPointerToNode.end());
        if (tie_rule == kTieEarlierFirst)  // reverse every run of equal sizes
          for (size_t a = 0; a < vPrevSizeAndPointerToNode.size();) {
            size_t b = a;
            while (b < vPrevSizeAndPointerToNode.size() &&
                   vPrevSizeAndPointerToNode[b].size == vPrevSizeAndPointerToNode[a].size)
              ++b;
            std::reverse(vPrevSizeAndPointerToNode.begin() + a, vPrevSizeAndPointerToNode.begin() + b);
            a = b;
          }
        std::vector<int> children(vPrevSizeAndPointerToNode.size(), 0);
        for (int j = vPrevSizeAndPointerToNode.size() - 1; j >= 0; j--) {
          ExtractorNode n1, n2, n3, n4;
          vPrevSizeAndPointerToNode[j].node->DivideNode(n1, n2, n3, n4);
          children[j] = (n1.vKeys.size() > 0) + (n2.vKeys.size() > 0) + (n3.vKeys.size() > 0) +
                        (n4.vKeys.size() > 0);
          push_child(n1, vSizeAndPointerToNode, nullptr);
          push_child(n2, vSizeAndPointerToNode, nullptr);
          push_child(n3, vSizeAndPointerToNode, nullptr);
          push_child(n4, vSizeAndPointerToNode, nullptr);
          lNodes.erase(vPrevSizeAndPointerToNode[j].node->lit);
          if ((int)lNodes.size() >= N) {
            // cut-off after node j: a straddle if the next (unsplit) node has j's size
            const int s = vPrevSizeAndPointerToNode[j].size;
            if (ties && j > 0 && vPrevSizeAndPointerToNode[j - 1].size == s) {
              ties->events++;
              for (int i = 0; i < (int)vPrevSizeAndPointerToNode.size(); ++i) {
                if (vPrevSizeAndPointerToNode[i].size != s) continue;
                ties->nodes++;
                ties->kps += i >= j ? children[i] : 1;
              }
            }
            break;
          }
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
      }
    }
  }
  std::vector<KeyPoint> vResultKeys;
  vResultKeys.reserve(lNodes.size());
  for (auto it = lNodes.begin(); it != lNodes.end(); it++) {
    std::vector<KeyPoint>& vNodeKeys = it->vKeys;
    KeyPoint* pKP = &vNodeKeys[0];
    float maxResponse = pKP->response;
    for (size_t k = 1; k < vNodeKeys.size(); k++) {
      if (vNodeKeys[k].response > maxResponse) {
        pKP = &vNodeKeys[k];
        maxResponse = vNodeKeys[k].response;
      }
    }
    vResultKeys.push_back(*pKP);
  }
  return vResultKeys;
}

// ------------------------------------------- quadtree with heap-address ties
// The reference's own tie-break, for the tie-rule study:
// DistributeOctTree with an ExtractorNode laid out exactly as
// include/ORBextractor.h:62-73 (std::vector<cv::KeyPoint> of 28-B keypoints,
// four cv::Point2i, a std::list iterator, a bool: 72 bytes, so a list node is
// an 88-byte malloc as in the reference), the reference's sequence of
// reserve / push_front / copy / erase / temporary destruction
// (src/ORBextractor.cc:831-1120), and the sorted rounds ordering
// pair<int, ExtractorNode*> by the real heap address (:1041). Only the heap
// state on entry differs from the reference process (OpenCV's own allocations
// before the call are not reproduced).
struct RefPoint2i {
  int x, y;
};
struct RefExtractorNode {
  std::vector<KeyPoint> vKeys;
  RefPoint2i UL, UR, BL, BR;
  std::list<RefExtractorNode>::iterator lit;
  bool bNoMore = false;
  void DivideNode(RefExtractorNode& n1, RefExtractorNode& n2, RefExtractorNode& n3, RefExtractorNode& n4) {
    const int halfX = ceil(static_cast<float>(UR.x - UL.x) / 2);
    const int halfY = ceil(static_cast<float>(BR.y - UL.y) / 2);
    n1.UL = UL;
    n1.UR = {UL.x + halfX, UL.y};
    n1.BL = {UL.x, UL.y + halfY};
    n1.BR = {UL.x + halfX, UL.y + halfY};
    n1.vKeys.reserve(vKeys.size());
    n2.UL = n1.UR;
    n2.UR = UR;
    n2.BL = n1.BR;
    n2.BR = {UR.x, UL.y + halfY};
    n2.vKeys.reserve(vKeys.size());
    n3.UL = n1.BL;
    n3.UR = n1.BR;
    n3.BL = BL;
    n3.BR = {n1.BR.x, BL.y};
    n3.vKeys.reserve(vKeys.size());
    n4.UL = n3.UR;
    n4.UR = n2.BR;
    n4.BL = n3.BR;
    n4.BR = BR;
    n4.vKeys.reserve(vKeys.size());
    for (const KeyPoint& kp : vKeys) {
      if (kp.x < n1.UR.x)
        (kp.y < n1.BR.y ? n1 : n3).vKeys.push_back(kp);
      else
        (kp.y < n1.BR.y ? n2 : n4).vKeys.push_back(kp);
    }
    for (RefExtractorNode* n : {&n1, &n2, &n3, &n4})
      if (n->vKeys.size() == 1) n->bNoMore = true;
  }
};
static_assert(sizeof(KeyPoint) == 28, "cv::KeyPoint is 28 bytes");
static_assert(sizeof(RefExtractorNode) == 72, "layout of the reference's ExtractorNode");

// Creation sequence of the pointer variant's nodes, kept beside the heap
// (fixed static table, no allocation during the call) so the study can see
// how address order relates to creation order: per sorted round, adjacent
// equal-size entries in address order counted as "later-created at the
// higher address" (concordant with rule 0) or not.
struct PtrSeqTable {
  static constexpr int kCap = 1 << 17;
  const void* key[kCap];
  long seq[kCap];
  long next = 0;
  long concordant = 0, discordant = 0;
  void clear() {
    std::memset(key, 0, sizeof(key));
    next = 0;
  }
  static size_t slot(const void* p) { return ((uintptr_t)p >> 4) * 0x9E3779B97F4A7C15ull >> (64 - 17); }
  void put(const void* p) {
    size_t i = slot(p);
    while (key[i] && key[i] != p) i = (i + 1) & (kCap - 1);
    key[i] = p;
    seq[i] = next++;
  }
  long get(const void* p) const {
    size_t i = slot(p);
    while (key[i] && key[i] != p) i = (i + 1) & (kCap - 1);
    return key[i] ? seq[i] : -1;
  }
};
PtrSeqTable* g_ptr_seq = nullptr;  // set by orc_tie_address_order (study only)

std::vector<KeyPoint> distribute_oct_tree_ptr(const std::vector<KeyPoint>& vToDistributeKeys, int minX, int maxX,
                                              int minY, int maxY, int N, int nfeatures) {
  if (g_ptr_seq) g_ptr_seq->clear();
  const int nIni = round(static_cast<float>(maxX - minX) / (maxY - minY));
  const float hX = static_cast<float>(maxX - minX) / nIni;
  std::list<RefExtractorNode> lNodes;
  std::vector<RefExtractorNode*> vpIniNodes;
  vpIniNodes.resize(nIni);
  for (int i = 0; i < nIni; i++) {
    RefExtractorNode ni;
    ni.UL = {(int)(hX * static_cast<float>(i)), 0};
    ni.UR = {(int)(hX * static_cast<float>(i + 1)), 0};
    ni.BL = {ni.UL.x, maxY - minY};
    ni.BR = {ni.UR.x, maxY - minY};
    ni.vKeys.reserve(vToDistributeKeys.size());
    lNodes.push_back(ni);  // copies an empty vector: the list node's vKeys starts with no buffer
    vpIniNodes[i] = &lNodes.back();
  }
  for (size_t i = 0; i < vToDistributeKeys.size(); i++) {
    const KeyPoint& kp = vToDistributeKeys[i];
    vpIniNodes[(size_t)(kp.x / hX)]->vKeys.push_back(kp);
  }
  auto lit = lNodes.begin();
  while (lit != lNodes.end()) {
    if (lit->vKeys.size() == 1) {
      lit->bNoMore = true;
      lit++;
    } else if (lit->vKeys.empty()) {
      lit = lNodes.erase(lit);
    } else {
      lit++;
    }
  }
  bool bFinish = false;
  std::vector<std::pair<int, RefExtractorNode*>> vSizeAndPointerToNode;
  vSizeAndPointerToNode.reserve(lNodes.size() * 4);
  // the reference's "add childs if they contain points" block, per child
  auto add_child = [&](RefExtractorNode& n, int* nToExpand) {
    if (n.vKeys.size() > 0) {
      lNodes.push_front(n);
      if (g_ptr_seq) g_ptr_seq->put(&lNodes.front());
      if (n.vKeys.size() > 1) {
        if (nToExpand) (*nToExpand)++;
        vSizeAndPointerToNode.push_back(std::make_pair((int)n.vKeys.size(), &lNodes.front()));
        lNodes.front().lit = lNodes.begin();
      }
    }
  };
  while (!bFinish) {
    int prevSize = lNodes.size();
    lit = lNodes.begin();
    int nToExpand = 0;
    vSizeAndPointerToNode.clear();
    while (lit != lNodes.end()) {
      if ((int)lNodes.size() >= N) {
        bFinish = true;
        break;
      }
      if (lit->bNoMore) {
        lit++;
        continue;
      }
      RefExtractorNode n1, n2, n3, n4;
      lit->DivideNode(n1, n2, n3, n4);
      add_child(n1, &nToExpand);
      add_child(n2, &nToExpand);
      add_child(n3, &nToExpand);
      add_child(n4, &nToExpand);
      lit = lNodes.erase(lit);
    }
    if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
      bFinish = true;
    } else if (((int)lNodes.size() + nToExpand * 3) > N) {
      while (!bFinish) {
        prevSize = lNodes.size();
        std::vector<std::pair<int, RefExtractorNode*>> vPrevSizeAndPointerToNode = vSizeAndPointerToNode;
        vSizeAndPointerToNode.clear();
        std::sort(vPrevSizeAndPointerToNode.begin(), vPrevSizeAndPointerToNode.end());  // ties: heap address
        if (g_ptr_seq)
          for (size_t a = 1; a < vPrevSizeAndPointerToNode.size(); ++a)
            if (vPrevSizeAndPointerToNode[a].first == vPrevSizeAndPointerToNode[a - 1].first) {
              const bool later_higher = g_ptr_seq->get(vPrevSizeAndPointerToNode[a].second) >
                                        g_ptr_seq->get(vPrevSizeAndPointerToNode[a - 1].second);
              (later_higher ? g_ptr_seq->concordant : g_ptr_seq->discordant)++;
            }
        for (int j = vPrevSizeAndPointerToNode.size() - 1; j >= 0; j--) {
          RefExtractorNode n1, n2, n3, n4;
          vPrevSizeAndPointerToNode[j].second->DivideNode(n1, n2, n3, n4);
          add_child(n1, nullptr);
          add_child(n2, nullptr);
          add_child(n3, nullptr);
          add_child(n4, nullptr);
          lNodes.erase(vPrevSizeAndPointerToNode[j].second->lit);
          if ((int)lNodes.size() >= N) break;
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
      }
    }
  }
  std::vector<KeyPoint> vResultKeys;
  vResultKeys.reserve(nfeatures);
  for (auto it = lNodes.begin(); it != lNodes.end(); it++) {
    std::vector<KeyPoint>& vNodeKeys = it->vKeys;
    KeyPoint* pKP = &vNodeKeys[0];
    float maxResponse = pKP->response;
    for (size_t k = 1; k < vNodeKeys.size(); k++) {
      if (vNodeKeys[k].response > maxResponse) {
        pKP = &vNodeKeys[k];
        maxResponse = vNodeKeys[k].response;
      }
    }
    vResultKeys.push_back(*pKP);
  }
  return vResultKeys;
}

// IC_Angle (src/ORBextractor.cc:164-191) on the unblurred level.
float ic_angle(const Mat8& image, float ptx, float pty, const std::vector<int>& u_max) {
  int m_01 = 0, m_10 = 0;
  const uint8_t* center = image.px.data() + (size_t)cv_round(pty) * image.w + cv_round(ptx);
  for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
  const int step = image.w;
  for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
    int v_sum = 0;
    int d = u_max[v];
    for (int u = -d; u <= d; ++u) {
      int val_plus = center[u + v * step], val_minus = center[u - v * step];
      v_sum += (val_plus - val_minus);
      m_10 += u * (val_plus + val_minus);
    }
    m_01 += v * v_sum;
  }
  return fast_atan2((float)m_01, (float)m_10);
}

// computeOrbDescriptor (src/ORBextractor.cc:195-233) on the blurred level.
const float factorPI = (float)(M_PI / 180.f);
void orb_descriptor(const KeyPoint& kpt, const Mat8& img, const signed char tests[256][4],
                    uint8_t* desc) {
  float angle = (float)kpt.angle * factorPI;
  float a = (float)cosf(angle), b = (float)sinf(angle);
  const uint8_t* center = img.px.data() + (size_t)cv_round(kpt.y) * img.w + cv_round(kpt.x);
  const int step = img.w;
  auto get = [&](int x, int y) {
    return center[cv_round(x * b + y * a) * step + cv_round(x * a - y * b)];
  };
  for (int i = 0; i < 32; ++i) {
    int val = 0;
    for (int k = 0; k < 8; ++k) {
      const signed char* t = tests[i * 8 + k];
      int t0 = get(t[0], t[1]), t1 = get(t[2], t[3]);
      val |= (t0 < t1) << k;
    }
    desc[i] = (uint8_t)val;
  }
}

// operator() CPU branch (src/ORBextractor.cc:1701-1809) + ComputeKeyPointsOctTree.
void Extractor::extract(const Mat8& image, std::vector<KeyPoint>& out, std::vector<uint8_t>& desc,
                        std::vector<TieStats>* ties) {
  out.clear();
  desc.clear();
  if (image.w == 0 || image.h == 0) return;
  if (ties) ties->assign(cfg.nlevels, TieStats{});
  compute_pyramid(image);
  std::vector<std::vector<KeyPoint>> allKeypoints(cfg.nlevels);
  std::vector<KeyPoint> cand;
  for (int level = 0; level < cfg.nlevels; ++level) {
    int bx[4];
    fast_level(level, cand, bx);
    std::vector<KeyPoint>& keypoints = allKeypoints[level];
    if (tie_rule == kTiePointer)
      keypoints = distribute_oct_tree_ptr(cand, bx[0], bx[1], bx[2], bx[3], mnFeaturesPerLevel[level], cfg.nfeatures);
    else
      keypoints = distribute_oct_tree(cand, bx[0], bx[1], bx[2], bx[3], mnFeaturesPerLevel[level],
                                      ties ? &(*ties)[level] : nullptr, tie_rule);
    const int scaledPatchSize = PATCH_SIZE * mvScaleFactor[level];
    for (auto& kp : keypoints) {
      kp.x += bx[0];
      kp.y += bx[2];
      kp.octave = level;
      kp.size = scaledPatchSize;
    }
  }
  for (int level = 0; level < cfg.nlevels; ++level)
    for (auto& kp : allKeypoints[level]) kp.angle = ic_angle(pyr[level], kp.x, kp.y, umax);
  for (int level = 0; level < cfg.nlevels; ++level) {
    std::vector<KeyPoint>& keypoints = allKeypoints[level];
    if (keypoints.empty()) continue;
    Mat8 working;
    gaussian_blur7(pyr[level], working);
    size_t off = desc.size();
    desc.resize(off + 32 * keypoints.size());
    for (size_t i = 0; i < keypoints.size(); ++i)
      orb_descriptor(keypoints[i], working, tests, desc.data() + off + 32 * i);
    if (level != 0) {
      float scale = mvScaleFactor[level];
      for (auto& kp : keypoints) { kp.x *= scale; kp.y *= scale; }
    }
    out.insert(out.end(), keypoints.begin(), keypoints.end());
  }
}

Mat8 wrap_image(const uint8_t* img, int w, int h, size_t stride) {
  Mat8 m;
  m.alloc(w, h);
  for (int y = 0; y < h; ++y) std::memcpy(m.row(y), img + (size_t)y * stride, w);
  return m;
}

// ------------------------------------------------------------------ matcher
const int TH_LOW = 50;
const int TH_HIGH = 100;  // src/ORBmatcher.cc:37
const int HISTO_LENGTH = 30;

int descriptor_distance(const uint8_t* a, const uint8_t* b) {
  const int32_t* pa = (const int32_t*)a;
  const int32_t* pb = (const int32_t*)b;
  int dist = 0;
  for (int i = 0; i < 8; i++, pa++, pb++) {
    unsigned int v = *pa ^ *pb;
    v = v - ((v >> 1) & 0x55555555);
    v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
    dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
  }
  return dist;
}

// ComputeThreeMaxima (src/ORBmatcher.cc:1601-1642).
void compute_three_maxima(const std::vector<int>* histo, const int L, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; i++) {
    const int s = histo[i].size();
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    ind3 = -1;
  }
}

const int FRAME_GRID_ROWS = 48;
const int FRAME_GRID_COLS = 64;

// The Frame fields SearchForInitialization touches (src/Frame.cc:229-391).
struct GridFrame {
  const KeyPoint* keys;
  const uint8_t* desc;
  int N;
  float mnMinX, mnMaxX, mnMinY, mnMaxY, invW, invH;
  std::vector<size_t> mGrid[FRAME_GRID_COLS][FRAME_GRID_ROWS];
  GridFrame(const KeyPoint* k, const uint8_t* d, int n, float minX, float maxX, float minY, float maxY)
      : keys(k), desc(d), N(n), mnMinX(minX), mnMaxX(maxX), mnMinY(minY), mnMaxY(maxY) {
    invW = static_cast<float>(FRAME_GRID_COLS) / static_cast<float>(mnMaxX - mnMinX);
    invH = static_cast<float>(FRAME_GRID_ROWS) / static_cast<float>(mnMaxY - mnMinY);
    for (int i = 0; i < N; i++) {
      int px, py;
      if (pos_in_grid(keys[i], px, py)) mGrid[px][py].push_back(i);
    }
  }
  bool pos_in_grid(const KeyPoint& kp, int& posX, int& posY) const {
    posX = round((kp.x - mnMinX) * invW);
    posY = round((kp.y - mnMinY) * invH);
    if (posX < 0 || posX >= FRAME_GRID_COLS || posY < 0 || posY >= FRAME_GRID_ROWS) return false;
    return true;
  }
  std::vector<size_t> features_in_area(const float& x, const float& y, const float& r,
                                       const int minLevel, const int maxLevel) const {
    std::vector<size_t> vIndices;
    const int nMinCellX = std::max(0, (int)floor((x - mnMinX - r) * invW));
    if (nMinCellX >= FRAME_GRID_COLS) return vIndices;
    const int nMaxCellX = std::min((int)FRAME_GRID_COLS - 1, (int)ceil((x - mnMinX + r) * invW));
    if (nMaxCellX < 0) return vIndices;
    const int nMinCellY = std::max(0, (int)floor((y - mnMinY - r) * invH));
    if (nMinCellY >= FRAME_GRID_ROWS) return vIndices;
    const int nMaxCellY = std::min((int)FRAME_GRID_ROWS - 1, (int)ceil((y - mnMinY + r) * invH));
    if (nMaxCellY < 0) return vIndices;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
      for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
        const std::vector<size_t>& vCell = mGrid[ix][iy];
        for (size_t j = 0; j < vCell.size(); j++) {
          const KeyPoint& kpUn = keys[vCell[j]];
          if (bCheckLevels) {
            if (kpUn.octave < minLevel) continue;
            if (maxLevel >= 0)
              if (kpUn.octave > maxLevel) continue;
          }
          const float distx = kpUn.x - x;
          const float disty = kpUn.y - y;
          if (fabs(distx) < r && fabs(disty) < r) vIndices.push_back(vCell[j]);
        }
      }
    }
    return vIndices;
  }
};

}  // namespace

// ===================================================================== C ABI
extern "C" {

int orc_level_info(const orc_config* cfg, int* level_w, int* level_h, float* scale,
                   float* inv_scale, float* sigma2, float* inv_sigma2, int* nfeat, int* umax16) {
  Extractor ex(*cfg);
  for (int l = 0; l < cfg->nlevels; ++l) {
    int w, h;
    ex.level_size(l, cfg->width, cfg->height, &w, &h);
    if (level_w) level_w[l] = w;
    if (level_h) level_h[l] = h;
    if (scale) scale[l] = ex.mvScaleFactor[l];
    if (inv_scale) inv_scale[l] = ex.mvInvScaleFactor[l];
    if (sigma2) sigma2[l] = ex.mvLevelSigma2[l];
    if (inv_sigma2) inv_sigma2[l] = ex.mvInvLevelSigma2[l];
    if (nfeat) nfeat[l] = ex.mnFeaturesPerLevel[l];
  }
  if (umax16)
    for (int v = 0; v <= HALF_PATCH_SIZE; ++v) umax16[v] = ex.umax[v];
  return 0;
}

int orc_extract(const orc_config* cfg, const uint8_t* img, int w, int h, size_t stride,
                orc_kp* kps, int cap, uint8_t* desc, int* n) {
  Extractor ex(*cfg);
  Mat8 im = wrap_image(img, w, h, stride);
  std::vector<KeyPoint> out;
  std::vector<uint8_t> d;
  ex.extract(im, out, d);
  *n = (int)out.size();
  if ((int)out.size() > cap) return -1;
  std::memcpy(kps, out.data(), out.size() * sizeof(KeyPoint));
  std::memcpy(desc, d.data(), d.size());
  return 0;
}

int orc_pyramid_level(const orc_config* cfg, const uint8_t* img, int w, int h, size_t stride,
                      int level, uint8_t* out) {
  Extractor ex(*cfg);
  ex.compute_pyramid(wrap_image(img, w, h, stride));
  std::memcpy(out, ex.pyr[level].px.data(), ex.pyr[level].px.size());
  return 0;
}

int orc_blur_level(const orc_config* cfg, const uint8_t* img, int w, int h, size_t stride,
                   int level, uint8_t* out) {
  Extractor ex(*cfg);
  ex.compute_pyramid(wrap_image(img, w, h, stride));
  Mat8 b;
  gaussian_blur7(ex.pyr[level], b);
  std::memcpy(out, b.px.data(), b.px.size());
  return 0;
}

int orc_fast_level(const orc_config* cfg, const uint8_t* img, int w, int h, size_t stride,
                   int level, orc_kp* kps, int cap, int* n) {
  Extractor ex(*cfg);
  ex.compute_pyramid(wrap_image(img, w, h, stride));
  std::vector<KeyPoint> cand;
  int bx[4];
  ex.fast_level(level, cand, bx);
  *n = (int)cand.size();
  if (*n > cap) return -1;
  std::memcpy(kps, cand.data(), cand.size() * sizeof(KeyPoint));
  return 0;
}

int orc_distribute(const orc_kp* keys, int nkeys, int minX, int maxX, int minY, int maxY, int N,
                   orc_kp* out, int cap, int* n) {
  std::vector<KeyPoint> in(keys, keys + nkeys);
  std::vector<KeyPoint> r = distribute_oct_tree(in, minX, maxX, minY, maxY, N);
  *n = (int)r.size();
  if (*n > cap) return -1;
  std::memcpy(out, r.data(), r.size() * sizeof(KeyPoint));
  return 0;
}

int orc_descriptor_distance(const uint8_t* a, const uint8_t* b) { return descriptor_distance(a, b); }

int orc_extract_tie_stats(const orc_config* cfg, const uint8_t* img, int w, int h, size_t stride, int* events,
                          int* nodes, int* kps) {
  Extractor ex(*cfg);
  std::vector<KeyPoint> out;
  std::vector<uint8_t> d;
  std::vector<TieStats> t;
  ex.extract(wrap_image(img, w, h, stride), out, d, &t);
  for (int l = 0; l < cfg->nlevels; ++l) {
    const TieStats z = l < (int)t.size() ? t[l] : TieStats{};
    if (events) events[l] = z.events;
    if (nodes) nodes[l] = z.nodes;
    if (kps) kps[l] = z.kps;
  }
  return 0;
}

int orc_extract_rule(const orc_config* cfg, int tie_rule, const uint8_t* img, int w, int h, size_t stride,
                     orc_kp* kps, int cap, uint8_t* desc, int* n) {
  Extractor ex(*cfg);
  ex.tie_rule = tie_rule;
  std::vector<KeyPoint> out;
  std::vector<uint8_t> d;
  ex.extract(wrap_image(img, w, h, stride), out, d);
  *n = (int)out.size();
  if ((int)out.size() > cap) return -1;
  std::memcpy(kps, out.data(), out.size() * sizeof(KeyPoint));
  if (desc) std::memcpy(desc, d.data(), d.size());
  return 0;
}

int orc_tie_sequence(const orc_config* cfg, const uint8_t* frames, int nframes, int w, int h, size_t stride,
                     size_t frame_bytes, int rule_a, int rule_b, int* differs, int* kept_diff) {
  // pass 1: every frame with rule_a in sequence, as the reference's Tracking
  // thread extracts them (one extractor, one heap history); pass 2: rule_b
  const int L = cfg->nlevels;
  std::vector<std::vector<std::vector<KeyPoint>>> res[2];
  for (int r = 0; r < 2; ++r) {
    Extractor ex(*cfg);
    ex.tie_rule = r ? rule_b : rule_a;
    res[r].resize(nframes);
    for (int f = 0; f < nframes; ++f) {
      std::vector<KeyPoint> out;
      std::vector<uint8_t> d;
      ex.extract(wrap_image(frames + (size_t)f * frame_bytes, w, h, stride), out, d);
      res[r][f].assign(L, {});
      for (const KeyPoint& k : out) res[r][f][k.octave].push_back(k);
    }
  }
  auto key = [](const KeyPoint& k) { return std::make_pair(k.y, k.x); };
  for (int f = 0; f < nframes; ++f)
    for (int l = 0; l < L; ++l) {
      const auto& a = res[0][f][l];
      const auto& b = res[1][f][l];
      bool same = a.size() == b.size();
      for (size_t i = 0; same && i < a.size(); ++i) same = std::memcmp(&a[i], &b[i], sizeof(KeyPoint)) == 0;
      differs[f * L + l] = !same;
      // keypoints kept by one rule and not the other (by position)
      std::vector<std::pair<float, float>> ka, kb, only;
      for (const auto& k : a) ka.push_back(key(k));
      for (const auto& k : b) kb.push_back(key(k));
      std::sort(ka.begin(), ka.end());
      std::sort(kb.begin(), kb.end());
      std::set_symmetric_difference(ka.begin(), ka.end(), kb.begin(), kb.end(), std::back_inserter(only));
      kept_diff[f * L + l] = (int)only.size();
    }
  return 0;
}

int orc_tie_address_order(const orc_config* cfg, const uint8_t* frames, int nframes, int w, int h, size_t stride,
                          size_t frame_bytes, long* concordant, long* discordant) {
  static PtrSeqTable table;  // static storage: the study allocates nothing on the heap per node
  g_ptr_seq = &table;
  table.concordant = table.discordant = 0;
  Extractor ex(*cfg);
  ex.tie_rule = kTiePointer;
  for (int f = 0; f < nframes; ++f) {
    std::vector<KeyPoint> out;
    std::vector<uint8_t> d;
    ex.extract(wrap_image(frames + (size_t)f * frame_bytes, w, h, stride), out, d);
  }
  *concordant = table.concordant;
  *discordant = table.discordant;
  g_ptr_seq = nullptr;
  return 0;
}

int orc_distribute_ties(const orc_kp* keys, int nkeys, int minX, int maxX, int minY, int maxY, int N, int* events,
                        int* nodes, int* kps) {
  std::vector<KeyPoint> in(keys, keys + nkeys);
  TieStats t;
  distribute_oct_tree(in, minX, maxX, minY, maxY, N, &t);
  *events = t.events;
  *nodes = t.nodes;
  *kps = t.kps;
  return 0;
}

void orc_pattern(int pattern_mode, signed char* out1024) {
  signed char t[256][4];
  std::memcpy(t, kOracleBriefTests, sizeof(t));
  if (pattern_mode == 1) t[kOracleForkIndex / 4][kOracleForkIndex % 4] = kOracleUpstreamValue;
  std::memcpy(out1024, t, sizeof(t));
}


int orc_compute_stereo_matches(const orc_kp* kpL, const uint8_t* descL, int nL, const orc_kp* kpR,
                               const uint8_t* descR, int nR, const uint8_t* const* pyrL, const size_t* strideL,
                               const uint8_t* const* pyrR, const size_t* strideR, const int* level_w,
                               const int* level_h, int nlevels, const float* scale, const float* inv_scale,
                               float mb, float mbf, float* uRight, float* depth) {
  // src/Frame.cc:465-639
  for (int i = 0; i < nL; i++) {
    uRight[i] = -1.0f;
    depth[i] = -1.0f;
  }
  const int TH_HIGH = 100, TH_LOW = 50;  // src/ORBmatcher.cc:37-38
  const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
  const int nRows = level_h[0];
  // row table: right keypoint iR is a candidate on rows [floor(y - r), ceil(y + r)] (:477-491)
  std::vector<std::vector<size_t>> vRowIndices(nRows);
  for (int iR = 0; iR < nR; iR++) {
    const orc_kp& kp = kpR[iR];
    const float kpY = kp.y;
    const float r = 2.0f * scale[kp.octave];
    const int maxr = (int)std::ceil(kpY + r);
    const int minr = (int)std::floor(kpY - r);
    for (int yi = minr; yi <= maxr; yi++)
      if (yi >= 0 && yi < nRows) vRowIndices[yi].push_back(iR);  // (rows off the image: UB in the reference)
  }
  const float minZ = mb;
  const float minD = 0;
  const float maxD = mbf / minZ;
  std::vector<std::pair<int, int>> vDistIdx;
  vDistIdx.reserve(nL);
  auto level_px = [&](const uint8_t* const* pyr, const size_t* stride, int l, int y, int x) {
    return (float)pyr[l][(size_t)y * stride[l] + x];
  };
  for (int iL = 0; iL < nL; iL++) {
    const orc_kp& kpL_ = kpL[iL];
    const int levelL = kpL_.octave;
    const float vL = kpL_.y;
    const float uL = kpL_.x;
    const size_t row = (size_t)vL;  // vRowIndices[vL]: float -> size_t
    if (row >= (size_t)nRows) continue;
    const std::vector<size_t>& vCandidates = vRowIndices[row];
    if (vCandidates.empty()) continue;
    const float minU = uL - maxD;
    const float maxU = uL - minD;
    if (maxU < 0) continue;
    int bestDist = TH_HIGH;
    size_t bestIdxR = 0;
    const uint8_t* dL = descL + (size_t)iL * 32;
    for (size_t iC = 0; iC < vCandidates.size(); iC++) {
      const size_t iR = vCandidates[iC];
      const orc_kp& kpR_ = kpR[iR];
      if (kpR_.octave < levelL - 1 || kpR_.octave > levelL + 1) continue;
      const float uR = kpR_.x;
      if (uR >= minU && uR <= maxU) {
        const int dist = descriptor_distance(dL, descR + iR * 32);
        if (dist < bestDist) {
          bestDist = dist;
          bestIdxR = iR;
        }
      }
    }
    if (bestDist >= thOrbDist) continue;
    // subpixel match by correlation (:549-606)
    const float uR0 = kpR[bestIdxR].x;
    const float scaleFactor = inv_scale[levelL];
    const float scaleduL = std::round(kpL_.x * scaleFactor);
    const float scaledvL = std::round(kpL_.y * scaleFactor);
    const float scaleduR0 = std::round(uR0 * scaleFactor);
    const int w = 5, L = 5;
    const int vl = (int)scaledvL, ul = (int)scaleduL;
    // a window reaching off the level is an OpenCV range assertion in the
    // reference (Mat::rowRange/colRange); here that keypoint gets no match
    if ((int)scaleduR0 < 10 || ul < 5 || ul + 5 >= level_w[levelL] || vl < 5 || vl + 5 >= level_h[levelL]) continue;
    float IL[11][11];
    const float cL = level_px(pyrL, strideL, levelL, vl, ul);
    for (int r = -w; r <= w; r++)
      for (int c = -w; c <= w; c++) IL[r + w][c + w] = level_px(pyrL, strideL, levelL, vl + r, ul + c) - cL;
    int bestDist2 = INT_MAX;
    int bestincR = 0;
    float vDists[2 * L + 1];
    const float iniu = scaleduR0 + L - w;
    const float endu = scaleduR0 + L + w + 1;
    if (iniu < 0 || endu >= level_w[levelL]) continue;
    const int ur0 = (int)scaleduR0;
    for (int incR = -L; incR <= +L; incR++) {
      const float cR = level_px(pyrR, strideR, levelL, vl, ur0 + incR);
      float dist = 0;  // cv::norm(IL, IR, NORM_L1): a sum of integers below 2^24, exact in any order
      for (int r = -w; r <= w; r++)
        for (int c = -w; c <= w; c++)
          dist += std::fabs(IL[r + w][c + w] - (level_px(pyrR, strideR, levelL, vl + r, ur0 + incR + c) - cR));
      if (dist < bestDist2) {
        bestDist2 = (int)dist;
        bestincR = incR;
      }
      vDists[L + incR] = dist;
    }
    if (bestincR == -L || bestincR == L) continue;
    const float dist1 = vDists[L + bestincR - 1];
    const float dist2 = vDists[L + bestincR];
    const float dist3 = vDists[L + bestincR + 1];
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) continue;
    float bestuR = scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
    float disparity = (uL - bestuR);
    if (disparity >= minD && disparity < maxD) {
      if (disparity <= 0) {
        disparity = 0.01;
        bestuR = uL - 0.01;
      }
      depth[iL] = mbf / disparity;
      uRight[iL] = bestuR;
      vDistIdx.push_back(std::pair<int, int>(bestDist2, iL));
    }
  }
  // outlier rejection by the median SAD (:620-638)
  if (vDistIdx.empty()) return 0;  // (the reference indexes an empty vector here)
  std::sort(vDistIdx.begin(), vDistIdx.end());
  const float median = vDistIdx[vDistIdx.size() / 2].first;
  const float thDist = 1.5f * 1.4f * median;
  int kept = (int)vDistIdx.size();
  for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
    if (vDistIdx[i].first < thDist) break;
    uRight[vDistIdx[i].second] = -1;
    depth[vDistIdx[i].second] = -1;
    --kept;
  }
  return kept;
}

float orc_fast_atan2(float y, float x) { return fast_atan2(y, x); }
void orc_sincosf(const float* x, int n, float* s, float* c) {
  for (int i = 0; i < n; ++i) {
    s[i] = sinf(x[i]);
    c[i] = cosf(x[i]);
  }
}

void orc_hamming_top2(const uint8_t* A, int nA, const uint8_t* B, int nB, int* best_idx,
                      int* best_dist, int* second_dist) {
  for (int i = 0; i < nA; ++i) {
    int bestDist1 = 256, bestIdx = -1, bestDist2 = 256;
    for (int j = 0; j < nB; ++j) {
      const int dist = descriptor_distance(A + 32 * (size_t)i, B + 32 * (size_t)j);
      if (dist < bestDist1) {
        bestDist2 = bestDist1;
        bestDist1 = dist;
        bestIdx = j;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    best_idx[i] = bestIdx;
    best_dist[i] = bestDist1;
    second_dist[i] = bestDist2;
  }
}

int orc_search_for_initialization(const orc_kp* kp1, const uint8_t* desc1, int n1,
                                  const orc_kp* kp2, const uint8_t* desc2, int n2, float min_x,
                                  float max_x, float min_y, float max_y, float* prev_xy,
                                  int windowSize, float mfNNratio, int mbCheckOrientation,
                                  int* vnMatches12, int* out_nmatches) {
  GridFrame F2(kp2, desc2, n2, min_x, max_x, min_y, max_y);
  int nmatches = 0;
  for (int i = 0; i < n1; ++i) vnMatches12[i] = -1;
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  std::vector<int> vMatchedDistance(n2, INT_MAX);
  std::vector<int> vnMatches21(n2, -1);
  for (int i1 = 0; i1 < n1; i1++) {
    const KeyPoint& kp1i = kp1[i1];
    int level1 = kp1i.octave;
    if (level1 > 0) continue;
    const float r = (float)windowSize;
    std::vector<size_t> vIndices2 =
        F2.features_in_area(prev_xy[2 * i1], prev_xy[2 * i1 + 1], r, level1, level1);
    if (vIndices2.empty()) continue;
    const uint8_t* d1 = desc1 + 32 * (size_t)i1;
    int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
    for (size_t i2 : vIndices2) {
      int dist = descriptor_distance(d1, desc2 + 32 * i2);
      if (vMatchedDistance[i2] <= dist) continue;
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestIdx2 = i2;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist <= TH_LOW) {
      if (bestDist < (float)bestDist2 * mfNNratio) {
        if (vnMatches21[bestIdx2] >= 0) {
          vnMatches12[vnMatches21[bestIdx2]] = -1;
          nmatches--;
        }
        vnMatches12[i1] = bestIdx2;
        vnMatches21[bestIdx2] = i1;
        vMatchedDistance[bestIdx2] = bestDist;
        nmatches++;
        if (mbCheckOrientation) {
          float rot = kp1[i1].angle - kp2[bestIdx2].angle;
          if (rot < 0.0) rot += 360.0f;
          int bin = round(rot * factor);
          if (bin == HISTO_LENGTH) bin = 0;
          rotHist[bin].push_back(i1);
        }
      }
    }
  }
  if (mbCheckOrientation) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    compute_three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (size_t j = 0; j < rotHist[i].size(); j++) {
        int idx1 = rotHist[i][j];
        if (vnMatches12[idx1] >= 0) {
          vnMatches12[idx1] = -1;
          nmatches--;
        }
      }
    }
  }
  for (int i1 = 0; i1 < n1; i1++)
    if (vnMatches12[i1] >= 0) {
      prev_xy[2 * i1] = kp2[vnMatches12[i1]].x;
      prev_xy[2 * i1 + 1] = kp2[vnMatches12[i1]].y;
    }
  *out_nmatches = nmatches;
  return 0;
}

int orc_search_by_bow(const uint8_t* descA, const float* angleA, const uint8_t* mpA, int nA,
                      const uint32_t* fvA_nodes, const int* fvA_off, const int* fvA_idx, int fvA_n,
                      const uint8_t* descB, const float* angleB, const uint8_t* mpB, int nB,
                      const uint32_t* fvB_nodes, const int* fvB_off, const int* fvB_idx, int fvB_n,
                      float mfNNratio, int mbCheckOrientation, int kf_vs_kf, int* out,
                      int* out_nmatches) {
  const int nout = kf_vs_kf ? nA : nB;
  for (int i = 0; i < nout; ++i) out[i] = -1;
  std::vector<char> vbMatched2(nB, 0);
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  int nmatches = 0;
  int ia = 0, ib = 0;
  while (ia < fvA_n && ib < fvB_n) {
    if (fvA_nodes[ia] == fvB_nodes[ib]) {
      for (int p = fvA_off[ia]; p < fvA_off[ia + 1]; ++p) {
        const int idx1 = fvA_idx[p];
        if (!mpA[idx1]) continue;  // !pMP || pMP->isBad()
        const uint8_t* d1 = descA + 32 * (size_t)idx1;
        int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
        for (int q = fvB_off[ib]; q < fvB_off[ib + 1]; ++q) {
          const int idx2 = fvB_idx[q];
          if (kf_vs_kf) {
            if (vbMatched2[idx2] || !mpB[idx2]) continue;
          } else {
            if (out[idx2] >= 0) continue;  // vpMapPointMatches[realIdxF] already set
          }
          const int dist = descriptor_distance(d1, descB + 32 * (size_t)idx2);
          if (dist < bestDist1) {
            bestDist2 = bestDist1;
            bestDist1 = dist;
            bestIdx2 = idx2;
          } else if (dist < bestDist2) {
            bestDist2 = dist;
          }
        }
        const bool pass_th = kf_vs_kf ? (bestDist1 < TH_LOW) : (bestDist1 <= TH_LOW);
        if (pass_th) {
          if (static_cast<float>(bestDist1) < mfNNratio * static_cast<float>(bestDist2)) {
            if (kf_vs_kf) {
              out[idx1] = bestIdx2;
              vbMatched2[bestIdx2] = 1;
            } else {
              out[bestIdx2] = idx1;
            }
            if (mbCheckOrientation) {
              float rot = angleA[idx1] - angleB[bestIdx2];
              if (rot < 0.0) rot += 360.0f;
              int bin = round(rot * factor);
              if (bin == HISTO_LENGTH) bin = 0;
              rotHist[bin].push_back(kf_vs_kf ? idx1 : bestIdx2);
            }
            nmatches++;
          }
        }
      }
      ia++;
      ib++;
    } else if (fvA_nodes[ia] < fvB_nodes[ib]) {
      ia = std::lower_bound(fvA_nodes + ia, fvA_nodes + fvA_n, fvB_nodes[ib]) - fvA_nodes;
    } else {
      ib = std::lower_bound(fvB_nodes + ib, fvB_nodes + fvB_n, fvA_nodes[ia]) - fvB_nodes;
    }
  }
  if (mbCheckOrientation) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    compute_three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (size_t j = 0; j < rotHist[i].size(); j++) {
        out[rotHist[i][j]] = -1;
        nmatches--;
      }
    }
  }
  *out_nmatches = nmatches;
  return 0;
}

// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th)
// (src/ORBmatcher.cc:45-118) with RadiusByViewingCos (:120-126). The MapPoint
// fields it reads are passed per point (orc_map_point_proj); the Frame's
// mvpMapPoints[idx] "has a MapPoint with Observations() > 0" state is
// `blocked`. out[idx] = index in vpMapPoints of the point the keypoint got in
// this call (the last one to write it), -1 if none.
int orc_search_by_projection(const orc_kp* kps, const uint8_t* desc, int n, const float* uright, float min_x,
                             float max_x, float min_y, float max_y, const float* scale, const uint8_t* blocked,
                             const orc_map_point_proj* mps, const uint8_t* mpdesc, int nmp, float th,
                             float mfNNratio, int* out, int* out_nmatches) {
  GridFrame F(kps, desc, n, min_x, max_x, min_y, max_y);
  std::vector<int> mp_of(n, -1);          // this call's assignments
  std::vector<uint8_t> blk(blocked, blocked + n);
  int nmatches = 0;
  const bool bFactor = th != 1.0;
  for (int iMP = 0; iMP < nmp; iMP++) {
    const orc_map_point_proj& pMP = mps[iMP];
    if (!pMP.track_in_view) continue;     // mbTrackInView (isBad() folded in by the caller)
    const int& nPredictedLevel = pMP.predicted_level;
    float r = pMP.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos
    if (bFactor) r *= th;
    const std::vector<size_t> vIndices = F.features_in_area(pMP.proj_x, pMP.proj_y, r * scale[nPredictedLevel],
                                                            nPredictedLevel - 1, nPredictedLevel);
    if (vIndices.empty()) continue;
    const uint8_t* MPdescriptor = mpdesc + (size_t)iMP * 32;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (size_t idx : vIndices) {
      if (blk[idx]) continue;  // F.mvpMapPoints[idx] && Observations() > 0
      if (uright && uright[idx] > 0) {
        const float er = fabs(pMP.proj_xr - uright[idx]);
        if (er > r * scale[nPredictedLevel]) continue;
      }
      const int dist = descriptor_distance(MPdescriptor, desc + 32 * idx);
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = kps[idx].octave;
        bestIdx = (int)idx;
      } else if (dist < bestDist2) {
        bestLevel2 = kps[idx].octave;
        bestDist2 = dist;
      }
    }
    if (bestDist <= TH_HIGH) {
      if (bestLevel == bestLevel2 && bestDist > mfNNratio * bestDist2) continue;
      mp_of[bestIdx] = iMP;                     // F.mvpMapPoints[bestIdx] = pMP
      blk[bestIdx] = pMP.obs_positive ? 1 : 0;  // later points see its Observations()
      nmatches++;
    }
  }
  for (int i = 0; i < n; ++i) out[i] = mp_of[i];
  *out_nmatches = nmatches;
  return 0;
}

// ======================================================= pose projection
// The SearchByProjection overloads that project world points with a pose
// (src/ORBmatcher.cc:290-403, 1328-1470, 1472-1599) and the cv::Mat
// arithmetic they run, restated from OpenCV 3.x (Appendix-A style, not
// vendored, PARITY UNPINNED at this boundary):
//  * R*x + t (MatExpr -> gemm(R, x, 1, t, 1), 3x3 times 3x1 float): gemm's
//    small-matrix path: t_r = a0*x0 + a1*x1 + a2*x2 summed in float, then
//    d_r = (float)(t_r*1.0 + c_r*1.0) in double (alpha = beta = 1.0).
//  * -R.t()*t (gemm with GEMM_1_T, alpha -1): the general path,
//    GEMMSingleMul<float,double>: double products summed in order, (float)(-s).
//  * cv::norm(v) (NORM_L2 of 3 floats): std::sqrt of the double sum of the
//    squares; Mat::dot of 3 floats: the double sum of double products.
//  * Mat / s: convertTo(alpha = 1/s): v * (float)(1.0/s) + 0.0f in float.
//  * log(float) in MapPoint::PredictScale and Frame's mfLogScaleFactor: the
//    float overload (glibc logf).
}  // extern "C"

namespace {

struct PoseMath {
  // R*x + t through gemm's small-matrix path
  static void rx_plus_t(const float* T, const float* x, float* d) {
    for (int r = 0; r < 3; ++r) {
      const float t = T[4 * r] * x[0] + T[4 * r + 1] * x[1] + T[4 * r + 2] * x[2];
      d[r] = (float)((double)t * 1.0 + (double)T[4 * r + 3] * 1.0);
    }
  }
  // -R.t()*t through the general gemm path
  static void neg_rt_t(const float* T, float* d) {
    for (int r = 0; r < 3; ++r) {
      double s = 0;
      for (int k = 0; k < 3; ++k) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
      d[r] = (float)(s * -1.0);
    }
  }
  static double norm3(const float* v) {
    double s = 0;
    for (int k = 0; k < 3; ++k) { double e = v[k]; s += e * e; }
    return std::sqrt(s);
  }
  static double dot3(const float* a, const float* b) {
    double s = 0;
    for (int k = 0; k < 3; ++k) s += (double)a[k] * b[k];
    return s;
  }
};

// MapPoint::PredictScale (src/MapPoint.cc:407-422). ceil(log(ratio)/mfLogScaleFactor)
// converted to int; a non-finite quotient converts like x86 cvttss2si (INT_MIN).
int predict_scale(float mfMaxDistance, float currentDist, float mfLogScaleFactor, int mnScaleLevels) {
  const float ratio = mfMaxDistance / currentDist;
  const float q = std::ceil(std::log(ratio) / mfLogScaleFactor);
  int nScale = (q >= -2147483648.0f && q < 2147483648.0f) ? (int)q : INT_MIN;
  if (nScale < 0)
    nScale = 0;
  else if (nScale >= mnScaleLevels)
    nScale = mnScaleLevels - 1;
  return nScale;
}

// Rotation consistency of the motion-model / relocalization overloads
// (src/ORBmatcher.cc:1423-1466, 1577-1596): assignments in bins outside the three
// largest are cleared (mvpMapPoints[i2] = NULL, recorded as -2).
void rotation_filter(std::vector<int>* rotHist, int* out, int& nmatches) {
  int ind1 = -1, ind2 = -1, ind3 = -1;
  compute_three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
  for (int i = 0; i < HISTO_LENGTH; i++) {
    if (i != ind1 && i != ind2 && i != ind3) {
      for (size_t j = 0, jend = rotHist[i].size(); j < jend; j++) {
        out[rotHist[i][j]] = -2;
        nmatches--;
      }
    }
  }
}

}  // namespace

extern "C" {

int orc_predict_scale(float max_distance, float current_dist, float scale_factor, int nlevels) {
  return predict_scale(max_distance, current_dist, std::log(scale_factor), nlevels);
}

void orc_predict_scale_ratios(const float* ratio, int n, float scale_factor, int nlevels, int* out) {
  const float logsf = std::log(scale_factor);
  // predict_scale(maxd, dist) with maxd / dist == ratio: maxd = ratio, dist = 1
  for (int i = 0; i < n; ++i) out[i] = predict_scale(ratio[i], 1.0f, logsf, nlevels);
}

// SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
// (src/ORBmatcher.cc:1328-1470).
int orc_search_by_projection_last_frame(const orc_kp* kps, const uint8_t* desc, int n, const float* uright,
                                        float min_x, float max_x, float min_y, float max_y, const float* scale,
                                        const uint8_t* blocked, const orc_camera* cur, const float* Tlw,
                                        const orc_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th,
                                        int bMono, int mbCheckOrientation, int* out, int* out_nmatches) {
  GridFrame F(kps, desc, n, min_x, max_x, min_y, max_y);
  std::vector<uint8_t> blk(blocked, blocked + n);  // mvpMapPoints[i2] && Observations() > 0
  for (int i = 0; i < n; ++i) out[i] = -1;
  int nmatches = 0;
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  // twc = -Rcw.t()*tcw; tlc = Rlw*twc + tlw  (:1338-1346)
  float twc[3], tlc[3];
  PoseMath::neg_rt_t(cur->Tcw, twc);
  PoseMath::rx_plus_t(Tlw, twc, tlc);
  const bool bForward = tlc[2] > cur->mb && !bMono;
  const bool bBackward = -tlc[2] > cur->mb && !bMono;
  for (int i = 0; i < nmp; i++) {
    const orc_map_point_world& pMP = mps[i];
    if (!pMP.valid) continue;  // pMP && !LastFrame.mvbOutlier[i]
    float x3Dc[3];
    PoseMath::rx_plus_t(cur->Tcw, pMP.pos, x3Dc);
    const float xc = x3Dc[0];
    const float yc = x3Dc[1];
    const float invzc = 1.0 / x3Dc[2];
    if (invzc < 0) continue;
    float u = cur->fx * xc * invzc + cur->cx;
    float v = cur->fy * yc * invzc + cur->cy;
    if (u < min_x || u > max_x) continue;
    if (v < min_y || v > max_y) continue;
    const int nLastOctave = pMP.octave;
    const float radius = th * scale[nLastOctave];
    std::vector<size_t> vIndices2;
    if (bForward)
      vIndices2 = F.features_in_area(u, v, radius, nLastOctave, -1);
    else if (bBackward)
      vIndices2 = F.features_in_area(u, v, radius, 0, nLastOctave);
    else
      vIndices2 = F.features_in_area(u, v, radius, nLastOctave - 1, nLastOctave + 1);
    if (vIndices2.empty()) continue;
    const uint8_t* dMP = mpdesc + 32 * (size_t)i;
    int bestDist = 256, bestIdx2 = -1;
    for (size_t i2 : vIndices2) {
      if (blk[i2]) continue;
      if (uright && uright[i2] > 0) {
        const float ur = u - cur->mbf * invzc;
        const float er = fabs(ur - uright[i2]);
        if (er > radius) continue;
      }
      const int dist = descriptor_distance(dMP, desc + 32 * i2);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = (int)i2;
      }
    }
    if (bestDist <= TH_HIGH) {
      out[bestIdx2] = i;  // CurrentFrame.mvpMapPoints[bestIdx2] = pMP
      blk[bestIdx2] = pMP.obs_positive;
      nmatches++;
      if (mbCheckOrientation) {
        float rot = pMP.angle - kps[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = round(rot * factor);
        if (bin == HISTO_LENGTH) bin = 0;
        rotHist[bin].push_back(bestIdx2);
      }
    }
  }
  if (mbCheckOrientation) rotation_filter(rotHist, out, nmatches);
  *out_nmatches = nmatches;
  return 0;
}

// SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, sAlreadyFound, th, ORBdist)
// (src/ORBmatcher.cc:1472-1599).
int orc_search_by_projection_keyframe(const orc_kp* kps, const uint8_t* desc, int n, float min_x, float max_x,
                                      float min_y, float max_y, const float* scale, int nlevels,
                                      float scale_factor, const uint8_t* has_mp, const orc_camera* cur,
                                      const orc_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th,
                                      int ORBdist, int mbCheckOrientation, int* out, int* out_nmatches) {
  GridFrame F(kps, desc, n, min_x, max_x, min_y, max_y);
  std::vector<uint8_t> taken(has_mp, has_mp + n);  // CurrentFrame.mvpMapPoints[i2] != NULL
  for (int i = 0; i < n; ++i) out[i] = -1;
  const float mfLogScaleFactor = std::log(scale_factor);
  float Ow[3];
  PoseMath::neg_rt_t(cur->Tcw, Ow);
  int nmatches = 0;
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  for (int i = 0; i < nmp; i++) {
    const orc_map_point_world& pMP = mps[i];
    if (!pMP.valid) continue;  // pMP && !isBad() && !sAlreadyFound.count(pMP)
    float x3Dc[3];
    PoseMath::rx_plus_t(cur->Tcw, pMP.pos, x3Dc);
    const float xc = x3Dc[0];
    const float yc = x3Dc[1];
    const float invzc = 1.0 / x3Dc[2];
    const float u = cur->fx * xc * invzc + cur->cx;
    const float v = cur->fy * yc * invzc + cur->cy;
    if (u < min_x || u > max_x) continue;
    if (v < min_y || v > max_y) continue;
    float PO[3];
    for (int k = 0; k < 3; ++k) PO[k] = pMP.pos[k] - Ow[k];
    const float dist3D = PoseMath::norm3(PO);
    const float maxDistance = 1.2f * pMP.max_distance;  // GetMaxDistanceInvariance
    const float minDistance = 0.8f * pMP.min_distance;  // GetMinDistanceInvariance
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    const int nPredictedLevel = predict_scale(pMP.max_distance, dist3D, mfLogScaleFactor, nlevels);
    const float radius = th * scale[nPredictedLevel];
    const std::vector<size_t> vIndices2 =
        F.features_in_area(u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1);
    if (vIndices2.empty()) continue;
    const uint8_t* dMP = mpdesc + 32 * (size_t)i;
    int bestDist = 256, bestIdx2 = -1;
    for (size_t i2 : vIndices2) {
      if (taken[i2]) continue;
      const int dist = descriptor_distance(dMP, desc + 32 * i2);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = (int)i2;
      }
    }
    if (bestDist <= ORBdist) {
      out[bestIdx2] = i;
      taken[bestIdx2] = 1;
      nmatches++;
      if (mbCheckOrientation) {
        float rot = pMP.angle - kps[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = round(rot * factor);
        if (bin == HISTO_LENGTH) bin = 0;
        rotHist[bin].push_back(bestIdx2);
      }
    }
  }
  if (mbCheckOrientation) rotation_filter(rotHist, out, nmatches);
  *out_nmatches = nmatches;
  return 0;
}

// SearchByProjection(KeyFrame* pKF, cv::Mat Scw, vpPoints, vpMatched, th)
// (src/ORBmatcher.cc:290-403) with KeyFrame::IsInImage (src/KeyFrame.cc:619-622)
// and KeyFrame::GetFeaturesInArea (:578-617, no level filter).
int orc_search_by_projection_sim3(const orc_kp* kps, const uint8_t* desc, int n, float min_x, float max_x,
                                  float min_y, float max_y, const float* scale, int nlevels, float scale_factor,
                                  const orc_camera* kf, const orc_map_point_world* mps, const uint8_t* mpdesc,
                                  int nmp, int th, const int* matched, int* out, int* out_nmatches) {
  GridFrame F(kps, desc, n, min_x, max_x, min_y, max_y);
  std::vector<uint8_t> taken(n);
  for (int i = 0; i < n; ++i) {
    taken[i] = matched && matched[i] >= 0;  // vpMatched[idx]
    out[i] = -1;
  }
  const float mfLogScaleFactor = std::log(scale_factor);
  // Decompose Scw (:298-304)
  const float* S = kf->Tcw;
  const float scw = std::sqrt(PoseMath::dot3(S, S));  // sRcw.row(0).dot(sRcw.row(0))
  const float a = (float)(1.0 / (double)scw);         // (Mat / scw): convertTo alpha
  float T[12];
  for (int k = 0; k < 12; ++k) T[k] = S[k] * a + 0.0f;  // Rcw = sRcw/scw, tcw = t/scw
  float Ow[3];
  PoseMath::neg_rt_t(T, Ow);
  int nmatches = 0;
  for (int iMP = 0; iMP < nmp; iMP++) {
    const orc_map_point_world& pMP = mps[iMP];
    if (!pMP.valid) continue;  // pMP->isBad() || spAlreadyFound.count(pMP)
    float p3Dc[3];
    PoseMath::rx_plus_t(T, pMP.pos, p3Dc);
    if (p3Dc[2] < 0.0) continue;
    const float invz = 1 / p3Dc[2];
    const float x = p3Dc[0] * invz;
    const float y = p3Dc[1] * invz;
    const float u = kf->fx * x + kf->cx;
    const float v = kf->fy * y + kf->cy;
    if (!(u >= min_x && u < max_x && v >= min_y && v < max_y)) continue;  // pKF->IsInImage
    const float maxDistance = 1.2f * pMP.max_distance;
    const float minDistance = 0.8f * pMP.min_distance;
    float PO[3];
    for (int k = 0; k < 3; ++k) PO[k] = pMP.pos[k] - Ow[k];
    const float dist = PoseMath::norm3(PO);
    if (dist < minDistance || dist > maxDistance) continue;
    if (PoseMath::dot3(PO, pMP.normal) < 0.5 * dist) continue;  // viewing angle < 60 deg
    const int nPredictedLevel = predict_scale(pMP.max_distance, dist, mfLogScaleFactor, nlevels);
    const float radius = th * scale[nPredictedLevel];
    const std::vector<size_t> vIndices = F.features_in_area(u, v, radius, -1, -1);
    if (vIndices.empty()) continue;
    const uint8_t* dMP = mpdesc + 32 * (size_t)iMP;
    int bestDist = 256, bestIdx = -1;
    for (size_t idx : vIndices) {
      if (taken[idx]) continue;
      const int& kpLevel = kps[idx].octave;
      if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
      const int dist = descriptor_distance(dMP, desc + 32 * idx);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = (int)idx;
      }
    }
    if (bestDist <= TH_LOW) {
      out[bestIdx] = iMP;  // vpMatched[bestIdx] = pMP
      taken[bestIdx] = 1;
      nmatches++;
    }
  }
  *out_nmatches = nmatches;
  return 0;
}

}  // extern "C"

// ===================================== Fuse, SearchBySim3, SearchForTriangulation
namespace {

// Sim3 decomposition of the loop-closing overloads (src/ORBmatcher.cc:298-304,
// 986-992): scw = sqrt(row0 . row0) (double dot), Rcw = sRcw/scw, tcw = t/scw.
void decompose_sim3(const float* S, float* T) {
  const float scw = std::sqrt(PoseMath::dot3(S, S));
  const float a = (float)(1.0 / (double)scw);
  for (int k = 0; k < 12; ++k) T[k] = S[k] * a + 0.0f;
}

// KeyFrame::IsInImage (src/KeyFrame.cc:619-622)
inline bool in_image(float u, float v, float min_x, float max_x, float min_y, float max_y) {
  return u >= min_x && u < max_x && v >= min_y && v < max_y;
}

}  // namespace

extern "C" {

// Fuse(KeyFrame*, const vector<MapPoint*>&, th) (src/ORBmatcher.cc:825-975), match part.
int orc_fuse(const orc_kp* kps, const uint8_t* desc, int n, const float* uright, float min_x, float max_x,
             float min_y, float max_y, const float* scale, const float* inv_sigma2, int nlevels, float scale_factor,
             const orc_camera* kf, const orc_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th, int* out,
             int* nfused) {
  GridFrame F(kps, desc, n, min_x, max_x, min_y, max_y);
  const float mfLogScaleFactor = std::log(scale_factor);
  const float* T = kf->Tcw;
  float Ow[3];
  PoseMath::neg_rt_t(T, Ow);  // pKF->GetCameraCenter()
  const float &fx = kf->fx, &fy = kf->fy, &cx = kf->cx, &cy = kf->cy, &bf = kf->mbf;
  int nFused = 0;
  for (int i = 0; i < nmp; i++) {
    out[i] = -1;
    const orc_map_point_world& pMP = mps[i];
    if (!pMP.valid) continue;  // !pMP || isBad() || IsInKeyFrame(pKF)
    float p3Dc[3];
    PoseMath::rx_plus_t(T, pMP.pos, p3Dc);
    if (p3Dc[2] < 0.0f) continue;
    const float invz = 1 / p3Dc[2];
    const float x = p3Dc[0] * invz;
    const float y = p3Dc[1] * invz;
    const float u = fx * x + cx;
    const float v = fy * y + cy;
    if (!in_image(u, v, min_x, max_x, min_y, max_y)) continue;
    const float ur = u - bf * invz;
    const float maxDistance = 1.2f * pMP.max_distance;
    const float minDistance = 0.8f * pMP.min_distance;
    float PO[3];
    for (int k = 0; k < 3; ++k) PO[k] = pMP.pos[k] - Ow[k];
    const float dist3D = PoseMath::norm3(PO);
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    if (PoseMath::dot3(PO, pMP.normal) < 0.5 * dist3D) continue;
    const int nPredictedLevel = predict_scale(pMP.max_distance, dist3D, mfLogScaleFactor, nlevels);
    const float radius = th * scale[nPredictedLevel];
    const std::vector<size_t> vIndices = F.features_in_area(u, v, radius, -1, -1);
    if (vIndices.empty()) continue;
    const uint8_t* dMP = mpdesc + 32 * (size_t)i;
    int bestDist = 256, bestIdx = -1;
    for (size_t idx : vIndices) {
      const KeyPoint& kp = kps[idx];
      const int& kpLevel = kp.octave;
      if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
      if (uright && uright[idx] >= 0) {
        const float& kpx = kp.x;
        const float& kpy = kp.y;
        const float& kpr = uright[idx];
        const float ex = u - kpx;
        const float ey = v - kpy;
        const float er = ur - kpr;
        const float e2 = ex * ex + ey * ey + er * er;
        if (e2 * inv_sigma2[kpLevel] > 7.8) continue;
      } else {
        const float ex = u - kp.x;
        const float ey = v - kp.y;
        const float e2 = ex * ex + ey * ey;
        if (e2 * inv_sigma2[kpLevel] > 5.99) continue;
      }
      const int dist = descriptor_distance(dMP, desc + 32 * idx);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = (int)idx;
      }
    }
    if (bestDist <= TH_LOW) {
      out[i] = bestIdx;
      nFused++;
    }
  }
  *nfused = nFused;
  return 0;
}

// Fuse(KeyFrame*, cv::Mat Scw, vpPoints, th, vpReplacePoint) (src/ORBmatcher.cc:977-1100), match part.
int orc_fuse_sim3(const orc_kp* kps, const uint8_t* desc, int n, float min_x, float max_x, float min_y,
                  float max_y, const float* scale, int nlevels, float scale_factor, const orc_camera* kf,
                  const orc_map_point_world* mps, const uint8_t* mpdesc, int nmp, float th, int* out, int* nfused) {
  GridFrame F(kps, desc, n, min_x, max_x, min_y, max_y);
  const float mfLogScaleFactor = std::log(scale_factor);
  float T[12], Ow[3];
  decompose_sim3(kf->Tcw, T);
  PoseMath::neg_rt_t(T, Ow);
  int nFused = 0;
  for (int iMP = 0; iMP < nmp; iMP++) {
    out[iMP] = -1;
    const orc_map_point_world& pMP = mps[iMP];
    if (!pMP.valid) continue;  // isBad() || spAlreadyFound.count(pMP)
    float p3Dc[3];
    PoseMath::rx_plus_t(T, pMP.pos, p3Dc);
    if (p3Dc[2] < 0.0f) continue;
    const float invz = 1.0 / p3Dc[2];
    const float x = p3Dc[0] * invz;
    const float y = p3Dc[1] * invz;
    const float u = kf->fx * x + kf->cx;
    const float v = kf->fy * y + kf->cy;
    if (!in_image(u, v, min_x, max_x, min_y, max_y)) continue;
    const float maxDistance = 1.2f * pMP.max_distance;
    const float minDistance = 0.8f * pMP.min_distance;
    float PO[3];
    for (int k = 0; k < 3; ++k) PO[k] = pMP.pos[k] - Ow[k];
    const float dist3D = PoseMath::norm3(PO);
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    if (PoseMath::dot3(PO, pMP.normal) < 0.5 * dist3D) continue;
    const int nPredictedLevel = predict_scale(pMP.max_distance, dist3D, mfLogScaleFactor, nlevels);
    const float radius = th * scale[nPredictedLevel];
    const std::vector<size_t> vIndices = F.features_in_area(u, v, radius, -1, -1);
    if (vIndices.empty()) continue;
    const uint8_t* dMP = mpdesc + 32 * (size_t)iMP;
    int bestDist = INT_MAX, bestIdx = -1;
    for (size_t idx : vIndices) {
      const int& kpLevel = kps[idx].octave;
      if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
      int dist = descriptor_distance(dMP, desc + 32 * idx);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = (int)idx;
      }
    }
    if (bestDist <= TH_LOW) {
      out[iMP] = bestIdx;
      nFused++;
    }
  }
  *nfused = nFused;
  return 0;
}

// SearchBySim3 (src/ORBmatcher.cc:1102-1326).
int orc_search_by_sim3(const orc_kp* kps1, const uint8_t* desc1, int n1, const float* bounds1, const float* scale1,
                       const orc_kp* kps2, const uint8_t* desc2, int n2, const float* bounds2, const float* scale2,
                       int nlevels, float scale_factor, const orc_camera* cam1, const float* T1w, const float* T2w,
                       float s12, const float* R12, const float* t12, const orc_map_point_world* mps1,
                       const uint8_t* mpdesc1, const orc_map_point_world* mps2, const uint8_t* mpdesc2, float th,
                       int* match1, int* vnMatch1_out, int* vnMatch2_out, int* nfound) {
  GridFrame F1(kps1, desc1, n1, bounds1[0], bounds1[1], bounds1[2], bounds1[3]);
  GridFrame F2(kps2, desc2, n2, bounds2[0], bounds2[1], bounds2[2], bounds2[3]);
  const float mfLogScaleFactor = std::log(scale_factor);
  const float &fx = cam1->fx, &fy = cam1->fy, &cx = cam1->cx, &cy = cam1->cy;
  // sR12 = s12*R12; sR21 = (1.0/s12)*R12.t(); t21 = -sR21*t12 (convertTo scaling, small gemm)
  float S12[12], S21[12];
  const float a12 = (float)(double)s12, a21 = (float)(1.0 / (double)s12);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      S12[4 * r + c] = R12[3 * r + c] * a12 + 0.0f;
      S21[4 * r + c] = R12[3 * c + r] * a21 + 0.0f;
    }
  for (int r = 0; r < 3; ++r) {
    S12[4 * r + 3] = t12[r];
    const float t = S21[4 * r] * t12[0] + S21[4 * r + 1] * t12[1] + S21[4 * r + 2] * t12[2];
    S21[4 * r + 3] = (float)((double)t * -1.0 + 0.0 * 0.0);
  }
  std::vector<int> vnMatch1(n1, -1), vnMatch2(n2, -1);
  // one direction: points of A through Taw then S (into B's camera), matched in B
  auto dir = [&](const orc_map_point_world* mps, const uint8_t* mpdesc, int nA, const float* Taw, const float* S,
                 const GridFrame& FB, const orc_kp* kpsB, const float* bB, const float* scaleB, std::vector<int>& vm) {
    for (int i1 = 0; i1 < nA; i1++) {
      const orc_map_point_world& pMP = mps[i1];
      if (!pMP.valid) continue;  // !pMP || vbAlreadyMatched || isBad()
      float p3Dc1[3], p3Dc2[3];
      PoseMath::rx_plus_t(Taw, pMP.pos, p3Dc1);
      PoseMath::rx_plus_t(S, p3Dc1, p3Dc2);
      if (p3Dc2[2] < 0.0) continue;
      const float invz = 1.0 / p3Dc2[2];
      const float x = p3Dc2[0] * invz;
      const float y = p3Dc2[1] * invz;
      const float u = fx * x + cx;
      const float v = fy * y + cy;
      if (!in_image(u, v, bB[0], bB[1], bB[2], bB[3])) continue;
      const float maxDistance = 1.2f * pMP.max_distance;
      const float minDistance = 0.8f * pMP.min_distance;
      const float dist3D = PoseMath::norm3(p3Dc2);
      if (dist3D < minDistance || dist3D > maxDistance) continue;
      const int nPredictedLevel = predict_scale(pMP.max_distance, dist3D, mfLogScaleFactor, nlevels);
      const float radius = th * scaleB[nPredictedLevel];
      const std::vector<size_t> vIndices = FB.features_in_area(u, v, radius, -1, -1);
      if (vIndices.empty()) continue;
      const uint8_t* dMP = mpdesc + 32 * (size_t)i1;
      int bestDist = INT_MAX, bestIdx = -1;
      for (size_t idx : vIndices) {
        const KeyPoint& kp = kpsB[idx];
        if (kp.octave < nPredictedLevel - 1 || kp.octave > nPredictedLevel) continue;
        const int dist = descriptor_distance(dMP, FB.desc + 32 * idx);
        if (dist < bestDist) {
          bestDist = dist;
          bestIdx = (int)idx;
        }
      }
      if (bestDist <= TH_HIGH) vm[i1] = bestIdx;
    }
  };
  dir(mps1, mpdesc1, n1, T1w, S21, F2, kps2, bounds2, scale2, vnMatch1);
  dir(mps2, mpdesc2, n2, T2w, S12, F1, kps1, bounds1, scale1, vnMatch2);
  int nFound = 0;
  for (int i1 = 0; i1 < n1; i1++) {
    match1[i1] = -1;
    const int idx2 = vnMatch1[i1];
    if (idx2 >= 0) {
      const int idx1 = vnMatch2[idx2];
      if (idx1 == i1) {
        match1[i1] = idx2;
        nFound++;
      }
    }
  }
  if (vnMatch1_out) std::copy(vnMatch1.begin(), vnMatch1.end(), vnMatch1_out);
  if (vnMatch2_out) std::copy(vnMatch2.begin(), vnMatch2.end(), vnMatch2_out);
  *nfound = nFound;
  return 0;
}

// SearchForTriangulation (src/ORBmatcher.cc:657-823) with CheckDistEpipolarLine (:140-157).
int orc_search_for_triangulation(const orc_kp* kps1, const uint8_t* desc1, const float* uright1,
                                 const uint8_t* has_mp1, int n1, const uint32_t* fv1_nodes, const int* fv1_off,
                                 const int* fv1_idx, int fv1_n, const orc_kp* kps2, const uint8_t* desc2,
                                 const float* uright2, const uint8_t* has_mp2, int n2, const uint32_t* fv2_nodes,
                                 const int* fv2_off, const int* fv2_idx, int fv2_n, const float* cw1,
                                 const float* T2w, const float* cam2, const float* scale2, const float* sigma2,
                                 const float* F12, int only_stereo, int check_ori, int* matches12, int* nmatches_out) {
  // Compute epipole in second image
  float C2[3];
  PoseMath::rx_plus_t(T2w, cw1, C2);  // C2 = R2w*Cw + t2w
  const float invz = 1.0f / C2[2];
  const float ex = cam2[0] * C2[0] * invz + cam2[2];
  const float ey = cam2[1] * C2[1] * invz + cam2[3];
  auto check_epipolar = [&](const KeyPoint& kp1, const KeyPoint& kp2) {
    const float a = kp1.x * F12[0] + kp1.y * F12[3] + F12[6];
    const float b = kp1.x * F12[1] + kp1.y * F12[4] + F12[7];
    const float c = kp1.x * F12[2] + kp1.y * F12[5] + F12[8];
    const float num = a * kp2.x + b * kp2.y + c;
    const float den = a * a + b * b;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * sigma2[kp2.octave];
  };
  int nmatches = 0;
  std::vector<bool> vbMatched2(n2, false);
  std::vector<int> vMatches12(n1, -1);
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  int f1 = 0, f2 = 0;
  while (f1 < fv1_n && f2 < fv2_n) {
    if (fv1_nodes[f1] == fv2_nodes[f2]) {
      for (int p1 = fv1_off[f1]; p1 < fv1_off[f1 + 1]; p1++) {
        const size_t idx1 = fv1_idx[p1];
        if (has_mp1[idx1]) continue;  // already a MapPoint
        const bool bStereo1 = uright1[idx1] >= 0;
        if (only_stereo)
          if (!bStereo1) continue;
        const KeyPoint& kp1 = kps1[idx1];
        const uint8_t* d1 = desc1 + 32 * idx1;
        int bestDist = TH_LOW;
        int bestIdx2 = -1;
        for (int p2 = fv2_off[f2]; p2 < fv2_off[f2 + 1]; p2++) {
          const size_t idx2 = fv2_idx[p2];
          if (vbMatched2[idx2] || has_mp2[idx2]) continue;
          const bool bStereo2 = uright2[idx2] >= 0;
          if (only_stereo)
            if (!bStereo2) continue;
          const int dist = descriptor_distance(d1, desc2 + 32 * idx2);
          if (dist > TH_LOW || dist > bestDist) continue;
          const KeyPoint& kp2 = kps2[idx2];
          if (!bStereo1 && !bStereo2) {
            const float distex = ex - kp2.x;
            const float distey = ey - kp2.y;
            if (distex * distex + distey * distey < 100 * scale2[kp2.octave]) continue;
          }
          if (check_epipolar(kp1, kp2)) {
            bestIdx2 = (int)idx2;
            bestDist = dist;
          }
        }
        if (bestIdx2 >= 0) {
          const KeyPoint& kp2 = kps2[bestIdx2];
          vMatches12[idx1] = bestIdx2;
          nmatches++;
          if (check_ori) {
            float rot = kp1.angle - kp2.angle;
            if (rot < 0.0) rot += 360.0f;
            int bin = round(rot * factor);
            if (bin == HISTO_LENGTH) bin = 0;
            rotHist[bin].push_back((int)idx1);
          }
        }
      }
      f1++;
      f2++;
    } else if (fv1_nodes[f1] < fv2_nodes[f2]) {
      f1 = (int)(std::lower_bound(fv1_nodes + f1, fv1_nodes + fv1_n, fv2_nodes[f2]) - fv1_nodes);
    } else {
      f2 = (int)(std::lower_bound(fv2_nodes + f2, fv2_nodes + fv2_n, fv1_nodes[f1]) - fv2_nodes);
    }
  }
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    compute_three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (size_t j = 0, jend = rotHist[i].size(); j < jend; j++) {
        vMatches12[rotHist[i][j]] = -1;
        nmatches--;
      }
    }
  }
  for (int i = 0; i < n1; ++i) matches12[i] = vMatches12[i];
  *nmatches_out = nmatches;
  return 0;
}

}  // extern "C"
