// Source-compatible replacement for the reference's include/ORBextractor.h
// (:75-197): the same class, constructor, operator() and getters, with the
// VisionWorks graph members (:119-196) replaced by one liborbx handle. Frame,
// Tracking and the rest compile against it unchanged.
#ifndef ORBEXTRACTOR_H
#define ORBEXTRACTOR_H

#include <chrono>
#include <list>
#include <string>
#include <vector>

#include <opencv2/core/core.hpp>

#include "orbx_c.h"

namespace ORB_SLAM2 {

class ORBextractor;

// Per-stage time records (include/ORBextractor.h:41-60): Tracking.cc also
// times its own stages with them (src/Tracking.cc:290-945).
struct times_t {
  int frame;
  std::string name;
  int level;
  long long time;
};

class GetTime {
 public:
  GetTime(ORBextractor* o, std::string name, int level);
  GetTime(std::vector<times_t>& times, int nFrame, std::string name, int level);
  ~GetTime();

 private:
  GetTime();
  ORBextractor* o;
  times_t t;
  std::chrono::steady_clock::time_point start;
  std::vector<times_t>& times;
};

class ORBextractor {
  friend class GetTime;

 public:
  enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int width, int height);
  ~ORBextractor();
  ORBextractor(const ORBextractor&) = delete;
  ORBextractor& operator=(const ORBextractor&) = delete;

  // Compute the ORB features and descriptors on an image (mask ignored, as
  // in the reference).
  void operator()(cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints,
                  cv::OutputArray descriptors);

  // The stereo Frame's two calls (src/Frame.cc:77-80, operator() on threadLeft
  // and threadRight) and ComputeStereoMatches (:89) with one device round trip
  // (orbm_stereo_frame): the same keypoints, descriptors, mvImagePyramid and
  // uRight / depth (mvuRight, mvDepth: one entry per left keypoint) as those
  // three steps. Images of different sizes or an empty one take the steps one
  // after the other. mb, mbf as Frame's.
  static void ExtractStereo(ORBextractor& left, ORBextractor& right, const cv::Mat& imLeft, const cv::Mat& imRight,
                            orbm_handle matcher, float mb, float mbf, std::vector<cv::KeyPoint>& keysLeft,
                            cv::OutputArray descLeft, std::vector<cv::KeyPoint>& keysRight, cv::OutputArray descRight,
                            std::vector<float>& uRight, std::vector<float>& depth);

  int inline GetLevels() { return nlevels; }
  float inline GetScaleFactor() { return (float)scaleFactor; }
  std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
  std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
  std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
  std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

  // The pyramid of the last call (src/ORBextractor.cc:1837-1863). Opt-in
  // (ORBX_HOST_PYRAMID=1): headers over the handle's pinned host copy, which
  // orbx_extract then fills beside the other kernels (orbx_set_host_pyramid).
  // Lifetime and aliasing differ from the reference's: the Mats do not own
  // their data; every level (level 0 is the call's input staging buffer) is
  // overwritten by the next operator() on this extractor, so a caller that
  // keeps a level across calls must clone() it (the reference allocates
  // fresh Mats per call, :1847). Off by default the levels stay empty: the
  // reference's only reader, ComputeStereoMatches (src/Frame.cc:472-579),
  // reads the device pyramids here (the Frame.cc body), and
  // the copy would cost ~30 us per call. A build that keeps the reference's
  // own Frame.cc body must set ORBX_HOST_PYRAMID=1.
  std::vector<cv::Mat> mvImagePyramid;

  // Per-stage device times of the last call, named as the reference's
  // GetTime records ("Pyramid/Resize", "FAST+Grid", ...).
  int GetStageTimes(std::vector<float>& ms, std::vector<const char*>& names);

  // The liborbx handle (its device pyramid of the last call is what
  // Frame::ComputeStereoMatches reads through orbm_compute_stereo_matches).
  orbx_handle handle() const { return h_; }

 protected:
  int nfeatures;
  double scaleFactor;
  int nlevels;
  int iniThFAST;
  int minThFAST;

  std::vector<int> mnFeaturesPerLevel;
  std::vector<float> mvScaleFactor;
  std::vector<float> mvInvScaleFactor;
  std::vector<float> mvLevelSigma2;
  std::vector<float> mvInvLevelSigma2;

  // the reference's per-extractor statistics (:145-148): operator()'s host
  // time, the frame count, and with ORBX_TIMING=1 the device stage times of
  // every call, written to times.csv by the destructor (src/ORBextractor.cc:800-820)
  long long totalTime = 0;
  unsigned int nFrame = 0;
  std::vector<times_t> times;

  void BeginCall(const cv::Mat& image, std::vector<cv::KeyPoint>& keypoints, cv::OutputArray descriptors);
  void EndCall(int n, std::vector<cv::KeyPoint>& keypoints, cv::OutputArray descriptors);

  orbx_handle h_ = nullptr;
  int cap_ = 0;
  bool timing_ = false;
  bool host_pyr_ = true;
  std::vector<int> lw_, lh_;  // level sizes (orbx_get_levels_info, refreshed on a new image size)
};

}  // namespace ORB_SLAM2

#endif
