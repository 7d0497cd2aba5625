// The slice of ORB_SLAM2::Frame (include/Frame.h) that the extractor and
// matcher shims read, with the reference's member names: N, mvKeys,
// mvKeysUn, mDescriptors, mBowVec, mFeatVec, mpORBvocabulary, the camera
// (static fx .. invfy, mb, mbf), stereo fields (mvKeysRight,
// mDescriptorsRight, mvuRight, mvDepth), the pose mTcw, mvpMapPoints,
// mvbOutlier, the scale tables and the static image bounds mnMinX..mnMaxY
// (Frame.h:110-186). ComputeBoW is src/Frame.cc:394-401; ComputeStereoMatches
// (:465-639) is the drop-in body in shim/src/Frame.cc. A test stand-in; a
// real build uses the reference's Frame with that one body replaced.
#ifndef ORBX_SHIM_FRAME_H
#define ORBX_SHIM_FRAME_H
#include <cmath>
#include <cstdlib>
#include <exception>
#include <thread>
#include <vector>

#include <opencv2/core/core.hpp>

#include "DBoW2.h"
#include "ORBVocabulary.h"
#include "ORBextractor.h"

namespace ORB_SLAM2 {
class MapPoint;

class Frame {
 public:
  Frame() = default;
  // The monocular constructor's extraction step (src/Frame.cc:172-190 ->
  // ExtractORB :246-252); no undistortion (mvKeysUn = mvKeys, zero
  // distortion), bounds from the image (ComputeImageBounds, :640-667).
  Frame(const cv::Mat& imGray, ORBextractor* extractor, ORBVocabulary* voc)
      : mpORBvocabulary(voc), mpORBextractorLeft(extractor) {
    scale_info();
    (*mpORBextractorLeft)(imGray, cv::noArray(), mvKeys, mDescriptors);
    N = (int)mvKeys.size();
    mvKeysUn = mvKeys;
    mvpMapPoints.assign(N, static_cast<MapPoint*>(nullptr));
    mvbOutlier.assign(N, false);
    image_bounds(imGray);
  }
  // The stereo constructor (src/Frame.cc:60-128); bf = baseline x fx, mb =
  // bf / fx. Its extraction and matching steps (:77-89) are the drop-in body
  // ExtractStereo (shim/src/Frame.cc: both extractions and ComputeStereoMatches
  // in one device round trip). ORBX_STEREO_THREADS=1 runs the reference's own
  // structure instead, for comparison: ExtractORB on two std::threads
  // (threadLeft / threadRight), an exception on either rethrown here after
  // both joined, then ComputeStereoMatches().
  Frame(const cv::Mat& imLeft, const cv::Mat& imRight, ORBextractor* extractorLeft, ORBextractor* extractorRight,
        ORBVocabulary* voc, float bf)
      : mpORBvocabulary(voc), mpORBextractorLeft(extractorLeft), mpORBextractorRight(extractorRight), mbf(bf) {
    scale_info();
    mb = mbf / fx;
    const char* th = std::getenv("ORBX_STEREO_THREADS");
    if (th && th[0] == '1') {
      std::exception_ptr errL, errR;
      std::thread threadLeft([&] {
        try {
          (*mpORBextractorLeft)(imLeft, cv::noArray(), mvKeys, mDescriptors);
        } catch (...) {
          errL = std::current_exception();
        }
      });
      std::thread threadRight([&] {
        try {
          (*mpORBextractorRight)(imRight, cv::noArray(), mvKeysRight, mDescriptorsRight);
        } catch (...) {
          errR = std::current_exception();
        }
      });
      threadLeft.join();
      threadRight.join();
      if (errL) std::rethrow_exception(errL);
      if (errR) std::rethrow_exception(errR);
      N = (int)mvKeys.size();
      ComputeStereoMatches();
    } else {
      ExtractStereo(imLeft, imRight);
    }
    mvKeysUn = mvKeys;
    image_bounds(imLeft);
    mvpMapPoints.assign(N, static_cast<MapPoint*>(nullptr));
    mvbOutlier.assign(N, false);
  }
  void ComputeBoW() {
    if (mBowVec.empty()) {
      std::vector<cv::Mat> vCurrentDesc;  // Converter::toDescriptorVector
      vCurrentDesc.reserve(mDescriptors.rows);
      for (int j = 0; j < mDescriptors.rows; j++) vCurrentDesc.push_back(mDescriptors.row(j));
      mpORBvocabulary->transform(vCurrentDesc, mBowVec, mFeatVec, 4);
    }
  }
  // Search a match for each keypoint in the left image to a keypoint in the
  // right image (shim/src/Frame.cc, over orbm_compute_stereo_matches)
  void ComputeStereoMatches();
  // The stereo constructor's ExtractORB threads and ComputeStereoMatches
  // (src/Frame.cc:77-89) in one call (shim/src/Frame.cc): mvKeys, mDescriptors,
  // mvKeysRight, mDescriptorsRight, N, mvuRight, mvDepth
  void ExtractStereo(const cv::Mat& imLeft, const cv::Mat& imRight);

  ORBVocabulary* mpORBvocabulary = nullptr;
  ORBextractor* mpORBextractorLeft = nullptr;
  ORBextractor* mpORBextractorRight = nullptr;
  static float fx, fy, cx, cy, invfx, invfy;
  float mbf = 0.f, mb = 0.f;
  int N = 0;
  std::vector<cv::KeyPoint> mvKeys, mvKeysRight, mvKeysUn;
  std::vector<float> mvuRight, mvDepth;
  DBoW2::BowVector mBowVec;
  DBoW2::FeatureVector mFeatVec;
  cv::Mat mDescriptors, mDescriptorsRight;
  std::vector<MapPoint*> mvpMapPoints;
  std::vector<bool> mvbOutlier;
  cv::Mat mTcw;
  int mnScaleLevels = 0;
  float mfScaleFactor = 0.f, mfLogScaleFactor = 0.f;
  std::vector<float> mvScaleFactors, mvInvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
  static float mnMinX, mnMaxX, mnMinY, mnMaxY;

 private:
  void scale_info() {  // src/Frame.cc:68-74
    mnScaleLevels = mpORBextractorLeft->GetLevels();
    mfScaleFactor = mpORBextractorLeft->GetScaleFactor();
    mfLogScaleFactor = std::log(mfScaleFactor);
    mvScaleFactors = mpORBextractorLeft->GetScaleFactors();
    mvInvScaleFactors = mpORBextractorLeft->GetInverseScaleFactors();
    mvLevelSigma2 = mpORBextractorLeft->GetScaleSigmaSquares();
    mvInvLevelSigma2 = mpORBextractorLeft->GetInverseScaleSigmaSquares();
  }
  static void image_bounds(const cv::Mat& im) {
    mnMinX = 0.0f;
    mnMaxX = (float)im.cols;
    mnMinY = 0.0f;
    mnMaxY = (float)im.rows;
  }
};
}  // namespace ORB_SLAM2
#endif
