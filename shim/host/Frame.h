// The slice of ORB_SLAM2::Frame (include/Frame.h) that the extractor and
// matcher shims read, with the reference's member names: N, mvKeys,
// mvKeysUn, mDescriptors, mBowVec, mFeatVec, mpORBvocabulary and the static
// image bounds mnMinX..mnMaxY (Frame.h:132-186). ComputeBoW is
// src/Frame.cc:394-401. A test stand-in; a real build uses the reference's
// Frame, unchanged.
#ifndef ORBX_SHIM_FRAME_H
#define ORBX_SHIM_FRAME_H
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
    (*mpORBextractorLeft)(imGray, cv::noArray(), mvKeys, mDescriptors);
    N = (int)mvKeys.size();
    mvKeysUn = mvKeys;
    mvpMapPoints.assign(N, static_cast<MapPoint*>(nullptr));
    mnMinX = 0.0f;
    mnMaxX = (float)imGray.cols;
    mnMinY = 0.0f;
    mnMaxY = (float)imGray.rows;
  }
  void ComputeBoW() {
    if (mBowVec.empty()) {
      std::vector<cv::Mat> vCurrentDesc;  // Converter::toDescriptorVector
      vCurrentDesc.reserve(mDescriptors.rows);
      for (int j = 0; j < mDescriptors.rows; j++) vCurrentDesc.push_back(mDescriptors.row(j));
      mpORBvocabulary->transform(vCurrentDesc, mBowVec, mFeatVec, 4);
    }
  }

  ORBVocabulary* mpORBvocabulary = nullptr;
  ORBextractor* mpORBextractorLeft = nullptr;
  int N = 0;
  std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
  DBoW2::BowVector mBowVec;
  DBoW2::FeatureVector mFeatVec;
  cv::Mat mDescriptors;
  std::vector<MapPoint*> mvpMapPoints;
  static float mnMinX, mnMaxX, mnMinY, mnMaxY;
};
}  // namespace ORB_SLAM2
#endif
