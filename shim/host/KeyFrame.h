// The slice of ORB_SLAM2::KeyFrame (include/KeyFrame.h) the BoW matchers
// read: mvKeysUn, mDescriptors, mFeatVec (KeyFrame.h:168-175) and
// GetMapPointMatches() (:91). A test stand-in built from a Frame, as
// KeyFrame::KeyFrame(Frame&, ...) copies these fields (src/KeyFrame.cc:29-45).
#ifndef ORBX_SHIM_KEYFRAME_H
#define ORBX_SHIM_KEYFRAME_H
#include <vector>

#include "Frame.h"
#include "MapPoint.h"

namespace ORB_SLAM2 {
class KeyFrame {
 public:
  explicit KeyFrame(const Frame& F)
      : N(F.N), mvKeysUn(F.mvKeysUn), mDescriptors(F.mDescriptors.clone()), mFeatVec(F.mFeatVec),
        mvpMapPoints(F.mvpMapPoints) {}
  std::vector<MapPoint*> GetMapPointMatches() { return mvpMapPoints; }
  const int N;
  const std::vector<cv::KeyPoint> mvKeysUn;
  const cv::Mat mDescriptors;
  DBoW2::FeatureVector mFeatVec;
  std::vector<MapPoint*> mvpMapPoints;
};
}  // namespace ORB_SLAM2
#endif
