// Source-compatible replacement for the reference's include/ORBmatcher.h
// (:36-110). Every public member is declared as in the reference and defined
// over liborbx in src/ORBmatcher.cc here: DescriptorDistance,
// SearchForInitialization, both SearchByBoW overloads, the four
// SearchByProjection overloads, SearchForTriangulation, SearchBySim3 and both
// Fuse overloads (whose map mutations run in the reference's order on the
// host). Additions, none of which changes a caller: Handle() (the calling
// thread's device workspace, also used by Frame::ComputeStereoMatches) and a
// private record builder that reads MapPoint::mfMinDistance / mfMaxDistance
// (a real build adds `friend class ORBmatcher;` to MapPoint).
#ifndef ORBMATCHER_H
#define ORBMATCHER_H

#include <set>
#include <utility>
#include <vector>

#include <opencv2/core/core.hpp>
#include <opencv2/features2d/features2d.hpp>

#include "orbx_c.h"

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"

namespace ORB_SLAM2 {

class ORBmatcher {
 public:
  ORBmatcher(float nnratio = 0.6, bool checkOri = true);

  // Computes the Hamming distance between two ORB descriptors
  static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b);

  int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3);
  int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono);
  int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                         const float th, const int ORBdist);
  int SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                         std::vector<MapPoint*>& vpMatched, int th);

  int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);
  int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12);

  int SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                              std::vector<int>& vnMatches12, int windowSize = 10);

  int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                             std::vector<std::pair<size_t, size_t> >& vMatchedPairs, const bool bOnlyStereo);
  int SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const float& s12,
                   const cv::Mat& R12, const cv::Mat& t12, const float th);
  int Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th = 3.0);
  int Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
           std::vector<MapPoint*>& vpReplacePoint);

 public:
  static const int TH_LOW;
  static const int TH_HIGH;
  static const int HISTO_LENGTH;

  // liborbx matcher workspace of the calling thread (Tracking, LocalMapping
  // and LoopClosing each run their own); the device is ORBX_DEVICE (default 0)
  static orbm_handle Handle();

 protected:
  float mfNNratio;
  bool mbCheckOrientation;

 private:
  // orbm_map_point_world of a MapPoint (GetWorldPos, GetNormal, mfMinDistance,
  // mfMaxDistance, Observations() > 0) for the pose-projection searches
  static orbm_map_point_world MapPointRecord(MapPoint* pMP, float angle, int octave, bool valid);
};

}  // namespace ORB_SLAM2

#endif
