// The slice of ORB_SLAM2::MapPoint (include/MapPoint.h) the matcher shim
// reads and the map mutations Fuse applies: GetWorldPos/GetNormal/
// GetDescriptor, Get{Min,Max}DistanceInvariance, Observations(), isBad(),
// IsInKeyFrame/GetIndexInKeyFrame, AddObservation, Replace and
// ComputeDistinctiveDescriptors (src/MapPoint.cc:80-370), and the tracking
// fields Frame::isInFrustum leaves (mTrackProj*, mbTrackInView, ...). A test
// stand-in with the reference's names; a real build uses the reference's
// MapPoint. Locks and the Map are omitted (one thread, no map).
#ifndef ORBX_SHIM_MAPPOINT_H
#define ORBX_SHIM_MAPPOINT_H
#include <algorithm>
#include <climits>
#include <map>
#include <vector>

#include <opencv2/core/core.hpp>

namespace ORB_SLAM2 {
class KeyFrame;

class MapPoint {
 public:
  explicit MapPoint(long unsigned int id, bool bad = false)
      : mnId(id), mWorldPos(3, 1, CV_32F), mNormalVector(3, 1, CV_32F), mDescriptor(1, 32, CV_8U), mbBad(bad) {
    for (int k = 0; k < 3; ++k) mWorldPos.at<float>(k) = mNormalVector.at<float>(k) = 0.f;
    for (int k = 0; k < 32; ++k) mDescriptor.data[k] = 0;
  }
  cv::Mat GetWorldPos() { return mWorldPos.clone(); }
  cv::Mat GetNormal() { return mNormalVector.clone(); }
  cv::Mat GetDescriptor() { return mDescriptor.clone(); }
  float GetMinDistanceInvariance() { return 0.8f * mfMinDistance; }  // MapPoint.cc:376-382
  float GetMaxDistanceInvariance() { return 1.2f * mfMaxDistance; }  // :384-388
  std::map<KeyFrame*, size_t> GetObservations() { return mObservations; }
  int Observations() { return nObs; }
  bool isBad() { return mbBad; }
  bool IsInKeyFrame(KeyFrame* pKF) { return mObservations.count(pKF) != 0; }
  int GetIndexInKeyFrame(KeyFrame* pKF) {
    auto it = mObservations.find(pKF);
    return it == mObservations.end() ? -1 : (int)it->second;
  }
  MapPoint* GetReplaced() { return mpReplaced; }
  // MapPoint.cc:80-93 (stereo observations count twice)
  void AddObservation(KeyFrame* pKF, size_t idx);
  // MapPoint.cc:140-179: this point's observations move to pMP (or are erased
  // where pMP is already seen), this point turns bad, pMP recomputes its descriptor
  void Replace(MapPoint* pMP);
  // MapPoint.cc:262-320: the observation descriptor with the least median
  // distance to the others (observations in std::map order)
  void ComputeDistinctiveDescriptors();

  long unsigned int mnId;
  // Frame::isInFrustum outputs (src/Frame.cc:277-324), read by SearchByProjection(F, vpMapPoints, th)
  float mTrackProjX = 0.f, mTrackProjY = 0.f, mTrackProjXR = 0.f;
  bool mbTrackInView = false;
  int mnTrackScaleLevel = 0;
  float mTrackViewCos = 0.f;
  // test scene setters
  cv::Mat mWorldPos, mNormalVector, mDescriptor;
  void SetScaleDistances(float minDistance, float maxDistance) {
    mfMinDistance = minDistance;
    mfMaxDistance = maxDistance;
  }
  int nObs = 0;

 protected:
  friend class ORBmatcher;  // the one-line addition a real build makes to include/MapPoint.h
  float mfMinDistance = 0.f, mfMaxDistance = 0.f;

 private:
  std::map<KeyFrame*, size_t> mObservations;
  bool mbBad;
  MapPoint* mpReplaced = nullptr;
};
}  // namespace ORB_SLAM2
#endif
