// The slice of ORB_SLAM2::KeyFrame (include/KeyFrame.h) the matcher shim
// reads and Fuse mutates: camera (fx .. mb, KeyFrame.h:161), keypoints,
// mvuRight, descriptors, mFeatVec, scale tables and image bounds
// (KeyFrame.h:165-192), the pose (GetPose / GetRotation / GetTranslation /
// GetCameraCenter, src/KeyFrame.cc:77-122) and the MapPoint matches
// (GetMapPointMatches / GetMapPoints / GetMapPoint / AddMapPoint /
// ReplaceMapPointMatch / EraseMapPointMatch, :190-260). A test stand-in with
// the reference's names, built from a Frame as KeyFrame::KeyFrame(Frame&, ...)
// copies it (src/KeyFrame.cc:40-75) or field by field by a test scene.
#ifndef ORBX_SHIM_KEYFRAME_H
#define ORBX_SHIM_KEYFRAME_H
#include <set>
#include <vector>

#include "Frame.h"
#include "MapPoint.h"

namespace ORB_SLAM2 {
class KeyFrame {
 public:
  KeyFrame() : Tcw(4, 4, CV_32F) { set_identity(); }
  explicit KeyFrame(const Frame& F)
      : fx(F.fx), fy(F.fy), cx(F.cx), cy(F.cy), invfx(F.invfx), invfy(F.invfy), mbf(F.mbf), mb(F.mb), N(F.N),
        mvKeys(F.mvKeys), mvKeysUn(F.mvKeysUn), mvuRight(F.mvuRight), mDescriptors(F.mDescriptors.clone()),
        mFeatVec(F.mFeatVec), mnScaleLevels(F.mnScaleLevels), mfScaleFactor(F.mfScaleFactor),
        mfLogScaleFactor(F.mfLogScaleFactor), mvScaleFactors(F.mvScaleFactors), mvLevelSigma2(F.mvLevelSigma2),
        mvInvLevelSigma2(F.mvInvLevelSigma2), mnMinX((int)F.mnMinX), mnMinY((int)F.mnMinY), mnMaxX((int)F.mnMaxX),
        mnMaxY((int)F.mnMaxY), Tcw(4, 4, CV_32F), mvpMapPoints(F.mvpMapPoints) {
    if (mvuRight.empty()) mvuRight.assign(N, -1.0f);
    if (!F.mTcw.empty()) SetPose(F.mTcw);
    else set_identity();
  }

  void SetPose(const cv::Mat& T) { T.copyTo(Tcw); }
  cv::Mat GetPose() { return Tcw.clone(); }
  cv::Mat GetRotation() { return Tcw.rowRange(0, 3).colRange(0, 3).clone(); }
  cv::Mat GetTranslation() { return Tcw.rowRange(0, 3).col(3).clone(); }
  // Ow = -Rcw^T tcw (KeyFrame::SetPose, src/KeyFrame.cc:77-92; cv::Mat gemm
  // accumulates in double)
  cv::Mat GetCameraCenter() {
    cv::Mat Ow(3, 1, CV_32F);
    for (int i = 0; i < 3; ++i) {
      double s = 0;
      for (int k = 0; k < 3; ++k) s += (double)Tcw.at<float>(k, i) * (double)Tcw.at<float>(k, 3);
      Ow.at<float>(i) = (float)-s;
    }
    return Ow;
  }

  std::vector<MapPoint*> GetMapPointMatches() { return mvpMapPoints; }
  std::set<MapPoint*> GetMapPoints() {
    std::set<MapPoint*> s;
    for (MapPoint* p : mvpMapPoints)
      if (p && !p->isBad()) s.insert(p);
    return s;
  }
  MapPoint* GetMapPoint(const size_t& idx) { return mvpMapPoints[idx]; }
  void AddMapPoint(MapPoint* pMP, const size_t& idx) { mvpMapPoints[idx] = pMP; }
  void ReplaceMapPointMatch(const size_t& idx, MapPoint* pMP) { mvpMapPoints[idx] = pMP; }
  void EraseMapPointMatch(const size_t& idx) { mvpMapPoints[idx] = static_cast<MapPoint*>(nullptr); }
  bool isBad() { return false; }

  float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0, mbf = 0, mb = 0;
  int N = 0;
  std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
  std::vector<float> mvuRight;
  cv::Mat mDescriptors;
  DBoW2::FeatureVector mFeatVec;
  int mnScaleLevels = 8;
  float mfScaleFactor = 1.2f, mfLogScaleFactor = 0.f;
  std::vector<float> mvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
  int mnMinX = 0, mnMinY = 0, mnMaxX = 0, mnMaxY = 0;

 private:
  void set_identity() {
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) Tcw.at<float>(r, c) = r == c ? 1.f : 0.f;
  }
  cv::Mat Tcw;

 public:
  std::vector<MapPoint*> mvpMapPoints;
};

// MapPoint members that need KeyFrame (src/MapPoint.cc:80-93, 140-179, 262-320)
inline void MapPoint::AddObservation(KeyFrame* pKF, size_t idx) {
  if (mObservations.count(pKF)) return;
  mObservations[pKF] = idx;
  nObs += (!pKF->mvuRight.empty() && pKF->mvuRight[idx] >= 0) ? 2 : 1;
}

inline void MapPoint::Replace(MapPoint* pMP) {
  if (pMP->mnId == mnId) return;
  std::map<KeyFrame*, size_t> obs = mObservations;
  mObservations.clear();
  mbBad = true;
  mpReplaced = pMP;
  for (auto& o : obs) {
    if (!pMP->IsInKeyFrame(o.first)) {
      o.first->ReplaceMapPointMatch(o.second, pMP);
      pMP->AddObservation(o.first, o.second);
    } else {
      o.first->EraseMapPointMatch(o.second);
    }
  }
  pMP->ComputeDistinctiveDescriptors();
}

inline int shim_descriptor_distance(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int k = 0; k < 32; ++k) d += __builtin_popcount((unsigned)(a[k] ^ b[k]));
  return d;
}

inline void MapPoint::ComputeDistinctiveDescriptors() {
  if (mbBad) return;
  std::vector<const uint8_t*> v;
  for (auto& o : mObservations)
    if (!o.first->isBad()) v.push_back(o.first->mDescriptors.ptr<uint8_t>((int)o.second));
  if (v.empty()) return;
  const size_t N = v.size();
  std::vector<std::vector<int>> D(N, std::vector<int>(N, 0));
  for (size_t i = 0; i < N; ++i)
    for (size_t j = i + 1; j < N; ++j) D[i][j] = D[j][i] = shim_descriptor_distance(v[i], v[j]);
  int best = INT_MAX;
  size_t bestIdx = 0;
  for (size_t i = 0; i < N; ++i) {
    std::vector<int> d = D[i];
    std::sort(d.begin(), d.end());
    const int median = d[(size_t)(0.5 * (N - 1))];
    if (median < best) {
      best = median;
      bestIdx = i;
    }
  }
  for (int k = 0; k < 32; ++k) mDescriptor.data[k] = v[bestIdx][k];
}
}  // namespace ORB_SLAM2
#endif
