// ORBmatcher over liborbx: DescriptorDistance (src/ORBmatcher.cc:1647-1663),
// SearchForInitialization (:405-520) and SearchByBoW (:159-288, :522-655).
// Frame / KeyFrame fields are flattened into the C-ABI's plain arrays and the
// returned feature indices are turned back into MapPoint pointers.
#include "ORBmatcher.h"

#include <stdexcept>
#include <string>

namespace ORB_SLAM2 {

const int ORBmatcher::TH_HIGH = 100;
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;

static void orbm_check(int rc) {
  if (rc != ORBX_OK) throw std::runtime_error(std::string("liborbx: ") + orbm_last_error());
}

// One device workspace per thread: Tracking, LocalMapping and LoopClosing
// each use their own ORBmatcher objects concurrently.
static orbm_handle matcher_handle() {
  struct Holder {
    orbm_handle h = nullptr;
    ~Holder() {
      if (h) orbm_destroy(h);
    }
  };
  thread_local Holder holder;
  if (!holder.h) orbm_check(orbm_create(0, 1, 8192, &holder.h));
  return holder.h;
}

ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  return orbm_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
}

int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize) {
  const int n1 = (int)F1.mvKeysUn.size(), n2 = (int)F2.mvKeysUn.size();
  vnMatches12.assign(n1, -1);
  if ((int)vbPrevMatched.size() < n1) throw std::runtime_error("vbPrevMatched shorter than F1.mvKeysUn");
  orbm_grid_bounds b = {Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY};
  int nmatches = 0;
  // cv::Point2f is two floats: vbPrevMatched is updated in place (:515-517)
  orbm_check(orbm_search_for_initialization(
      matcher_handle(), reinterpret_cast<const orbx_kp*>(F1.mvKeysUn.data()), F1.mDescriptors.ptr<uint8_t>(), n1,
      reinterpret_cast<const orbx_kp*>(F2.mvKeysUn.data()), F2.mDescriptors.ptr<uint8_t>(), n2, b,
      reinterpret_cast<float*>(vbPrevMatched.data()), windowSize, mfNNratio, mbCheckOrientation,
      vnMatches12.data(), &nmatches));
  return nmatches;
}

namespace {
// DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>) as CSR, in map order
struct FeatVecCSR {
  std::vector<uint32_t> nodes;
  std::vector<int> off{0}, idx;
  explicit FeatVecCSR(const DBoW2::FeatureVector& fv) {
    nodes.reserve(fv.size());
    for (const auto& kv : fv) {
      nodes.push_back(kv.first);
      idx.insert(idx.end(), kv.second.begin(), kv.second.end());
      off.push_back((int)idx.size());
    }
  }
  orbm_feature_vector view() const { return {nodes.data(), off.data(), idx.data(), (int)nodes.size()}; }
};

std::vector<uint8_t> good_map_points(const std::vector<MapPoint*>& v) {  // pMP && !pMP->isBad()
  std::vector<uint8_t> m(v.size());
  for (size_t i = 0; i < v.size(); ++i) m[i] = v[i] && !v[i]->isBad();
  return m;
}

std::vector<float> angles(const std::vector<cv::KeyPoint>& k) {
  std::vector<float> a(k.size());
  for (size_t i = 0; i < k.size(); ++i) a[i] = k[i].angle;
  return a;
}
}  // namespace

int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
  const std::vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
  vpMapPointMatches = std::vector<MapPoint*>(F.N, static_cast<MapPoint*>(nullptr));
  const FeatVecCSR fvA(pKF->mFeatVec), fvB(F.mFeatVec);
  const std::vector<uint8_t> mpA = good_map_points(vpMapPointsKF);
  const std::vector<float> angA = angles(pKF->mvKeysUn), angB = angles(F.mvKeys);  // (:236)
  std::vector<int> out(F.N, -1);
  int n = 0;
  orbm_check(orbm_search_by_bow(matcher_handle(), pKF->mDescriptors.ptr<uint8_t>(), angA.data(), mpA.data(),
                                (int)vpMapPointsKF.size(), fvA.view(), F.mDescriptors.ptr<uint8_t>(), angB.data(),
                                nullptr, F.N, fvB.view(), mfNNratio, mbCheckOrientation, /*kf_vs_kf=*/0, out.data(),
                                &n));
  for (int j = 0; j < F.N; ++j) vpMapPointMatches[j] = out[j] >= 0 ? vpMapPointsKF[out[j]] : nullptr;
  return n;
}

int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
  const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
  const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
  vpMatches12 = std::vector<MapPoint*>(vpMapPoints1.size(), static_cast<MapPoint*>(nullptr));
  const FeatVecCSR fv1(pKF1->mFeatVec), fv2(pKF2->mFeatVec);
  const std::vector<uint8_t> mp1 = good_map_points(vpMapPoints1), mp2 = good_map_points(vpMapPoints2);
  const std::vector<float> ang1 = angles(pKF1->mvKeysUn), ang2 = angles(pKF2->mvKeysUn);  // (:608)
  std::vector<int> out(vpMapPoints1.size(), -1);
  int n = 0;
  orbm_check(orbm_search_by_bow(matcher_handle(), pKF1->mDescriptors.ptr<uint8_t>(), ang1.data(), mp1.data(),
                                (int)vpMapPoints1.size(), fv1.view(), pKF2->mDescriptors.ptr<uint8_t>(), ang2.data(),
                                mp2.data(), (int)vpMapPoints2.size(), fv2.view(), mfNNratio, mbCheckOrientation,
                                /*kf_vs_kf=*/1, out.data(), &n));
  for (size_t i = 0; i < out.size(); ++i) vpMatches12[i] = out[i] >= 0 ? vpMapPoints2[out[i]] : nullptr;
  return n;
}

}  // namespace ORB_SLAM2
