// ORBmatcher over liborbx: every method of the reference's src/ORBmatcher.cc
// marshals Frame / KeyFrame / MapPoint fields into the C-ABI's plain arrays
// (include/orbx_c.h) and turns the returned indices back into the
// reference's side effects (MapPoint pointers stored in mvpMapPoints /
// vpMatched / vpMatches12, vMatchedPairs, Fuse's map mutations in point order).
#include "ORBmatcher.h"

#include <cstdlib>
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
orbm_handle ORBmatcher::Handle() {
  struct Holder {
    orbm_handle h = nullptr;
    ~Holder() {
      if (h) orbm_destroy(h);
    }
  };
  thread_local Holder holder;
  if (!holder.h) {
    const char* dev = getenv("ORBX_DEVICE");
    orbm_check(orbm_create(dev ? atoi(dev) : 0, 1, 8192, &holder.h));
  }
  return holder.h;
}

ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  return orbm_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
}

namespace {
const orbx_kp* kps(const std::vector<cv::KeyPoint>& v) { return reinterpret_cast<const orbx_kp*>(v.data()); }

orbm_grid_bounds frame_bounds() { return {Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY}; }
orbm_grid_bounds kf_bounds(const KeyFrame* pKF) {
  return {(float)pKF->mnMinX, (float)pKF->mnMaxX, (float)pKF->mnMinY, (float)pKF->mnMaxY};
}

// fx, fy, cx, cy, mb, mbf and rows 0..2 of a 4x4 (or 3x4) float pose
orbm_camera camera(float fx, float fy, float cx, float cy, float mb, float mbf, const cv::Mat& T) {
  orbm_camera c{fx, fy, cx, cy, mb, mbf, {}};
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 4; ++k) c.Tcw[4 * r + k] = T.at<float>(r, k);
  return c;
}

void pose_rows(const cv::Mat& T, float out[12]) {
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 4; ++k) out[4 * r + k] = T.at<float>(r, k);
}

// DBoW2::FeatureVector (std::map<NodeId, vector<uint>>) as CSR, in map order
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

// descriptors of the points in record order (zero rows for NULL pointers)
cv::Mat point_descriptors(const std::vector<MapPoint*>& v) {
  cv::Mat D(std::max<int>((int)v.size(), 1), 32, CV_8U);
  for (size_t i = 0; i < v.size(); ++i) {
    uint8_t* row = D.ptr<uint8_t>((int)i);
    if (v[i]) {
      const cv::Mat d = v[i]->GetDescriptor();
      for (int k = 0; k < 32; ++k) row[k] = d.ptr<uint8_t>()[k];
    } else {
      for (int k = 0; k < 32; ++k) row[k] = 0;
    }
  }
  return D;
}

// mvuRight of a frame or keyframe (NULL for a monocular one)
const float* uright(const std::vector<float>& u, int n) { return (int)u.size() >= n && n > 0 ? u.data() : nullptr; }
}  // namespace

orbm_map_point_world ORBmatcher::MapPointRecord(MapPoint* pMP, float angle, int octave, bool valid) {
  orbm_map_point_world r{};
  if (!pMP) return r;
  const cv::Mat X = pMP->GetWorldPos(), Pn = pMP->GetNormal();
  for (int k = 0; k < 3; ++k) {
    r.pos[k] = X.at<float>(k);
    r.normal[k] = Pn.at<float>(k);
  }
  r.min_distance = pMP->mfMinDistance;
  r.max_distance = pMP->mfMaxDistance;
  r.angle = angle;
  r.octave = octave;
  r.valid = valid;
  r.obs_positive = pMP->Observations() > 0;
  return r;
}

// ------------------------------------------------------------------- Tracking
int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize) {
  const int n1 = (int)F1.mvKeysUn.size(), n2 = (int)F2.mvKeysUn.size();
  vnMatches12.assign(n1, -1);
  if ((int)vbPrevMatched.size() < n1) throw std::runtime_error("vbPrevMatched shorter than F1.mvKeysUn");
  int nmatches = 0;
  // cv::Point2f is two floats: vbPrevMatched is updated in place (:515-517)
  orbm_check(orbm_search_for_initialization(Handle(), kps(F1.mvKeysUn), F1.mDescriptors.ptr<uint8_t>(), n1,
                                            kps(F2.mvKeysUn), F2.mDescriptors.ptr<uint8_t>(), n2, frame_bounds(),
                                            reinterpret_cast<float*>(vbPrevMatched.data()), windowSize, mfNNratio,
                                            mbCheckOrientation, vnMatches12.data(), &nmatches));
  return nmatches;
}

// SearchByProjection(F, vpMapPoints, th) (:45-118): Tracking::SearchLocalPoints (Tracking.cc:1277)
int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th) {
  const int M = (int)vpMapPoints.size();
  std::vector<orbm_map_point_proj> mp(std::max(M, 1));
  for (int j = 0; j < M; ++j) {
    MapPoint* p = vpMapPoints[j];
    mp[j] = {p->mTrackProjX, p->mTrackProjY, p->mTrackProjXR, p->mTrackViewCos, p->mnTrackScaleLevel,
             (uint8_t)(p->mbTrackInView && !p->isBad()), (uint8_t)(p->Observations() > 0), {0, 0}};
  }
  const cv::Mat D = point_descriptors(vpMapPoints);
  std::vector<uint8_t> blocked(std::max(F.N, 1));
  for (int i = 0; i < F.N; ++i) blocked[i] = F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0;
  std::vector<int> out(std::max(F.N, 1), -1);
  int n = 0;
  orbm_check(orbm_search_by_projection(Handle(), kps(F.mvKeysUn), F.mDescriptors.ptr<uint8_t>(), F.N,
                                       uright(F.mvuRight, F.N), frame_bounds(), F.mvScaleFactors.data(),
                                       (int)F.mvScaleFactors.size(), blocked.data(), mp.data(), D.data, M, th,
                                       mfNNratio, out.data(), &n));
  for (int i = 0; i < F.N; ++i)
    if (out[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[out[i]];
  return n;
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono) (:1328-1470): Tracking::TrackWithMotionModel (Tracking.cc:962, 968)
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
  const int NL = LastFrame.N, NC = CurrentFrame.N;
  std::vector<orbm_map_point_world> mp(std::max(NL, 1));
  for (int i = 0; i < NL; ++i) {
    MapPoint* p = LastFrame.mvpMapPoints[i];
    mp[i] = MapPointRecord(p, LastFrame.mvKeysUn[i].angle, LastFrame.mvKeys[i].octave,
                           p && !LastFrame.mvbOutlier[i]);
  }
  const cv::Mat D = point_descriptors(LastFrame.mvpMapPoints);
  std::vector<uint8_t> blocked(std::max(NC, 1));
  for (int i = 0; i < NC; ++i)
    blocked[i] = CurrentFrame.mvpMapPoints[i] && CurrentFrame.mvpMapPoints[i]->Observations() > 0;
  const orbm_camera cur = camera(Frame::fx, Frame::fy, Frame::cx, Frame::cy, CurrentFrame.mb, CurrentFrame.mbf,
                                 CurrentFrame.mTcw);
  float Tlw[12];
  pose_rows(LastFrame.mTcw, Tlw);
  std::vector<int> out(std::max(NC, 1), -1);
  int n = 0;
  orbm_check(orbm_search_by_projection_last_frame(
      Handle(), kps(CurrentFrame.mvKeysUn), CurrentFrame.mDescriptors.ptr<uint8_t>(), NC,
      uright(CurrentFrame.mvuRight, NC), frame_bounds(), CurrentFrame.mvScaleFactors.data(),
      (int)CurrentFrame.mvScaleFactors.size(), blocked.data(), &cur, Tlw, mp.data(), D.data, NL, th, bMono,
      mbCheckOrientation, out.data(), &n));
  for (int i = 0; i < NC; ++i) {
    if (out[i] >= 0) CurrentFrame.mvpMapPoints[i] = LastFrame.mvpMapPoints[out[i]];
    else if (out[i] == -2) CurrentFrame.mvpMapPoints[i] = static_cast<MapPoint*>(nullptr);  // rotation check
  }
  return n;
}

// SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (:1472-1599): Tracking::Relocalization (Tracking.cc:1540, 1554)
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                                   const float th, const int ORBdist) {
  const std::vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
  const int M = (int)vpMPs.size(), NC = CurrentFrame.N;
  std::vector<orbm_map_point_world> mp(std::max(M, 1));
  for (int i = 0; i < M; ++i) {
    MapPoint* p = vpMPs[i];
    mp[i] = MapPointRecord(p, pKF->mvKeysUn[i].angle, 0, p && !p->isBad() && !sAlreadyFound.count(p));
  }
  const cv::Mat D = point_descriptors(vpMPs);
  std::vector<uint8_t> has_mp(std::max(NC, 1));
  for (int i = 0; i < NC; ++i) has_mp[i] = CurrentFrame.mvpMapPoints[i] != nullptr;
  const orbm_camera cur = camera(Frame::fx, Frame::fy, Frame::cx, Frame::cy, CurrentFrame.mb, CurrentFrame.mbf,
                                 CurrentFrame.mTcw);
  std::vector<int> out(std::max(NC, 1), -1);
  int n = 0;
  orbm_check(orbm_search_by_projection_keyframe(
      Handle(), kps(CurrentFrame.mvKeysUn), CurrentFrame.mDescriptors.ptr<uint8_t>(), NC, frame_bounds(),
      CurrentFrame.mvScaleFactors.data(), (int)CurrentFrame.mvScaleFactors.size(), CurrentFrame.mfScaleFactor,
      has_mp.data(), &cur, mp.data(), D.data, M, th, ORBdist, mbCheckOrientation, out.data(), &n));
  for (int i = 0; i < NC; ++i) {
    if (out[i] >= 0) CurrentFrame.mvpMapPoints[i] = vpMPs[out[i]];
    else if (out[i] == -2) CurrentFrame.mvpMapPoints[i] = static_cast<MapPoint*>(nullptr);
  }
  return n;
}

// SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (:290-403): LoopClosing::ComputeSim3 (LoopClosing.cc:414)
int ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                                   std::vector<MapPoint*>& vpMatched, int th) {
  const int M = (int)vpPoints.size(), N = pKF->N;
  const std::set<MapPoint*> already = [&] {  // spAlreadyFound (:306-307)
    std::set<MapPoint*> s(vpMatched.begin(), vpMatched.end());
    s.erase(static_cast<MapPoint*>(nullptr));
    return s;
  }();
  std::vector<orbm_map_point_world> mp(std::max(M, 1));
  for (int i = 0; i < M; ++i) {
    MapPoint* p = vpPoints[i];
    mp[i] = MapPointRecord(p, 0.f, 0, !p->isBad() && !already.count(p));
  }
  const cv::Mat D = point_descriptors(vpPoints);
  std::vector<int> matched(std::max(N, 1), -1);
  for (int i = 0; i < N; ++i) matched[i] = vpMatched[i] ? 0 : -1;
  const orbm_camera kf = camera(pKF->fx, pKF->fy, pKF->cx, pKF->cy, 0.f, 0.f, Scw);
  std::vector<int> out(std::max(N, 1), -1);
  int n = 0;
  orbm_check(orbm_search_by_projection_sim3(Handle(), kps(pKF->mvKeysUn), pKF->mDescriptors.ptr<uint8_t>(), N,
                                            kf_bounds(pKF), pKF->mvScaleFactors.data(),
                                            (int)pKF->mvScaleFactors.size(), pKF->mfScaleFactor, &kf, mp.data(),
                                            D.data, M, th, matched.data(), out.data(), &n));
  for (int i = 0; i < N; ++i)
    if (out[i] >= 0) vpMatched[i] = vpPoints[out[i]];
  return n;
}

// -------------------------------------------------------------------- BoW
int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
  const std::vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
  vpMapPointMatches = std::vector<MapPoint*>(F.N, static_cast<MapPoint*>(nullptr));
  const FeatVecCSR fvA(pKF->mFeatVec), fvB(F.mFeatVec);
  const std::vector<uint8_t> mpA = good_map_points(vpMapPointsKF);
  const std::vector<float> angA = angles(pKF->mvKeysUn), angB = angles(F.mvKeys);  // (:236)
  std::vector<int> out(std::max(F.N, 1), -1);
  int n = 0;
  orbm_check(orbm_search_by_bow(Handle(), pKF->mDescriptors.ptr<uint8_t>(), angA.data(), mpA.data(),
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
  std::vector<int> out(std::max<size_t>(vpMapPoints1.size(), 1), -1);
  int n = 0;
  orbm_check(orbm_search_by_bow(Handle(), pKF1->mDescriptors.ptr<uint8_t>(), ang1.data(), mp1.data(),
                                (int)vpMapPoints1.size(), fv1.view(), pKF2->mDescriptors.ptr<uint8_t>(), ang2.data(),
                                mp2.data(), (int)vpMapPoints2.size(), fv2.view(), mfNNratio, mbCheckOrientation,
                                /*kf_vs_kf=*/1, out.data(), &n));
  for (size_t i = 0; i < vpMapPoints1.size(); ++i) vpMatches12[i] = out[i] >= 0 ? vpMapPoints2[out[i]] : nullptr;
  return n;
}

// --------------------------------------------------------------- LocalMapping
// SearchForTriangulation (:657-823): LocalMapping::CreateNewMapPoints (LocalMapping.cc:301)
int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                                       std::vector<std::pair<size_t, size_t> >& vMatchedPairs,
                                       const bool bOnlyStereo) {
  const int N1 = pKF1->N, N2 = pKF2->N;
  auto has_mp = [](KeyFrame* K) {
    std::vector<uint8_t> h(std::max(K->N, 1));
    for (int i = 0; i < K->N; ++i) h[i] = K->GetMapPoint(i) != nullptr;
    return h;
  };
  auto ur = [](KeyFrame* K) {
    std::vector<float> u(K->mvuRight);
    u.resize(std::max(K->N, 1), -1.0f);
    return u;
  };
  const std::vector<uint8_t> h1 = has_mp(pKF1), h2 = has_mp(pKF2);
  const std::vector<float> u1 = ur(pKF1), u2 = ur(pKF2);
  const FeatVecCSR fv1(pKF1->mFeatVec), fv2(pKF2->mFeatVec);
  const cv::Mat Cw = pKF1->GetCameraCenter();
  const float cw1[3] = {Cw.at<float>(0), Cw.at<float>(1), Cw.at<float>(2)};
  float T2w[12];
  pose_rows(pKF2->GetPose(), T2w);
  const float cam2[4] = {pKF2->fx, pKF2->fy, pKF2->cx, pKF2->cy};
  float F[9];
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k) F[3 * r + k] = F12.at<float>(r, k);
  std::vector<int> m12(std::max(N1, 1), -1);
  int n = 0;
  orbm_check(orbm_search_for_triangulation(
      Handle(), kps(pKF1->mvKeysUn), pKF1->mDescriptors.ptr<uint8_t>(), u1.data(), h1.data(), N1, fv1.view(),
      kps(pKF2->mvKeysUn), pKF2->mDescriptors.ptr<uint8_t>(), u2.data(), h2.data(), N2, fv2.view(), cw1, T2w, cam2,
      pKF2->mvScaleFactors.data(), pKF2->mvLevelSigma2.data(), (int)pKF2->mvScaleFactors.size(), F, bOnlyStereo,
      mbCheckOrientation, m12.data(), &n));
  vMatchedPairs.clear();
  vMatchedPairs.reserve(n);
  for (int i = 0; i < N1; ++i)
    if (m12[i] >= 0) vMatchedPairs.push_back(std::make_pair((size_t)i, (size_t)m12[i]));
  return n;
}

// Fuse(pKF, vpMapPoints, th) (:825-975): LocalMapping::SearchInNeighbors (LocalMapping.cc:525, 550).
// The device matches every point against pKF as it is at call time; the
// reference's tail (:951-971) then runs in point order. A point that turned
// bad or became part of pKF since the call (an earlier fusion of the same
// pointer) is skipped as the reference's loop head (:846-850) skips it; every
// fusion leaves its survivor in pKF, so no later point's match can change.
int ORBmatcher::Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th) {
  const int M = (int)vpMapPoints.size(), N = pKF->N;
  std::vector<orbm_map_point_world> mp(std::max(M, 1));
  for (int i = 0; i < M; ++i) {
    MapPoint* p = vpMapPoints[i];
    mp[i] = MapPointRecord(p, 0.f, 0, p && !p->isBad() && !p->IsInKeyFrame(pKF));
  }
  const cv::Mat D = point_descriptors(vpMapPoints);
  const orbm_camera kf = camera(pKF->fx, pKF->fy, pKF->cx, pKF->cy, 0.f, pKF->mbf, pKF->GetPose());
  std::vector<int> out(std::max(M, 1), -1);
  int n = 0;
  orbm_check(orbm_fuse(Handle(), kps(pKF->mvKeysUn), pKF->mDescriptors.ptr<uint8_t>(), N, uright(pKF->mvuRight, N),
                       kf_bounds(pKF), pKF->mvScaleFactors.data(), pKF->mvInvLevelSigma2.data(),
                       (int)pKF->mvScaleFactors.size(), pKF->mfScaleFactor, &kf, mp.data(), D.data, M, th,
                       out.data(), &n));
  int nFused = 0;
  for (int i = 0; i < M; ++i) {
    MapPoint* pMP = vpMapPoints[i];
    if (!pMP || out[i] < 0 || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
    const int bestIdx = out[i];
    MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);
    if (pMPinKF) {
      if (!pMPinKF->isBad()) {
        if (pMPinKF->Observations() > pMP->Observations())
          pMP->Replace(pMPinKF);
        else
          pMPinKF->Replace(pMP);
      }
    } else {
      pMP->AddObservation(pKF, bestIdx);
      pKF->AddMapPoint(pMP, bestIdx);
    }
    nFused++;
  }
  return nFused;
}

// Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:977-1100): LoopClosing::SearchAndFuse (LoopClosing.cc:654)
int ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
                     std::vector<MapPoint*>& vpReplacePoint) {
  const int M = (int)vpPoints.size(), N = pKF->N;
  const std::set<MapPoint*> spAlreadyFound = pKF->GetMapPoints();
  std::vector<orbm_map_point_world> mp(std::max(M, 1));
  for (int i = 0; i < M; ++i) {
    MapPoint* p = vpPoints[i];
    mp[i] = MapPointRecord(p, 0.f, 0, !p->isBad() && !spAlreadyFound.count(p));
  }
  const cv::Mat D = point_descriptors(vpPoints);
  const orbm_camera kf = camera(pKF->fx, pKF->fy, pKF->cx, pKF->cy, 0.f, 0.f, Scw);
  std::vector<int> out(std::max(M, 1), -1);
  int n = 0;
  orbm_check(orbm_fuse_sim3(Handle(), kps(pKF->mvKeysUn), pKF->mDescriptors.ptr<uint8_t>(), N, kf_bounds(pKF),
                            pKF->mvScaleFactors.data(), (int)pKF->mvScaleFactors.size(), pKF->mfScaleFactor, &kf,
                            mp.data(), D.data, M, th, out.data(), &n));
  int nFused = 0;
  for (int i = 0; i < M; ++i) {  // the reference's tail (:1081-1096), in point order
    if (out[i] < 0) continue;
    MapPoint* pMP = vpPoints[i];
    MapPoint* pMPinKF = pKF->GetMapPoint(out[i]);
    if (pMPinKF) {
      if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
    } else {
      pMP->AddObservation(pKF, out[i]);
      pKF->AddMapPoint(pMP, out[i]);
    }
    nFused++;
  }
  return nFused;
}

// --------------------------------------------------------------- LoopClosing
// SearchBySim3 (:1102-1326): LoopClosing::ComputeSim3 (LoopClosing.cc:362)
int ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const float& s12,
                             const cv::Mat& R12, const cv::Mat& t12, const float th) {
  const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
  const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
  const int N1 = (int)vpMapPoints1.size(), N2 = (int)vpMapPoints2.size();
  std::vector<bool> vbAlreadyMatched1(N1, false), vbAlreadyMatched2(N2, false);  // (:1129-1142)
  for (int i = 0; i < N1; i++) {
    MapPoint* pMP = vpMatches12[i];
    if (pMP) {
      vbAlreadyMatched1[i] = true;
      const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
      if (idx2 >= 0 && idx2 < N2) vbAlreadyMatched2[idx2] = true;
    }
  }
  std::vector<orbm_map_point_world> r1(std::max(N1, 1)), r2(std::max(N2, 1));
  for (int i = 0; i < N1; ++i) {
    MapPoint* p = vpMapPoints1[i];
    r1[i] = MapPointRecord(p, 0.f, 0, p && !vbAlreadyMatched1[i] && !p->isBad());
  }
  for (int i = 0; i < N2; ++i) {
    MapPoint* p = vpMapPoints2[i];
    r2[i] = MapPointRecord(p, 0.f, 0, p && !vbAlreadyMatched2[i] && !p->isBad());
  }
  const cv::Mat D1 = point_descriptors(vpMapPoints1), D2 = point_descriptors(vpMapPoints2);
  float T1w[12], T2w[12], R[9], t[3];
  pose_rows(pKF1->GetPose(), T1w);
  pose_rows(pKF2->GetPose(), T2w);
  for (int r = 0; r < 3; ++r) {
    for (int k = 0; k < 3; ++k) R[3 * r + k] = R12.at<float>(r, k);
    t[r] = t12.at<float>(r);
  }
  const orbm_camera cam1 = camera(pKF1->fx, pKF1->fy, pKF1->cx, pKF1->cy, 0.f, 0.f, pKF1->GetPose());
  std::vector<int> m12(std::max(N1, 1), -1);
  int nFound = 0;
  orbm_check(orbm_search_by_sim3(Handle(), kps(pKF1->mvKeysUn), pKF1->mDescriptors.ptr<uint8_t>(), N1,
                                 kf_bounds(pKF1), T1w, r1.data(), D1.data, kps(pKF2->mvKeysUn),
                                 pKF2->mDescriptors.ptr<uint8_t>(), N2, kf_bounds(pKF2), T2w, r2.data(), D2.data,
                                 pKF2->mvScaleFactors.data(), (int)pKF2->mvScaleFactors.size(), pKF2->mfScaleFactor,
                                 &cam1, s12, R, t, th, m12.data(), &nFound));
  for (int i = 0; i < N1; ++i)
    if (m12[i] >= 0) vpMatches12[i] = vpMapPoints2[m12[i]];
  return nFound;
}

}  // namespace ORB_SLAM2
