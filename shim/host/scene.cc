// Scene mode of the shim host: rebuilds Frames / KeyFrames / MapPoints from a
// binary scene file (written by tests/shimscene.py), calls ONE ORBmatcher
// method the way the reference's threads call it, and writes the resulting
// pointer state as MapPoint indices for tests/test_shim.py to compare with
// the oracle:
//   op 1 SearchByProjection(F, vpMapPoints, th)           Tracking.cc:1277
//   op 2 SearchByProjection(CurrentFrame, LastFrame, ...)  Tracking.cc:962, 968
//   op 3 SearchByProjection(CurrentFrame, pKF, found, ...) Tracking.cc:1540, 1554
//   op 4 SearchByProjection(pKF, Scw, vpPoints, vpMatched) LoopClosing.cc:414
//   op 5 Fuse(pKF, vpMapPoints, th)                       LocalMapping.cc:525, 550
//   op 6 Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)     LoopClosing.cc:654
//   op 7 SearchBySim3(pKF1, pKF2, vpMatches12, ...)        LoopClosing.cc:362
//   op 8 SearchForTriangulation(pKF1, pKF2, F12, ...)      LocalMapping.cc:301
//   op 9 SearchByBoW(pKF, F, vpMapPointMatches)            Tracking.cc:842, 1465
// --scene-latency: the same scene rebuilt per call, only the method call on
// the host clock (median / p99 over the calls after the warm ones).
// Scene file: records of [u32 name length][name][u32 dtype 0 u8 / 1 i32 /
// 2 f32][u32 count][count elements].
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"
#include "ORBmatcher.h"

using namespace ORB_SLAM2;

namespace {
struct Rec {
  int dtype = 0;
  std::vector<char> bytes;
  template <typename T> const T* p() const { return reinterpret_cast<const T*>(bytes.data()); }
  template <typename T> size_t n() const { return bytes.size() / sizeof(T); }
};

struct Scene {
  std::map<std::string, Rec> r;
  bool has(const std::string& k) const { return r.count(k) != 0; }
  const Rec& at(const std::string& k) const {
    auto it = r.find(k);
    if (it == r.end()) throw std::runtime_error("scene lacks " + k);
    return it->second;
  }
  template <typename T> std::vector<T> vec(const std::string& k) const {
    const Rec& x = at(k);
    return std::vector<T>(x.p<T>(), x.p<T>() + x.n<T>());
  }
  float f(const std::string& k) const { return at(k).p<float>()[0]; }
  int i(const std::string& k) const { return at(k).p<int>()[0]; }
};

Scene load(const std::string& path) {
  Scene s;
  FILE* fp = fopen(path.c_str(), "rb");
  if (!fp) throw std::runtime_error("cannot read " + path);
  for (;;) {
    uint32_t len = 0;
    if (fread(&len, 4, 1, fp) != 1) break;
    std::string name(len, '\0');
    uint32_t dt = 0, cnt = 0;
    if (fread(&name[0], 1, len, fp) != len || fread(&dt, 4, 1, fp) != 1 || fread(&cnt, 4, 1, fp) != 1)
      throw std::runtime_error("truncated scene");
    Rec rec;
    rec.dtype = (int)dt;
    rec.bytes.resize((size_t)cnt * (dt == 0 ? 1 : 4));
    if (!rec.bytes.empty() && fread(rec.bytes.data(), 1, rec.bytes.size(), fp) != rec.bytes.size())
      throw std::runtime_error("truncated scene");
    s.r[name] = std::move(rec);
  }
  fclose(fp);
  return s;
}

// the scene's MapPoints (mp_*), indexed by their row
std::vector<std::unique_ptr<MapPoint>> map_points(const Scene& s) {
  std::vector<std::unique_ptr<MapPoint>> pool;
  if (!s.has("mp_desc")) return pool;
  const int M = (int)(s.at("mp_desc").n<uint8_t>() / 32);
  const auto desc = s.vec<uint8_t>("mp_desc");
  for (int i = 0; i < M; ++i) {
    const bool bad = s.has("mp_bad") && s.at("mp_bad").p<uint8_t>()[i];
    pool.emplace_back(new MapPoint((unsigned long)i, bad));
    MapPoint* p = pool.back().get();
    for (int k = 0; k < 32; ++k) p->mDescriptor.data[k] = desc[(size_t)i * 32 + k];
    if (s.has("mp_pos"))
      for (int k = 0; k < 3; ++k) p->mWorldPos.at<float>(k) = s.at("mp_pos").p<float>()[3 * i + k];
    if (s.has("mp_normal"))
      for (int k = 0; k < 3; ++k) p->mNormalVector.at<float>(k) = s.at("mp_normal").p<float>()[3 * i + k];
    if (s.has("mp_dist")) p->SetScaleDistances(s.at("mp_dist").p<float>()[2 * i], s.at("mp_dist").p<float>()[2 * i + 1]);
    if (s.has("mp_track")) {
      const float* t = s.at("mp_track").p<float>() + 4 * i;
      p->mTrackProjX = t[0];
      p->mTrackProjY = t[1];
      p->mTrackProjXR = t[2];
      p->mTrackViewCos = t[3];
      p->mnTrackScaleLevel = s.at("mp_level").p<int>()[i];
      p->mbTrackInView = s.at("mp_inview").p<uint8_t>()[i] != 0;
    }
  }
  return pool;
}

MapPoint* ptr_of(const std::vector<std::unique_ptr<MapPoint>>& pool, int i) { return i >= 0 ? pool.at(i).get() : nullptr; }
int id_of(const MapPoint* p) { return p ? (int)p->mnId : -1; }

cv::Mat pose4(const Scene& s, const std::string& k) {
  const auto v = s.vec<float>(k);  // 12 (3x4) or 16 (4x4) row-major
  cv::Mat T(4, 4, CV_32F);
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) T.at<float>(r, c) = r < 3 ? v[4 * r + c] : (r == c ? 1.f : 0.f);
  return T;
}

// common fields of side X ("A" or "B"): keypoints, descriptors, uright, scale tables
template <typename F>
void fill_common(const Scene& s, const std::string& X, F& f) {
  const Rec& k = s.at(X + "_kps");
  const int n = (int)(k.bytes.size() / sizeof(cv::KeyPoint));
  f.mvKeys.resize(n);
  if (n) memcpy(f.mvKeys.data(), k.bytes.data(), k.bytes.size());
  f.mvKeysUn = f.mvKeys;
  f.N = n;
  f.mDescriptors.create(std::max(n, 1), 32, CV_8U);
  f.mDescriptors.rows = n;
  if (n) memcpy(f.mDescriptors.data, s.at(X + "_desc").bytes.data(), (size_t)n * 32);
  if (s.has(X + "_uright")) f.mvuRight = s.vec<float>(X + "_uright");
  else f.mvuRight.clear();
  f.mvScaleFactors = s.vec<float>(X + "_scale");
  f.mnScaleLevels = (int)f.mvScaleFactors.size();
  f.mfScaleFactor = s.has(X + "_sf") ? s.f(X + "_sf") : 1.2f;
  f.mfLogScaleFactor = std::log(f.mfScaleFactor);
  if (s.has(X + "_sigma2")) f.mvLevelSigma2 = s.vec<float>(X + "_sigma2");
  if (s.has(X + "_invsigma2")) f.mvInvLevelSigma2 = s.vec<float>(X + "_invsigma2");
}

std::unique_ptr<Frame> frame(const Scene& s, const std::string& X, const std::vector<std::unique_ptr<MapPoint>>& pool) {
  std::unique_ptr<Frame> F(new Frame());
  fill_common(s, X, *F);
  const auto cam = s.vec<float>(X + "_cam");  // fx fy cx cy mb mbf
  Frame::fx = cam[0];
  Frame::fy = cam[1];
  Frame::cx = cam[2];
  Frame::cy = cam[3];
  Frame::invfx = 1.0f / cam[0];
  Frame::invfy = 1.0f / cam[1];
  F->mb = cam[4];
  F->mbf = cam[5];
  const auto b = s.vec<float>(X + "_bounds");
  Frame::mnMinX = b[0];
  Frame::mnMaxX = b[1];
  Frame::mnMinY = b[2];
  Frame::mnMaxY = b[3];
  if (s.has(X + "_T")) F->mTcw = pose4(s, X + "_T");
  F->mvpMapPoints.assign(F->N, nullptr);
  if (s.has(X + "_mps")) {
    const auto m = s.vec<int>(X + "_mps");
    for (int i = 0; i < F->N; ++i) F->mvpMapPoints[i] = ptr_of(pool, m[i]);
  }
  if (s.has(X + "_fv_nodes")) {
    const auto nodes = s.vec<int>(X + "_fv_nodes");
    const auto off = s.vec<int>(X + "_fv_off");
    const auto idx = s.vec<int>(X + "_fv_idx");
    for (size_t j = 0; j < nodes.size(); ++j)
      F->mFeatVec[(unsigned)nodes[j]] = std::vector<unsigned>(idx.begin() + off[j], idx.begin() + off[j + 1]);
  }
  F->mvbOutlier.assign(F->N, false);
  if (s.has(X + "_outlier")) {
    const auto o = s.vec<uint8_t>(X + "_outlier");
    for (int i = 0; i < F->N; ++i) F->mvbOutlier[i] = o[i] != 0;
  }
  return F;
}

std::unique_ptr<KeyFrame> keyframe(const Scene& s, const std::string& X,
                                   const std::vector<std::unique_ptr<MapPoint>>& pool) {
  std::unique_ptr<KeyFrame> K(new KeyFrame());
  fill_common(s, X, *K);
  if (K->mvuRight.empty()) K->mvuRight.assign(K->N, -1.0f);
  const auto cam = s.vec<float>(X + "_cam");
  K->fx = cam[0];
  K->fy = cam[1];
  K->cx = cam[2];
  K->cy = cam[3];
  K->invfx = 1.0f / cam[0];
  K->invfy = 1.0f / cam[1];
  K->mb = cam[4];
  K->mbf = cam[5];
  const auto b = s.vec<float>(X + "_bounds");
  K->mnMinX = (int)b[0];
  K->mnMaxX = (int)b[1];
  K->mnMinY = (int)b[2];
  K->mnMaxY = (int)b[3];
  if (s.has(X + "_T")) K->SetPose(pose4(s, X + "_T"));
  K->mvpMapPoints.assign(K->N, nullptr);
  if (s.has(X + "_mps")) {
    const auto m = s.vec<int>(X + "_mps");
    for (int i = 0; i < K->N; ++i) K->mvpMapPoints[i] = ptr_of(pool, m[i]);
  }
  if (s.has(X + "_fv_nodes")) {
    const auto nodes = s.vec<int>(X + "_fv_nodes");
    const auto off = s.vec<int>(X + "_fv_off");
    const auto idx = s.vec<int>(X + "_fv_idx");
    for (size_t j = 0; j < nodes.size(); ++j)
      K->mFeatVec[(unsigned)nodes[j]] = std::vector<unsigned>(idx.begin() + off[j], idx.begin() + off[j + 1]);
  }
  return K;
}

// observations: the points each keyframe holds (AddObservation, src/KeyFrame.cc
// holds the reverse link), then Observations() as the scene sets it (mp_nobs)
void observe(KeyFrame* K, const Scene& s, const std::vector<std::unique_ptr<MapPoint>>& pool) {
  for (int i = 0; i < K->N; ++i)
    if (K->mvpMapPoints[i]) K->mvpMapPoints[i]->AddObservation(K, i);
}
void set_nobs(const Scene& s, const std::vector<std::unique_ptr<MapPoint>>& pool) {
  if (!s.has("mp_nobs")) return;
  const auto n = s.vec<int>("mp_nobs");
  for (size_t i = 0; i < pool.size(); ++i) pool[i]->nObs = n[i];
}

std::vector<MapPoint*> pointers(const Scene& s, const std::string& k,
                                const std::vector<std::unique_ptr<MapPoint>>& pool) {
  std::vector<MapPoint*> v;
  for (int i : s.vec<int>(k)) v.push_back(ptr_of(pool, i));
  return v;
}

void write_ints(const std::string& path, const std::vector<int>& v) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f || (!v.empty() && fwrite(v.data(), 4, v.size(), f) != v.size())) throw std::runtime_error("cannot write " + path);
  fclose(f);
}
}  // namespace

// One method call on the scene's state (built here), its results as int32
// arrays (see each op) and its host time in *ms (the call alone).
static void run_op(const Scene& s, std::vector<int>& res, double* ms) {
  const int op = s.i("op");
  auto pool = map_points(s);
  ORBmatcher matcher(s.has("nnratio") ? s.f("nnratio") : 0.6f, s.has("check_ori") ? s.i("check_ori") != 0 : true);
  using clk = std::chrono::steady_clock;
  clk::time_point t0;
  auto tic = [&]() { t0 = clk::now(); };
  auto toc = [&]() { *ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count(); };
  switch (op) {
    case 1: {  // -> [n, F.mvpMapPoints...]
      auto F = frame(s, "A", pool);
      set_nobs(s, pool);
      const std::vector<MapPoint*> vp = pointers(s, "vp", pool);
      tic();
      const int n = matcher.SearchByProjection(*F, vp, s.f("th"));
      toc();
      res.push_back(n);
      for (MapPoint* p : F->mvpMapPoints) res.push_back(id_of(p));
      break;
    }
    case 2: {  // -> [n, CurrentFrame.mvpMapPoints...]
      auto Last = frame(s, "B", pool);
      auto Cur = frame(s, "A", pool);  // A last: the Frame statics are the current frame's
      set_nobs(s, pool);
      tic();
      const int n = matcher.SearchByProjection(*Cur, *Last, s.f("th"), s.i("mono") != 0);
      toc();
      res.push_back(n);
      for (MapPoint* p : Cur->mvpMapPoints) res.push_back(id_of(p));
      break;
    }
    case 3: {  // -> [n, CurrentFrame.mvpMapPoints...]
      auto K = keyframe(s, "B", pool);
      auto Cur = frame(s, "A", pool);
      set_nobs(s, pool);
      std::set<MapPoint*> found;
      for (MapPoint* p : pointers(s, "already", pool)) found.insert(p);
      tic();
      const int n = matcher.SearchByProjection(*Cur, K.get(), found, s.f("th"), s.i("orb_dist"));
      toc();
      res.push_back(n);
      for (MapPoint* p : Cur->mvpMapPoints) res.push_back(id_of(p));
      break;
    }
    case 4: {  // -> [n, vpMatched...]
      auto K = keyframe(s, "A", pool);
      set_nobs(s, pool);
      std::vector<MapPoint*> matched = pointers(s, "matched", pool);
      const cv::Mat Scw = pose4(s, "Scw");
      const std::vector<MapPoint*> vp = pointers(s, "vp", pool);
      tic();
      const int n = matcher.SearchByProjection(K.get(), Scw, vp, matched, s.i("thi"));
      toc();
      res.push_back(n);
      for (MapPoint* p : matched) res.push_back(id_of(p));
      break;
    }
    case 5: {  // -> [nFused, pKF->mvpMapPoints..., per point: bad, Observations()]
      auto K = keyframe(s, "A", pool);
      observe(K.get(), s, pool);
      set_nobs(s, pool);
      const std::vector<MapPoint*> vp = pointers(s, "vp", pool);
      tic();
      const int n = matcher.Fuse(K.get(), vp, s.f("th"));
      toc();
      res.push_back(n);
      for (MapPoint* p : K->mvpMapPoints) res.push_back(id_of(p));
      for (auto& p : pool) res.push_back(p->isBad() ? 1 : 0);
      for (auto& p : pool) res.push_back(p->Observations());
      break;
    }
    case 6: {  // -> [nFused, pKF->mvpMapPoints..., vpReplacePoint...]
      auto K = keyframe(s, "A", pool);
      observe(K.get(), s, pool);
      set_nobs(s, pool);
      const std::vector<MapPoint*> vp = pointers(s, "vp", pool);
      std::vector<MapPoint*> replace(vp.size(), nullptr);
      const cv::Mat Scw = pose4(s, "Scw");
      tic();
      const int n = matcher.Fuse(K.get(), Scw, vp, s.f("th"), replace);
      toc();
      res.push_back(n);
      for (MapPoint* p : K->mvpMapPoints) res.push_back(id_of(p));
      for (MapPoint* p : replace) res.push_back(id_of(p));
      break;
    }
    case 7: {  // -> [nFound, vpMatches12...]
      auto K1 = keyframe(s, "A", pool);
      auto K2 = keyframe(s, "B", pool);
      observe(K1.get(), s, pool);
      observe(K2.get(), s, pool);
      set_nobs(s, pool);
      std::vector<MapPoint*> m12 = pointers(s, "matched", pool);
      const auto R = s.vec<float>("R12"), t = s.vec<float>("t12");
      cv::Mat R12(3, 3, CV_32F), t12(3, 1, CV_32F);
      for (int k = 0; k < 9; ++k) R12.at<float>(k / 3, k % 3) = R[k];
      for (int k = 0; k < 3; ++k) t12.at<float>(k) = t[k];
      const float s12 = s.f("s12");
      tic();
      const int n = matcher.SearchBySim3(K1.get(), K2.get(), m12, s12, R12, t12, s.f("th"));
      toc();
      res.push_back(n);
      for (MapPoint* p : m12) res.push_back(id_of(p));
      break;
    }
    case 8: {  // -> [n, (idx1, idx2)...]
      auto K1 = keyframe(s, "A", pool);
      auto K2 = keyframe(s, "B", pool);
      const auto Fv = s.vec<float>("F12");
      cv::Mat F12(3, 3, CV_32F);
      for (int k = 0; k < 9; ++k) F12.at<float>(k / 3, k % 3) = Fv[k];
      std::vector<std::pair<size_t, size_t>> pairs;
      tic();
      const int n = matcher.SearchForTriangulation(K1.get(), K2.get(), F12, pairs, s.i("only_stereo") != 0);
      toc();
      res.push_back(n);
      for (auto& pr : pairs) {
        res.push_back((int)pr.first);
        res.push_back((int)pr.second);
      }
      break;
    }
    case 9: {  // -> [n, vpMapPointMatches...]
      auto K = keyframe(s, "B", pool);
      auto F = frame(s, "A", pool);
      std::vector<MapPoint*> matches;
      tic();
      const int n = matcher.SearchByBoW(K.get(), *F, matches);
      toc();
      res.push_back(n);
      for (MapPoint* p : matches) res.push_back(id_of(p));
      break;
    }
    default:
      throw std::runtime_error("unknown scene op " + std::to_string(op));
  }
}

// Returns 0 on success; results in OUT as int32 arrays (see each op).
int run_scene(const std::string& in, const std::string& out) {
  const Scene s = load(in);
  std::vector<int> res;
  double ms = 0;
  run_op(s, res, &ms);
  write_ints(out, res);
  return 0;
}

// Per-call host time of the scene's method (the state rebuilt before every
// call, outside the clock): one JSON object on stdout.
int run_scene_latency(const std::string& in, int ncalls, int warm) {
  const Scene s = load(in);
  std::vector<double> t;
  int n = 0;
  for (int i = 0; i < warm + ncalls; ++i) {
    std::vector<int> res;
    double ms = 0;
    run_op(s, res, &ms);
    if (i >= warm) t.push_back(ms);
    n = res.empty() ? 0 : res[0];
  }
  std::sort(t.begin(), t.end());
  const double med = t[t.size() / 2], p99 = t[std::min(t.size() - 1, (size_t)(0.99 * (double)t.size()))];
  printf("{\"op\": %d, \"calls\": %d, \"median_ms\": %.4f, \"p99_ms\": %.4f, \"matches\": %d}\n", s.i("op"), ncalls,
         med, p99, n);
  return 0;
}
