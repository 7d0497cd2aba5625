// A minimal C++ host over the drop-in classes, calling them the way the
// reference's Tracking does: Frame construction -> ORBextractor::operator()
// (src/Frame.cc:172-190, 246-252), MonocularInitialization's
// SearchForInitialization (src/Tracking.cc:640-660), Frame::ComputeBoW and
// TrackReferenceKeyFrame's SearchByBoW(KF, F) (src/Tracking.cc:825-842), and
// LoopClosing's SearchByBoW(KF, KF) (src/LoopClosing.cc:246). Results are
// written as raw arrays for tests/test_shim.py to compare with the oracle.
//
//   orbx_shim_driver --version
//   orbx_shim_driver FRAMES.u8 NFRAMES W H VOC.txt|- OUTDIR
//   orbx_shim_driver --scene SCENE.bin OUT.bin   (one ORBmatcher method on a test scene, scene.cc)
//   orbx_shim_driver --stereo LEFT.u8 RIGHT.u8 NPAIRS W H BF OUTDIR
//                                 (stereo Frames, two extraction threads each, + ComputeStereoMatches)
//   orbx_shim_driver --latency MONO.u8 LEFT.u8 RIGHT.u8 NFRAMES W H NCALLS WARM
//                                 (per-call host times of the drop-in path, one JSON line)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"
#include "ORBVocabulary.h"
#include "ORBextractor.h"
#include "ORBmatcher.h"

using namespace ORB_SLAM2;

static void write_file(const std::string& path, const void* p, size_t n) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f || (n && fwrite(p, 1, n, f) != n)) {
    fprintf(stderr, "cannot write %s\n", path.c_str());
    exit(2);
  }
  fclose(f);
}

// MapPoint index in the test's pool (-1 = none), for writing matches out
static std::vector<int> ids(const std::vector<MapPoint*>& v) {
  std::vector<int> r(v.size());
  for (size_t i = 0; i < v.size(); ++i) r[i] = v[i] ? (int)v[i]->mnId : -1;
  return r;
}

int run_scene(const std::string& in, const std::string& out);  // scene.cc
int run_scene_latency(const std::string& in, int ncalls, int warm);  // scene.cc

// The stereo Frame constructor (src/Frame.cc:60-128) over NPAIRS stereo
// pairs: two extractors, Frame::ExtractStereo (or, ORBX_STEREO_THREADS=1, left
// and right extraction on two std::threads as the reference's :77-80, then
// ComputeStereoMatches); writes each
// pair's left / right keypoints, mvuRight and mvDepth.
static int run_stereo(const char* left, const char* right, int npairs, int W, int H, float bf,
                      const std::string& out) {
  const size_t plane = (size_t)W * H;
  std::vector<uint8_t> L(plane * npairs), R(plane * npairs);
  for (auto& lr : {std::make_pair(left, &L), std::make_pair(right, &R)}) {
    FILE* f = fopen(lr.first, "rb");
    if (!f || fread(lr.second->data(), 1, lr.second->size(), f) != lr.second->size()) {
      fprintf(stderr, "cannot read %s\n", lr.first);
      return 2;
    }
    fclose(f);
  }
  ORBextractor left_ext(2000, 1.2f, 8, 20, 7, W, H), right_ext(2000, 1.2f, 8, 20, 7, W, H);
  // Frame::fx from K (src/Frame.cc:103-108): the KITTI calibration
  Frame::fx = 718.856f;
  Frame::fy = 718.856f;
  Frame::cx = 607.1928f;
  Frame::cy = 185.2157f;
  Frame::invfx = 1.0f / Frame::fx;
  Frame::invfy = 1.0f / Frame::fy;
  for (int i = 0; i < npairs; ++i) {
    Frame F(cv::Mat(H, W, CV_8U, L.data() + i * plane, W), cv::Mat(H, W, CV_8U, R.data() + i * plane, W), &left_ext,
            &right_ext, nullptr, bf);
    const std::string k = std::to_string(i);
    write_file(out + "/kpL" + k + ".bin", F.mvKeys.data(), F.mvKeys.size() * sizeof(cv::KeyPoint));
    write_file(out + "/descL" + k + ".bin", F.mDescriptors.data, (size_t)F.N * 32);
    write_file(out + "/kpR" + k + ".bin", F.mvKeysRight.data(), F.mvKeysRight.size() * sizeof(cv::KeyPoint));
    write_file(out + "/descR" + k + ".bin", F.mDescriptorsRight.data, F.mvKeysRight.size() * 32);
    write_file(out + "/uright" + k + ".bin", F.mvuRight.data(), F.mvuRight.size() * 4);
    write_file(out + "/depth" + k + ".bin", F.mvDepth.data(), F.mvDepth.size() * 4);
    const float mb = F.mb;
    write_file(out + "/mb.bin", &mb, 4);
  }
  return 0;
}

static bool read_file(const char* path, std::vector<uint8_t>& v) {
  FILE* f = fopen(path, "rb");
  const bool ok = f && fread(v.data(), 1, v.size(), f) == v.size();
  if (f) fclose(f);
  if (!ok) fprintf(stderr, "cannot read %s\n", path);
  return ok;
}

// median / p99 of per-call times (ms) as a JSON object
static std::string stats(std::vector<double> t) {
  std::sort(t.begin(), t.end());
  const double med = t[t.size() / 2], p99 = t[std::min(t.size() - 1, (size_t)(0.99 * (double)t.size()))];
  char buf[128];
  snprintf(buf, sizeof buf, "{\"median\": %.4f, \"p99\": %.4f, \"calls\": %zu}", med, p99, t.size());
  return buf;
}

// The per-frame cost of the drop-in classes as Tracking pays it (bench.py's
// shim_latency leg): NCALLS timed calls after WARM untimed ones, cycling over
// NFRAMES images, each call timed on the host clock around
//   orbx_extract        the C-ABI call alone (its own handle, host buffers)
//   operator()          ORBextractor::operator() (src/Frame.cc:246-252), with
//                       and without the pinned host pyramid (ORBX_HOST_PYRAMID)
//   stereo Frame        the stereo constructor (src/Frame.cc:60-128): its drop-in
//                       body (Frame::ExtractStereo, one device round trip) and the
//                       reference's structure (left and right operator() on two
//                       std::threads + ComputeStereoMatches, ORBX_STEREO_THREADS=1)
// Prints one JSON object.
static int run_latency(const char* mono, const char* left, const char* right, int nfr, int W, int H, int ncalls,
                       int warm) {
  const size_t plane = (size_t)W * H;
  std::vector<uint8_t> M(plane * nfr), Lp(plane * nfr), Rp(plane * nfr);
  if (!read_file(mono, M) || !read_file(left, Lp) || !read_file(right, Rp)) return 2;
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); };
  std::string out = "{";
  {
    orbx_config c = {};
    c.nfeatures = 2000;
    c.scale_factor = 1.2f;
    c.nlevels = 8;
    c.ini_th_fast = 20;
    c.min_th_fast = 7;
    c.width = W;
    c.height = H;
    c.max_batch = 1;
    const char* dev = getenv("ORBX_DEVICE");
    c.device = dev ? atoi(dev) : 0;
    orbx_handle h = nullptr;
    if (orbx_create(&c, &h) != ORBX_OK) throw std::runtime_error(orbx_last_error());
    const int cap = orbx_frame_capacity(h);
    std::vector<orbx_kp> kp(cap);
    std::vector<uint8_t> desc((size_t)cap * 32);
    std::vector<double> t;
    for (int i = 0; i < warm + ncalls; ++i) {
      int n = 0;
      const auto t0 = clk::now();
      if (orbx_extract(h, M.data() + (size_t)(i % nfr) * plane, W, H, W, kp.data(), cap, desc.data(), &n) != ORBX_OK)
        throw std::runtime_error(orbx_last_error());
      if (i >= warm) t.push_back(ms_since(t0));
    }
    orbx_destroy(h);
    out += "\"orbx_extract_ms\": " + stats(t);
  }
  for (int hp = 1; hp >= 0; --hp) {
    setenv("ORBX_HOST_PYRAMID", hp ? "1" : "0", 1);
    ORBextractor ext(2000, 1.2f, 8, 20, 7, W, H);
    std::vector<cv::KeyPoint> kps;
    cv::Mat desc;
    std::vector<double> t;
    for (int i = 0; i < warm + ncalls; ++i) {
      cv::Mat im(H, W, CV_8U, M.data() + (size_t)(i % nfr) * plane, W);
      const auto t0 = clk::now();
      ext(im, cv::noArray(), kps, desc);
      if (i >= warm) t.push_back(ms_since(t0));
    }
    out += std::string(", \"operator_ms") + (hp ? "_host_pyramid" : "") + "\": " + stats(t);
  }
  Frame::fx = Frame::fy = 718.856f;
  Frame::cx = 607.1928f;
  Frame::cy = 185.2157f;
  Frame::invfx = Frame::invfy = 1.0f / 718.856f;
  const float bf = 0.54f * 718.856f;
  // the stereo constructor: the drop-in body (one device round trip), with and
  // without the host pyramid, then the reference's two-thread structure
  for (int v = 0; v < 3; ++v) {
    const int hp = v == 1;
    setenv("ORBX_HOST_PYRAMID", hp ? "1" : "0", 1);
    setenv("ORBX_STEREO_THREADS", v == 2 ? "1" : "0", 1);
    ORBextractor le(2000, 1.2f, 8, 20, 7, W, H), re(2000, 1.2f, 8, 20, 7, W, H);
    std::vector<double> t;
    size_t kept = 0;
    for (int i = 0; i < warm + ncalls; ++i) {
      const size_t o = (size_t)(i % nfr) * plane;
      cv::Mat l(H, W, CV_8U, Lp.data() + o, W), r(H, W, CV_8U, Rp.data() + o, W);
      const auto t0 = clk::now();
      Frame F(l, r, &le, &re, nullptr, bf);
      if (i >= warm) {
        t.push_back(ms_since(t0));
        for (float u : F.mvuRight) kept += u >= 0;
      }
    }
    char buf[96];
    snprintf(buf, sizeof buf, "\"stereo_matches_per_frame\": %.1f, ", (double)kept / ncalls);
    const char* key = v == 0 ? "stereo_frame_ms" : v == 1 ? "stereo_frame_ms_host_pyramid" : "stereo_frame_threads_ms";
    out += std::string(", ") + (v == 0 ? buf : "") + "\"" + key + "\": " + stats(t);
  }
  unsetenv("ORBX_STEREO_THREADS");
  {
    // the stereo constructor's parts (no host pyramid): the two extraction
    // threads alone, the two extractions on one thread, ComputeStereoMatches alone
    setenv("ORBX_HOST_PYRAMID", "0", 1);
    ORBextractor le(2000, 1.2f, 8, 20, 7, W, H), re(2000, 1.2f, 8, 20, 7, W, H);
    std::vector<double> t2, t1, tm;
    std::vector<cv::KeyPoint> kl, kr;
    cv::Mat dl, dr;
    for (int i = 0; i < warm + ncalls; ++i) {
      const size_t o = (size_t)(i % nfr) * plane;
      cv::Mat l(H, W, CV_8U, Lp.data() + o, W), r(H, W, CV_8U, Rp.data() + o, W);
      auto t0 = clk::now();
      std::thread a([&] { le(l, cv::noArray(), kl, dl); });
      std::thread b([&] { re(r, cv::noArray(), kr, dr); });
      a.join();
      b.join();
      if (i >= warm) t2.push_back(ms_since(t0));
      t0 = clk::now();
      le(l, cv::noArray(), kl, dl);
      re(r, cv::noArray(), kr, dr);
      if (i >= warm) t1.push_back(ms_since(t0));
      std::vector<float> u(kl.size()), d(kl.size());
      int k = 0;
      t0 = clk::now();
      if (orbm_compute_stereo_matches_last(ORBmatcher::Handle(), le.handle(), re.handle(), 0.54f, bf, u.data(),
                                           d.data(), (int)kl.size(), &k) != ORBX_OK)
        throw std::runtime_error(orbm_last_error());
      if (i >= warm) tm.push_back(ms_since(t0));
    }
    // the two std::threads' own cost (spawn + join with no work), which the
    // reference's stereo constructor pays as well (src/Frame.cc:77-80)
    std::vector<double> ts;
    for (int i = 0; i < warm + ncalls; ++i) {
      const auto t0 = clk::now();
      std::thread a([] {});
      std::thread b([] {});
      a.join();
      b.join();
      if (i >= warm) ts.push_back(ms_since(t0));
    }
    out += ", \"stereo_parts\": {\"thread_spawn_join_ms\": " + stats(ts) +
           ", \"extract_two_threads_ms\": " + stats(t2) +
           ", \"extract_one_thread_ms\": " + stats(t1) + ", \"compute_stereo_matches_ms\": " + stats(tm);
    // ComputeStereoMatches' workgroups per pair (ORBX_STEREO_GROUPS, read per call)
    for (int g : {8, 16, 32, 64}) {
      setenv("ORBX_STEREO_GROUPS", std::to_string(g).c_str(), 1);
      std::vector<double> tg;
      std::vector<float> u(kl.size()), d(kl.size());
      for (int i = 0; i < warm + ncalls; ++i) {
        int k = 0;
        const auto t0 = clk::now();
        if (orbm_compute_stereo_matches_last(ORBmatcher::Handle(), le.handle(), re.handle(), 0.54f, bf, u.data(),
                                             d.data(), (int)kl.size(), &k) != ORBX_OK)
          throw std::runtime_error(orbm_last_error());
        if (i >= warm) tg.push_back(ms_since(t0));
      }
      out += ", \"compute_stereo_matches_g" + std::to_string(g) + "_ms\": " + stats(tg);
    }
    unsetenv("ORBX_STEREO_GROUPS");
    out += "}";
  }
  unsetenv("ORBX_HOST_PYRAMID");
  printf("%s}\n", out.c_str());
  return 0;
}

int main(int argc, char** argv) {
  if (argc == 2 && std::string(argv[1]) == "--version") {
    printf("%s\n", orbx_version());
    return 0;
  }
  try {
    if (argc == 4 && std::string(argv[1]) == "--scene") return run_scene(argv[2], argv[3]);
    if (argc == 5 && std::string(argv[1]) == "--scene-latency") return run_scene_latency(argv[2], atoi(argv[3]), atoi(argv[4]));
    if (argc == 10 && std::string(argv[1]) == "--latency")
      return run_latency(argv[2], argv[3], argv[4], atoi(argv[5]), atoi(argv[6]), atoi(argv[7]), atoi(argv[8]),
                         atoi(argv[9]));
    if (argc == 9 && std::string(argv[1]) == "--stereo")
      return run_stereo(argv[2], argv[3], atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), (float)atof(argv[7]), argv[8]);
  } catch (const std::exception& e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 4;
  }
  if (argc != 7) {
    fprintf(stderr, "usage: %s FRAMES.u8 NFRAMES W H VOC.txt|- OUTDIR\n", argv[0]);
    return 1;
  }
  const std::string out = argv[6];
  const int nfr = atoi(argv[2]), W = atoi(argv[3]), H = atoi(argv[4]);
  std::vector<uint8_t> pix((size_t)nfr * W * H);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(pix.data(), 1, pix.size(), f) != pix.size()) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  fclose(f);
  std::unique_ptr<ORBVocabulary> voc;
  if (std::string(argv[5]) != "-") {
    voc.reset(new ORBVocabulary);
    if (!voc->loadFromTextFile(argv[5])) {
      fprintf(stderr, "vocabulary load failed: %s\n", orbv_last_error());
      return 3;
    }
  }
  try {
    setenv("ORBX_HOST_PYRAMID", "1", 1);  // the test reads mvImagePyramid
    // Tracking's monocular extractors: mpIniORBextractor has 2x nFeatures (src/Tracking.cc:145-150)
    // ORBX_DRIVER_CTOR_WH=0: the ctor gets width/height 0, as Tracking passes
    // them for the reference's mono yamls (Examples/Monocular/KITTI00-02.yaml
    // has no Camera.width/height, src/Tracking.cc:124-133); the scale getters
    // are recorded before the first call
    const char* wh = getenv("ORBX_DRIVER_CTOR_WH");
    const bool zero_wh = wh && wh[0] == '0';
    ORBextractor extractor(2000, 1.2f, 8, 20, 7, zero_wh ? 0 : W, zero_wh ? 0 : H);
    {
      std::vector<float> sc = extractor.GetScaleFactors(), isc = extractor.GetInverseScaleFactors(),
                         s2 = extractor.GetScaleSigmaSquares(), is2 = extractor.GetInverseScaleSigmaSquares();
      sc.insert(sc.end(), isc.begin(), isc.end());
      sc.insert(sc.end(), s2.begin(), s2.end());
      sc.insert(sc.end(), is2.begin(), is2.end());
      write_file(out + "/scales_pre.bin", sc.data(), sc.size() * 4);
    }
    std::vector<Frame> frames;
    for (int i = 0; i < nfr; ++i) {
      cv::Mat im(H, W, CV_8U, pix.data() + (size_t)i * W * H, W);
      frames.emplace_back(im, &extractor, voc.get());
      const Frame& F = frames.back();
      write_file(out + "/kp" + std::to_string(i) + ".bin", F.mvKeys.data(), F.mvKeys.size() * sizeof(cv::KeyPoint));
      write_file(out + "/desc" + std::to_string(i) + ".bin", F.mDescriptors.data, (size_t)F.N * 32);
      // mvImagePyramid of this frame's extraction, every level (read by stereo
      // matching), rows at the level width
      for (size_t l = 0; l < extractor.mvImagePyramid.size(); ++l) {
        const cv::Mat Ll = extractor.mvImagePyramid[l].clone();
        write_file(out + "/pyr" + std::to_string(l) + "_" + std::to_string(i) + ".bin", Ll.data,
                   (size_t)Ll.rows * Ll.step);
      }
    }
    if (nfr >= 2) {
      Frame &F1 = frames[0], &F2 = frames[1];
      // MonocularInitialization: mvbPrevMatched = F1 keypoints (src/Tracking.cc:645-647)
      std::vector<cv::Point2f> prev(F1.mvKeysUn.size());
      for (size_t i = 0; i < prev.size(); ++i) prev[i] = F1.mvKeysUn[i].pt;
      std::vector<int> m12;
      ORBmatcher matcher(0.9f, true);
      const int nm = matcher.SearchForInitialization(F1, F2, prev, m12, 100);
      std::vector<int> rec(1, nm);
      rec.insert(rec.end(), m12.begin(), m12.end());
      write_file(out + "/init.bin", rec.data(), rec.size() * 4);
      write_file(out + "/init_prev.bin", prev.data(), prev.size() * sizeof(cv::Point2f));
      const int d01 = ORBmatcher::DescriptorDistance(F1.mDescriptors.row(0), F2.mDescriptors.row(0));
      write_file(out + "/dist.bin", &d01, 4);
      if (voc) {
        F1.ComputeBoW();
        F2.ComputeBoW();
        // keyframe MapPoints: every 4th feature has none, every 7th is bad
        std::vector<std::unique_ptr<MapPoint>> pool;
        for (Frame* F : {&F1, &F2})
          for (int i = 0; i < F->N; ++i) {
            if (i % 4 == 3) continue;
            pool.emplace_back(new MapPoint(i, i % 7 == 5));
            F->mvpMapPoints[i] = pool.back().get();
          }
        KeyFrame kf1(F1), kf2(F2);
        std::vector<MapPoint*> vpMatches;
        ORBmatcher m07(0.7f, true);  // Tracking::TrackReferenceKeyFrame (src/Tracking.cc:832)
        const int nb = m07.SearchByBoW(&kf1, F2, vpMatches);
        std::vector<int> r(1, nb), id = ids(vpMatches);
        r.insert(r.end(), id.begin(), id.end());
        write_file(out + "/bow_kf_f.bin", r.data(), r.size() * 4);
        ORBmatcher m075(0.75f, true);  // LoopClosing::ComputeSim3 (src/LoopClosing.cc:239)
        std::vector<MapPoint*> vpMatches12;
        const int nkk = m075.SearchByBoW(&kf1, &kf2, vpMatches12);
        std::vector<int> r2(1, nkk), id2 = ids(vpMatches12);
        r2.insert(r2.end(), id2.begin(), id2.end());
        write_file(out + "/bow_kf_kf.bin", r2.data(), r2.size() * 4);
      }
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 4;
  }
  printf("ok %d frames\n", nfr);
  return 0;
}
