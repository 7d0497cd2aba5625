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
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
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

// The stereo Frame constructor (src/Frame.cc:60-128) over NPAIRS stereo
// pairs: two extractors, left and right extraction on two std::threads
// (Frame.h, as the reference's :77-80), ComputeStereoMatches; writes each
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

int main(int argc, char** argv) {
  if (argc == 2 && std::string(argv[1]) == "--version") {
    printf("%s\n", orbx_version());
    return 0;
  }
  try {
    if (argc == 4 && std::string(argv[1]) == "--scene") return run_scene(argv[2], argv[3]);
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
    // Tracking's monocular extractors: mpIniORBextractor has 2x nFeatures (src/Tracking.cc:145-150)
    ORBextractor extractor(2000, 1.2f, 8, 20, 7, W, H);
    std::vector<Frame> frames;
    for (int i = 0; i < nfr; ++i) {
      cv::Mat im(H, W, CV_8U, pix.data() + (size_t)i * W * H, W);
      frames.emplace_back(im, &extractor, voc.get());
      const Frame& F = frames.back();
      write_file(out + "/kp" + std::to_string(i) + ".bin", F.mvKeys.data(), F.mvKeys.size() * sizeof(cv::KeyPoint));
      write_file(out + "/desc" + std::to_string(i) + ".bin", F.mDescriptors.data, (size_t)F.N * 32);
      // mvImagePyramid of this frame's extraction, level 1 (read by stereo matching)
      const cv::Mat& L1 = extractor.mvImagePyramid[1];
      write_file(out + "/pyr1_" + std::to_string(i) + ".bin", L1.data, (size_t)L1.rows * L1.step);
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
