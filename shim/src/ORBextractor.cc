// ORBextractor over liborbx: replaces the reference's src/ORBextractor.cc
// (constructor :496-560, operator() :1538-1548 / CPU branch :1710-1808).
#include "ORBextractor.h"

#include <chrono>
#include <climits>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <stdexcept>
#include <string>

namespace ORB_SLAM2 {

static void orbx_check(int rc) {
  if (rc != ORBX_OK) throw std::runtime_error(std::string("liborbx: ") + orbx_last_error());  // NVXIO_SAFE_CALL
}

static_assert(sizeof(cv::KeyPoint) == sizeof(orbx_kp), "cv::KeyPoint must be layout-identical to orbx_kp");

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST,
                           int width, int height)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST) {
  orbx_config c = {};
  c.nfeatures = _nfeatures;
  c.scale_factor = _scaleFactor;
  c.nlevels = _nlevels;
  c.ini_th_fast = _iniThFAST;
  c.min_th_fast = _minThFAST;
  c.width = width;
  c.height = height;
  // Device and parity modes, read once per extractor (environment table):
  //   ORBX_DEVICE      HIP device (default 0)
  //   ORBX_SCALE_MODE  U = the 1.2^l geometry (default; the reference's own map.yml was
  //                    written with it, tests/test_pins.py) or F = the fork's buildGraph
  //                    override of the scale tables (src/ORBextractor.cc:674-680)
  //   ORBX_PATTERN     fork = bit_pattern_31_ with the fork's entry 96 (default) or upstream
  const char* dev = getenv("ORBX_DEVICE");
  const char* sm = getenv("ORBX_SCALE_MODE");
  const char* pm = getenv("ORBX_PATTERN");
  c.device = dev ? atoi(dev) : 0;
  c.max_batch = 1;
  c.scale_mode = ORBX_SCALE_U;
  if (sm && (sm[0] == 'F' || sm[0] == 'f' || sm[0] == '1')) c.scale_mode = ORBX_SCALE_F;
  else if (sm && !(sm[0] == 'U' || sm[0] == 'u' || sm[0] == '0'))
    throw std::runtime_error(std::string("ORBX_SCALE_MODE must be U or F, not ") + sm);
  c.pattern_mode = ORBX_PATTERN_FORK;
  if (pm && std::string(pm) == "upstream") c.pattern_mode = ORBX_PATTERN_UPSTREAM;
  else if (pm && std::string(pm) != "fork")
    throw std::runtime_error(std::string("ORBX_PATTERN must be fork or upstream, not ") + pm);
  orbx_check(orbx_create(&c, &h_));
  mvScaleFactor.resize(nlevels);
  mvInvScaleFactor.resize(nlevels);
  mvLevelSigma2.resize(nlevels);
  mvInvLevelSigma2.resize(nlevels);
  orbx_check(orbx_get_scales(h_, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                             mvInvLevelSigma2.data()));
  lw_.resize(nlevels);
  lh_.resize(nlevels);
  mnFeaturesPerLevel.resize(nlevels);
  int nl = 0;
  orbx_check(orbx_get_levels_info(h_, &nl, lw_.data(), lh_.data(), mnFeaturesPerLevel.data()));
  cap_ = orbx_frame_capacity(h_);
  // width/height 0 (a mono yaml without Camera.width/height, src/Tracking.cc:124-133):
  // the handle plans on the first image, and operator() re-reads the capacity then
  if (cap_ <= 0 && !(width == 0 && height == 0)) throw std::runtime_error("liborbx: bad frame capacity");
  // ORBX_HOST_PYRAMID=1: mvImagePyramid filled on every call (opt-in: the copy
  // costs ~30 us per call, bench.py shim_latency, and the reference's only
  // reader, ComputeStereoMatches, reads the device pyramids here)
  const char* hp = getenv("ORBX_HOST_PYRAMID");
  host_pyr_ = hp && hp[0] == '1';
  orbx_check(orbx_set_host_pyramid(h_, host_pyr_ ? 1 : 0));
  mvImagePyramid.resize(nlevels);
  // ORBX_TIMING=1: the library records its stage events (orbx_create reads the
  // same variable) and every call's stage times go to `times`
  const char* tm = getenv("ORBX_TIMING");
  timing_ = tm && atoi(tm) != 0;
}

// The reference's destructor (src/ORBextractor.cc:800-820): average host time
// per frame on stdout, the time records appended to times.csv in its layout.
ORBextractor::~ORBextractor() {
  if (nFrame) std::cout << "Avg computed frame ORB: " << ((double)totalTime / nFrame) / 1000000.0 << "ms" << std::endl;
  if (!times.empty()) {
    std::ofstream timesFile;
    timesFile.open("times.csv", std::ios_base::app);
    timesFile << "#Frame;Name Processing function;Level;Time spent (ns);Time spent (ms)" << std::endl;
    for (const times_t& t : times) {
      timesFile << t.frame << ";" << t.name << ";" << t.level << ";" << t.time << ";" << t.time / 1000000.0 << ";"
                << std::endl;
    }
  }
  if (h_) orbx_destroy(h_);
}

// Before a call: outputs sized to the capacity (keypoints and descriptors are
// written straight into them and trimmed to the count, no staging copy); a
// new image size re-plans the handle (the reference accepts any size per
// call): one call with no outputs plans it, then the capacity is known.
void ORBextractor::BeginCall(const cv::Mat& image, std::vector<cv::KeyPoint>& keypoints, cv::OutputArray descriptors) {
  if (image.cols != lw_[0] || image.rows != lh_[0]) {
    int n = 0;
    orbx_check(orbx_extract(h_, image.data, image.cols, image.rows, image.step, nullptr, INT_MAX, nullptr, &n));
    cap_ = orbx_frame_capacity(h_);
    int nl = 0;
    orbx_check(orbx_get_levels_info(h_, &nl, lw_.data(), lh_.data(), mnFeaturesPerLevel.data()));
  }
  keypoints.resize(cap_);
  descriptors.create(cap_, 32, CV_8U);
}

// After a call that left n keypoints: outputs trimmed, mvImagePyramid and the
// time records of the call.
void ORBextractor::EndCall(int n, std::vector<cv::KeyPoint>& keypoints, cv::OutputArray descriptors) {
  cv::Mat& desc = descriptors.getMatRef();
  keypoints.resize(n);
  if (n == 0)
    descriptors.release();  // :1716-1717
  else
    desc = desc.rowRange(0, n);  // _descriptors.create(nkeypoints, 32, CV_8U) :1719
  // mvImagePyramid: headers over the pinned host copy of this call's pyramid
  if (host_pyr_) {
    const uint8_t* lv[16];
    size_t lp[16];
    orbx_check(orbx_get_host_pyramid(h_, lv, lp, 16));
    for (int l = 0; l < nlevels; ++l)
      mvImagePyramid[l] = cv::Mat(lh_[l], lw_[l], CV_8U, const_cast<uint8_t*>(lv[l]), lp[l]);
  }
  if (timing_) {
    // the device stages under the reference's GetTime names; one launch covers
    // every pyramid level, so the level field is -1 (as the VX branch's
    // whole-graph records, :1561-1700)
    std::vector<float> ms;
    std::vector<const char*> names;
    const int n_st = GetStageTimes(ms, names);
    for (int i = 0; i < n_st; ++i) times.push_back(times_t{(int)nFrame, names[i], -1, (long long)(ms[i] * 1e6)});
  }
}

void ORBextractor::operator()(cv::InputArray _image, cv::InputArray /*_mask*/, std::vector<cv::KeyPoint>& _keypoints,
                              cv::OutputArray _descriptors) {
  if (_image.empty()) {  // :1542-1543, no outputs
    // the handle's last extraction becomes an empty one, so ComputeStereoMatches
    // after an empty right image matches nothing (the reference's empty mvKeysRight)
    int n = 0;
    orbx_check(orbx_extract(h_, nullptr, 0, 0, 0, nullptr, 0, nullptr, &n));
    return;
  }
  cv::Mat image = _image.getMat();
  assert(image.type() == CV_8UC1);  // :1546
  const auto start = std::chrono::steady_clock::now();
  {
    GetTime total(this, "Total Time ORB extraction", -1);  // :1548 (recorded only with ORBX_TIMING=1)
    BeginCall(image, _keypoints, _descriptors);
    int n = 0;
    orbx_check(orbx_extract(h_, image.data, image.cols, image.rows, image.step,
                            reinterpret_cast<orbx_kp*>(_keypoints.data()), cap_, _descriptors.getMatRef().data, &n));
    EndCall(n, _keypoints, _descriptors);
  }
  totalTime += std::chrono::duration<long long, std::nano>(std::chrono::steady_clock::now() - start).count();  // :1810-1814
  nFrame++;
}

void ORBextractor::ExtractStereo(ORBextractor& left, ORBextractor& right, const cv::Mat& imLeft, const cv::Mat& imRight,
                                 orbm_handle matcher, float mb, float mbf, std::vector<cv::KeyPoint>& keysLeft,
                                 cv::OutputArray descLeft, std::vector<cv::KeyPoint>& keysRight,
                                 cv::OutputArray descRight, std::vector<float>& uRight, std::vector<float>& depth) {
  auto matcher_check = [](int rc) {
    if (rc != ORBX_OK) throw std::runtime_error(std::string("liborbx: ") + orbm_last_error());
  };
  if (imLeft.empty() || imRight.empty() || imLeft.rows != imRight.rows || imLeft.cols != imRight.cols ||
      &left == &right) {
    // the two operator() calls one after the other, then the matching
    left(imLeft, cv::noArray(), keysLeft, descLeft);
    right(imRight, cv::noArray(), keysRight, descRight);
    uRight.assign(keysLeft.size(), -1.0f);
    depth.assign(keysLeft.size(), -1.0f);
    if (keysLeft.empty()) return;
    int kept = 0;
    matcher_check(orbm_compute_stereo_matches_last(matcher, left.h_, right.h_, mb, mbf, uRight.data(), depth.data(),
                                                   (int)keysLeft.size(), &kept));
    return;
  }
  assert(imLeft.type() == CV_8UC1 && imRight.type() == CV_8UC1);
  const auto start = std::chrono::steady_clock::now();
  {
    // both extractors record the pair's time as their total (ORBX_TIMING=1)
    GetTime totalL(&left, "Total Time ORB extraction", -1), totalR(&right, "Total Time ORB extraction", -1);
    left.BeginCall(imLeft, keysLeft, descLeft);
    right.BeginCall(imRight, keysRight, descRight);
    uRight.assign(left.cap_, -1.0f);
    depth.assign(left.cap_, -1.0f);
    int nL = 0, nR = 0, kept = 0;
    matcher_check(orbm_stereo_frame(matcher, left.h_, right.h_, imLeft.data, imLeft.step, imRight.data, imRight.step,
                                    imLeft.cols, imLeft.rows, mb, mbf, reinterpret_cast<orbx_kp*>(keysLeft.data()),
                                    left.cap_, descLeft.getMatRef().data, &nL,
                                    reinterpret_cast<orbx_kp*>(keysRight.data()), right.cap_,
                                    descRight.getMatRef().data, &nR, uRight.data(), depth.data(), &kept));
    uRight.resize(nL);
    depth.resize(nL);
    left.EndCall(nL, keysLeft, descLeft);
    right.EndCall(nR, keysRight, descRight);
  }
  const long long ns = std::chrono::duration<long long, std::nano>(std::chrono::steady_clock::now() - start).count();
  for (ORBextractor* e : {&left, &right}) {
    e->totalTime += ns;
    e->nFrame++;
  }
}

GetTime::GetTime(std::vector<times_t>& times, int nFrame, std::string name, int level) : o(nullptr), times(times) {
  t.frame = nFrame;
  t.name = name;
  t.level = level;
  start = std::chrono::steady_clock::now();
}

GetTime::GetTime(ORBextractor* o, std::string name, int level) : o(o), times(o->times) {
  t.frame = (int)o->nFrame;
  t.name = name;
  t.level = level;
  start = std::chrono::steady_clock::now();
}

// Records on destruction (src/ORBextractor.cc:1896-1904); an extractor's own
// records only when its timing is on (ORBX_TIMING=1), Tracking's always.
GetTime::~GetTime() {
  if (o && !o->timing_) return;
  t.time = std::chrono::duration<long long, std::nano>(std::chrono::steady_clock::now() - start).count();
  times.push_back(t);
}

int ORBextractor::GetStageTimes(std::vector<float>& ms, std::vector<const char*>& names) {
  ms.assign(16, 0.f);
  names.assign(16, nullptr);
  int n = 0;
  orbx_check(orbx_get_stage_times(h_, ms.data(), names.data(), 16, &n));
  ms.resize(n);
  names.resize(n);
  return n;
}

}  // namespace ORB_SLAM2
