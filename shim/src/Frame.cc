// Frame's statics (src/Frame.cc:31-34 defines them for the reference) and the
// drop-in body of Frame::ComputeStereoMatches (src/Frame.cc:465-639): the
// keypoints, descriptors and pyramids of the two extractors' last calls are
// matched where they lie on the device (orbm_compute_stereo_matches_last),
// which fills mvuRight and mvDepth (-1 where a keypoint has no stereo match).
#include "Frame.h"

#include <stdexcept>
#include <string>

#include "ORBmatcher.h"

namespace ORB_SLAM2 {
float Frame::fx, Frame::fy, Frame::cx, Frame::cy, Frame::invfx, Frame::invfy;
float Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY;

void Frame::ComputeStereoMatches() {
  mvuRight = std::vector<float>(N, -1.0f);
  mvDepth = std::vector<float>(N, -1.0f);
  if (N == 0) return;
  int kept = 0;
  // the stereo constructor calls this right after its two extractions
  // (src/Frame.cc:77-89): the keypoints and descriptors are read where those
  // calls left them on the device, only mvuRight / mvDepth come back
  const int rc = orbm_compute_stereo_matches_last(ORBmatcher::Handle(), mpORBextractorLeft->handle(),
                                                  mpORBextractorRight->handle(), mb, mbf, mvuRight.data(),
                                                  mvDepth.data(), N, &kept);
  if (rc != ORBX_OK) throw std::runtime_error(std::string("liborbx: ") + orbm_last_error());
}

// The stereo constructor's extraction and matching steps (src/Frame.cc:77-89:
// ExtractORB on threadLeft / threadRight, N = mvKeys.size(), then
// ComputeStereoMatches) as one call with one device round trip: both
// extraction chains are issued from this thread and run concurrently on the
// device, the stereo kernel follows them there, and the keypoints,
// descriptors, mvuRight and mvDepth come back together (orbm_stereo_frame).
// Same results as those steps.
void Frame::ExtractStereo(const cv::Mat& imLeft, const cv::Mat& imRight) {
  ORBextractor::ExtractStereo(*mpORBextractorLeft, *mpORBextractorRight, imLeft, imRight, ORBmatcher::Handle(), mb, mbf,
                              mvKeys, mDescriptors, mvKeysRight, mDescriptorsRight, mvuRight, mvDepth);
  N = (int)mvKeys.size();
}
}  // namespace ORB_SLAM2
