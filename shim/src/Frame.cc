// Frame's statics (src/Frame.cc:31-34 defines them for the reference) and the
// drop-in body of Frame::ComputeStereoMatches (src/Frame.cc:465-639): the
// keypoints of both images and the two extractors' pyramids of this frame's
// extraction go to orbm_compute_stereo_matches, which fills mvuRight and
// mvDepth (-1 where a keypoint has no stereo match).
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
  const int rc = orbm_compute_stereo_matches(
      ORBmatcher::Handle(), mpORBextractorLeft->handle(), mpORBextractorRight->handle(),
      reinterpret_cast<const orbx_kp*>(mvKeys.data()), mDescriptors.ptr<uint8_t>(), N,
      reinterpret_cast<const orbx_kp*>(mvKeysRight.data()), mDescriptorsRight.ptr<uint8_t>(),
      (int)mvKeysRight.size(), mb, mbf, mvuRight.data(), mvDepth.data(), &kept);
  if (rc != ORBX_OK) throw std::runtime_error(std::string("liborbx: ") + orbm_last_error());
}
}  // namespace ORB_SLAM2
