// The slice of ORB_SLAM2::MapPoint (include/MapPoint.h) the BoW matchers read:
// isBad() (src/ORBmatcher.cc:194-197, 559-560, 589-590). A test stand-in;
// a real build uses the reference's MapPoint.
#ifndef ORBX_SHIM_MAPPOINT_H
#define ORBX_SHIM_MAPPOINT_H
namespace ORB_SLAM2 {
class MapPoint {
 public:
  explicit MapPoint(long unsigned int id, bool bad = false) : mnId(id), mbBad(bad) {}
  bool isBad() const { return mbBad; }
  long unsigned int mnId;

 private:
  bool mbBad;
};
}  // namespace ORB_SLAM2
#endif
