// Replacement for the reference's include/ORBVocabulary.h
// (typedef DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> ORBVocabulary)
// for the members the hot path calls: loadFromTextFile (System.cc:61-68,
// TemplatedVocabulary.h:1338-1418) and transform(features, BowVector,
// FeatureVector, levelsup) (Frame::ComputeBoW, Frame.cc:394-401;
// TemplatedVocabulary.h:1127-1256), over liborbx's orbv_* entry points.
// The database-side members (score, KeyFrameDatabase) stay DBoW2's.
#ifndef ORBVOCABULARY_H
#define ORBVOCABULARY_H

#include <string>
#include <vector>

#include <opencv2/core/core.hpp>

#include "DBoW2.h"
#include "orbx_c.h"

namespace ORB_SLAM2 {

class ORBVocabulary {
 public:
  ORBVocabulary() = default;
  ~ORBVocabulary();
  ORBVocabulary(const ORBVocabulary&) = delete;
  ORBVocabulary& operator=(const ORBVocabulary&) = delete;

  bool loadFromTextFile(const std::string& filename);
  void transform(const std::vector<cv::Mat>& features, DBoW2::BowVector& v, DBoW2::FeatureVector& fv,
                 int levelsup) const;
  unsigned int size() const;  // number of words
  bool empty() const { return h_ == nullptr; }
  int getBranchingFactor() const;
  int getDepthLevels() const;

 private:
  orbv_handle h_ = nullptr;
};

}  // namespace ORB_SLAM2

#endif
