// ORBVocabulary over liborbx's orbv_*: DBoW2 TemplatedVocabulary's
// loadFromTextFile (TemplatedVocabulary.h:1338-1418) and transform with
// FeatureVector (:1127-1256), as Frame::ComputeBoW calls it.
#include "ORBVocabulary.h"

#include <cstring>
#include <stdexcept>
#include <string>

namespace ORB_SLAM2 {

ORBVocabulary::~ORBVocabulary() {
  if (h_) orbv_destroy(h_);
}

bool ORBVocabulary::loadFromTextFile(const std::string& filename) {
  if (h_) orbv_destroy(h_), h_ = nullptr;
  return orbv_load_text(filename.c_str(), /*device=*/0, &h_) == ORBX_OK;
}

void ORBVocabulary::transform(const std::vector<cv::Mat>& features, DBoW2::BowVector& v, DBoW2::FeatureVector& fv,
                              int levelsup) const {
  v.clear();
  fv.clear();
  if (!h_) throw std::runtime_error("ORBVocabulary: empty vocabulary");
  const int n = (int)features.size();
  if (n == 0) return;  // (:1140-1143)
  std::vector<uint8_t> desc((size_t)n * 32);
  for (int i = 0; i < n; ++i) memcpy(&desc[(size_t)i * 32], features[i].ptr<uint8_t>(0), 32);
  std::vector<uint32_t> words(n), nodes(n);
  std::vector<double> values(n);
  std::vector<int> off(n + 1), idx(n);
  int bn = 0, fn = 0;
  if (orbv_transform(h_, desc.data(), n, levelsup, words.data(), values.data(), &bn, nodes.data(), off.data(),
                     idx.data(), &fn, nullptr, nullptr, nullptr) != ORBX_OK)
    throw std::runtime_error(std::string("liborbx: ") + orbv_last_error());
  for (int i = 0; i < bn; ++i) v.emplace_hint(v.end(), words[i], values[i]);
  for (int k = 0; k < fn; ++k)
    fv.emplace_hint(fv.end(), nodes[k], std::vector<unsigned int>(idx.begin() + off[k], idx.begin() + off[k + 1]));
}

unsigned int ORBVocabulary::size() const {
  int k, L, s, w, nn, nw = 0;
  if (!h_ || orbv_info(h_, &k, &L, &s, &w, &nn, &nw) != ORBX_OK) return 0;
  return (unsigned)nw;
}

int ORBVocabulary::getBranchingFactor() const {
  int k = 0, L, s, w, nn, nw;
  if (h_) orbv_info(h_, &k, &L, &s, &w, &nn, &nw);
  return k;
}

int ORBVocabulary::getDepthLevels() const {
  int k, L = 0, s, w, nn, nw;
  if (h_) orbv_info(h_, &k, &L, &s, &w, &nn, &nw);
  return L;
}

}  // namespace ORB_SLAM2
