// Stand-ins for the two DBoW2 containers the hot path exchanges
// (Thirdparty/DBoW2/DBoW2/BowVector.h, FeatureVector.h): the same std::map
// shapes, so code iterating them compiles unchanged.
#ifndef ORBX_SHIM_DBOW2_H
#define ORBX_SHIM_DBOW2_H
#include <map>
#include <vector>

namespace DBoW2 {
typedef unsigned int WordId;
typedef double WordValue;
typedef unsigned int NodeId;
class BowVector : public std::map<WordId, WordValue> {};
class FeatureVector : public std::map<NodeId, std::vector<unsigned int> > {};
}  // namespace DBoW2
#endif
