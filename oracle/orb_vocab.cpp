// orb_vocab.cpp — CPU ORACLE of the DBoW2 vocabulary transform used by
// Frame::ComputeBoW (src/Frame.cc:394-401). Test infrastructure only (see
// orb_oracle.h); the product never links it.
//
// Restates, from Thirdparty/DBoW2/DBoW2 (vendored in the reference):
//   TemplatedVocabulary::loadFromTextFile   TemplatedVocabulary.h:1338-1418
//   TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)
//                                           TemplatedVocabulary.h:1127-1192
//   TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)
//                                           TemplatedVocabulary.h:1214-1256
//   BowVector::addWeight / addIfNotExist / normalize   BowVector.cpp:34-84
//   FeatureVector::addFeature               FeatureVector.cpp:31-45
//   FORB::distance (Hamming), FORB::fromString   FORB.cpp:81-135
//   ScoringObject MUST_NORMALIZE / norm per scoring type   ScoringObject.h:74-89
// Decisions where the reference is undefined (documented in DESIGN.md):
//   * a line without tokens (the trailing newline of a text file) is skipped;
//     the reference appends a root child with an uninitialised descriptor;
//   * a descent that ends at a leaf above level L - levelsup reports the leaf
//     as its node id (the reference leaves the caller's NodeId uninitialised).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "orb_oracle.h"

namespace {

struct Node {
  int id = 0, parent = 0;
  std::vector<int> children;
  uint8_t desc[32] = {};
  double weight = 0;   // Node(): weight(0)
  uint32_t word_id = 0;  // Node(): word_id(0)
};

struct Voc {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<Node> nodes;
  int nwords = 0;
};

int hamming(const uint8_t* a, const uint8_t* b) {
  // FORB::distance over 8 int32 words (FORB.cpp:81-101): the bit-parallel
  // popcount is an exact popcount
  int d = 0;
  for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

void build(Voc& v, int n, const int* parent, const uint8_t* leaf, const uint8_t* desc, const double* weight) {
  v.nodes.assign(n, Node());
  v.nwords = 0;
  for (int i = 0; i < n; ++i) {
    Node& nd = v.nodes[i];
    nd.id = i;
    if (i > 0) {
      nd.parent = parent[i];
      v.nodes[parent[i]].children.push_back(i);  // file order (:1389-1390)
    }
    memcpy(nd.desc, desc + (size_t)i * 32, 32);
    nd.weight = weight[i];
    if (i > 0 && leaf[i]) nd.word_id = (uint32_t)v.nwords++;  // m_words in file order (:1405-1412)
  }
}

// transform(feature, word_id, weight, nid, levelsup) (:1214-1256)
void transform_one(const Voc& v, const uint8_t* f, uint32_t& word, double& w, uint32_t& nid, int levelsup) {
  const int nid_level = v.L - levelsup;
  if (nid_level <= 0) nid = 0;
  int final_id = 0, level = 0;
  do {
    ++level;
    const std::vector<int>& ch = v.nodes[final_id].children;
    final_id = ch[0];
    double best_d = hamming(f, v.nodes[final_id].desc);
    for (size_t c = 1; c < ch.size(); ++c) {
      const double d = hamming(f, v.nodes[ch[c]].desc);
      if (d < best_d) {
        best_d = d;
        final_id = ch[c];
      }
    }
    if (level == nid_level) nid = (uint32_t)final_id;
  } while (!v.nodes[final_id].children.empty());
  if (nid_level > level) nid = (uint32_t)final_id;  // see header: shallow leaf
  word = v.nodes[final_id].word_id;
  w = v.nodes[final_id].weight;
}

bool must_normalize(int scoring, int* l1) {
  // L1 0, L2 1, CHI_SQUARE 2, KL 3, BHATTACHARYYA 4, DOT_PRODUCT 5 (ScoringObject.h:74-89)
  *l1 = scoring != 1;
  return scoring != 5;
}

}  // namespace

extern "C" {

int orc_voc_load_text(const char* path, int* k, int* L, int* scoring, int* weighting, int* n_nodes, int cap,
                      int* parent, uint8_t* leaf, uint8_t* desc, double* weight) {
  // TemplatedVocabulary::loadFromTextFile (:1338-1418), iostream parsing as there
  std::ifstream f(path);
  if (!f.is_open()) return -1;
  std::string s;
  std::getline(f, s);
  std::stringstream ss;
  ss << s;
  int kk = 0, LL = 0, n1 = 0, n2 = 0;
  ss >> kk >> LL >> n1 >> n2;
  if (kk < 0 || kk > 20 || LL < 1 || LL > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return -2;
  *k = kk;
  *L = LL;
  *scoring = n1;
  *weighting = n2;
  int n = 1;
  if (cap < 1) return -3;
  parent[0] = 0;
  leaf[0] = 0;
  memset(desc, 0, 32);
  weight[0] = 0;
  while (!f.eof()) {
    std::string snode;
    std::getline(f, snode);
    if (snode.find_first_not_of(" \t\r\n") == std::string::npos) continue;  // see header
    if (n >= cap) return -3;
    std::stringstream ssnode;
    ssnode << snode;
    int pid = 0, isleaf = 0;
    ssnode >> pid;
    ssnode >> isleaf;
    if (pid < 0 || pid >= n) return -4;
    std::stringstream ssd;
    for (int i = 0; i < 32; ++i) {
      std::string e;
      ssnode >> e;
      ssd << e << " ";
    }
    // FORB::fromString (FORB.cpp:120-135)
    std::stringstream sd(ssd.str());
    uint8_t* p = desc + (size_t)n * 32;
    for (int i = 0; i < 32; ++i) {
      int v = 0;
      sd >> v;
      p[i] = sd.fail() ? 0 : (uint8_t)v;
    }
    double w = 0;
    ssnode >> w;
    parent[n] = pid;
    leaf[n] = isleaf > 0;
    weight[n] = w;
    ++n;
  }
  *n_nodes = n;
  return 0;
}

int orc_voc_transform(int k, int L, int weighting, int scoring, int n_nodes, const int* parent, const uint8_t* leaf,
                      const uint8_t* node_desc, const double* node_weight, const uint8_t* desc, int n, int levelsup,
                      uint32_t* word_out, uint32_t* nid_out, double* w_out, uint32_t* bow_words,
                      double* bow_values, int* bow_n, uint32_t* fv_nodes, int* fv_off, int* fv_idx, int* fv_n) {
  (void)k;
  Voc v;
  v.L = L;
  v.scoring = scoring;
  v.weighting = weighting;
  build(v, n_nodes, parent, leaf, node_desc, node_weight);
  std::map<uint32_t, double> bow;                 // DBoW2::BowVector
  std::map<uint32_t, std::vector<int>> fv;        // DBoW2::FeatureVector
  if (v.nwords > 0) {                             // if(empty()) return (:1131-1134)
    int l1 = 1;
    const bool must = must_normalize(scoring, &l1);
    const bool tf = weighting == 0 || weighting == 1;  // TF_IDF 0, TF 1, IDF 2, BINARY 3
    for (int i = 0; i < n; ++i) {
      uint32_t word = 0, nid = 0;
      double w = 0;
      transform_one(v, desc + (size_t)i * 32, word, w, nid, levelsup);
      if (word_out) word_out[i] = word;
      if (nid_out) nid_out[i] = nid;
      if (w_out) w_out[i] = w;
      if (w > 0) {
        if (tf) {
          auto it = bow.lower_bound(word);  // addWeight
          if (it != bow.end() && it->first == word) it->second += w;
          else bow.insert(it, {word, w});
        } else {
          if (!bow.count(word)) bow[word] = w;  // addIfNotExist
        }
        fv[nid].push_back(i);
      }
    }
    if (tf && !bow.empty() && !must) {
      const double nd = bow.size();
      for (auto& e : bow) e.second /= nd;
    }
    if (must) {  // BowVector::normalize (BowVector.cpp:62-84)
      double norm = 0.0;
      if (l1)
        for (auto& e : bow) norm += std::fabs(e.second);
      else {
        for (auto& e : bow) norm += e.second * e.second;
        norm = std::sqrt(norm);
      }
      if (norm > 0.0)
        for (auto& e : bow) e.second /= norm;
    }
  }
  int b = 0;
  for (auto& e : bow) {
    bow_words[b] = e.first;
    bow_values[b] = e.second;
    ++b;
  }
  *bow_n = b;
  int f = 0, o = 0;
  fv_off[0] = 0;
  for (auto& e : fv) {
    fv_nodes[f] = e.first;
    for (int i : e.second) fv_idx[o++] = i;
    fv_off[++f] = o;
  }
  *fv_n = f;
  return 0;
}

}  // extern "C"
