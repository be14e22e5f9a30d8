// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// CPU restatement of the bag-of-words part of the path:
//   DBoW2 (vendored, Thirdparty/DBoW2):
//     TemplatedVocabulary::loadFromTextFile   DBoW2/TemplatedVocabulary.h:1338-1424
//     TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
//                                             :1127-1194, per feature :1217-1259
//     BowVector::addWeight / addIfNotExist / normalize     DBoW2/BowVector.cpp
//     FeatureVector::addFeature               DBoW2/FeatureVector.cpp:31-45
//     FORB::distance (256-bit Hamming)        DBoW2/FORB.cpp; FORB::fromString
//     mustNormalize per scoring type          DBoW2/ScoringObject.h:53-89
//   Frame::ComputeBoW = transform(mDescriptors rows, mBowVec, mFeatVec, 4)
//                                             src/Frame.cc:495-502 (KeyFrame.cc:64-72)
//   ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
//                                             src/ORBmatcher.cc:159-288 (TH_LOW 50,
//                                             HISTO_LENGTH 30, ComputeThreeMaxima :1601-1642)
//
// Vocabulary file quirks kept (they are the reference's behaviour when it loads
// ORBvoc.txt, System.cc:64):
//   * the loop `while(!f.eof()) { getline(f, snode); ... }` turns the empty string
//     after a final newline into one more node: `ssnode >> pid` fails and stores 0
//     (C++11), so it becomes a child of the root with no children (a leaf), word_id
//     0 (Node()), weight 0 (a stop word).  FORB::fromString leaves its descriptor
//     uninitialised (a.create without fill) -- indeterminate in the reference;
//     pinned here to all-zero bytes.
//   * a feature whose descent reaches a leaf before level m_L - levelsup leaves
//     `nid` unassigned in the reference (indeterminate); pinned here to the leaf.
//     The in-repo vocabularies have no leaf above that level (tools/make_vocab.py).
// Float: weights parse as double (istream >> double); BowVector sums and the L1/L2
// norm run in word-id order in double exactly as the std::map loops do.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace oracle {
namespace bow {

struct Node {
    int parent = 0;
    std::vector<int> children;
    uint8_t desc[32] = {0};
    double weight = 0.0;
    unsigned word_id = 0;
    bool leaf() const { return children.empty(); }
};

struct Vocabulary {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    std::vector<Node> nodes;
    int n_words = 0;
};

// DBoW2 FORB::distance: popcount of the XOR over eight 32-bit words
inline int distance(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

bool load_text(const std::string& text, Vocabulary& V) {
    std::istringstream f(text);
    std::string s;
    std::getline(f, s);
    std::stringstream ss;
    ss << s;
    int n1 = 0, n2 = 0;
    ss >> V.k >> V.L >> n1 >> n2;
    if (V.k < 0 || V.k > 20 || V.L < 1 || V.L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return false;
    V.scoring = n1;
    V.weighting = n2;
    V.nodes.assign(1, Node());
    V.n_words = 0;
    while (!f.eof()) {
        std::string snode;
        std::getline(f, snode);
        std::stringstream ssnode;
        ssnode << snode;
        const int nid = (int)V.nodes.size();
        V.nodes.emplace_back();
        int pid = 0;
        ssnode >> pid;  // 0 when the line is empty (C++11 failed extraction)
        if (pid < 0 || pid >= nid) return false;
        V.nodes[nid].parent = pid;
        V.nodes[pid].children.push_back(nid);
        int is_leaf = 0;
        ssnode >> is_leaf;
        std::stringstream ssd;
        for (int i = 0; i < 32; i++) {
            std::string e;
            ssnode >> e;
            ssd << e << " ";
        }
        for (int i = 0; i < 32; i++) {  // FORB::fromString: bytes that fail to parse stay unset (zero here)
            int n;
            ssd >> n;
            if (!ssd.fail()) V.nodes[nid].desc[i] = (uint8_t)n;
        }
        double w = 0.0;
        ssnode >> w;
        V.nodes[nid].weight = w;
        if (is_leaf > 0) V.nodes[nid].word_id = (unsigned)V.n_words++;
    }
    return true;
}

// TemplatedVocabulary::transform(feature, word_id, weight, &nid, levelsup)
void transform_one(const Vocabulary& V, const uint8_t* feature, unsigned* word, double* weight, unsigned* nid,
                   int levelsup) {
    const int nid_level = V.L - levelsup;
    unsigned node = 0;
    if (nid_level <= 0) *nid = 0;
    bool set = nid_level <= 0;
    int level = 0;
    do {
        ++level;
        const std::vector<int>& ch = V.nodes[node].children;
        unsigned best = (unsigned)ch[0];
        double best_d = distance(feature, V.nodes[best].desc);
        for (size_t c = 1; c < ch.size(); c++) {
            const double d = distance(feature, V.nodes[ch[c]].desc);
            if (d < best_d) {
                best_d = d;
                best = (unsigned)ch[c];
            }
        }
        node = best;
        if (level == nid_level) {
            *nid = node;
            set = true;
        }
    } while (!V.nodes[node].leaf());
    if (!set) *nid = node;  // indeterminate in the reference (see header)
    *word = V.nodes[node].word_id;
    *weight = V.nodes[node].weight;
}

}  // namespace bow
}  // namespace oracle

extern "C" {

void* oracle_bow_load(const char* text, long long len, int* k, int* L, int* n_nodes, int* n_words) {
    auto* V = new oracle::bow::Vocabulary();
    if (!oracle::bow::load_text(std::string(text, (size_t)len), *V)) {
        delete V;
        return nullptr;
    }
    *k = V->k;
    *L = V->L;
    *n_nodes = (int)V->nodes.size();
    *n_words = V->n_words;
    return V;
}

void oracle_bow_free(void* v) { delete (oracle::bow::Vocabulary*)v; }

// Per feature: word id, weight, node id at levelsup (TemplatedVocabulary.h:1217-1259).
void oracle_bow_words(const void* v, const uint8_t* desc, int n, int levelsup, uint32_t* word, double* weight,
                      uint32_t* nid) {
    const auto& V = *(const oracle::bow::Vocabulary*)v;
    for (int i = 0; i < n; i++) oracle::bow::transform_one(V, desc + 32 * i, &word[i], &weight[i], &nid[i], levelsup);
}

// TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup): BowVector as sorted
// (word, value) pairs, FeatureVector as sorted node ids with CSR feature lists (fv_start has n_fv + 1
// entries).  Returns 0, or -1 for an empty vocabulary (both vectors cleared).
int oracle_bow_transform(const void* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words,
                         double* bow_values, int* n_bow, uint32_t* fv_nodes, int32_t* fv_start,
                         int32_t* fv_features, int* n_fv) {
    using namespace oracle::bow;
    const auto& V = *(const Vocabulary*)v;
    *n_bow = *n_fv = 0;
    if (V.nodes.size() <= 1) return -1;
    std::map<unsigned, double> bv;
    std::map<unsigned, std::vector<unsigned>> fv;
    const bool tf = V.weighting == 0 || V.weighting == 1;  // TF_IDF, TF
    // mustNormalize: every scoring but DOT_PRODUCT (5); L2 norm only for L2_NORM (1)
    const bool must = V.scoring != 5;
    const bool l2 = V.scoring == 1;
    for (int i = 0; i < n; i++) {
        unsigned id, nid;
        double w;
        transform_one(V, desc + 32 * i, &id, &w, &nid, levelsup);
        if (w > 0) {
            auto it = bv.lower_bound(id);
            if (it != bv.end() && it->first == id) {
                if (tf) it->second += w;  // addWeight; addIfNotExist keeps the first
            } else {
                bv.insert(it, {id, w});
            }
            fv[nid].push_back((unsigned)i);
        }
    }
    if (tf && !bv.empty() && !must) {
        const double nd = (double)bv.size();
        for (auto& e : bv) e.second /= nd;
    }
    if (must) {  // BowVector::normalize
        double norm = 0.0;
        if (!l2) {
            for (auto& e : bv) norm += std::fabs(e.second);
        } else {
            for (auto& e : bv) norm += e.second * e.second;
            norm = std::sqrt(norm);
        }
        if (norm > 0.0)
            for (auto& e : bv) e.second /= norm;
    }
    int j = 0;
    for (auto& e : bv) {
        bow_words[j] = e.first;
        bow_values[j++] = e.second;
    }
    *n_bow = j;
    j = 0;
    int m = 0;
    for (auto& e : fv) {
        fv_nodes[j] = e.first;
        fv_start[j++] = m;
        for (unsigned f : e.second) fv_features[m++] = (int32_t)f;
    }
    fv_start[j] = m;
    *n_fv = j;
    return 0;
}

// ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vpMapPointMatches) (src/ORBmatcher.cc:159-288).
// kf_has_point[i]: pKF->GetMapPointMatches()[i] && !isBad(); angles: mvKeysUn / mvKeys angles.
// match[i] (i < F.N): the keyframe feature whose map point F's feature i receives, -1 if none.
int oracle_search_by_bow(const uint8_t* kf_desc, const float* kf_angle, const uint8_t* kf_has_point,
                         const uint32_t* kf_nodes, const int32_t* kf_start, const int32_t* kf_feat, int kf_n_fv,
                         const uint8_t* f_desc, const float* f_angle, int f_n, const uint32_t* f_nodes,
                         const int32_t* f_start, const int32_t* f_feat, int f_n_fv, float nn_ratio, int check_ori,
                         int32_t* match) {
    using oracle::bow::distance;
    constexpr int kHisto = 30, kThLow = 50;
    for (int i = 0; i < f_n; i++) match[i] = -1;
    std::vector<int> rot_hist[kHisto];
    const float factor = 1.0f / kHisto;
    int nmatches = 0;
    int a = 0, b = 0;
    while (a < kf_n_fv && b < f_n_fv) {
        if (kf_nodes[a] == f_nodes[b]) {
            for (int p = kf_start[a]; p < kf_start[a + 1]; p++) {
                const int ikf = kf_feat[p];
                if (!kf_has_point[ikf]) continue;
                int best1 = 256, best_idx = -1, best2 = 256;
                for (int q = f_start[b]; q < f_start[b + 1]; q++) {
                    const int jf = f_feat[q];
                    if (match[jf] >= 0) continue;
                    const int d = distance(kf_desc + 32 * ikf, f_desc + 32 * jf);
                    if (d < best1) {
                        best2 = best1;
                        best1 = d;
                        best_idx = jf;
                    } else if (d < best2) {
                        best2 = d;
                    }
                }
                if (best1 <= kThLow && (float)best1 < nn_ratio * (float)best2) {
                    match[best_idx] = ikf;
                    if (check_ori) {
                        float rot = kf_angle[ikf] - f_angle[best_idx];
                        if (rot < 0.0f) rot += 360.0f;
                        int bin = (int)std::round(rot * factor);
                        if (bin == kHisto) bin = 0;
                        rot_hist[bin].push_back(best_idx);
                    }
                    nmatches++;
                }
            }
            a++;
            b++;
        } else if (kf_nodes[a] < f_nodes[b]) {
            while (a < kf_n_fv && kf_nodes[a] < f_nodes[b]) a++;  // lower_bound
        } else {
            while (b < f_n_fv && f_nodes[b] < kf_nodes[a]) b++;
        }
    }
    if (check_ori) {  // ComputeThreeMaxima (src/ORBmatcher.cc:1601-1642)
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < kHisto; i++) {
            const int s = (int)rot_hist[i].size();
            if (s > max1) {
                max3 = max2; max2 = max1; max1 = s;
                ind3 = ind2; ind2 = ind1; ind1 = i;
            } else if (s > max2) {
                max3 = max2; max2 = s;
                ind3 = ind2; ind2 = i;
            } else if (s > max3) {
                max3 = s;
                ind3 = i;
            }
        }
        if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if (max3 < 0.1f * (float)max1) ind3 = -1;
        for (int i = 0; i < kHisto; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j : rot_hist[i]) {
                match[j] = -1;
                nmatches--;
            }
        }
    }
    return nmatches;
}

}  // extern "C"
