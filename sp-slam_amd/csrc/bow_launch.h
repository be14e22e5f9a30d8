// Host-side entry points of bow_kernels.hip (DBoW2 transform = Frame::ComputeBoW,
// ORBmatcher::SearchByBoW).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"

namespace spslam {

// A DBoW2 TemplatedVocabulary resident in HBM (structure of arrays).  Children of
// node n: child_ids[child_begin[n] .. child_begin[n] + child_count[n]) in the
// order loadFromTextFile pushed them (the first-minimum tie-break follows it).
struct VocabDev {
    int n_nodes = 0, k = 0, L = 0, scoring = 0, weighting = 0;
    const uint4* desc = nullptr;        // [n_nodes][2] 32-byte node descriptors
    const int* child_begin = nullptr;   // [n_nodes]
    const int* child_count = nullptr;   // [n_nodes]
    const int* child_ids = nullptr;     // [n_nodes - 1]
    const double* weight = nullptr;     // [n_nodes] (0 = stop word / internal node)
    const uint32_t* word_id = nullptr;  // [n_nodes]
};

// Per-frame BowVector / FeatureVector outputs at f * cap (fv_start at f * (cap + 1)).
struct BowOut {
    uint32_t* bow_words;
    double* bow_values;
    int* n_bow;
    uint32_t* fv_nodes;
    int32_t* fv_start;
    int32_t* fv_features;
    int* n_fv;
};

// Frame f's descriptors at desc + f * cap * 32, counts[f] of them.  Scratch:
// word / weight / node per feature slot (n_frames * cap each).
hipError_t bow_transform_launch(const VocabDev& V, int n_frames, const uint8_t* desc, const int* counts, int cap,
                                int levelsup, uint32_t* s_word, double* s_weight, uint32_t* s_node,
                                const BowOut& out, hipStream_t s, KernelTimer* timer);

// The keyframe / frame sides of SearchByBoW pairs: features of slot f at f * cap
// (descriptors, keypoints for the angle, has_point flags of the keyframe side),
// FeatureVectors in the BowOut layout.
struct BowSide {
    const uint8_t* desc;
    const spslam_keypoint* keys;
    const uint8_t* has_point;  // keyframe side only (may be NULL on the frame side)
    const int* counts;
    const uint32_t* fv_nodes;
    const int32_t* fv_start;
    const int32_t* fv_features;
    const int* n_fv;
    int cap;
};

hipError_t bow_search_launch(int n_pairs, const int2* pairs, const BowSide& kf, const BowSide& fr, float nn_ratio,
                             int check_ori, int32_t* match, int* nmatches, hipStream_t s, KernelTimer* timer);

}  // namespace spslam
