// Host-side entry points of match_kernels.hip (ORBmatcher::SearchByProjection).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"

namespace spslam {

struct MatchGeom {
    float fx, fy, cx, cy, bf;          // mK, mbf
    float min_x, max_x, min_y, max_y;  // ComputeImageBounds
    float ginv_x, ginv_y;              // mfGridElementWidthInv / HeightInv
    float scale[8];                    // mvScaleFactors
};

struct MatchCurrent {
    const spslam_keypoint* kun;
    const uint8_t* desc;
    const float* uright;
    const int32_t* grid_off;
    const int32_t* grid_idx;
    const int* counts;
    int cap;
};

// Per-point search state between the two kernels (scratch, n_frames * max_points entries), with the K smallest
// keys per point: the in-order walks re-scan a point's window only when in-loop assignments took (all but one of)
// them.  Small batches keep kProjKeys / kLocalKeys = 6 (with 3, a B = 1 frame re-scanned 2.6 last-frame and 12.5
// local windows of ~10 us each); large batches keep 3, whose window kernels cost less (kSmallBatchKeys).  The
// results do not depend on K.
constexpr int kProjKeys = 6, kLocalKeys = 6, kFewKeys = 3, kSmallBatchKeys = 16;
template <int K>
struct MatchWindowK {
    float u, v, r, invzc;
    int16_t x0, x1, y0, y1;   // GetFeaturesInArea cell range (x0 > x1: empty)
    int8_t min_level, max_level, valid, pad;
    uint32_t best[K];          // the smallest (distance << 20) | CSR position over the window; ~0u: none
    int32_t kp[K];             // their keypoints (grid_idx of the CSR position), -1: none
    float kang[K];             // and those keypoints' angles
};
using MatchWindow = MatchWindowK<kProjKeys>;  // (the scratch is sized for the larger K)

// Local-map search state per point (SearchLocalPoints).
template <int K>
struct LocalWindowK {
    float u, v, rs, ur;      // mTrackProjX / Y, r * mvScaleFactors[level], mTrackProjXR
    int16_t x0, x1, y0, y1;
    int8_t level, in_view, pad[2];
    uint32_t best[K];        // smallest keys over the window without the initially taken keypoints
    int32_t kp[K];           // their keypoints, -1: none
    int8_t oct[K];           // and those keypoints' octaves
    int8_t pad2[(8 - K % 8) % 8];
};
using LocalWindow = LocalWindowK<kLocalKeys>;

struct LocalConsts {
    float th, nn_ratio, view_cos_limit, log_scale_factor;
    int n_levels;
    const int32_t* seen;  // per-frame seen stamps (spslam_local_frame.seen_offset / stamp), may be NULL
};

hipError_t local_match_launch(int n_frames, const spslam_local_frame* frames, const spslam_local_point* points,
                              int max_points, const MatchCurrent& cur, const MatchGeom& g, const LocalConsts& P,
                              const uint8_t* taken_in, LocalWindow* win, int32_t* match, int* nmatches,
                              uint8_t* in_view, hipStream_t s, KernelTimer* timer);

hipError_t match_launch(int n_frames, const spslam_proj_frame* frames, const spslam_proj_point* points,
                        int max_points, const MatchCurrent& cur, const MatchGeom& g, const spslam_match_params& P,
                        MatchWindow* win, int2* pushes, int32_t* match, int* nmatches, hipStream_t s,
                        KernelTimer* timer);

}  // namespace spslam
