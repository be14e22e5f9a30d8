// Host-side entry points of supposed_kernels.hip (Frame::GeneratePlanesFromBoundries).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"
#include "plane_launch.h"

namespace spslam {

constexpr int kMaxLinesPerBoundary = 4;       // Frame.cc:960 `for (j = 0; j < 4; j++)`
constexpr int kSuppRndTable = 1 << 21;        // >= 1001 trials x 1000 checks x 2 draws of one segment()
constexpr int kMaxPatchSteps = 64;
constexpr int kMaxSuppPerFrame = 32;         // appended (supposed) planes stored per frame

// One SACSegmentation LINE result on a boundary (scratch, per frame x plane x j).
struct LineCand {
    float line[6];     // refined coefficients: point (centroid) + direction
    int n_inliers;     // selectWithinDistance(refined) size
    int iterations;    // RANSAC trials
    int flags;         // 1 fitted (>= Line.Ratio * boundary), 2 LineInRange, 4 IsBorderLine
    int idx_off;       // line points (organized-cloud indices) at frame scratch + idx_off
};

struct SuppParams {
    double line_ratio;     // Line.Ratio
    float sqr_th_f;        // largest float s with (double)s < (double)th * th (th = Line.DistanceThreshold)
    float min_x, max_x, min_y, max_y;  // Frame::mnMinX .. mnMaxY
    int supp_cap;          // appended planes per frame
    int line_cap;          // line index capacity per frame
    int n_steps;           // CaculatePlanes patch loop length per axis
    float steps[kMaxPatchSteps];
};

struct SuppBuffers {
    const uint32_t* rnd;   // kSuppRndTable draws of mt19937(12345) >> 1
    LineCand* cand;        // [F][kMaxPlanesPerFrame][kMaxLinesPerBoundary]
    int* n_cand;           // [F][kMaxPlanesPerFrame]
    int32_t* line_idx;     // [F][contour_cap] line point indices, per boundary at its contour offset
    float4* big;           // [F][contour_cap] point scratch for boundaries beyond the LDS tile
    int* big_sh;           // [F][contour_cap]
    uint8_t* big_flag;     // [F][contour_cap]
    long long* prof;       // [F][kMaxPlanesPerFrame][8] phase clocks of the SPSLAM_SUPP_PROF diagnostic build
};

hipError_t supp_launch(const PlaneGeom& g, const PlaneBuffers& pb, const SuppParams& sp, const SuppBuffers& sb,
                       int n, const float* depth, long long depth_fs, int depth_stride, const spslam_plane* planes,
                       const int* plane_counts, const int32_t* contours, spslam_supposed_plane* out, int* out_counts,
                       int32_t* out_line_idx, float* out_patch, hipStream_t s, KernelTimer* timer);

// Frame::PlaneNotSeen of m candidates against n planes (4 floats each), device buffers: out[k] = 1 if not seen.
hipError_t plane_not_seen_debug_launch(const float* planes, int n, const float* coefs, int m, int* out,
                                       hipStream_t s);

}  // namespace spslam
