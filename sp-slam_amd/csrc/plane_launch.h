// Host-side entry points of plane_kernels.hip (Frame::ComputePlanesFromOrganizedPointCloud).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"

namespace spslam {

constexpr int kMaxPlanesPerFrame = 64;   // models kept per frame (reference: unbounded, <= N/MinSize)

struct PlaneGeom {
    int w, h;            // depth image
    int ds;              // Cloud.Dis
    int W, H, N;         // organized cloud (ceil(w/ds) x ceil(h/ds))
    float fx, fy, cx, cy;
    int min_size;        // Plane.MinSize
    float ang_cos;       // cosf(0.017453 * Plane.AngleThreshold)
    float dist_th;       // Plane.DistanceThreshold
    int inlier_cap;      // per-frame inlier index capacity
    int contour_cap;     // per-frame contour index capacity
    int pad_;
};

// Per-frame scratch, frame f at base + f * stride (element counts).
struct PlaneBuffers {
    float* cloud;        // [F][3][N]  x | y | z planes
    float* dist;         // [F][N]
    double* integral;    // [F][(W+1)*(H+1)][6]  (dx xyz, dy xyz)
    float* normal;       // [F][3][N]
    float* pd;           // [F][N]  plane_d = p . n
    uint32_t* labels;    // [F][N]
    int* work;           // [F][N + 4*N] misc (ranks, sizes, member lists)
    int* grown;          // [F][N] refinement grow events (target | model << 24), reference order
    uint8_t* maps;       // [F][2N] component tag / model map + contour masks (when not in LDS)
    long long* ts;       // [F][16] segmentation phase stamps (s_memrealtime, 100 MHz), diagnostics
    long long cloud_fs, dist_fs, integral_fs, normal_fs, pd_fs, labels_fs, work_fs, grown_fs, maps_fs;
};

hipError_t plane_launch(const PlaneGeom& g, const PlaneBuffers& b, int n, const float* depth, long long depth_fs,
                        int depth_stride, spslam_plane* planes, int* plane_counts, int planes_cap,
                        int32_t* inliers, int32_t* contours, hipStream_t s, KernelTimer* timer);

// Segmentation stage alone (plane_segment.hip); needs cloud/normal/pd filled.
hipError_t plane_segment_launch(const PlaneGeom& g, const PlaneBuffers& b, int n, spslam_plane* planes,
                                int* plane_counts, int planes_cap, int32_t* inliers, int32_t* contours,
                                hipStream_t s);

}  // namespace spslam
