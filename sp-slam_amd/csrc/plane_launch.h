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
    // wave: the wavefront kernel's skewed pass-1 distance map (wave_index: one step's cells are contiguous)
    float* wave;         // [F][wave_size]
    float* dist;         // [F][N]  distance map
    double* integral;    // [F][(W+1)*(H+2)][6]  (dx xyz, dy xyz); row H+1 absorbs padding lanes
    float* normal;       // [F][3][N]
    float* pd;           // [F][N]  plane_d = p . n
    uint32_t* labels;    // [F][N] connected-component labels (global instance: also its union-find parents)
    int* work;           // [F][N + 4*N] misc (ranks, sizes, member lists)
    int* grown;          // [F][N] refinement grow events (target | model << 24), reference order
    uint8_t* maps;       // [F][2N] component tag / model map + contour masks (when not in LDS)
    long long* ts;       // [F][16] segmentation phase stamps (s_memrealtime, 100 MHz), diagnostics
    long long cloud_fs, wave_fs, dist_fs, integral_fs, normal_fs, pd_fs, labels_fs, work_fs, grown_fs, maps_fs;
    int keep_labels;     // the LDS instance also stores the connected-component labels in `labels` (test hook)
};

// Skewed wavefront layout: entry (st, r) = cloud cell (r, c = st - 2r), the cell wavefront step st
// visits in row r, at (st + kWaveChunk) * pitch + r.  pitch = H rounded up to a wave (every lane of
// the wavefront workgroup owns an entry, so its loads and stores need no bounds test); steps are
// padded to a multiple of kWaveChunk (the kernel's prefetch unit) plus one chunk of prefetch slack
// on either side.
constexpr int kWaveChunk = 8;
__host__ __device__ inline int wave_pitch(int H) { return (H + 63) / 64 * 64; }
__host__ __device__ inline int wave_steps(int W, int H) {
    return (2 * (H - 1) + W + kWaveChunk - 1) / kWaveChunk * kWaveChunk;
}
__host__ __device__ inline long long wave_size(int W, int H) {
    return (long long)(wave_steps(W, H) + 2 * kWaveChunk) * wave_pitch(H);
}
__host__ __device__ inline long long wave_index(int r, int c, int H) {
    return (long long)(c + 2 * r + kWaveChunk) * wave_pitch(H) + r;
}

hipError_t plane_launch(const PlaneGeom& g, const PlaneBuffers& b, int n, const float* depth, long long depth_fs,
                        int depth_stride, spslam_plane* planes, int* plane_counts, int planes_cap,
                        int32_t* inliers, int32_t* contours, hipStream_t s, KernelTimer* timer,
                        bool have_cloud = false);  // have_cloud: b.cloud already holds the depth's cloud

// Segmentation stage alone (plane_segment.hip); needs cloud/normal/pd filled.
// dynamic LDS bytes of the segmentation kernel; *in_lds: the per-frame maps (and 16-bit labels) live in LDS
size_t plane_segment_lds_bytes(const PlaneGeom& g, bool* in_lds);
hipError_t plane_segment_launch(const PlaneGeom& g, const PlaneBuffers& b, int n, spslam_plane* planes,
                                int* plane_counts, int planes_cap, int32_t* inliers, int32_t* contours,
                                hipStream_t s);

}  // namespace spslam
