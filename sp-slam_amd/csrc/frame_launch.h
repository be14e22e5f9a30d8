// Host-side entry points of frame_kernels.hip (RGB-D Frame per-keypoint steps).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"

namespace spslam {

struct FrameGeom {
    float fx, fy, cx, cy;
    float dist[5];      // mDistCoef: k1 k2 p1 p2 k3
    float bf;           // mbf
    int undistort;      // mDistCoef.at<float>(0) != 0 (Frame.cc:506)
    float min_x, max_x, min_y, max_y;  // ComputeImageBounds
    float ginv_x, ginv_y;              // mfGridElementWidthInv / HeightInv
};

hipError_t frame_launch(const FrameGeom& g, int n, const spslam_keypoint* kps, const int* counts, int cap,
                        const float* depth, long long depth_fs, int stride, spslam_keypoint* keys_un, float* dout,
                        float* urout, int32_t* grid_off, int32_t* grid_idx, int* plane_counts, int* supp_counts,
                        hipStream_t s, KernelTimer* timer);

}  // namespace spslam
