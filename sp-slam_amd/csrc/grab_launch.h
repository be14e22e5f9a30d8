// Host-side entry point of grab_kernels.hip (Tracking::GrabImageRGBD's image preparation).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"

namespace spslam {

struct GrabArgs {
    const uint8_t* color;
    size_t color_frame_stride;  // bytes
    int color_stride;           // bytes per row
    const void* depth;
    size_t depth_frame_stride;  // elements
    int depth_stride;           // elements per row
    int w, h;
    spslam_grab_params p;
    uint8_t* gray;
    float* depth_out;
    // the organized cloud of Frame::ComputePlanesFromOrganizedPointCloud (Frame.cc:857-874) made in the same pass
    // (spslam_grab_fuse_cloud): cloud == nullptr = none; frame f's x | y | z planes at cloud + f * cloud_fs
    float* cloud;
    long long cloud_fs;
    int ds, cW, cN;  // Cloud.Dis, the cloud's width and size (plane configuration)
    float fx, fy, cx, cy;
};

hipError_t grab_launch(int n_frames, const GrabArgs& a, hipStream_t s, KernelTimer* timer);

}  // namespace spslam
