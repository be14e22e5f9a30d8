// Host-side entry point of track_kernels.hip (the Tracking-side bookkeeping that
// turns matches and plane associations into PoseOptimization graphs).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"

namespace spslam {

struct TrackArgs {
    spslam_track_batch b;
    float inv_sigma2[kMaxLevels];
};

hipError_t track_launch(int n_frames, int stage, const TrackArgs& a, hipStream_t s, KernelTimer* timer);

}  // namespace spslam
