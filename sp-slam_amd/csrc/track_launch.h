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

// mpReferenceKF per frame (spslam_track_refkf_vote_batch_device)
hipError_t refkf_vote_launch(int n_frames, const spslam_track_batch& mm, const spslam_refkf_vote& v, hipStream_t s);
// TrackWithMotionModel's failure test and the TrackReferenceKeyFrame switch (spslam_track_refkf_batch_device)
hipError_t refkf_launch(int n_frames, int stage, const spslam_track_batch& mm, const spslam_refkf_batch& rk,
                        hipStream_t s);

constexpr int kMaxFrameRegions = 32;
struct FrameRegions {
    spslam_frame_region r[kMaxFrameRegions];
    int n;
};
hipError_t masked_frame_copy_launch(int n_frames, const uint8_t* flags, const FrameRegions& regions, hipStream_t s);

}  // namespace spslam
