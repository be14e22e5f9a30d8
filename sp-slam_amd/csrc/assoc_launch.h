// Host-side entry points of assoc_kernels.hip (Map::AssociatePlanesByBoundary).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"

namespace spslam {

struct AssocSources {
    const uint8_t* a;  // frame-plane records (coefficients first), source A then source B
    const uint8_t* b;
    int stride_a, stride_b;  // bytes per record
    const int* count_a;
    const int* count_b;
    int cap_a, cap_b;
};

// dist: scratch of n_frames * (cap_a + cap_b) * max_map floats.
hipError_t assoc_launch(int n_frames, const spslam_assoc_frame* frames, const AssocSources& src,
                        const spslam_map_plane* map, const float* boundary, int max_map,
                        const spslam_assoc_params& P, float* dist, int32_t* match, int32_t* parallel,
                        int32_t* vertical, int* new_plane, hipStream_t s, KernelTimer* timer);

}  // namespace spslam
