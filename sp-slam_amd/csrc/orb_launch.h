// Host-side entry points of orb_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_geom.h"

namespace spslam {

struct OrbBuffers {
    uint32_t* cand;      // [frames][cells][kCellCap] packed FAST survivors
    uint16_t* cand_cnt;  // [frames][cells]
    uint32_t* keys;      // [frames][keys_per_frame] DistributeOctTree key scratch
    uint16_t* keynode;   // [frames][keys_per_frame]
    LevelKp* lvl_kp;     // [frames][lvl_kp_per_frame]
    int* lvl_cnt;        // [frames][kMaxLevels]
};

hipError_t orb_upload_tables(const int umax[16]);
hipError_t orb_launch(const OrbGeom& g, const OrbBuffers& b, int n, int iniTh, int minTh, spslam_keypoint* kps,
                      uint8_t* desc, int* counts, int cap_per_frame, hipStream_t s);

}  // namespace spslam
