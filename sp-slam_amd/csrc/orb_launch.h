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

// Kernel kinds for the per-kind HIP-event timers (spslam_kernel_times).
enum KernelKind {
    kKindLevel = 0, kKindFast, kKindOctree, kKindDesc, kKindPose,
    kKindPlaneCloud, kKindPlaneDist, kKindPlaneIntegral, kKindPlaneNormal, kKindPlaneSegment,
    kKindSuppLines, kKindSuppAssemble, kKindFrame, kKindLba, kKindAssoc, kKindMatch, kKindLocalMatch,
    kKindTrack, kKindGrab, kKindBowWords, kKindBowVectors, kKindBowMatch, kNumKernelKinds
};
const char* kernel_kind_name(int kind);

// Optional timer: begin/end are called on the launch stream around each kernel
// kind (the level kind spans its per-level launches).
struct KernelTimer {
    virtual void begin(int kind, hipStream_t s) = 0;
    virtual void end(int kind, hipStream_t s) = 0;
    virtual ~KernelTimer() = default;
};

hipError_t orb_upload_tables(const int umax[16]);
// aux / ev_fork / ev_join (optional): a second stream for the small levels' chain (orb_kernels.hip)
hipError_t orb_launch(const OrbGeom& g, const OrbBuffers& b, int n, int iniTh, int minTh, spslam_keypoint* kps,
                      uint8_t* desc, int* counts, int cap_per_frame, hipStream_t s, KernelTimer* timer,
                      hipStream_t aux = nullptr, hipEvent_t ev_fork = nullptr, hipEvent_t ev_join = nullptr);

}  // namespace spslam
