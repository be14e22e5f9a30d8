// Issue priority of the tracking tail's waves.
//
// In the pipelined step the tracking tail (frame steps, matching, association,
// graphs, PoseOptimization: one latency-bound workgroup per frame, barrier
// after barrier) shares every CU with the next batch's ORB and plane
// extraction (wide, high-occupancy kernels).  The HIP stream priority only
// orders workgroup dispatch; once resident, a tail wave competes for issue
// slots with the extraction waves on its SIMD and every dependent step of its
// chain stretches.  s_setprio raises the wave's issue priority in the SIMD
// arbiter so the chain advances first and the extraction waves fill the gaps.
#pragma once
#include <hip/hip_runtime.h>

// Off by default since round 6: with the ORB stream at high dispatch priority (the C2 step's critical path,
// bench.py --orb-priority) the raised tail waves cost the ORB chain more than they gain: C2 step 42.7K -> 43.3K
// frames/s without them, B = 1 unchanged (profiles/r06/ab_wave_priority.txt).  -DSPSLAM_TAIL_PRIO=1 restores it.
#ifndef SPSLAM_TAIL_PRIO
#define SPSLAM_TAIL_PRIO 0
#endif

namespace spslam {
__device__ __forceinline__ void tail_wave_priority() {
#if SPSLAM_TAIL_PRIO
    __builtin_amdgcn_s_setprio(3);
#endif
}
// Measurement knob: the ORB chain's waves (the C2 step's critical path) at issue priority SPSLAM_ORB_PRIO.
__device__ __forceinline__ void orb_wave_priority() {
#ifdef SPSLAM_ORB_PRIO
    __builtin_amdgcn_s_setprio(SPSLAM_ORB_PRIO);
#endif
}
}  // namespace spslam
