// Host-side entry points of pose_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"

namespace spslam {

// Derived constants of PoseOptimization (src/Optimizer.cc:553-554, 681-693).
struct PoseConsts {
    double delta_mono, delta_stereo;        // (float)sqrt(5.991), (float)sqrt(7.815)
    double angle_info, dis_info, par_info, ver_info;
    double plane_chi, vp_chi;
    double delta_plane, delta_vp;           // (float)sqrt(Chi), (float)sqrt(VPChi)
    int spin_cap;                           // bound of the kernel's internal waits (spslam_debug_pose_spin_cap)
    unsigned fail_mask;                     // test hook: bit q = LM trial q's LDLT reports failure
                                            //   (spslam_debug_force_solve_failures; 0 otherwise)
};

PoseConsts make_pose_consts(const spslam_plane_config& c);
hipError_t libm64_debug_launch(int kind, const double* a, const double* b, int n, double* out, hipStream_t s);
hipError_t pose_launch(int n, const spslam_pose_problem* probs, const spslam_point_obs* pts,
                       const spslam_plane_obs* pls, const PoseConsts& K, const spslam_pose_result* init_from,
                       spslam_pose_result* res, uint8_t* pout, uint8_t* plout, hipStream_t s);

}  // namespace spslam
