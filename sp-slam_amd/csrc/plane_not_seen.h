// Frame::PlaneNotSeen's pair test (src/Frame.cc:1116-1130), shared by the
// plane-extraction dedupe (plane_segment.hip, Frame.cc:912-934) and the
// supposed-plane dedupe (supposed_kernels.hip, Frame.cc:1090).
//
// FP: the reference is built -O3 -march=native (CMakeLists.txt:10-11).  GCC
// contracts PlaneNotSeen's dot product pM . coef as
//   fma(p2, c2, fma(p1, c1, p0 * c0))
// (the coef loads are hoisted out of the loop, which reorders the operands
// compared with AssociatePlanesByBoundary's fma(a2, b2, fma(a0, b0, a1 * b1))),
// and compares d and angle in double against the double literals.  Checked
// against g++ -O3 -march=native on cv::Mat-like accessors in
// tests/test_oracle_planes_kat.py; the oracle states the same expression.
#pragma once
#include <hip/hip_runtime.h>

namespace spslam {

// true when coefficient vector cf duplicates plane pm (|d diff| <= 0.2 and |cos| >= 0.9397)
__host__ __device__ __forceinline__ bool plane_seen_by(const float* pm, const float* cf) {
    const float d = pm[3] - cf[3];
    const float angle = __builtin_fmaf(pm[2], cf[2], __builtin_fmaf(pm[1], cf[1], pm[0] * cf[0]));
    if ((double)d > 0.2 || (double)d < -0.2) return false;
    if ((double)angle < 0.9397 && (double)angle > -0.9397) return false;
    return true;
}

}  // namespace spslam
