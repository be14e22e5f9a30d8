// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// Correctly rounded double sin / cos / atan2 / x^3 for the CPU oracle, computed independently of the
// device's double-double code (sp-slam_amd/csrc/libm64_cr.h): the x87 extended-precision routines of the
// host libm (sinl, cosl, atan2l: error a few ulps of a 64-bit significand) give the result when both ends
// of a 2^-60 relative interval around them round to the same double; otherwise (about 1 call in 20) the
// quad-precision routines of libquadmath (113-bit significand) decide.  The pinned semantics this
// realizes, and why, are in libm64_cr.h's header and DESIGN.md section 3.3.
#pragma once
#include <quadmath.h>

#include <cmath>

// ORACLE_NS: the namespace of the g2o / Eigen restatement -- "oracle", or "oracle_fma" when the Makefile compiles
// pose_oracle.cpp / lba_oracle.cpp a second time with GCC's FP contraction (the FMA diagnostic mode)
#ifndef ORACLE_NS
#define ORACLE_NS oracle
#endif

namespace ORACLE_NS {
namespace libm_cr {

inline bool settle(long double v, double* out) {
    const long double e = fabsl(v) * 0x1p-60L;
    const double a = (double)(v - e), b = (double)(v + e);
    *out = a;
    return a == b;
}
inline double sin(double x) {
    double r;
    if (!std::isfinite(x)) return x - x;
    if (settle(sinl((long double)x), &r)) return r;
    return (double)sinq((__float128)x);
}
inline double cos(double x) {
    double r;
    if (!std::isfinite(x)) return x - x;
    if (settle(cosl((long double)x), &r)) return r;
    return (double)cosq((__float128)x);
}
inline double atan2(double y, double x) {
    double r;
    if (std::isnan(x) || std::isnan(y)) return x + y;
    if (settle(atan2l((long double)y, (long double)x), &r)) return r;
    return (double)atan2q((__float128)y, (__float128)x);
}
inline double cube(double x) {  // x * x is exact in quad precision; one rounding of the product to 113 bits
    const __float128 q = (__float128)x * (__float128)x * (__float128)x;
    return (double)q;
}

}  // namespace libm_cr
}  // namespace oracle
