// glibc float math restated for the GPU (and the host, for the CPU check).
//
// The reference calls these through Eigen/PCL float code on the host
// (pcl::computeRoots: std::atan2(float, float), std::cos(float),
// std::sin(float)); the CPU oracle calls the system libm.  The device
// versions below reproduce glibc 2.35's results bit for bit so the GPU path
// yields the same plane / line eigenvectors as the host:
//   atanf / atan2f: sysdeps/ieee754/flt-32/s_atanf.c, e_atan2f.c (fdlibm);
//   sinf / cosf   : sysdeps/ieee754/flt-32/s_sincosf.h (|x| < 120 branch).
// tests/test_libm_restated.py checks the host build of this header against
// the system libm (exhaustively over the arguments computeRoots can pass).
#pragma once
#if defined(__HIP__)
#include <hip/hip_runtime.h>
#else  // host-only build (tests/test_libm_restated.py compiles this header with g++)
#define __host__
#define __device__
#endif

#include <cstdint>

namespace spslam {
namespace libm {

__host__ __device__ inline uint32_t f2u(float x) {
    union { float f; uint32_t u; } v;
    v.f = x;
    return v.u;
}
__host__ __device__ inline float u2f(uint32_t x) {
    union { float f; uint32_t u; } v;
    v.u = x;
    return v.f;
}

// fdlibm __atanf.
__host__ __device__ inline float atanf_(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT[11] = {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                          9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                          4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};
    const int32_t hx = (int32_t)f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {   // |x| < 0.4375
        if (ix < 0x31000000) return x;  // |x| < 2^-29
        id = -1;
    } else {
        x = x < 0.f ? -x : x;
        if (ix < 0x3f980000) {        // |x| < 1.1875
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

// fdlibm __ieee754_atan2f.
__host__ __device__ inline float atan2f_(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)f2u(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)f2u(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return atanf_(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else {
        const float q = y / x;
        z = atanf_(q < 0.f ? -q : q);
    }
    switch (m) {
        case 0: return z;
        case 1: return u2f(f2u(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// glibc sinf / cosf for |x| < 120 (s_sincosf.h, the ranges computeRoots and
// the ORB angles use); double-precision polynomials.  glibc's second
// coefficient table is the first with the cosine terms negated, which equals
// negating the cosine polynomial's (double) value exactly.
__host__ __device__ inline float sincos_poly(double x, double x2, bool neg_cos, int n) {
    const double c0 = 0x1p0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5, c3 = -0x1.6c087e89a359dp-10,
                 c4 = 0x1.99343027bf8c3p-16, s1c = -0x1.555545995a603p-3, s2c = 0x1.1107605230bc4p-7,
                 s3c = -0x1.994eb3774cf24p-13;
    if ((n & 1) == 0) {
        const double x3 = x * x2, s1 = s2c + x2 * s3c, x7 = x3 * x2, s = x + x3 * s1c;
        return (float)(s + x7 * s1);
    }
    const double x4 = x2 * x2, cc2 = c3 + x2 * c4, cc1 = c0 + x2 * c1, x6 = x4 * x2, c = cc1 + x4 * c2;
    const double v = c + x6 * cc2;
    return (float)(neg_cos ? -v : v);
}
__host__ __device__ inline uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }
__host__ __device__ inline void sincosf_(float y, float* sn, float* cs) {
    const double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) { *sn = y; *cs = 1.0f; return; }
        *sn = sincos_poly(x, x * x, false, 0);
        *cs = sincos_poly(x, x * x, false, 1);
        return;
    }
    const double hpi_inv = 0x1.45F306DC9C883p+23, hpi = 0x1.921FB54442D18p0;
    const double r = x * hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    const double xr = x - n * hpi;
    const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    const bool neg = (n & 2) != 0;
    *sn = sincos_poly(xr * s, xr * xr, neg, n);
    *cs = sincos_poly(xr * s, xr * xr, neg, n ^ 1);
}

}  // namespace libm
}  // namespace spslam
