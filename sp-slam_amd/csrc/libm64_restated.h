// Double-precision sin / cos / atan2 and x^3, written once for the GPU and the
// host, so that PoseOptimization gives the same bits on both.
//
// The reference gets these from glibc through g2o / Eigen / g2oAddition
// (SE3Quat::exp: std::sin, std::cos, std::pow(theta, 3); Plane3D::azimuth /
// elevation: std::atan2; AngleAxis: std::sin / std::cos).  glibc 2.35's double
// routines are table-driven (IBM Accurate Mathematical Library) and not worth
// restating bit for bit; ocml's are a different set of polynomials.  The
// PoseOptimization kernel and the oracle's device-order mode
// (oracle/pose_oracle.cpp) both call the functions below instead:
//   sin / cos : fdlibm 5.3 __kernel_sin / __kernel_cos + the medium-size
//               __ieee754_rem_pio2 (three-part pi/2, up to three rounds), one
//               reduction for both (sincos_);
//   atan2     : fdlibm 5.3 __ieee754_atan2 / atan;
//   cube      : x*x*x with the two products carried exactly (fma), rounded
//               once -- the value glibc's pow(x, 3.0) returns.
// tests/test_libm64_restated.py checks the host build against the system libm
// (sin / cos / atan2 within 1 ulp, cube identical to pow(x, 3)).
#pragma once
#if defined(__HIP__)
#include <hip/hip_runtime.h>
#else  // host build (oracle, tests)
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#include <cmath>
#endif

#include <cstdint>

namespace spslam {
namespace libm64 {

__host__ __device__ inline uint64_t d2u(double x) {
    union { double d; uint64_t u; } v;
    v.d = x;
    return v.u;
}
__host__ __device__ inline double u2d(uint64_t x) {
    union { double d; uint64_t u; } v;
    v.u = x;
    return v.d;
}
__host__ __device__ inline int32_t hi_word(double x) { return (int32_t)(d2u(x) >> 32); }
__host__ __device__ inline uint32_t lo_word(double x) { return (uint32_t)d2u(x); }

// The routines below are written select-style (both sides of a data-dependent choice computed, one kept):
// on the GPU the lanes of a wave take different branches for different angles, and branch code would run
// every taken path one after the other.  The host build runs the same expressions.

// __kernel_sin(x, y, iy): sin(x + y), |x| <= pi/4, y the tail of x
__host__ __device__ inline double k_sin(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const int32_t ix = hi_word(x) & 0x7fffffff;
    const double z = x * x, v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double p = iy == 0 ? x + v * (S1 + z * r) : x - ((z * (0.5 * y - v * r) - y) - v * S1);
    return ix < 0x3e400000 ? x : p;  // |x| < 2^-27 (fdlibm's (int)x == 0 always holds there)
}

// __kernel_cos(x, y): cos(x + y), |x| <= pi/4
__host__ __device__ inline double k_cos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const int32_t ix = hi_word(x) & 0x7fffffff;
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double small = 1.0 - (0.5 * z - (z * r - x * y));  // |x| < 0.3
    const double qx = ix > 0x3fe90000 ? 0.28125 : u2d((uint64_t)(uint32_t)(ix - 0x00200000) << 32);  // x/4
    const double hz = 0.5 * z - qx, a = 1.0 - qx;
    const double large = a - (hz - (z * r - x * y));
    return ix < 0x3e400000 ? 1.0 : (ix < 0x3fd33333 ? small : large);
}

// __ieee754_rem_pio2's medium-size algorithm for finite x: x = n * pi/2 + (y0 + y1).  fdlibm special-cases
// |x| < 3pi/4 with the same first round; here one algorithm serves every magnitude (the path's arguments are
// angles of at most a few pi; beyond 2^19 pi/2 the result stays deterministic and identical on host and
// device, only less accurate).  The second and third rounds (cancellation near a multiple of pi/2) are rare.
__host__ __device__ inline int rem_pio2(double x, double* y0, double* y1) {
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    const int32_t hx = hi_word(x), ix = hx & 0x7fffffff;
    const double t0 = hx < 0 ? -x : x;
    const int n = (int)(t0 * invpio2 + 0.5);
    const double fn = (double)n;
    double r = t0 - fn * pio2_1;
    double w = fn * pio2_1t;  // first round: good to 85 bits
    const int32_t j = ix >> 20;
    double y = r - w;
    if (j - ((hi_word(y) >> 20) & 0x7ff) > 16) {  // cancellation: second round, good to 118 bits
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        y = r - w;
        if (j - ((hi_word(y) >> 20) & 0x7ff) > 49) {  // third round, 151 bits
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            y = r - w;
        }
    }
    const double yt = (r - y) - w;
    *y0 = hx < 0 ? -y : y;
    *y1 = hx < 0 ? -yt : yt;
    return hx < 0 ? -n : n;
}

// sin and cos of one argument (fdlibm s_sin.c / s_cos.c: kernels at |x| <= pi/4, else reduced)
__host__ __device__ inline void sincos_(double x, double* sn, double* cs) {
    const int32_t ix = hi_word(x) & 0x7fffffff;
    double a, b;
    const int n = rem_pio2(x, &a, &b);
    const double ks = k_sin(a, b, 1), kc = k_cos(a, b);
    const int m = n & 3;
    double s = (m & 1) ? kc : ks, c = (m & 1) ? ks : kc;
    s = (m & 2) ? -s : s;
    c = ((m + 1) & 2) ? -c : c;  // cos: +kc, -ks, -kc, +ks
    const bool direct = ix <= 0x3fe921fb;
    const bool special = ix >= 0x7ff00000;  // inf or NaN
    *sn = special ? x - x : (direct ? k_sin(x, 0.0, 0) : s);
    *cs = special ? x - x : (direct ? k_cos(x, 0.0) : c);
}
__host__ __device__ inline double sin_(double x) {
    double s, c;
    sincos_(x, &s, &c);
    return s;
}
__host__ __device__ inline double cos_(double x) {
    double s, c;
    sincos_(x, &s, &c);
    return c;
}

// fdlibm atan: the five argument ranges share one division num / den
__host__ __device__ inline double atan_(double x0) {
    const double aT[11] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                           -1.11111104054623557880e-01, 9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                           6.66107313738753120669e-02,  -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                           -3.65315727442169155270e-02, 1.62858201153657823623e-02};
    const int32_t hx = hi_word(x0), ix = hx & 0x7fffffff;
    const double ax = x0 < 0 ? -x0 : x0;
    // id -1: |x| < 0.4375; 0: < 11/16; 1: < 1.1875; 2: < 2.4375; 3: beyond
    const int id = ix < 0x3fdc0000 ? -1 : (ix < 0x3fe60000 ? 0 : (ix < 0x3ff30000 ? 1 : (ix < 0x40038000 ? 2 : 3)));
    const double num = id < 0 ? x0 : (id == 0 ? 2.0 * ax - 1.0 : (id == 1 ? ax - 1.0 : (id == 2 ? ax - 1.5 : -1.0)));
    const double den = id < 0 ? 1.0 : (id == 0 ? 2.0 + ax : (id == 1 ? ax + 1.0 : (id == 2 ? 1.0 + 1.5 * ax : ax)));
    const double x = num / den;  // id -1: x0 / 1 = x0 exactly
    const double z = x * x, w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    const double hi = id == 0 ? 4.63647609000806093515e-01
                              : (id == 1 ? 7.85398163397448278999e-01
                                         : (id == 2 ? 9.82793723247329054082e-01 : 1.57079632679489655800e+00));
    const double lo = id == 0 ? 2.26987774529616870924e-17
                              : (id == 1 ? 3.06161699786838301793e-17
                                         : (id == 2 ? 1.39033110312309984516e-17 : 6.12323399573676603587e-17));
    const double rr = hi - ((x * (s1 + s2) - lo) - x);
    const double red = id < 0 ? x - x * (s1 + s2) : (hx < 0 ? -rr : rr);
    const double big = hx > 0 ? 1.57079632679489655800e+00 + 6.12323399573676603587e-17
                              : -1.57079632679489655800e+00 - 6.12323399573676603587e-17;
    const bool nan = ix > 0x7ff00000 || (ix == 0x7ff00000 && lo_word(x0) != 0);
    return nan ? x0 + x0 : (ix >= 0x44100000 ? big : (ix < 0x3e200000 ? x0 : red));  // |x| >= 2^66, < 2^-29
}

// fdlibm __ieee754_atan2 (zero / infinite / NaN arguments keep fdlibm's branches; the finite path selects)
__host__ __device__ inline double atan2_(double y, double x) {
    const double tiny = 1.0e-300, pi_o_4 = 7.8539816339744827900e-01, pi_o_2 = 1.5707963267948965580e+00,
                 pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    const int32_t hx = hi_word(x), ix = hx & 0x7fffffff;
    const uint32_t lx = lo_word(x);
    const int32_t hy = hi_word(y), iy = hy & 0x7fffffff;
    const uint32_t ly = lo_word(y);
    if ((ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000 || (iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000)
        return x + y;  // NaN
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if ((iy | ly) == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if ((ix | lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7ff00000) {
        if (iy == 0x7ff00000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0 * pi_o_4 + tiny;
                default: return -3.0 * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0;
            case 1: return -0.0;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7ff00000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const bool x_is_one = hx == 0x3ff00000 && lx == 0;  // atan2(y, 1) = atan(y)
    const int32_t k = (iy - ix) >> 20;
    const double q = y / x;
    const double aq = x_is_one ? y : (q < 0 ? -q : q);
    const double at = atan_(aq);
    if (x_is_one) return at;
    const double z = k > 60 ? pi_o_2 + 0.5 * pi_lo : ((hx < 0 && k < -60) ? 0.0 : at);  // |y/x| > 2^60, < -2^60
    return m == 0 ? z : (m == 1 ? -z : (m == 2 ? pi - (z - pi_lo) : (z - pi_lo) - pi));
}

// x^3 rounded once: x*x = h + l exactly, h*x = p + e exactly, x^3 = p + (e + l*x) (l*x rounded: its error is
// ~2^-106 of the result).  Equal to a correctly rounded pow(x, 3.0) except in midpoint cases of probability
// ~2^-50.
__host__ __device__ inline double cube_(double x) {
    const double h = x * x;
    const double l = fma(x, x, -h);
    const double p = h * x;
    const double e = fma(h, x, -p);
    return p + (e + l * x);
}

}  // namespace libm64
}  // namespace spslam
