// How far is this host's glibc float libm (2.35: sinf / cosf / atan2f, the functions the path restates bit for
// bit in csrc/libm_restated.h) from the correctly rounded float functions, on the arguments the path feeds them
// ?
//   * sinf, cosf: every float in [0, 2 pi) -- ORB's `cos(angle)`, `sin(angle)` of kpt.angle * pi / 180
//     (src/ORBextractor.cc:115-116) and pcl::computeRoots' cos / sin of theta in [0, pi / 3];
//   * atan2f: N random (y >= 0, x) pairs of pcl::computeRoots' atan2(sqrt(-q), half_c0) magnitudes.
// Reference: the x87 long double function rounded to float; arguments whose long double result lies within
// 2^-56 (relative) of a float rounding boundary are settled with libquadmath.
//   g++ -O2 -fopenmp -o /tmp/float_libm_cr tools/float_libm_cr.cpp -lquadmath && /tmp/float_libm_cr [N]
#include <quadmath.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

static float as_float(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
static uint32_t as_u32(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

// v rounded to float, or NaN when v is too close to a rounding boundary to decide from long double
static float round_or_nan(long double v) {
    const float f = (float)v;
    const float lo = nextafterf(f, -INFINITY), hi = nextafterf(f, INFINITY);
    const long double m1 = ((long double)f + (long double)lo) / 2, m2 = ((long double)f + (long double)hi) / 2;
    const long double tol = fabsl(v) * 0x1p-56L;
    if (fabsl(v - m1) <= tol || fabsl(v - m2) <= tol) return NAN;
    return f;
}

static float cr_sin(float x) {
    const float f = round_or_nan(sinl((long double)x));
    return std::isnan(f) ? (float)sinq((__float128)x) : f;
}
static float cr_cos(float x) {
    const float f = round_or_nan(cosl((long double)x));
    return std::isnan(f) ? (float)cosq((__float128)x) : f;
}
static float cr_atan2(float y, float x) {
    const float f = round_or_nan(atan2l((long double)y, (long double)x));
    return std::isnan(f) ? (float)atan2q((__float128)y, (__float128)x) : f;
}

int main(int argc, char** argv) {
    const long n_pairs = argc > 1 ? atol(argv[1]) : 20000000;
    const uint32_t top = as_u32(6.2831855f);  // 2 pi rounded up
    long bad_sin = 0, bad_cos = 0, total = 0;
    uint32_t ex_sin = 0, ex_cos = 0;
#pragma omp parallel for reduction(+ : bad_sin, bad_cos, total) schedule(dynamic, 1 << 20)
    for (long u = 0; u < (long)top; u++) {
        const float x = as_float((uint32_t)u);
        total++;
        if (sinf(x) != cr_sin(x)) {
            bad_sin++;
            ex_sin = (uint32_t)u;
        }
        if (cosf(x) != cr_cos(x)) {
            bad_cos++;
            ex_cos = (uint32_t)u;
        }
    }
    std::printf("sinf: %ld of %ld floats in [0, 2pi) differ from the correctly rounded value%s", bad_sin, total,
                bad_sin ? "" : "\n");
    if (bad_sin) std::printf(" (e.g. x = %a)\n", as_float(ex_sin));
    std::printf("cosf: %ld of %ld floats in [0, 2pi) differ from the correctly rounded value%s", bad_cos, total,
                bad_cos ? "" : "\n");
    if (bad_cos) std::printf(" (e.g. x = %a)\n", as_float(ex_cos));
    long bad_at = 0;
    float ey = 0, ex = 0;
#pragma omp parallel reduction(+ : bad_at)
    {
        std::mt19937_64 rng(12345);
        rng.discard(0);
#pragma omp for
        for (long i = 0; i < n_pairs; i++) {
            std::mt19937_64 r(i * 0x9E3779B97F4A7C15ull);
            // magnitudes over the covariance eigenvalue range (|q|, |c0| from 1e-12 to 1e2), any sign of x
            const double ly = std::uniform_real_distribution<double>(-12, 2)(r);
            const double lx = std::uniform_real_distribution<double>(-12, 2)(r);
            const float y = (float)std::pow(10.0, ly);
            const float x = (float)(((r() & 1) ? -1.0 : 1.0) * std::pow(10.0, lx));
            if (atan2f(y, x) != cr_atan2(y, x)) {
                bad_at++;
                ey = y;
                ex = x;
            }
        }
    }
    std::printf("atan2f: %ld of %ld random (y > 0, x) pairs differ from the correctly rounded value", bad_at, n_pairs);
    if (bad_at) std::printf(" (e.g. atan2f(%a, %a))", ey, ex);
    std::printf("\n");
    return 0;
}
