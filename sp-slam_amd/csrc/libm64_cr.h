// Correctly rounded double sin / cos / atan2 / x^3 for the GPU (and a host build of the same code for tests).
//
// The reference reaches these through g2o / Eigen / g2oAddition (SE3Quat::exp: std::sin / std::cos;
// Plane3D::azimuth / elevation: std::atan2; AngleAxis: std::sin / std::cos) and so through glibc's double
// routines, the IBM Accurate Mathematical Library.  That library was designed to return the correctly
// rounded result and did so, through multi-precision fallbacks, in the glibc of ORB-SLAM2's tested
// platforms (Ubuntu 14.04 / 16.04: glibc 2.19 / 2.23); glibc 2.28 (sin, cos) and 2.34 (atan2) dropped the
// fallbacks, and glibc 2.35's fast paths misround ~0.1 % of arguments (measured in tests/test_libm64_cr.py).  The
// reference does not pin its glibc, so the path pins the libm semantics to correct rounding (DESIGN.md
// section 3.3): the unique result of round-to-nearest applied to the exact value, whatever implementation
// produces it.  The CPU oracle gets it independently (x87 long double with a quad-precision fallback,
// oracle/libm_cr_oracle.h); tests/test_libm64_cr.py checks this header's host build and
// tests/test_gpu_libm.py its gfx950 build against the oracle, bit for bit.
//
// Method (Ziv's strategy): a quick double-double evaluation (relative error well below 2^-80) whose result
// is accepted when both ends of its error interval round to the same double; otherwise (probability
// ~2^-16) an accurate double-double evaluation (relative error < 2^-100) decides.  Products are exact
// through fma (two_prod); the build keeps fp contraction off, so every other operation rounds once, on
// the GPU and on the host alike.
//   sin / cos : x = k pi/2 + r (three-part pi/2, exact first product), r = j/64 + t with |t| <= 1/128,
//               sin / cos of j/64 from a double-double table, Taylor series in t.
//   atan2     : z = min(|y|,|x|) / max(|y|,|x|) as a double-double, atan z = atan(i/64) + atan(u),
//               u = (z - i/64) / (1 + z i/64), |u| <= 1/128; then pi/2 - . , pi - . and the sign.
// Domain of the guarantee: sin / cos for |x| < 2^20 (beyond, or within ~2^-40 of a multiple of pi/2 where
// the three-part reduction loses bits, the result is still the accurate path's, possibly not correctly
// rounded); atan2 everywhere.
#pragma once
#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define SPSLAM_CR_TABLE(T, name, dims) __device__ constexpr T name dims
#else  // host build (tests)
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#include <cmath>
#define SPSLAM_CR_TABLE(T, name, dims) constexpr T name dims
#endif

namespace spslam {
namespace libm64cr {

#include "libm64_cr_tables.inc"

struct dd { double hi, lo; };

__host__ __device__ inline dd two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline dd fast_two_sum(double a, double b) {  // |a| >= |b| or a == 0
    const double s = a + b;
    return {s, b - (s - a)};
}
__host__ __device__ inline dd dmul(dd a, dd b) {
    const double p = a.hi * b.hi;
    double e = fma(a.hi, b.hi, -p);
    e = fma(a.hi, b.lo, e);
    e = fma(a.lo, b.hi, e);
    return fast_two_sum(p, e);
}
__host__ __device__ inline dd dmul_d(dd a, double b) {
    const double p = a.hi * b;
    double e = fma(a.hi, b, -p);
    e = fma(a.lo, b, e);
    return fast_two_sum(p, e);
}
__host__ __device__ inline dd dadd(dd a, dd b) {
    const dd s = two_sum(a.hi, b.hi);
    return fast_two_sum(s.hi, s.lo + (a.lo + b.lo));
}
__host__ __device__ inline dd dadd_d(dd a, double b) {
    const dd s = two_sum(a.hi, b);
    return fast_two_sum(s.hi, s.lo + a.lo);
}
__host__ __device__ inline dd dneg(dd a) { return {-a.hi, -a.lo}; }
__host__ __device__ inline dd ddiv(dd a, dd b) {
    const double q1 = a.hi / b.hi;
    const dd r = dadd(a, dneg(dmul_d(b, q1)));
    return fast_two_sum(q1, r.hi / b.hi);
}
// a / b through one reciprocal instead of two divisions (the quick paths: q1 within a few ulps of a / b, the
// double-double remainder exact to ~2^-106, so the quotient's error stays near 2^-103 -- far inside kQuickEps)
__host__ __device__ inline dd ddiv_r(dd a, dd b) {
    const double r = 1.0 / b.hi;
    const double q1 = a.hi * r;
    const dd rem = dadd(a, dneg(dmul_d(b, q1)));
    return fast_two_sum(q1, rem.hi * r);
}

// Round-to-nearest of a value known to lie within eps |r.hi| of r.hi + r.lo: true when both ends of that
// interval round to the same double (rounding is monotone), which is then the correctly rounded result.
// eps includes the rounding of r.lo -+ e itself (|r.lo| <= 2^-53 |r.hi| after fast_two_sum).
__host__ __device__ inline bool rounds_to(dd r, double eps, double* out) {
    const double e = eps * fabs(r.hi);
    const double a = r.hi + (r.lo - e), b = r.hi + (r.lo + e);
    *out = a;
    return a == b;
}

constexpr double kQuickEps = 0x1p-70;     // quick evaluations: error < 2^-80 (margin 2^10)
constexpr double kAccurateEps = 0x1p-98;  // accurate evaluations: error < 2^-100

// ---- sin / cos ---------------------------------------------------------------------------------------------
// sin(t) and cos(t) - 1 for |t| <= 1/128 (+ rounding).  Quick: the series' leading coefficient in
// double-double, the tail in double.  Accurate: Horner in double-double through t^23 / t^22.
template <bool kAccurate>
__host__ __device__ inline void sin_cm1(dd t, dd* s, dd* cm1) {
    const dd t2 = dmul(t, t);
    if (!kAccurate) {
        const double q = t2.hi;
        const double ps = kSinC[2][0] + q * (kSinC[3][0] + q * (kSinC[4][0] + q * kSinC[5][0]));
        const dd P = dadd_d(dd{kSinC[1][0], kSinC[1][1]}, q * ps);
        *s = dadd(t, dmul(dmul(t, t2), P));
        const double pc = kCosC[2][0] + q * (kCosC[3][0] + q * (kCosC[4][0] + q * kCosC[5][0]));
        *cm1 = dadd(dd{-0.5 * t2.hi, -0.5 * t2.lo}, dd{q * (q * pc), 0.0});
    } else {
        dd P{kSinC[11][0], kSinC[11][1]}, C{kCosC[11][0], kCosC[11][1]};
        for (int k = 10; k >= 1; k--) {
            P = dadd(dmul(P, t2), dd{kSinC[k][0], kSinC[k][1]});
            C = dadd(dmul(C, t2), dd{kCosC[k][0], kCosC[k][1]});
        }
        *s = dadd(t, dmul(dmul(t, t2), P));  // t (1 + t^2 P)
        *cm1 = dmul(t2, C);                    // t^2 (-1/2 + t^2 ...)
    }
}

// sin(r), cos(r) for |r| <= pi/4 (+ a little), r a double-double
template <bool kAccurate>
__host__ __device__ inline void sincos_reduced(dd r, dd* s, dd* c) {
    const double jf = rint(r.hi * 64.0);
    const int j = (int)jf;
    const dd t = two_sum(r.hi - jf * 0.015625, r.lo);  // r.hi - j/64 is exact (Sterbenz)
    dd st, cm1;
    sin_cm1<kAccurate>(t, &st, &cm1);
    // |j| <= 51 for every argument the reduction handles (|x| < 2^20 pi/2); the clamp only keeps a wild argument
    // (a diverged LM step) from indexing past the table -- its result is then garbage, as the reduction's
    const int aj = (int)fmin(fabs(jf), 64.0);
    const double sg = j < 0 ? -1.0 : 1.0;
    const dd S{sg * kSinCos64[aj][0], sg * kSinCos64[aj][1]}, C{kSinCos64[aj][2], kSinCos64[aj][3]};
    // sin(a + t) = S + (S (cos t - 1) + C sin t), cos(a + t) = C + (C (cos t - 1) - S sin t)
    *s = dadd(S, dadd(dmul(S, cm1), dmul(C, st)));
    *c = dadd(C, dadd(dmul(C, cm1), dneg(dmul(S, st))));
}

// x = k pi/2 + r: k = rint(x 2/pi); k P1 carried exactly (its high part cancels against x exactly by
// Sterbenz), P2 exactly, P3 rounded (|k P3| < 2^-87 for |k| < 2^20)
__host__ __device__ inline dd reduce_pio2(double x, int* k) {
    const double kf = rint(x * kInvPio2);
    *k = (int)(kf - 4.0 * floor(kf * 0.25));  // the quadrant (k mod 4), without overflow for any x
    const double ph = kf * kPio2_1, pl = fma(kf, kPio2_1, -ph);
    const double qh = kf * kPio2_2, ql = fma(kf, kPio2_2, -qh);
    const dd a = two_sum(x - ph, -qh);
    const dd b = two_sum(a.hi, -pl);
    return fast_two_sum(b.hi, ((a.lo + b.lo) - ql) - kf * kPio2_3);
}

template <bool kAccurate>
__host__ __device__ inline void sincos_eval(double x, dd* s, dd* c) {
    int k;
    const dd r = reduce_pio2(x, &k);
    dd sr, cr;
    sincos_reduced<kAccurate>(r, &sr, &cr);
    const int n = k & 3;  // sin: s, c, -s, -c; cos: c, -s, -c, s
    const dd a = (n & 1) ? cr : sr, b = (n & 1) ? sr : cr;
    *s = (n & 2) ? dneg(a) : a;
    *c = ((n + 1) & 2) ? dneg(b) : b;
}

// The accurate paths run for ~2^-16 of the arguments: kept out of line, so that the callers' inlined code holds
// the quick paths only (the pose kernel inlines ~20 sin / cos / atan2 sites; inlining both paths at every site
// made its body ~5x the instruction cache)
#if defined(__HIP__)
#define SPSLAM_CR_COLD __attribute__((noinline))
#else
#define SPSLAM_CR_COLD
#endif
__host__ __device__ SPSLAM_CR_COLD inline dd sincos_accurate(double x) {
    dd s, c;
    sincos_eval<true>(x, &s, &c);
    double rs, rc;
    rounds_to(s, kAccurateEps, &rs);
    rounds_to(c, kAccurateEps, &rc);
    return dd{rs, rc};
}

// The quick path without branches: special arguments select their result at the end (the evaluation then runs
// on a stand-in argument), so that two evaluations placed side by side form one straight-line block whose
// dependent chains the scheduler interleaves.  Returns false when the accurate path must decide.
__host__ __device__ inline bool sincos_quick(double x, double* sn, double* cs) {
    const double ax = fabs(x);
    const bool nonfinite = !(ax <= 1.7976931348623157e308);  // inf / NaN: both x - x
    const bool tiny = ax < 0x1p-27;  // sin x = x - x^3/6 and cos x = 1 - x^2/2 both round to their first term
    const bool special = nonfinite || tiny;
    dd s, c;
    sincos_eval<false>(special ? 1.0 : x, &s, &c);
    double rs, rc;
    const bool ok_s = rounds_to(s, kQuickEps, &rs), ok_c = rounds_to(c, kQuickEps, &rc);
    *sn = nonfinite ? x - x : (tiny ? x : rs);
    *cs = nonfinite ? x - x : (tiny ? 1.0 : rc);
    return special || (ok_s && ok_c);
}

__host__ __device__ inline void sincos_(double x, double* sn, double* cs) {
    if (!sincos_quick(x, sn, cs)) {
        const dd a = sincos_accurate(x);
        *sn = a.hi;
        *cs = a.lo;
    }
}
// sin / cos of two arguments, evaluated side by side
__host__ __device__ inline void sincos2_(double x0, double x1, double* s0, double* c0, double* s1, double* c1) {
    const bool ok0 = sincos_quick(x0, s0, c0), ok1 = sincos_quick(x1, s1, c1);
    if (!(ok0 && ok1)) {
        if (!ok0) { const dd a = sincos_accurate(x0); *s0 = a.hi; *c0 = a.lo; }
        if (!ok1) { const dd a = sincos_accurate(x1); *s1 = a.hi; *c1 = a.lo; }
    }
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

// ---- atan2 -------------------------------------------------------------------------------------------------
// atan(u), |u| <= 1/128 (+ rounding)
template <bool kAccurate>
__host__ __device__ inline dd atan_small(dd u) {
    const dd u2 = dmul(u, u);
    dd P;
    if (!kAccurate) {
        const double q = u2.hi;
        const double pa = kAtanC[2][0] +
                          q * (kAtanC[3][0] + q * (kAtanC[4][0] + q * (kAtanC[5][0] + q * (kAtanC[6][0] + q * kAtanC[7][0]))));
        P = dadd_d(dd{kAtanC[1][0], kAtanC[1][1]}, q * pa);
    } else {
        P = dd{kAtanC[11][0], kAtanC[11][1]};
        for (int k = 10; k >= 1; k--) P = dadd(dmul(P, u2), dd{kAtanC[k][0], kAtanC[k][1]});
    }
    return dadd(u, dmul(dmul(u, u2), P));  // u (1 + u^2 P)
}

// atan2 of finite, nonzero-denominator arguments as a double-double (ax = |x|, ay = |y|, not both zero)
template <bool kAccurate>
__host__ __device__ inline dd atan2_eval(double y, double x) {
    const double ax = fabs(x), ay = fabs(y);
    const bool swap = ay > ax;
    const double num = swap ? ax : ay, den = swap ? ay : ax;
    // z = num / den as a double-double: the accurate path divides twice (the remainder is exact), the quick path
    // multiplies by one reciprocal (zh within a few ulps, z still exact to ~2^-103)
    double zh, zl;
    if (kAccurate) {
        zh = num / den;
        zl = fma(-zh, den, num) / den;
    } else {
        const double rd = 1.0 / den;
        zh = num * rd;
        zl = fma(-zh, den, num) * rd;
    }
    const dd z{zh, zl};
    const double fi = rint(zh * 64.0);
    const int i = (int)fi;
    const double c = fi * 0.015625;
    const dd nm = two_sum(zh - c, z.lo);               // z - i/64 (the high difference is exact)
    const dd dn = dadd_d(dmul_d(z, c), 1.0);           // 1 + z i/64
    const dd uq = kAccurate ? ddiv(nm, dn) : ddiv_r(nm, dn);  // computed for i = 0 too: a select, not a branch
    const dd u{i == 0 ? z.hi : uq.hi, i == 0 ? z.lo : uq.lo};
    dd a = dadd(dd{kAtan64[i][0], kAtan64[i][1]}, atan_small<kAccurate>(u));
    // pi/2 - a, pi - a and the sign as selects (no branches inside the quick path)
    const dd a1 = dadd(dd{kPio2_hi, kPio2_lo}, dneg(a));
    a = dd{swap ? a1.hi : a.hi, swap ? a1.lo : a.lo};
    const dd a2 = dadd(dd{kPi_hi, kPi_lo}, dneg(a));
    a = dd{x < 0 ? a2.hi : a.hi, x < 0 ? a2.lo : a.lo};
    return dd{y < 0 ? -a.hi : a.hi, y < 0 ? -a.lo : a.lo};
}

__host__ __device__ SPSLAM_CR_COLD inline double atan2_accurate(double y, double x) {
    // |y / x| below 2^-900 with x > 0: atan2 = y/x (1 - (y/x)^2/3), which rounds like y/x (y / x is never a
    // midpoint) -- and the double-double quotient's low part would be subnormal
    if (!__builtin_signbit(x) && fabs(y) < fabs(x) * 0x1p-900) return y / x;
    double out;
    rounds_to(atan2_eval<true>(y, x), kAccurateEps, &out);
    return out;
}

// The quick path without branches (see sincos_quick); false when the accurate path must decide.
__host__ __device__ inline bool atan2_quick(double y, double x, double* out) {
    const double ax = fabs(x), ay = fabs(y);
    const double inf = 1.7976931348623157e308 * 2.0;
    const double sy = __builtin_signbit(y) ? -1.0 : 1.0;  // sign of y, zeros included (NaN: overridden below)
    const bool xneg = __builtin_signbit(x);
    const bool nan = x != x || y != y;
    const bool zy = ay == 0, zx = ax == 0, infs = ax == inf || ay == inf;
    // |y / x| below 2^-900 with x > 0 (y / x, see atan2_accurate): left to the slow path
    const bool small = !xneg && ay < ax * 0x1p-900;
    const bool special = nan || zy || zx || infs;
    double sp = 0.0;
    if (infs) sp = ax == inf && ay == inf ? sy * (xneg ? k3Pio4_hi : kPio4_hi)
                                          : (ax == inf ? (xneg ? sy * kPi_hi : sy * 0.0) : sy * kPio2_hi);
    if (zx) sp = sy * kPio2_hi;
    if (zy) sp = xneg ? sy * kPi_hi : y;                         // atan2(+-0, x): +-pi or +-0
    if (nan) sp = x + y;
    // the reciprocal 1 / max(|x|, |y|) must be a normal double: extreme magnitudes are left to the slow path
    const double den = ax > ay ? ax : ay;
    const bool extreme = !(den >= 0x1p-1000 && den <= 0x1p1000);
    const bool stand_in = special || small || extreme;
    const dd r = atan2_eval<false>(stand_in ? 1.0 : y, stand_in ? 1.0 : x);
    double q;
    const bool ok = rounds_to(r, kQuickEps, &q) && !small && !extreme;
    *out = special ? sp : q;
    return special || ok;
}

__host__ __device__ inline double atan2_(double y, double x) {
    double out;
    if (!atan2_quick(y, x, &out)) out = atan2_accurate(y, x);
    return out;
}
// atan2 of two argument pairs, evaluated side by side
__host__ __device__ inline void atan2x2_(double y0, double x0, double y1, double x1, double* r0, double* r1) {
    const bool ok0 = atan2_quick(y0, x0, r0), ok1 = atan2_quick(y1, x1, r1);
    if (!(ok0 && ok1)) {
        if (!ok0) *r0 = atan2_accurate(y0, x0);
        if (!ok1) *r1 = atan2_accurate(y1, x1);
    }
}

// ---- x^3 (pow(x, 3) in SE3Quat::exp and the LM damping update) ---------------------------------------------
// x*x = h + l exactly, h*x = p + e exactly, x^3 = p + (e + l*x): l*x's rounding is ~2^-106 of the result, so
// this is the correctly rounded cube except in midpoint cases of probability ~2^-50 (tests/test_libm64_cr.py
// checks it against exact rationals).
__host__ __device__ inline double cube_(double x) {
    const double h = x * x;
    const double l = fma(x, x, -h);
    const double p = h * x;
    const double e = fma(h, x, -p);
    if (x == 0 || !(fabs(p) <= 1.7976931348623157e308)) return p;  // +-0, +-inf (overflow included), NaN
    return p + (e + l * x);
}

}  // namespace libm64cr
}  // namespace spslam
