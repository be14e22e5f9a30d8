// g2o / Eigen / g2oAddition math on the device (fp64), shared by the
// PoseOptimization (pose_kernels.hip) and LocalBundleAdjustment
// (lba_kernels.hip) kernels: SE3Quat (Thirdparty/g2o/g2o/types/se3quat.h),
// Eigen quaternion / rotation conversions, g2oAddition/Plane3D.h.
// See oracle/g2o_restated.h for the CPU restatement of the same routines.
// sin / cos / atan2 / pow(x, 3) are correctly rounded (libm64_cr.h, the path's pinned libm semantics,
// DESIGN.md section 3.3), not ocml's.
#pragma once
#include <hip/hip_runtime.h>

#include "libm64_cr.h"

namespace spslam {
namespace g2od {

// Measurement knob only (never the product build): SPSLAM_LIBM64_OCML swaps the correctly rounded routines for
// ocml's to price them (tools/pose_phases.py); results then differ from the oracle.
#ifdef SPSLAM_LIBM64_OCML
namespace lm {
__device__ __forceinline__ void sincos_(double x, double* s, double* c) { ::sincos(x, s, c); }
__device__ __forceinline__ double atan2_(double y, double x) { return ::atan2(y, x); }
__device__ __forceinline__ void sincos2_(double a, double b, double* sa, double* ca, double* sb, double* cb) {
    ::sincos(a, sa, ca);
    ::sincos(b, sb, cb);
}
__device__ __forceinline__ void atan2x2_(double y0, double x0, double y1, double x1, double* r0, double* r1) {
    *r0 = ::atan2(y0, x0);
    *r1 = ::atan2(y1, x1);
}
__device__ __forceinline__ double cube_(double x) { return libm64cr::cube_(x); }
}  // namespace lm
#else
namespace lm = libm64cr;
#endif

struct V3 { double x, y, z; };
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

struct Q { double w, x, y, z; };
struct SE3 { Q r; V3 t; };
struct M3 { double a[9]; };  // row-major

__device__ __forceinline__ V3 mv(const M3& R, V3 v) {
    return {R.a[0] * v.x + R.a[1] * v.y + R.a[2] * v.z, R.a[3] * v.x + R.a[4] * v.y + R.a[5] * v.z,
            R.a[6] * v.x + R.a[7] * v.y + R.a[8] * v.z};
}
__device__ __forceinline__ V3 mtv(const M3& R, V3 v) {  // R^T v
    return {R.a[0] * v.x + R.a[3] * v.y + R.a[6] * v.z, R.a[1] * v.x + R.a[4] * v.y + R.a[7] * v.z,
            R.a[2] * v.x + R.a[5] * v.y + R.a[8] * v.z};
}

template <int I, int J, int K>
__device__ __forceinline__ void q_case(const M3& R, Q& q) {
    double t = sqrt(R.a[4 * I] - R.a[4 * J] - R.a[4 * K] + 1.0);
    const double ci = 0.5 * t;
    t = 0.5 / t;
    q.w = (R.a[3 * K + J] - R.a[3 * J + K]) * t;
    const double cj = (R.a[3 * J + I] + R.a[3 * I + J]) * t;
    const double ck = (R.a[3 * K + I] + R.a[3 * I + K]) * t;
    q.x = I == 0 ? ci : (J == 0 ? cj : ck);
    q.y = I == 1 ? ci : (J == 1 ? cj : ck);
    q.z = I == 2 ? ci : (J == 2 ? cj : ck);
}

// Eigen Quaternion(Matrix3)
__device__ __forceinline__ Q q_from_rot(const M3& R) {
    Q q;
    double t = R.a[0] + R.a[4] + R.a[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (R.a[7] - R.a[5]) * t;
        q.y = (R.a[2] - R.a[6]) * t;
        q.z = (R.a[3] - R.a[1]) * t;
    } else {
        // largest diagonal i, j = (i+1)%3, k = (j+1)%3; one branch per i so every index is a
        // constant (a dynamically indexed R would live in scratch memory)
        int i = 0;
        if (R.a[4] > R.a[0]) i = 1;
        if (R.a[8] > (i == 0 ? R.a[0] : R.a[4])) i = 2;
        if (i == 0) q_case<0, 1, 2>(R, q);
        else if (i == 1) q_case<1, 2, 0>(R, q);
        else q_case<2, 0, 1>(R, q);
    }
    return q;
}
__device__ M3 q_to_rot(const Q& q) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    return M3{{1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx, txz - twy, tyz + twx,
               1 - (txx + tyy)}};
}
__device__ __forceinline__ Q q_mul(const Q& a, const Q& b) {
    return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
            a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ V3 q_rot(const Q& q, V3 v) {  // Eigen _transformVector
    const V3 qv{q.x, q.y, q.z};
    V3 uv = cross(qv, v);
    uv = uv + uv;
    return v + q.w * uv + cross(qv, uv);
}
__device__ __forceinline__ void q_normalize(Q& q) {  // SE3Quat::normalizeRotation
    if (q.w < 0) { q.w = -q.w; q.x = -q.x; q.y = -q.y; q.z = -q.z; }
    const double n = sqrt(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
    q.w /= n; q.x /= n; q.y /= n; q.z /= n;
}
__device__ __forceinline__ SE3 se3_mul(const SE3& a, const SE3& b) {
    SE3 r = a;
    r.t = r.t + q_rot(a.r, b.t);
    r.r = q_mul(r.r, b.r);
    q_normalize(r.r);
    return r;
}
// SE3Quat::exp (types/se3quat.h:223-257)
__device__ __forceinline__ SE3 se3_exp(const double* u) {
    const V3 w{u[0], u[1], u[2]}, ups{u[3], u[4], u[5]};
    const double theta = sqrt(dot(w, w));
    const double O[9] = {0, -w.z, w.y, w.z, 0, -w.x, -w.y, w.x, 0};
    double O2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
    M3 R, V;
    if (theta < 0.00001) {
        for (int k = 0; k < 9; k++) R.a[k] = (k % 4 == 0 ? 1.0 : 0.0) + O[k] + O2[k];
        V = R;
    } else {
        double st, ct;
        lm::sincos_(theta, &st, &ct);
        const double a = st / theta, b = (1 - ct) / (theta * theta), c = (theta - st) / lm::cube_(theta);
        for (int k = 0; k < 9; k++) {
            R.a[k] = (k % 4 == 0 ? 1.0 : 0.0) + a * O[k] + b * O2[k];
            V.a[k] = (k % 4 == 0 ? 1.0 : 0.0) + b * O[k] + c * O2[k];
        }
    }
    SE3 s;
    s.r = q_from_rot(R);
    s.t = mv(V, ups);
    q_normalize(s.r);
    return s;
}

// ---- g2oAddition/Plane3D.h ------------------------------------------------
struct P4 { double c[4]; };
__device__ __forceinline__ void p_normalize(double* v) {
    const double n = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    for (int i = 0; i < 4; i++) v[i] = v[i] * (1. / n);
    if (v[3] < 0.0)
        for (int i = 0; i < 4; i++) v[i] = -v[i];
}
__device__ __forceinline__ double azimuth(V3 v) { return lm::atan2_(v.y, v.x); }
__device__ __forceinline__ double elevation(V3 v) { return lm::atan2_(v.z, sqrt(v.x * v.x + v.y * v.y)); }
// Plane3D::rotation: (AngleAxis(az, Z) * AngleAxis(-el, Y)).toRotationMatrix()
// (the two angles, then the two sin / cos pairs, are evaluated side by side: independent dependent chains)
__device__ __forceinline__ void az_el(V3 v, double* az, double* el) {
    lm::atan2x2_(v.y, v.x, v.z, sqrt(v.x * v.x + v.y * v.y), az, el);
}
__device__ __forceinline__ M3 p_rotation(V3 v) {
    double az, el;
    az_el(v, &az, &el);
    const double ha = 0.5 * az, he = 0.5 * (-el);
    double sa, ca, se, ce;
    lm::sincos2_(ha, he, &sa, &ca, &se, &ce);
    const Q a{ca, 0.0 * sa, 0.0 * sa, 1.0 * sa};
    const Q e{ce, 0.0 * se, 1.0 * se, 0.0 * se};
    return q_to_rot(q_mul(a, e));
}
// Eigen AngleAxis(M_PI / 2, ax).toRotationMatrix() * v (Plane3D::ominus_ver's only angle): sin and cos of the
// double nearest pi/2, correctly rounded (tests/test_gpu_libm.py checks both against the oracle)
__device__ __forceinline__ V3 aa_apply_half_pi(V3 ax, V3 v) {
    const double s = 1.0, c = 6.123233995736766e-17;
    const V3 sa = s * ax;
    const V3 c1 = (1 - c) * ax;
    M3 r;
    double tmp;
    tmp = c1.x * ax.y; r.a[1] = tmp - sa.z; r.a[3] = tmp + sa.z;
    tmp = c1.x * ax.z; r.a[2] = tmp + sa.y; r.a[6] = tmp - sa.y;
    tmp = c1.y * ax.z; r.a[5] = tmp - sa.x; r.a[7] = tmp + sa.x;
    r.a[0] = c1.x * ax.x + c; r.a[4] = c1.y * ax.y + c; r.a[8] = c1.z * ax.z + c;
    return mv(r, v);
}

// plane-edge error: (T * world).ominus{,_par,_ver}(meas)
__device__ __forceinline__ void plane_error(int kind, const SE3& T, const P4& world, const P4& meas, double* e) {
    const M3 R = q_to_rot(T.r);
    const V3 n2 = mv(R, V3{world.c[0], world.c[1], world.c[2]});
    double v[4] = {n2.x, n2.y, n2.z, world.c[3] - dot(T.t, n2)};
    if (v[3] < 0.0)
        for (int i = 0; i < 4; i++) v[i] = -v[i];
    p_normalize(v);
    const V3 ln{v[0], v[1], v[2]}, mn{meas.c[0], meas.c[1], meas.c[2]};
    V3 ref = ln;
    if (kind == 1) {
        if (dot(mn, ln) < 0) ref = -1.0 * ln;
    } else if (kind == 2) {
        const V3 a = cross(ln, mn);
        ref = aa_apply_half_pi((1.0 / sqrt(dot(a, a))) * a, ln);
    }
    const V3 n = mtv(p_rotation(ref), mn);
    az_el(n, &e[0], &e[1]);
    if (kind == 0) e[2] = (-v[3]) - (-meas.c[3]);
}

struct E3 { double e0, e1, e2; };
// plane_error returning the error by value (no address-taken array: keeps it in registers)
__device__ __forceinline__ E3 plane_error3(int kind, const SE3& T, const P4& world, const P4& meas) {
    double e[3] = {0, 0, 0};
    plane_error(kind, T, world, meas, e);
    return E3{e[0], e[1], e[2]};
}

// ---- the same error on a pair of adjacent lanes (2k, 2k + 1: half = lane & 1) -----------------------------
// A plane-edge error is ~2,300 fp64 instructions, 80 % of them the three pairs of correctly rounded functions
// (azimuth / elevation of the reference normal, the two half-angle sincos, azimuth / elevation of the rotated
// measurement), and one wave issues them one after the other.  Here each lane of the pair computes one member
// of every pair and the two halves are exchanged (DPP within the quad): about 1,000 instructions per lane, both
// lanes end with the whole error.  Same operations on the same operands: bit-identical to plane_error.  Both
// lanes of a pair must evaluate the same (kind, T, world, meas) and be active together.
__device__ __forceinline__ double pair_xchg(double v) {
    // quad_perm [1, 0, 3, 2]: every lane reads its pair partner
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// this lane's member of (atan2(v.y, v.x), atan2(v.z, |v.xy|)) -- azimuth on the even lane, elevation on the odd
// -- and the partner's, as (azimuth, elevation)
__device__ __forceinline__ void az_el_pair(V3 v, bool half, double* az, double* el) {
    const double mine = lm::atan2_(half ? v.z : v.y, half ? sqrt(v.x * v.x + v.y * v.y) : v.x);
    const double other = pair_xchg(mine);
    *az = half ? other : mine;
    *el = half ? mine : other;
}
__device__ __forceinline__ E3 plane_error_pair(int kind, const SE3& T, const P4& world, const P4& meas, bool half) {
    const M3 R = q_to_rot(T.r);
    const V3 n2 = mv(R, V3{world.c[0], world.c[1], world.c[2]});
    double v[4] = {n2.x, n2.y, n2.z, world.c[3] - dot(T.t, n2)};
    if (v[3] < 0.0)
        for (int i = 0; i < 4; i++) v[i] = -v[i];
    p_normalize(v);
    const V3 ln{v[0], v[1], v[2]}, mn{meas.c[0], meas.c[1], meas.c[2]};
    V3 ref = ln;
    if (kind == 1) {
        if (dot(mn, ln) < 0) ref = -1.0 * ln;
    } else if (kind == 2) {
        const V3 a = cross(ln, mn);
        ref = aa_apply_half_pi((1.0 / sqrt(dot(a, a))) * a, ln);
    }
    // p_rotation(ref): sincos of 0.5 * az on the even lane, of 0.5 * (-el) on the odd one
    double az, el;
    az_el_pair(ref, half, &az, &el);
    double s, c;
    lm::sincos_(half ? 0.5 * (-el) : 0.5 * az, &s, &c);
    const double so = pair_xchg(s), co = pair_xchg(c);
    const double sa = half ? so : s, ca = half ? co : c, se = half ? s : so, ce = half ? c : co;
    const Q qa{ca, 0.0 * sa, 0.0 * sa, 1.0 * sa};
    const Q qe{ce, 0.0 * se, 1.0 * se, 0.0 * se};
    const V3 n = mtv(q_to_rot(q_mul(qa, qe)), mn);
    E3 e;
    az_el_pair(n, half, &e.e0, &e.e1);
    e.e2 = kind == 0 ? (-v[3]) - (-meas.c[3]) : 0.0;
    return e;
}

// Plane3D::oplus (g2oAddition/Plane3D.h:72-85)
__device__ void p_oplus(P4& p, const double* v) {
    double s, c, s0, c0;
    lm::sincos2_(v[1], v[0], &s, &c, &s0, &c0);
    const V3 n{c * c0, c * s0, s};
    const M3 R = p_rotation(V3{p.c[0], p.c[1], p.c[2]});
    const double d = -p.c[3] + v[2];
    const V3 rn = mv(R, n);
    p.c[0] = rn.x; p.c[1] = rn.y; p.c[2] = rn.z;
    p.c[3] = -d;
    p_normalize(p.c);
}

}  // namespace g2od
}  // namespace spslam
