// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// g2o / Eigen / g2oAddition math restated for the CPU oracle, shared by
// pose_oracle.cpp (PoseOptimization) and lba_oracle.cpp (LocalBundleAdjustment):
//   SE3Quat + VertexSE3Expmap::oplus (Thirdparty/g2o/g2o/types/se3quat.h,
//     types_six_dof_expmap.h:73-76), Eigen Quaternion(Matrix3) / toRotationMatrix
//     / product / _transformVector, AngleAxis;
//   g2oAddition/Plane3D.h (normalize, rotation, operator*(Isometry3D, Plane3D),
//     ominus / ominus_par / ominus_ver, oplus);
//   RobustKernelHuber (core/robust_kernel_impl.cpp:78-91).
// All arithmetic is double, like the reference.
#pragma once
#include <cmath>
#include <cstring>

#include "libm_cr_oracle.h"

// ORACLE_NS: the namespace of the g2o / Eigen restatement -- "oracle", or "oracle_fma" when the Makefile compiles
// pose_oracle.cpp / lba_oracle.cpp a second time with GCC's FP contraction (the FMA diagnostic mode)
#ifndef ORACLE_NS
#define ORACLE_NS oracle
#endif
#ifdef ORACLE_FMA_VARIANT
#define ORACLE_ENTRY(name) name##_fma
#else
#define ORACLE_ENTRY(name) name
#endif

namespace ORACLE_NS {
namespace g2o_math {

// Elementary functions: correctly rounded by default (libm_cr_oracle.h: the
// semantics the path pins, which the GPU's libm64_cr.h reproduces); libm mode 1 switches the calling thread
// to the host glibc's double routines (glibc 2.35 here: fast paths that misround ~0.1 % of arguments) -- a
// diagnostic of the path's sensitivity to the libm, and the CPU baseline's speed-representative libm.
inline int& libm_mode() {
    static thread_local int mode = 0;
    return mode;
}
inline double o_sin(double x) { return libm_mode() ? std::sin(x) : libm_cr::sin(x); }
inline double o_cos(double x) { return libm_mode() ? std::cos(x) : libm_cr::cos(x); }
inline double o_atan2(double y, double x) { return libm_mode() ? std::atan2(y, x) : libm_cr::atan2(y, x); }
inline double o_cube(double x) { return libm_mode() ? std::pow(x, 3) : libm_cr::cube(x); }

struct V3 { double x, y, z; };
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline double norm(V3 a) { return std::sqrt(dot(a, a)); }

struct M3 { double m[3][3]; };
inline V3 mul(const M3& R, V3 v) {
    return {R.m[0][0] * v.x + R.m[0][1] * v.y + R.m[0][2] * v.z, R.m[1][0] * v.x + R.m[1][1] * v.y + R.m[1][2] * v.z,
            R.m[2][0] * v.x + R.m[2][1] * v.y + R.m[2][2] * v.z};
}
inline M3 transpose(const M3& R) {
    M3 T;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T.m[i][j] = R.m[j][i];
    return T;
}
inline M3 mul(const M3& A, const M3& B) {
    M3 C;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C.m[i][j] = A.m[i][0] * B.m[0][j] + A.m[i][1] * B.m[1][j] + A.m[i][2] * B.m[2][j];
    return C;
}

struct Quat { double w, x, y, z; };
// Eigen::Quaternion(const Matrix3&) (Eigen/src/Geometry/Quaternion.h quaternionbase_assign_impl)
inline Quat quat_from_rot(const M3& R) {
    Quat q;
    double t = R.m[0][0] + R.m[1][1] + R.m[2][2];
    if (t > 0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (R.m[2][1] - R.m[1][2]) * t;
        q.y = (R.m[0][2] - R.m[2][0]) * t;
        q.z = (R.m[1][0] - R.m[0][1]) * t;
    } else {
        int i = 0;
        if (R.m[1][1] > R.m[0][0]) i = 1;
        if (R.m[2][2] > R.m[i][i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(R.m[i][i] - R.m[j][j] - R.m[k][k] + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (R.m[k][j] - R.m[j][k]) * t;
        c[j] = (R.m[j][i] + R.m[i][j]) * t;
        c[k] = (R.m[k][i] + R.m[i][k]) * t;
        q.x = c[0]; q.y = c[1]; q.z = c[2];
    }
    return q;
}
inline M3 quat_to_rot(const Quat& q) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    M3 R;
    R.m[0][0] = 1 - (tyy + tzz); R.m[0][1] = txy - twz; R.m[0][2] = txz + twy;
    R.m[1][0] = txy + twz; R.m[1][1] = 1 - (txx + tzz); R.m[1][2] = tyz - twx;
    R.m[2][0] = txz - twy; R.m[2][1] = tyz + twx; R.m[2][2] = 1 - (txx + tyy);
    return R;
}
inline Quat quat_mul(const Quat& a, const Quat& b) {
    return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
            a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}
// Eigen QuaternionBase::_transformVector
inline V3 quat_rotate(const Quat& q, V3 v) {
    V3 qv{q.x, q.y, q.z};
    V3 uv = cross(qv, v);
    uv = uv + uv;
    return v + q.w * uv + cross(qv, uv);
}
inline void quat_normalize_rotation(Quat& q) {  // SE3Quat::normalizeRotation
    if (q.w < 0) { q.w = -q.w; q.x = -q.x; q.y = -q.y; q.z = -q.z; }
    double n = std::sqrt(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
    q.w /= n; q.x /= n; q.y /= n; q.z /= n;
}

struct SE3 {
    Quat r{1, 0, 0, 0};
    V3 t{0, 0, 0};
    static SE3 from_Rt(const M3& R, V3 t) { SE3 s; s.r = quat_from_rot(R); s.t = t; quat_normalize_rotation(s.r); return s; }
    V3 map(V3 X) const { return quat_rotate(r, X) + t; }
    SE3 operator*(const SE3& b) const {
        SE3 res = *this;
        res.t = res.t + quat_rotate(r, b.t);
        res.r = quat_mul(res.r, b.r);
        quat_normalize_rotation(res.r);
        return res;
    }
    // SE3Quat::exp, types/se3quat.h:223-257
    static SE3 exp(const double u[6]) {
        V3 w{u[0], u[1], u[2]}, ups{u[3], u[4], u[5]};
        double theta = norm(w);
        M3 O{{{0, -w.z, w.y}, {w.z, 0, -w.x}, {-w.y, w.x, 0}}};
        M3 R, V;
        if (theta < 0.00001) {
            M3 O2 = mul(O, O);
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) R.m[i][j] = (i == j ? 1.0 : 0.0) + O.m[i][j] + O2.m[i][j];
            V = R;
        } else {
            M3 O2 = mul(O, O);
            double a = o_sin(theta) / theta, b = (1 - o_cos(theta)) / (theta * theta),
                   c = (theta - o_sin(theta)) / o_cube(theta);
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) {
                    R.m[i][j] = (i == j ? 1.0 : 0.0) + a * O.m[i][j] + b * O2.m[i][j];
                    V.m[i][j] = (i == j ? 1.0 : 0.0) + b * O.m[i][j] + c * O2.m[i][j];
                }
        }
        SE3 s;
        s.r = quat_from_rot(R);
        s.t = mul(V, ups);
        quat_normalize_rotation(s.r);
        return s;
    }
};

// --- g2oAddition/Plane3D.h -------------------------------------------------
struct Plane {
    double c[4];
    V3 normal() const { return {c[0], c[1], c[2]}; }
    double distance() const { return -c[3]; }
    static void normalize(double* v) {
        double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        for (int i = 0; i < 4; i++) v[i] = v[i] * (1. / n);
        if (v[3] < 0.0)
            for (int i = 0; i < 4; i++) v[i] = -v[i];
    }
    static Plane from(const double* v) { Plane p; std::memcpy(p.c, v, sizeof p.c); normalize(p.c); return p; }
};
inline double azimuth(V3 v) { return o_atan2(v.y, v.x); }
inline double elevation(V3 v) { return o_atan2(v.z, std::sqrt(v.x * v.x + v.y * v.y)); }
inline Quat aa_quat(double angle, V3 axis) {  // Eigen Quaternion(AngleAxis)
    double ha = 0.5 * angle, s = o_sin(ha);
    return {o_cos(ha), s * axis.x, s * axis.y, s * axis.z};
}
inline M3 aa_rot(double angle, V3 a) {  // Eigen AngleAxis::toRotationMatrix
    V3 sa = o_sin(angle) * a;
    double c = o_cos(angle);
    V3 c1 = (1 - c) * a;
    M3 r;
    double tmp;
    tmp = c1.x * a.y; r.m[0][1] = tmp - sa.z; r.m[1][0] = tmp + sa.z;
    tmp = c1.x * a.z; r.m[0][2] = tmp + sa.y; r.m[2][0] = tmp - sa.y;
    tmp = c1.y * a.z; r.m[1][2] = tmp - sa.x; r.m[2][1] = tmp + sa.x;
    r.m[0][0] = c1.x * a.x + c; r.m[1][1] = c1.y * a.y + c; r.m[2][2] = c1.z * a.z + c;
    return r;
}
inline M3 plane_rotation(V3 v) {  // Plane3D::rotation
    Quat q = quat_mul(aa_quat(azimuth(v), {0, 0, 1}), aa_quat(-elevation(v), {0, 1, 0}));
    return quat_to_rot(q);
}
// operator*(Isometry3D, Plane3D)
inline Plane transform(const SE3& T, const Plane& p) {
    M3 R = quat_to_rot(T.r);
    V3 n2 = mul(R, p.normal());
    double v2[4] = {n2.x, n2.y, n2.z, p.c[3] - dot(T.t, n2)};
    if (v2[3] < 0.0)
        for (double& e : v2) e = -e;
    return Plane::from(v2);
}
inline void ominus(const Plane& a, const Plane& b, double* e) {
    M3 R = transpose(plane_rotation(a.normal()));
    V3 n = mul(R, b.normal());
    e[0] = azimuth(n); e[1] = elevation(n); e[2] = a.distance() - b.distance();
}
inline void ominus_par(const Plane& a, const Plane& b, double* e) {
    V3 nor = a.normal();
    if (dot(b.normal(), nor) < 0) nor = -1.0 * nor;
    M3 R = transpose(plane_rotation(nor));
    V3 n = mul(R, b.normal());
    e[0] = azimuth(n); e[1] = elevation(n);
}
inline void ominus_ver(const Plane& a, const Plane& b, double* e) {
    V3 v = cross(a.normal(), b.normal());
    V3 ax = (1.0 / norm(v)) * v;
    V3 bb = mul(aa_rot(M_PI / 2, ax), a.normal());
    M3 R = transpose(plane_rotation(bb));
    V3 n = mul(R, b.normal());
    e[0] = azimuth(n); e[1] = elevation(n);
}

// --- edges -------------------------------------------------------------------
struct Huber {
    bool on = true;
    double delta = 0, dsqr = 0;
    void set(double d) { delta = d; dsqr = d * d; }
    void robustify(double e, double rho[3]) const {
        if (e <= dsqr) { rho[0] = e; rho[1] = 1.; rho[2] = 0.; }
        else { double s = std::sqrt(e); rho[0] = 2 * s * delta - dsqr; rho[1] = delta / s; rho[2] = -0.5 * rho[1] / e; }
    }
};


// Plane3D::oplus (g2oAddition/Plane3D.h:72-85): azimuth/elevation/distance update.
inline void plane_oplus(Plane& p, const double* v) {
    const double az = v[0], el = v[1];
    const double s = o_sin(el), c = o_cos(el);
    const V3 n{c * o_cos(az), c * o_sin(az), s};
    const M3 R = plane_rotation(p.normal());
    const double d = p.distance() + v[2];
    const V3 rn = mul(R, n);
    p.c[0] = rn.x; p.c[1] = rn.y; p.c[2] = rn.z;
    p.c[3] = -d;
    Plane::normalize(p.c);
}

}  // namespace g2o_math
}  // namespace oracle
