// gfx950 LocalBundleAdjustment (reference: src/Optimizer.cc:1154-1977 on the
// vendored g2o BlockSolver_6_3 + Levenberg-Marquardt, g2oAddition plane
// edges).  Semantics: oracle/lba_oracle.cpp.
//
// One 512-thread workgroup per problem runs the whole schedule --
// optimize(5), relabel, optimize(10), outlier flags -- with no host round
// trip; problems of a batch (keyframes of many sequences) run side by side.
// Per LM iteration:
//   edges      thread per edge: error, Huber weight, analytic (points) or
//              central-difference (planes, both vertices) Jacobians, and the
//              edge's quadratic-form terms (Hll, bl, Hpl, Hpp, bp) -> HBM;
//   landmarks  thread per landmark: Hll, bl and its (landmark, pose) blocks
//              summed over its edges in insertion order;
//   poses      wave per pose: Hpp, bp summed over the pose's edges.
// Per LM trial (lambda):
//   landmarks  thread per landmark: (Hll + lambda)^-1 (Eigen 3x3 cofactor
//              inverse), Dinv bl, B Dinv per block;
//   Schur      wave per pose pair (p1 <= p2): Hpp + lambda - sum_l B Dinv B^T
//              over the landmarks both poses see (64-bit pose masks, lanes
//              stride over landmarks, 36 accumulators per lane), and
//              bp - sum_l B Dinv bl per pose;
//   solve      LDL^T of the reduced 6P x 6P system, right-looking (the same
//              per-entry operation order as the oracle's factorisation);
//   update     landmark back-substitution, exp(x) * T, X + x, Plane3D::oplus;
//   errors     thread per edge, robust chi2 (tree reduction), accept/reject.
// All arithmetic is fp64; reductions are tree-ordered and the landmark order
// is the caller's list order, so results match the oracle to rounding
// (north-star bar 1e-4), not bitwise.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "g2o_device.h"
#include "lba_launch.h"

namespace spslam {
namespace lba {

using namespace g2od;

constexpr int kThreads = 256, kWaves = kThreads / 64;

struct Shared {
    double red[kWaves][8];
    double lambda, ni, currentChi, iniChi, rho;
    int nBad, stop, ok, qmax, its;
    int np, nl_active;
    int pose_hidx[kLbaMaxKeyframes];
    int hidx_pose[kLbaMaxKeyframes];
    int pose_act[kLbaMaxKeyframes];
    int wsum[kWaves];
    long long t_phase[8];   // wall_clock64 ticks per phase (100 MHz), thread 0
    long long t_mark;
    int trials;
};

// Phase timer (diagnostics): thread 0 charges the time since the last mark to phase p.
__device__ __forceinline__ void mark(Shared& S, int p) {
    if (threadIdx.x == 0) {
        const long long now = wall_clock64();
        S.t_phase[p] += now - S.t_mark;
        S.t_mark = now;
    }
}

struct Ctx {
    int K, Np, Nq, E, Ep, L;
    const spslam_lba_keyframe* kf;
    const spslam_lba_point* pt;
    const spslam_lba_point_obs* pobs;
    const spslam_lba_plane* pl;
    const spslam_lba_plane_obs* plobs;
    double *pose, *pose_b, *X, *X_b, *P, *P_b, *err, *con, *lmH, *lmb, *Dinv, *db, *xl, *blkH, *blkBD, *S, *bs, *dd, *y,
        *Hpp, *bp;
    int *pose_hidx_g, *hidx_pose_g, *e_lm, *e_kf, *e_type, *e_level, *e_blk, *e_src, *lm_boff, *lm_nb, *blk_pose,
        *lm_act;
    uint64_t* lm_mask;
};

__device__ __forceinline__ SE3 load_pose(const double* p) { return SE3{Q{p[0], p[1], p[2], p[3]}, V3{p[4], p[5], p[6]}}; }
__device__ __forceinline__ void store_pose(double* p, const SE3& T) {
    p[0] = T.r.w; p[1] = T.r.x; p[2] = T.r.y; p[3] = T.r.z; p[4] = T.t.x; p[5] = T.t.y; p[6] = T.t.z;
}
// Converter::toPlane3D (flip d < 0) + Plane3D(v) normalisation
__device__ __forceinline__ P4 plane_from_f(const float* c) {
    P4 p{{c[0], c[1], c[2], c[3]}};
    if (c[3] < 0.0f)
        for (int i = 0; i < 4; i++) p.c[i] = -p.c[i];
    p_normalize(p.c);
    return p;
}
// operator*(Isometry3D, Plane3D)
__device__ P4 plane_transform(const SE3& T, const P4& w) {
    const M3 R = q_to_rot(T.r);
    const V3 n2 = mv(R, V3{w.c[0], w.c[1], w.c[2]});
    P4 v{{n2.x, n2.y, n2.z, w.c[3] - dot(T.t, n2)}};
    if (v.c[3] < 0.0)
        for (int i = 0; i < 4; i++) v.c[i] = -v.c[i];
    p_normalize(v.c);
    return v;
}
// (T * world).ominus{,_par,_ver}(meas) for edge types 2 / 3 / 4
__device__ void plane_edge_error(int type, const SE3& T, const P4& world, const P4& meas, double* e) {
    plane_error(type - 2, T, world, meas, e);
}

__device__ __forceinline__ int edge_dim(int type) { return type == 0 ? 2 : (type == 1 || type == 2) ? 3 : 2; }

__device__ void info_of(const Ctx& c, const LbaConsts& C, int e, double* info) {
    const int t = c.e_type[e];
    if (t <= 1) {
        const double s = (double)c.pobs[c.e_src[e]].inv_sigma2;
        info[0] = info[1] = info[2] = s;
    } else if (t == 2) {
        info[0] = info[1] = C.angle_info; info[2] = C.dis_info;
    } else {
        info[0] = info[1] = t == 3 ? C.par_info : C.ver_info;
        info[2] = 0;
    }
}

__device__ void edge_error(const Ctx& c, int e, const SE3& T, const double* X, const P4* P, double* err) {
    const int t = c.e_type[e];
    if (t <= 1) {
        const spslam_lba_point_obs& o = c.pobs[c.e_src[e]];
        const spslam_lba_keyframe& k = c.kf[c.e_kf[e]];
        const V3 p = q_rot(T.r, V3{X[0], X[1], X[2]}) + T.t;
        if (t == 0) {
            err[0] = (double)o.u - (p.x / p.z * (double)k.fx + (double)k.cx);
            err[1] = (double)o.v - (p.y / p.z * (double)k.fy + (double)k.cy);
        } else {
            const float invz = (float)(1.0f / p.z);
            const double r0 = p.x * invz * (double)k.fx + (double)k.cx, r1 = p.y * invz * (double)k.fy + (double)k.cy;
            const double r2 = r0 - (double)(k.bf * invz);  // cam_project(..., const float& bf)
            err[0] = (double)o.u - r0;
            err[1] = (double)o.v - r1;
            err[2] = (double)o.ur - r2;
        }
        return;
    }
    plane_edge_error(t, T, *P, plane_from_f(c.plobs[c.e_src[e]].meas), err);
}

__device__ __forceinline__ const double* lm_state(const Ctx& c, int lm) {
    return lm < c.Np ? c.X + 3 * lm : c.P + 4 * (lm - c.Np);
}
__device__ __forceinline__ double chi2_of(const double* err, const double* info, int dim) {
    double s = 0;
    for (int i = 0; i < dim; i++) s += err[i] * info[i] * err[i];
    return s;
}
__device__ __forceinline__ void huber(double chi, double delta, bool on, double* rho0, double* rho1) {
    const double dsqr = delta * delta;
    if (!on || chi <= dsqr) { *rho0 = chi; *rho1 = 1.0; return; }
    const double s = sqrt(chi);
    *rho0 = 2 * s * delta - dsqr;
    *rho1 = delta / s;
}
__device__ __forceinline__ double delta_of(const LbaConsts& C, int t) {
    return t == 0 ? C.delta_mono : t == 1 ? C.delta_stereo : t == 2 ? C.delta_plane : C.delta_vp;
}

__device__ bool depth_positive(const Ctx& c, int e) {
    const SE3 T = load_pose(c.pose + 7 * c.e_kf[e]);
    const int lm = c.e_lm[e];
    if (c.e_type[e] <= 1) {
        const double* X = c.X + 3 * lm;
        return (q_rot(T.r, V3{X[0], X[1], X[2]}) + T.t).z > 0.0;
    }
    const double* pp = c.P + 4 * (lm - c.Np);
    const P4 w{{pp[0], pp[1], pp[2], pp[3]}};
    return -plane_transform(T, w).c[3] > 0;
}

// Block-wide sum of NV doubles per thread; result valid in every thread.
template <int NV>
__device__ void block_sum(double (&v)[NV], Shared& S) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; k++) {
        double x = v[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
        if (lane == 0) S.red[w][k] = x;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; k++) {
        double s = 0;
        for (int j = 0; j < kWaves; j++) s += S.red[j][k];
        v[k] = s;
    }
    __syncthreads();
}
__device__ double block_max(double v, Shared& S) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    if (lane == 0) S.red[w][0] = v;
    __syncthreads();
    double m = 0;
    for (int j = 0; j < kWaves; j++) m = fmax(m, S.red[j][0]);
    __syncthreads();
    return m;
}
// exclusive block scan of one int per thread; *total = sum
__device__ int block_scan(int v, int* total, Shared& S) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) S.wsum[w] = x;
    __syncthreads();
    int base = 0, tot = 0;
    for (int j = 0; j < kWaves; j++) {
        if (j < w) base += S.wsum[j];
        tot += S.wsum[j];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// Robust chi2 of all active edges at the current estimates (errors cached per edge).
__device__ double active_chi2(const Ctx& c, const LbaConsts& C, bool robust, Shared& S) {
    double acc[1] = {0.0};
    for (int e = threadIdx.x; e < c.E; e += kThreads) {
        if (c.e_level[e] != 0) continue;
        const int lm = c.e_lm[e];
        const SE3 T = load_pose(c.pose + 7 * c.e_kf[e]);
        double* err = c.err + 3 * e;
        P4 P;
        if (lm >= c.Np) {
            const double* pp = c.P + 4 * (lm - c.Np);
            P = P4{{pp[0], pp[1], pp[2], pp[3]}};
        }
        edge_error(c, e, T, lm < c.Np ? c.X + 3 * lm : nullptr, &P, err);
        double info[3];
        info_of(c, C, e, info);
        const int t = c.e_type[e];
        double r0, r1;
        huber(chi2_of(err, info, edge_dim(t)), delta_of(C, t), robust, &r0, &r1);
        acc[0] += r0;
    }
    block_sum(acc, S);
    return acc[0];
}

// Edge Jacobians: A (landmark, dim x 3), B (pose, dim x 6); fixed vertices skipped.
__device__ void edge_jacobians(const Ctx& c, int e, bool pose_free, double (&A)[3][3], double (&B)[3][6]) {
    const int t = c.e_type[e], lm = c.e_lm[e];
    const SE3 T = load_pose(c.pose + 7 * c.e_kf[e]);
    if (t <= 1) {
        const spslam_lba_keyframe& k = c.kf[c.e_kf[e]];
        const double fx = k.fx, fy = k.fy, bf = k.bf;
        const double* X = c.X + 3 * lm;
        const V3 p = q_rot(T.r, V3{X[0], X[1], X[2]}) + T.t;
        const double x = p.x, y = p.y, z = p.z, z_2 = z * z;
        const M3 R = q_to_rot(T.r);
        if (t == 0) {
            const double tmp[2][3] = {{fx, 0, -x / z * fx}, {0, fy, -y / z * fy}};
            const double s = -1. / z;
            for (int r = 0; r < 2; r++) {
                const double t0 = s * tmp[r][0], t1 = s * tmp[r][1], t2 = s * tmp[r][2];
                for (int q = 0; q < 3; q++) A[r][q] = t0 * R.a[q] + t1 * R.a[3 + q] + t2 * R.a[6 + q];
            }
        } else {
            for (int q = 0; q < 3; q++) {
                A[0][q] = -fx * R.a[q] / z + fx * x * R.a[6 + q] / z_2;
                A[1][q] = -fy * R.a[3 + q] / z + fy * y * R.a[6 + q] / z_2;
                A[2][q] = A[0][q] - bf * R.a[6 + q] / z_2;
            }
        }
        B[0][0] = x * y / z_2 * fx; B[0][1] = -(1 + (x * x / z_2)) * fx; B[0][2] = y / z * fx;
        B[0][3] = -1. / z * fx; B[0][4] = 0; B[0][5] = x / z_2 * fx;
        B[1][0] = (1 + y * y / z_2) * fy; B[1][1] = -x * y / z_2 * fy; B[1][2] = -x / z * fy;
        B[1][3] = 0; B[1][4] = -1. / z * fy; B[1][5] = y / z_2 * fy;
        if (t == 1) {
            B[2][0] = B[0][0] - bf * y / z_2; B[2][1] = B[0][1] + bf * x / z_2; B[2][2] = B[0][2];
            B[2][3] = B[0][3]; B[2][4] = 0; B[2][5] = B[0][5] - bf / z_2;
        }
        return;
    }
    const double delta = 1e-9, scalar = 1.0 / (2 * delta);
    const double* pp = c.P + 4 * (lm - c.Np);
    const P4 P0{{pp[0], pp[1], pp[2], pp[3]}};
    const P4 meas = plane_from_f(c.plobs[c.e_src[e]].meas);
    const int dim = edge_dim(t);
    double ep[3], em[3];
    for (int d = 0; d < 3; d++) {
        double add[3] = {0, 0, 0};
        add[d] = delta;
        P4 P = P0;
        p_oplus(P, add);
        plane_edge_error(t, T, P, meas, ep);
        add[d] = -delta;
        P = P0;
        p_oplus(P, add);
        plane_edge_error(t, T, P, meas, em);
#pragma unroll
        for (int i = 0; i < 3; i++) A[i][d] = i < dim ? scalar * (ep[i] - em[i]) : 0.0;
    }
    if (!pose_free) return;
    for (int d = 0; d < 6; d++) {
        double add[6] = {0, 0, 0, 0, 0, 0};
        add[d] = delta;
        plane_edge_error(t, se3_mul(se3_exp(add), T), P0, meas, ep);
        add[d] = -delta;
        plane_edge_error(t, se3_mul(se3_exp(add), T), P0, meas, em);
#pragma unroll
        for (int i = 0; i < 3; i++) B[i][d] = i < dim ? scalar * (ep[i] - em[i]) : 0.0;
    }
}

// Eigen compute_inverse<Matrix3d>
__device__ void inverse3(const double (&m)[3][3], double* r) {
    auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1];
    };
    const double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    const double det = (c0 * m[0][0] + c1 * m[1][0]) + c2 * m[2][0];
    const double invdet = 1.0 / det;
    r[0] = c0 * invdet; r[1] = c1 * invdet; r[2] = c2 * invdet;
    r[3] = cof(0, 1) * invdet; r[4] = cof(1, 1) * invdet; r[5] = cof(2, 1) * invdet;
    r[6] = cof(0, 2) * invdet; r[7] = cof(1, 2) * invdet; r[8] = cof(2, 2) * invdet;
}

// initializeOptimization(0): active poses (by id) / landmarks, (landmark, pose) blocks.
__device__ void initialize(Ctx& c, Shared& S) {
    const int t = threadIdx.x;
    if (t < c.K) S.pose_act[t] = 0;
    for (int l = t; l < c.L; l += kThreads) c.lm_act[l] = 0;
    __syncthreads();
    for (int e = t; e < c.E; e += kThreads)
        if (c.e_level[e] == 0) {
            atomicOr(&S.pose_act[c.e_kf[e]], 1);
            c.lm_act[c.e_lm[e]] = 1;  // benign race: every writer stores 1
        }
    __syncthreads();
    if (t == 0) {
        int np = 0;
        for (int k = 0; k < c.K; k++) S.pose_hidx[k] = -1;
        for (int k = 0; k < c.K; k++) {  // non-fixed active poses in id order (insertion sort, K <= 64)
            const spslam_lba_keyframe& kk = c.kf[k];
            if (!S.pose_act[k] || kk.fixed || kk.id == 0) continue;
            int j = np++;
            while (j > 0 && c.kf[S.hidx_pose[j - 1]].id > kk.id) { S.hidx_pose[j] = S.hidx_pose[j - 1]; j--; }
            S.hidx_pose[j] = k;
        }
        for (int j = 0; j < np; j++) S.pose_hidx[S.hidx_pose[j]] = j;
        S.np = np;
    }
    __syncthreads();
    // blocks: unique free poses among a landmark's active edges, sorted by hessian index
    const int nchunk = (c.L + kThreads - 1) / kThreads;
    int base = 0;
    for (int ch = 0; ch < nchunk; ch++) {
        const int l = ch * kThreads + t;
        uint64_t mask = 0;
        int e_beg = 0, e_end = 0;
        if (l < c.L) {
            // edges of a landmark are contiguous: points first (Ep edges), then planes
            e_beg = c.lm_boff[l];
            e_end = e_beg + c.lm_nb[l];
        }
        for (int e = e_beg; e < e_end; e++)
            if (c.e_level[e] == 0) {
                const int h = S.pose_hidx[c.e_kf[e]];
                if (h >= 0) mask |= 1ull << h;
            }
        const int nb = __popcll(mask);
        int tot;
        const int off = block_scan(nb, &tot, S) + base;
        if (l < c.L) {
            c.lm_mask[l] = mask;
            // blocks of l at [off, off + nb): pose hidx in increasing order
            uint64_t m = mask;
            for (int j = 0; j < nb; j++) {
                const int h = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                c.blk_pose[off + j] = h;
            }
            for (int e = e_beg; e < e_end; e++) {
                const int h = S.pose_hidx[c.e_kf[e]];
                c.e_blk[e] = (c.e_level[e] == 0 && h >= 0) ? off + __popcll(mask & ((1ull << h) - 1)) : -1;
            }
        }
        base += tot;
        // block offsets per landmark are recovered from the mask + the running offset
        if (l < c.L) c.lm_act[l] = c.lm_act[l] ? (off + 1) : 0;  // store off+1 (0 = inactive)
    }
    __syncthreads();
}

__device__ __forceinline__ int lm_block_base(const Ctx& c, int l) { return c.lm_act[l] - 1; }

// buildSystem: edge terms, landmark / pose sums.  Returns max |diag| (lambda init).
__device__ double build_system(Ctx& c, const LbaConsts& C, bool robust, Shared& S) {
    const int t = threadIdx.x;
    for (int e = t; e < c.E; e += kThreads) {
        if (c.e_level[e] != 0) continue;
        const int ty = c.e_type[e], dim = edge_dim(ty);
        const bool pfree = S.pose_hidx[c.e_kf[e]] >= 0;
        double A[3][3] = {}, B[3][6] = {};
        edge_jacobians(c, e, pfree, A, B);
        double info[3];
        info_of(c, C, e, info);
        const double* err = c.err + 3 * e;
        double r0, w;
        huber(chi2_of(err, info, dim), delta_of(C, ty), robust, &r0, &w);
        double W[3] = {0, 0, 0}, om[3] = {0, 0, 0};
#pragma unroll
        for (int r = 0; r < 3; r++)
            if (r < dim) {
                W[r] = robust ? w * info[r] : info[r];
                om[r] = -(info[r] * err[r]);
                if (robust) om[r] *= w;
            }
        // rows >= dim of A, B, W, om are zero: the padded terms add exact zeros
        double* o = c.con + (size_t)kLbaCon * e;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            o[9 + i] = (A[0][i] * om[0] + A[1][i] * om[1]) + A[2][i] * om[2];
#pragma unroll
            for (int j = 0; j < 3; j++)
                o[3 * i + j] = ((A[0][i] * W[0]) * A[0][j] + (A[1][i] * W[1]) * A[1][j]) + (A[2][i] * W[2]) * A[2][j];
#pragma unroll
            for (int j = 0; j < 6; j++)
                o[12 + 6 * i + j] = pfree ? ((A[0][i] * W[0]) * B[0][j] + (A[1][i] * W[1]) * B[1][j]) +
                                                (A[2][i] * W[2]) * B[2][j]
                                          : 0.0;
        }
        if (pfree) {
            int q = 30;
#pragma unroll
            for (int i = 0; i < 6; i++)
#pragma unroll
                for (int j = i; j < 6; j++)
                    o[q++] = ((B[0][i] * W[0]) * B[0][j] + (B[1][i] * W[1]) * B[1][j]) + (B[2][i] * W[2]) * B[2][j];
#pragma unroll
            for (int i = 0; i < 6; i++) o[51 + i] = (B[0][i] * om[0] + B[1][i] * om[1]) + B[2][i] * om[2];
        }
    }
    __syncthreads();
    mark(S, 2);
    double mx = 0.0;
    // landmarks: Hll, bl, blocks (edges of a landmark are contiguous, summed in order)
    for (int l = t; l < c.L; l += kThreads) {
        const int b0 = lm_block_base(c, l);
        if (b0 < 0) continue;
        const int nb = __popcll(c.lm_mask[l]);
        for (int j = 0; j < nb * 18; j++) c.blkH[(size_t)b0 * 18 + j] = 0.0;
        double H[9] = {}, b[3] = {};
        for (int e = c.lm_boff[l]; e < c.lm_boff[l] + c.lm_nb[l]; e++) {
            if (c.e_level[e] != 0) continue;
            const double* o = c.con + (size_t)kLbaCon * e;
            for (int j = 0; j < 9; j++) H[j] += o[j];
            for (int j = 0; j < 3; j++) b[j] += o[9 + j];
            const int bk = c.e_blk[e];
            if (bk >= 0)
                for (int j = 0; j < 18; j++) c.blkH[(size_t)bk * 18 + j] += o[12 + j];
        }
        for (int j = 0; j < 9; j++) c.lmH[9 * l + j] = H[j];
        for (int j = 0; j < 3; j++) c.lmb[3 * l + j] = b[j];
        mx = fmax(mx, fmax(fabs(H[0]), fmax(fabs(H[4]), fabs(H[8]))));
    }
    // poses: wave per pose, lanes stride over edges
    const int lane = t & 63, wave = t >> 6;
    for (int h = wave; h < S.np; h += kWaves) {
        const int k = S.hidx_pose[h];
        double acc[27];
#pragma unroll
        for (int j = 0; j < 27; j++) acc[j] = 0.0;
        for (int e = lane; e < c.E; e += 64) {
            if (c.e_level[e] != 0 || c.e_kf[e] != k) continue;
            const double* o = c.con + (size_t)kLbaCon * e + 30;
#pragma unroll
            for (int j = 0; j < 27; j++) acc[j] += o[j];
        }
#pragma unroll
        for (int j = 0; j < 27; j++) {
            double x = acc[j];
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
            acc[j] = x;
        }
        if (lane == 0) {
            double* H = c.Hpp + 36 * h;
            int q = 0;
#pragma unroll
            for (int i = 0; i < 6; i++)
#pragma unroll
                for (int j = i; j < 6; j++) { H[6 * i + j] = acc[q]; H[6 * j + i] = acc[q]; q++; }
#pragma unroll
            for (int i = 0; i < 6; i++) c.bp[6 * h + i] = acc[21 + i];
            mx = fmax(mx, fmax(fmax(fabs(acc[0]), fabs(acc[6])), fmax(fmax(fabs(acc[11]), fabs(acc[15])),
                                                                      fmax(fabs(acc[18]), fabs(acc[20])))));
        }
    }
    __syncthreads();
    return block_max(mx, S);
}

// Schur complement + reduced solve + landmark back-substitution.  Returns false on a zero pivot.
__device__ bool solve(Ctx& c, double lam, Shared& S) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int np = S.np, n = 6 * np;
    // landmarks: Dinv, db, B Dinv per block
    for (int l = t; l < c.L; l += kThreads) {
        const int b0 = lm_block_base(c, l);
        if (b0 < 0) continue;
        double D[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) D[i][j] = c.lmH[9 * l + 3 * i + j] + (i == j ? lam : 0.0);
        double Di[9];
        inverse3(D, Di);
        for (int j = 0; j < 9; j++) c.Dinv[9 * l + j] = Di[j];
        const double* bl = c.lmb + 3 * l;
        for (int i = 0; i < 3; i++) c.db[3 * l + i] = (Di[3 * i] * bl[0] + Di[3 * i + 1] * bl[1]) + Di[3 * i + 2] * bl[2];
        const int nb = __popcll(c.lm_mask[l]);
        for (int a = 0; a < nb; a++) {
            const double* H = c.blkH + (size_t)(b0 + a) * 18;  // 3 x 6 (landmark x pose)
            double* BD = c.blkBD + (size_t)(b0 + a) * 18;     // 6 x 3
            for (int r = 0; r < 6; r++)
                for (int q = 0; q < 3; q++) BD[3 * r + q] = (H[r] * Di[q] + H[6 + r] * Di[3 + q]) + H[12 + r] * Di[6 + q];
        }
    }
    __syncthreads();
    // Schur blocks: wave per pose pair (p1 <= p2); lanes stride over landmarks
    const int npairs = np * (np + 1) / 2;
    for (int pr = wave; pr < npairs + np; pr += kWaves) {
        if (pr < npairs) {
            int p1 = 0, rem = pr;
            while (rem >= np - p1) { rem -= np - p1; p1++; }
            const int p2 = p1 + rem;
            const uint64_t need = (1ull << p1) | (1ull << p2);
            double acc[36];
#pragma unroll
            for (int j = 0; j < 36; j++) acc[j] = 0.0;
            for (int l = lane; l < c.L; l += 64) {
                const uint64_t m = c.lm_mask[l];
                if ((m & need) != need) continue;
                const int b0 = lm_block_base(c, l);
                const int a = b0 + __popcll(m & ((1ull << p1) - 1)), b = b0 + __popcll(m & ((1ull << p2) - 1));
                const double* BD = c.blkBD + (size_t)a * 18;
                const double* H = c.blkH + (size_t)b * 18;
                double bd[18], hh[18];
#pragma unroll
                for (int j = 0; j < 18; j++) { bd[j] = BD[j]; hh[j] = H[j]; }
#pragma unroll
                for (int r = 0; r < 6; r++)
#pragma unroll
                    for (int q = 0; q < 6; q++)
                        acc[6 * r + q] += (bd[3 * r] * hh[q] + bd[3 * r + 1] * hh[6 + q]) + bd[3 * r + 2] * hh[12 + q];
            }
#pragma unroll
            for (int j = 0; j < 36; j++) {
                double x = acc[j];
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
                acc[j] = x;
            }
            if (lane < 36) {
                const int r = lane / 6, q = lane % 6;
                double v = 0.0;
#pragma unroll
                for (int j = 0; j < 36; j++) if (j == lane) v = acc[j];
                double base = 0.0;
                if (p1 == p2) base = c.Hpp[36 * p1 + lane] + (r == q ? lam : 0.0);
                c.S[(size_t)(6 * p1 + r) * n + 6 * p2 + q] = base - v;
            }
        } else {
            const int p = pr - npairs;
            double acc[6] = {0, 0, 0, 0, 0, 0};
            for (int l = lane; l < c.L; l += 64) {
                const uint64_t m = c.lm_mask[l];
                if (!((m >> p) & 1)) continue;
                const int a = lm_block_base(c, l) + __popcll(m & ((1ull << p) - 1));
                const double* H = c.blkH + (size_t)a * 18;
                const double* db = c.db + 3 * l;
#pragma unroll
                for (int r = 0; r < 6; r++) acc[r] += (H[r] * db[0] + H[6 + r] * db[1]) + H[12 + r] * db[2];
            }
#pragma unroll
            for (int j = 0; j < 6; j++) {
                double x = acc[j];
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
                acc[j] = x;
            }
            if (lane < 6) {
                double v = 0.0;
#pragma unroll
                for (int j = 0; j < 6; j++) if (j == lane) v = acc[j];
                c.bs[6 * p + lane] = c.bp[6 * p + lane] - v;
            }
        }
    }
    __syncthreads();
    mark(S, 4);
    // LDL^T of the upper triangle, right-looking: entry (r, q), r <= q, loses (L[q][k] d_k) L[r][k]
    // at step k; L[i][j] is kept in the lower triangle of S.
    for (int j = 0; j < n; j++) {
        const double dj = c.S[(size_t)j * n + j];
        if (dj == 0.0) { __syncthreads(); return false; }
        for (int i = j + 1 + t; i < n; i += kThreads) c.S[(size_t)i * n + j] = c.S[(size_t)j * n + i] / dj;
        if (t == 0) c.dd[j] = dj;
        __syncthreads();
        const int m = n - j - 1;
        for (int idx = t; idx < m * m; idx += kThreads) {
            const int r = j + 1 + idx / m, q = j + 1 + idx % m;
            if (r > q) continue;
            c.S[(size_t)r * n + q] -= (c.S[(size_t)q * n + j] * dj) * c.S[(size_t)r * n + j];
        }
        __syncthreads();
    }
    mark(S, 5);
    for (int i = t; i < n; i += kThreads) c.y[i] = c.bs[i];
    __syncthreads();
    for (int k = 0; k < n; k++) {  // forward: y[i] -= L[i][k] y[k], k increasing
        const double yk = c.y[k];
        __syncthreads();
        for (int i = k + 1 + t; i < n; i += kThreads) c.y[i] -= c.S[(size_t)i * n + k] * yk;
        __syncthreads();
    }
    for (int i = t; i < n; i += kThreads) c.y[i] /= c.dd[i];
    __syncthreads();
    for (int k = n - 1; k >= 0; k--) {  // backward: y[i] -= L[k][i] y[k], k decreasing
        const double yk = c.y[k];
        __syncthreads();
        for (int i = t; i < k; i += kThreads) c.y[i] -= c.S[(size_t)k * n + i] * yk;
        __syncthreads();
    }
    // landmarks: xl = Dinv (bl - Hpl^T xp)
    for (int l = t; l < c.L; l += kThreads) {
        const int b0 = lm_block_base(c, l);
        if (b0 < 0) continue;
        double cl[3] = {c.lmb[3 * l], c.lmb[3 * l + 1], c.lmb[3 * l + 2]};
        uint64_t m = c.lm_mask[l];
        for (int a = 0; m; a++) {
            const int h = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const double* H = c.blkH + (size_t)(b0 + a) * 18;
            for (int i = 0; i < 3; i++) {
                double s = 0;
                for (int j = 0; j < 6; j++) s += H[6 * i + j] * (-c.y[6 * h + j]);
                cl[i] += s;
            }
        }
        const double* Di = c.Dinv + 9 * l;
        for (int i = 0; i < 3; i++) c.xl[3 * l + i] = (Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1]) + Di[3 * i + 2] * cl[2];
    }
    __syncthreads();
    mark(S, 6);
    return true;
}

__device__ void push_state(Ctx& c, Shared& S) {
    for (int i = threadIdx.x; i < 7 * c.K; i += kThreads) c.pose_b[i] = c.pose[i];
    for (int i = threadIdx.x; i < 3 * c.Np; i += kThreads) c.X_b[i] = c.X[i];
    for (int i = threadIdx.x; i < 4 * c.Nq; i += kThreads) c.P_b[i] = c.P[i];
    __syncthreads();
}
__device__ void pop_state(Ctx& c, Shared& S) {
    for (int i = threadIdx.x; i < 7 * c.K; i += kThreads) c.pose[i] = c.pose_b[i];
    for (int i = threadIdx.x; i < 3 * c.Np; i += kThreads) c.X[i] = c.X_b[i];
    for (int i = threadIdx.x; i < 4 * c.Nq; i += kThreads) c.P[i] = c.P_b[i];
    __syncthreads();
}
__device__ void apply_update(Ctx& c, Shared& S) {
    const int t = threadIdx.x;
    if (t < S.np) {
        const int k = S.hidx_pose[t];
        double u[6];
        for (int j = 0; j < 6; j++) u[j] = c.y[6 * t + j];
        store_pose(c.pose + 7 * k, se3_mul(se3_exp(u), load_pose(c.pose + 7 * k)));
    }
    for (int l = t; l < c.L; l += kThreads) {
        if (lm_block_base(c, l) < 0) continue;
        const double* u = c.xl + 3 * l;
        if (l < c.Np) {
            for (int j = 0; j < 3; j++) c.X[3 * l + j] += u[j];
        } else {
            double* pp = c.P + 4 * (l - c.Np);
            P4 P{{pp[0], pp[1], pp[2], pp[3]}};
            p_oplus(P, u);
            for (int j = 0; j < 4; j++) pp[j] = P.c[j];
        }
    }
    __syncthreads();
}
// computeScale: sum x (lambda x + b) over poses then landmarks
__device__ double step_scale(Ctx& c, double lam, Shared& S) {
    double acc[1] = {0.0};
    const int n = 6 * S.np;
    for (int i = threadIdx.x; i < n; i += kThreads) acc[0] += c.y[i] * (lam * c.y[i] + c.bp[i]);
    for (int l = threadIdx.x; l < c.L; l += kThreads) {
        if (lm_block_base(c, l) < 0) continue;
        for (int j = 0; j < 3; j++) acc[0] += c.xl[3 * l + j] * (lam * c.xl[3 * l + j] + c.lmb[3 * l + j]);
    }
    block_sum(acc, S);
    return acc[0];
}

// SparseOptimizer::optimize(iterations), OptimizationAlgorithmLevenberg.
__device__ int optimize(Ctx& c, const LbaConsts& C, bool robust, int iterations, Shared& S) {
    if (S.np == 0 && c.L == 0) return 0;
    int its = 0;
    for (int it = 0; it < iterations; it++) {
        mark(S, 7);
        const double chi = active_chi2(c, C, robust, S);
        mark(S, 1);
        if (threadIdx.x == 0) { S.currentChi = chi; S.iniChi = chi; }
        const double mx = build_system(c, C, robust, S);
        mark(S, 3);
        if (threadIdx.x == 0 && it == 0) { S.lambda = 1e-5 * mx; S.ni = 2; S.nBad = 0; }
        if (threadIdx.x == 0) S.qmax = 0;
        __syncthreads();
        double rho = 0;
        do {
            push_state(c, S);
            mark(S, 7);
            const bool ok = solve(c, S.lambda, S);
            if (ok) apply_update(c, S);
            mark(S, 7);
            const double tempChi0 = active_chi2(c, C, robust, S);
            mark(S, 1);
            const double scale = ok ? step_scale(c, S.lambda, S) : 0.0;
            if (threadIdx.x == 0) {
                const double tempChi = ok ? tempChi0 : DBL_MAX;
                rho = (S.currentChi - tempChi) / (scale + 1e-3);
                if (rho > 0 && isfinite(tempChi)) {
                    double alpha = 1. - pow((2 * rho - 1), 3);
                    alpha = fmin(alpha, 2. / 3.);
                    S.lambda *= fmax(1. / 3., alpha);
                    S.ni = 2;
                    S.currentChi = tempChi;
                    S.ok = 1;
                } else {
                    S.lambda *= S.ni;
                    S.ni *= 2;
                    S.ok = 0;
                }
                S.qmax++;
                S.trials++;
                S.rho = rho;
            }
            __syncthreads();
            rho = S.rho;
            if (!S.ok) pop_state(c, S);
        } while (rho < 0 && S.qmax < 10);
        its++;
        if (S.qmax == 10 || rho == 0) break;
        if (threadIdx.x == 0) {
            if ((S.iniChi - S.currentChi) * 1e3 < S.iniChi) S.nBad++;
            else S.nBad = 0;
        }
        __syncthreads();
        if (S.nBad >= 3) break;
    }
    return its;
}

__global__ __launch_bounds__(kThreads) void lba_kernel(
    const spslam_lba_problem* __restrict__ probs, const long long* __restrict__ scratch_off,
    const spslam_lba_keyframe* __restrict__ kfs, const spslam_lba_point* __restrict__ pts,
    const spslam_lba_point_obs* __restrict__ pobs, const spslam_lba_plane* __restrict__ pls,
    const spslam_lba_plane_obs* __restrict__ plobs, LbaConsts C, uint8_t* __restrict__ scratch,
    float* __restrict__ kf_out, float* __restrict__ pt_out, float* __restrict__ pl_out,
    uint8_t* __restrict__ pobs_out, uint8_t* __restrict__ plobs_out, spslam_lba_result* __restrict__ res) {
    __shared__ Shared S;
    const spslam_lba_problem pb = probs[blockIdx.x];
    const int t = threadIdx.x;
    Ctx c;
    c.K = pb.n_kf; c.Np = pb.n_points; c.Nq = pb.n_planes;
    c.Ep = pb.n_point_obs; c.E = pb.n_point_obs + pb.n_plane_obs; c.L = c.Np + c.Nq;
    c.kf = kfs + pb.kf_offset; c.pt = pts + pb.point_offset; c.pl = pls + pb.plane_offset;
    c.pobs = pobs; c.plobs = plobs;
    spslam_lba_result* R = res + blockIdx.x;
    if (t < 8) S.t_phase[t] = 0;
    if (t == 0) { S.t_mark = wall_clock64(); S.trials = 0; }
    __syncthreads();
    if (c.K > kLbaMaxKeyframes) {
        if (t == 0) { R->status = -2; R->iterations[0] = R->iterations[1] = 0; }
        return;
    }
    const LbaLayout Ly = lba_layout(c.K, c.Np, c.Nq, c.E);
    uint8_t* base = scratch + scratch_off[blockIdx.x];
    c.pose = (double*)(base + Ly.pose); c.pose_b = (double*)(base + Ly.pose_b);
    c.X = (double*)(base + Ly.pt); c.X_b = (double*)(base + Ly.pt_b);
    c.P = (double*)(base + Ly.pl); c.P_b = (double*)(base + Ly.pl_b);
    c.err = (double*)(base + Ly.e_err); c.con = (double*)(base + Ly.e_con);
    c.lmH = (double*)(base + Ly.lm_H); c.lmb = (double*)(base + Ly.lm_b); c.Dinv = (double*)(base + Ly.lm_Dinv);
    c.db = (double*)(base + Ly.lm_db); c.xl = (double*)(base + Ly.lm_x);
    c.blkH = (double*)(base + Ly.blk_H); c.blkBD = (double*)(base + Ly.blk_BD);
    c.S = (double*)(base + Ly.S); c.bs = (double*)(base + Ly.bs); c.dd = (double*)(base + Ly.dd);
    c.y = (double*)(base + Ly.y); c.Hpp = (double*)(base + Ly.Hpp); c.bp = (double*)(base + Ly.bp);
    c.pose_hidx_g = (int*)(base + Ly.pose_hidx); c.hidx_pose_g = (int*)(base + Ly.hidx_pose);
    c.e_lm = (int*)(base + Ly.e_lm); c.e_kf = (int*)(base + Ly.e_kf); c.e_type = (int*)(base + Ly.e_type);
    c.e_level = (int*)(base + Ly.e_level); c.e_blk = (int*)(base + Ly.e_blk); c.e_src = (int*)(base + Ly.e_src);
    c.lm_boff = (int*)(base + Ly.lm_boff); c.lm_nb = (int*)(base + Ly.lm_nb); c.blk_pose = (int*)(base + Ly.blk_pose);
    c.lm_act = (int*)(base + Ly.lm_act); c.lm_mask = (uint64_t*)(base + Ly.lm_mask);

    // ---- vertices: Converter::toSE3Quat / toVector3d / toPlane3D
    for (int k = t; k < c.K; k += kThreads) {
        const float* T = c.kf[k].Tcw;
        M3 Rm;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) Rm.a[3 * i + j] = T[4 * i + j];
        SE3 s;
        s.r = q_from_rot(Rm);
        s.t = V3{T[3], T[7], T[11]};
        q_normalize(s.r);
        store_pose(c.pose + 7 * k, s);
    }
    for (int i = t; i < c.Np; i += kThreads)
        for (int j = 0; j < 3; j++) c.X[3 * i + j] = c.pt[i].xw[j];
    for (int i = t; i < c.Nq; i += kThreads) {
        const P4 p = plane_from_f(c.pl[i].world);
        for (int j = 0; j < 4; j++) c.P[4 * i + j] = p.c[j];
    }
    // ---- edges in insertion order: point observations (points in list order), then plane observations
    {
        int base_e = 0;
        for (int ch = 0; ch < c.L; ch += kThreads) {
            const int l = ch + t;
            const int n_obs = l < c.Np ? c.pt[l].n_obs : (l < c.L ? c.pl[l - c.Np].n_obs : 0);
            int tot;
            const int off = block_scan(n_obs, &tot, S) + base_e;
            if (l < c.L) {
                c.lm_boff[l] = off;  // first edge of the landmark (edges contiguous)
                c.lm_nb[l] = n_obs;
                const int src0 = l < c.Np ? c.pt[l].obs_offset : c.pl[l - c.Np].obs_offset;
                for (int o = 0; o < n_obs; o++) {
                    const int e = off + o;
                    c.e_lm[e] = l;
                    c.e_src[e] = src0 + o;
                    c.e_level[e] = 0;
                    if (l < c.Np) {
                        const spslam_lba_point_obs& ob = c.pobs[src0 + o];
                        c.e_kf[e] = ob.kf;
                        c.e_type[e] = ob.ur < 0 ? 0 : 1;
                    } else {
                        const spslam_lba_plane_obs& ob = c.plobs[src0 + o];
                        c.e_kf[e] = ob.kf;
                        c.e_type[e] = ob.kind == SPSLAM_PLANE_EDGE ? 2 : (ob.kind == SPSLAM_PARALLEL_EDGE ? 3 : 4);
                    }
                }
            }
            base_e += tot;
        }
    }
    __syncthreads();
    int its[2] = {0, 0};
    mark(S, 0);
    if (c.E > 0) {
        for (int phase = 0; phase < 2; phase++) {
            initialize(c, S);
            mark(S, 0);
            its[phase] = optimize(c, C, phase == 0, phase == 0 ? 5 : 10, S);
            if (phase == 0) {  // relabel with the errors cached by the last computeActiveErrors
                for (int e = t; e < c.E; e += kThreads) {
                    double info[3];
                    info_of(c, C, e, info);
                    const int ty = c.e_type[e];
                    const double chi = chi2_of(c.err + 3 * e, info, edge_dim(ty));
                    bool bad;
                    if (ty == 0) bad = chi > 5.991 || !depth_positive(c, e);
                    else if (ty == 1) bad = chi > 7.815 || !depth_positive(c, e);
                    else if (ty == 2) bad = chi > C.plane_chi;
                    else bad = chi > C.vp_chi;
                    if (bad) c.e_level[e] = 1;
                }
                __syncthreads();
            }
        }
    }
    // ---- outlier flags (cached errors), write back
    int npo = 0, nplo = 0;
    for (int e = t; e < c.E; e += kThreads) {
        double info[3];
        info_of(c, C, e, info);
        const int ty = c.e_type[e];
        const double chi = chi2_of(c.err + 3 * e, info, edge_dim(ty));
        if (ty <= 1) {
            const bool bad = chi > (ty == 0 ? 5.991 : 7.815) || !depth_positive(c, e);
            pobs_out[c.e_src[e]] = bad;
            npo += bad;
        } else {
            const bool bad = ty == 2 ? chi > C.plane_chi : chi > C.vp_chi;
            plobs_out[c.e_src[e]] = bad;
            nplo += bad;
        }
    }
    double cnt[2] = {(double)npo, (double)nplo};
    block_sum(cnt, S);
    for (int k = t; k < c.K; k += kThreads) {
        float* o = kf_out + 16 * ((size_t)pb.kf_offset + k);
        if (c.kf[k].fixed) {
            for (int j = 0; j < 16; j++) o[j] = c.kf[k].Tcw[j];
            continue;
        }
        const SE3 T = load_pose(c.pose + 7 * k);
        const M3 Rm = q_to_rot(T.r);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) o[4 * i + j] = (float)Rm.a[3 * i + j];
        o[3] = (float)T.t.x; o[7] = (float)T.t.y; o[11] = (float)T.t.z;
        o[12] = 0.f; o[13] = 0.f; o[14] = 0.f; o[15] = 1.f;
    }
    for (int i = t; i < c.Np; i += kThreads)
        for (int j = 0; j < 3; j++) pt_out[3 * ((size_t)pb.point_offset + i) + j] = (float)c.X[3 * i + j];
    for (int i = t; i < c.Nq; i += kThreads)
        for (int j = 0; j < 4; j++) pl_out[4 * ((size_t)pb.plane_offset + i) + j] = (float)c.P[4 * i + j];
    if (t == 0) {
        R->iterations[0] = its[0];
        R->iterations[1] = its[1];
        R->n_point_outliers = (int)cnt[0];
        R->n_plane_outliers = (int)cnt[1];
        R->status = 0;
        R->trials = S.trials;
        for (int k = 0; k < 8; k++) R->phase_us[k] = (float)(S.t_phase[k] * 0.01);  // 100 MHz ticks
    }
}

}  // namespace lba

hipError_t lba_launch(int n, const spslam_lba_problem* d_probs, const long long* d_scratch_off,
                      const spslam_lba_keyframe* kfs, const spslam_lba_point* pts, const spslam_lba_point_obs* pobs,
                      const spslam_lba_plane* pls, const spslam_lba_plane_obs* plobs, const LbaConsts& C,
                      uint8_t* scratch, float* kf_out, float* pt_out, float* pl_out, uint8_t* pobs_out,
                      uint8_t* plobs_out, spslam_lba_result* res, hipStream_t s, KernelTimer* timer) {
    if (timer) timer->begin(kKindLba, s);
    hipLaunchKernelGGL(lba::lba_kernel, dim3(n), dim3(lba::kThreads), 0, s, d_probs, d_scratch_off, kfs, pts, pobs,
                       pls, plobs, C, scratch, kf_out, pt_out, pl_out, pobs_out, plobs_out, res);
    if (timer) timer->end(kKindLba, s);
    return hipGetLastError();
}

}  // namespace spslam
