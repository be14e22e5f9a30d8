// gfx950 PoseOptimization (reference: src/Optimizer.cc:519-1152 on the
// vendored g2o Levenberg-Marquardt + g2oAddition plane edges).
//
// One 256-thread workgroup per frame problem runs all 4 rounds x <= 10 LM
// iterations (x <= 10 trials) with no host round trip.  Per LM iteration:
//   pass A  (all threads)  per-edge error, Huber weight and Jacobian, the edge's
//                          robust chi2, lower J^T W J (21 terms) and J^T W e (6),
//                          staged in LDS a chunk of edges at a time
//   chain                  28 lanes add the staged terms edge by edge in g2o's
//                          insertion order (BlockSolver::buildSystem,
//                          SparseOptimizer::activeRobustChi2): the reference's
//                          sums, not a tree
//   solve   (lane q % K)   (H + lambda_q I) x = b by LDLT with diagonal pivoting
//                          (Eigen::LDLT, solvers/linear_solver_dense.h:103-110)
//                          for K damping trials at once, poses by readlane
//   pass B  (all threads)  robust chi2 of every edge at exp(x_q) * T for the K
//                          trials, chained in edge order by K lanes, then the
//                          reference's accept/reject walk, redundantly
// Outlier relabeling after each round reproduces the reference's use of the
// errors cached by the LAST computeActiveErrors (which may belong to a
// rejected trial): those errors are recomputed at that trial pose.
// All arithmetic is fp64 like g2o/Eigen, per edge in Eigen's expression
// structure (oracle/pose_oracle.cpp quadratic_form) with contraction off, and
// sin / cos / atan2 / pow(x, 3) are correctly rounded (libm64_cr.h): the
// oracle's default mode restates the same arithmetic and this kernel matches
// it bit for bit.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "wave_priority.h"

#include "../../include/spslam_gpu.h"
#include "g2o_device.h"
#include "pose_launch.h"

// Phase profile (diagnostic build only: make prof -> libspslam_gpu_prof.so).  Thread 0 of every problem
// accumulates wall_clock64 ticks (100 MHz) per phase; spslam_pose_prof_read returns the grid totals.
#ifdef SPSLAM_POSE_PROF
__device__ unsigned long long g_pose_prof[16];
#define PROF_MARK(k)                                   \
    do {                                               \
        if (t == 0) {                                  \
            const unsigned long long now_ = wall_clock64(); \
            prof_acc[k] += now_ - prof_t;              \
            prof_t = now_;                             \
        }                                              \
    } while (0)
#define PROF_COUNT(k) do { if (t == 0) prof_acc[k]++; } while (0)
#else
#define PROF_MARK(k) do {} while (0)
#define PROF_COUNT(k) do {} while (0)
#endif

namespace spslam {
namespace pose {

using namespace g2od;

struct Cam { double fx, fy, cx, cy, bf; };

__device__ __forceinline__ E3 point_error(const spslam_point_obs& o, const SE3& T, const Cam& c, V3& pc) {
    const V3 p = q_rot(T.r, V3{(double)o.xw[0], (double)o.xw[1], (double)o.xw[2]}) + T.t;
    pc = p;
    if (o.ur < 0) {
        return E3{(double)o.u - (p.x / p.z * c.fx + c.cx), (double)o.v - (p.y / p.z * c.fy + c.cy), 0.0};
    }
    const float invz = (float)(1.0f / p.z);  // float reciprocal, types_six_dof_expmap.cpp:300
    const double r0 = p.x * invz * c.fx + c.cx, r1 = p.y * invz * c.fy + c.cy;
    return E3{(double)o.u - r0, (double)o.v - r1, (double)o.ur - (r0 - c.bf * invz)};
}

// Eigen::LDLT (lower, diagonal pivoting) + solve on H + lambda I.  Returns
// false when the factor is not positive (LinearSolverDense::solve returns
// false, x unchanged).  Fully unrolled over the 6x6 matrix so that it lives in
// registers; the data-dependent pivot swaps are unrolled over the candidate
// rows, so the arithmetic (and its order) is exactly Eigen's unblocked LDLT.
__device__ __forceinline__ void swapd(double& a, double& b) { const double t = a; a = b; b = t; }

__device__ __forceinline__ bool ldlt_solve(const double (*H)[6], double lambda, const double* b, double* x) {
    constexpr int n = 6;
    double m[n][n];
#pragma unroll
    for (int i = 0; i < n; i++)
#pragma unroll
        for (int j = 0; j < n; j++) m[i][j] = i == j ? H[i][j] + lambda : H[i][j];
    int tr[n];
    int sign = 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = fabs(m[k][k]);
#pragma unroll
        for (int i = k + 1; i < n; i++)
            if (fabs(m[i][i]) > bv) { bv = fabs(m[i][i]); big = i; }
        tr[k] = big;
#pragma unroll
        for (int c = k + 1; c < n; c++) {
            if (big == c) {
#pragma unroll
                for (int j = 0; j < k; j++) swapd(m[k][j], m[c][j]);
#pragma unroll
                for (int i = c + 1; i < n; i++) swapd(m[i][k], m[i][c]);
                swapd(m[k][k], m[c][c]);
#pragma unroll
                for (int i = k + 1; i < c; ++i) swapd(m[i][k], m[c][i]);
            }
        }
        if (k > 0) {
            double temp[n];
#pragma unroll
            for (int j = 0; j < k; j++) temp[j] = m[j][j] * m[k][j];
            double s = 0;
#pragma unroll
            for (int j = 0; j < k; j++) s += m[k][j] * temp[j];
            m[k][k] -= s;
#pragma unroll
            for (int i = k + 1; i < n; i++) {
                double t = 0;
#pragma unroll
                for (int j = 0; j < k; j++) t += m[i][j] * temp[j];
                m[i][k] -= t;
            }
        }
        const double akk = m[k][k];
        const bool valid = fabs(akk) > 0;
        if (k == 0 && !valid) return false;
        if (k + 1 < n && valid) {
#pragma unroll
            for (int i = k + 1; i < n; i++) m[i][k] /= akk;
        }
        if (sign == 1) { if (akk < 0) sign = 3; }
        else if (sign == 2) { if (akk > 0) sign = 3; }
        else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
    }
    if (!(sign == 1 || sign == 0)) return false;
    double y[n];
#pragma unroll
    for (int i = 0; i < n; i++) y[i] = b[i];
#pragma unroll
    for (int k = 0; k < n; k++)
#pragma unroll
        for (int c = k + 1; c < n; c++)
            if (tr[k] == c) swapd(y[k], y[c]);
#pragma unroll
    for (int i = 0; i < n; i++)
#pragma unroll
        for (int j = 0; j < i; j++) y[i] -= m[i][j] * y[j];
#pragma unroll
    for (int i = 0; i < n; i++) y[i] = fabs(m[i][i]) > 2.2250738585072014e-308 ? y[i] / m[i][i] : 0.0;
#pragma unroll
    for (int i = n - 1; i >= 0; i--)
#pragma unroll
        for (int j = i + 1; j < n; j++) y[i] -= m[j][i] * y[j];
#pragma unroll
    for (int k = n - 1; k >= 0; k--)
#pragma unroll
        for (int c = k + 1; c < n; c++)
            if (tr[k] == c) swapd(y[k], y[c]);
#pragma unroll
    for (int i = 0; i < n; i++) x[i] = y[i];
    return true;
}

// Four waves per problem (measured: one wave per problem frees SIMDs for the
// pipelined extraction but makes the edge passes 4x longer -- a net loss).
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kRed = 28;  // robust chi2, 21 upper-triangle H terms, 6 b terms
constexpr int kPlaneChunk = 64;  // plane edges whose 13 errors (12 perturbed poses + T) are evaluated together
constexpr int kMaxTrials = 10;   // OptimizationAlgorithmLevenberg: qmax < 10

constexpr int kStage = 256;      // edges per chained chunk
constexpr int kStageStride = kRed + 1;  // odd stride in doubles: the 64 lanes' row writes spread over the banks

template <int kSpec>
struct Shared {
    double stage[kStage][kStageStride];  // per-edge terms of one chunk (pass A: 28, pass B: kSpec)
    double tot[kRed];                 // the chained totals, for every thread
    double red[2][kWaves][kRed];      // wave totals of the workgroup sums, double-buffered
    double perr[kPlaneChunk][13][3];  // plane errors at the 12 perturbed poses and at T
    double perrB[kPlaneChunk][kSpec][3];  // plane errors at the trial poses of the last pass B
    double perrT[kPlaneChunk][3];     // plane errors at the accepted trial pose = the next iteration's T
    double hb[kRed];                  // the iteration's H (lower, 21) and b (6), slot 0 unused
    SE3 tlast[kWaves];                // each wave's copy of the last trial pose (the relabel's active-edge pose)
    SE3 Eadd[12];                     // exp(+-1e-9 e_d), d = 0..5 (numeric Jacobian steps)
};

// Workgroup sum of NV doubles per thread; every thread returns the same totals.  Fixed order (the oracle's
// device-order mode restates it, oracle/pose_oracle.cpp): xor butterfly over the 64 lanes of each wave (all
// lanes end with the wave total), then ((0 + w0) + w1) + w2) + w3 from LDS in every thread.  One barrier;
// consecutive calls alternate the two LDS buffers, so a buffer is only rewritten after the next call's
// barrier has seen every thread finish reading it.
template <int NV, class Sh>
__device__ __forceinline__ void wg_sum(double (&v)[NV], Sh& S, int& buf) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int k = 0; k < NV; k++) v[k] += __shfl_xor(v[k], off);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; k++) S.red[buf][w][k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; k++) {
        double s = 0;
#pragma unroll
        for (int j = 0; j < kWaves; j++) s += S.red[buf][j][k];
        v[k] = s;
    }
    buf ^= 1;
}

__device__ __forceinline__ void huber(double chi, double delta, bool on, double* rho0, double* rho1) {
    const double dsqr = delta * delta;
    if (!on || chi <= dsqr) { *rho0 = chi; *rho1 = 1.0; return; }
    const double s = sqrt(chi);
    *rho0 = 2 * s * delta - dsqr;
    *rho1 = delta / s;
}

// acc += col[0], col[stride], ... col[(cnt - 1) stride] one after the other (the reference's order); the
// loads of the next group of 8 are in flight while the current group's dependent adds run (the prefetch past
// the last group reads stage rows that are never used -- unconditional, so the waits stay per group)
__device__ __forceinline__ void chain_add(double& acc, const double* col, int cnt) {
    static_assert((kStage & (kStage - 1)) == 0, "row wrap");
    const int full = cnt & ~7;
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = col[k * kStageStride];
    for (int i = 0; i < full; i += 8) {
        double w[8];
#pragma unroll
        for (int k = 0; k < 8; k++) w[k] = col[((i + 8 + k) & (kStage - 1)) * kStageStride];
#pragma unroll
        for (int k = 0; k < 8; k++) acc += v[k];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = w[k];
    }
    for (int i = full; i < cnt; i++) acc += col[i * kStageStride];
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ SE3 readlane_se3(const SE3& a, int l) {
    SE3 r;
    r.r.w = readlane_d(a.r.w, l); r.r.x = readlane_d(a.r.x, l);
    r.r.y = readlane_d(a.r.y, l); r.r.z = readlane_d(a.r.z, l);
    r.t.x = readlane_d(a.t.x, l); r.t.y = readlane_d(a.t.y, l); r.t.z = readlane_d(a.t.z, l);
    return r;
}

}  // namespace pose

using namespace pose;

// Every thread holds the whole LM state (pose, lambda, chi2 values, H, b): the workgroup sums hand every
// thread the same totals and every decision is computed redundantly from them, so no thread waits on another
// except inside wg_sum.  The damping trials of one LM iteration are evaluated kSpec at a time: after a
// rejected trial the reference only multiplies lambda by ni and doubles ni (optimization_algorithm_levenberg
// .cpp:145-160), so trial q's lambda is known in advance; lane q % kSpec of every wave solves trial q, the
// trial poses are broadcast with readlane, one pass over the edges evaluates all kSpec robust chi2 sums, and
// the accept / reject walk then replays the reference's sequence over them.  Results do not depend on kSpec.
#ifndef SPSLAM_POSE_MINW
#define SPSLAM_POSE_MINW 1  // waves per SIMD the register allocation leaves room for
#endif
template <int kSpec>
__global__ __launch_bounds__(kThreads, SPSLAM_POSE_MINW) void pose_kernel(const spslam_pose_problem* __restrict__ probs,
                                                         const spslam_point_obs* __restrict__ pts_all,
                                                         const spslam_plane_obs* __restrict__ pls_all, PoseConsts K,
                                                         const spslam_pose_result* __restrict__ init_from,
                                                         spslam_pose_result* __restrict__ results,
                                                         uint8_t* __restrict__ pout_all, uint8_t* __restrict__ plout_all) {
    tail_wave_priority();
    __shared__ Shared<kSpec> S;
    const int t = threadIdx.x, lane = t & 63;
#ifdef SPSLAM_POSE_PROF
    unsigned long long prof_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long prof_t = wall_clock64();
#endif
    const spslam_pose_problem P = probs[blockIdx.x];
    const spslam_point_obs* pts = pts_all + P.point_offset;
    const spslam_plane_obs* pls = pls_all + P.plane_offset;
    uint8_t* pout = pout_all + P.point_offset;
    uint8_t* plout = plout_all + P.plane_offset;
    spslam_pose_result* res = results + blockIdx.x;
    const float* Tin = init_from ? init_from[blockIdx.x].Tcw : probs[blockIdx.x].Tcw;
    const int np = P.n_points, nl = P.n_planes, ne = np + nl;
    const Cam cam{P.fx, P.fy, P.cx, P.cy, P.bf};

    for (int i = t; i < np; i += kThreads) pout[i] = 0;
    for (int i = t; i < nl; i += kThreads) plout[i] = 0;
    if (np < 3) {  // nInitialCorrespondences < 3 (:653): no SetPose
        if (t < 16) res->Tcw[t] = Tin[t];
        if (t == 0) { res->n_inliers = 0; res->lm_iterations = 0; }
        return;
    }
    if (t < 12 && nl > 0) {
        double add[6] = {0, 0, 0, 0, 0, 0};
        add[t >> 1] = (t & 1) ? -1e-9 : 1e-9;
        S.Eadd[t] = se3_exp(add);
    }
    SE3 T0;  // Converter::toSE3Quat: Quaterniond(R) of the float pose, normalized (every thread)
    {
        M3 R;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R.a[3 * i + j] = Tin[4 * i + j];
        T0.r = q_from_rot(R);
        T0.t = V3{Tin[3], Tin[7], Tin[11]};
        q_normalize(T0.r);
    }
    __syncthreads();

    // edge e < np: point e; else plane e - np.  Per-edge info/delta:
    auto edge_info = [&](int e, double* info, double* delta) __attribute__((always_inline)) {
        if (e < np) {
            const spslam_point_obs& o = pts[e];
            info[0] = info[1] = info[2] = (double)o.inv_sigma2;
            *delta = o.ur < 0 ? K.delta_mono : K.delta_stereo;
        } else {
            const int kind = pls[e - np].kind;
            if (kind == 0) { info[0] = info[1] = K.angle_info; info[2] = K.dis_info; *delta = K.delta_plane; }
            else { info[0] = info[1] = kind == 1 ? K.par_info : K.ver_info; info[2] = 0; *delta = K.delta_vp; }
        }
    };
    auto plane_of = [&](int e, P4& w, P4& m) __attribute__((always_inline)) {
        const spslam_plane_obs& o = pls[e - np];
        for (int k = 0; k < 4; k++) { w.c[k] = o.world[k]; m.c[k] = o.meas[k]; }
        if (o.world[3] < 0.0f) for (int k = 0; k < 4; k++) w.c[k] = -w.c[k];  // Converter::toPlane3D
        if (o.meas[3] < 0.0f) for (int k = 0; k < 4; k++) m.c[k] = -m.c[k];
        p_normalize(w.c);
        p_normalize(m.c);
    };
    auto error_at = [&](int e, const SE3& T, double* err, V3* pc) __attribute__((always_inline)) {
        E3 r;
        if (e < np) {
            V3 p;
            r = point_error(pts[e], T, cam, p);
            if (pc) *pc = p;
        } else {
            P4 w, m;
            plane_of(e, w, m);
            r = plane_error3(pls[e - np].kind, T, w, m);
        }
        err[0] = r.e0; err[1] = r.e1; err[2] = r.e2;
    };
    auto chi2_of = [](const double* err, const double* info) __attribute__((always_inline)) {
        // e . (Omega e) (base_edge.h chi2); rows beyond the edge's dimension hold a zero error: their +0 terms
        // leave chi unchanged
        return (err[0] * (info[0] * err[0]) + err[1] * (info[1] * err[1])) + err[2] * (info[2] * err[2]);
    };
    auto is_outlier = [&](int e) __attribute__((always_inline)) -> bool { return e < np ? pout[e] != 0 : plout[e - np] != 0; };

    int buf = 0;
    bool robust = true;
    int nBad = 0, total_its = 0;
    SE3 T;
    for (int round = 0; round < 4; round++) {
        PROF_MARK(0);  // setup / previous relabel
        T = T0;
        // any active edge?
        int act = 0;
        for (int e = t; e < ne; e += kThreads) act |= !is_outlier(e);
        act = __syncthreads_or(act);
        if (act) {
            double lambda = 0, ni = 2;
            int lmBad = 0;
            bool tValid = false;  // perrT holds the plane errors at T (set when a trial is accepted)
            for (int it = 0; it < 10; it++) {
                // ---- pass A: errors, robust chi2, quadratic form at T, chained in edge order
                // one edge's terms into row t of the stage: its robust chi2, the lower triangle of its
                // H_e (BaseUnaryEdge / BaseBinaryEdge::constructQuadraticForm in Eigen's order: the
                // temporary A^T (rho' Omega) times A) and -s_e with b -= s_e (unary: ((rho' A^T) Omega) e;
                // binary, pose = vertex 1: B^T (rho' Omega e))
                auto stage_terms = [&](const double (&J)[3][6], const double* err, const double* info, double delta,
                                       bool binary) __attribute__((always_inline)) {
                    double* row = S.stage[t];
                    double rho0, rho1;
                    huber(chi2_of(err, info), delta, robust, &rho0, &rho1);
                    row[0] = rho0;
                    double wo[3], q[3];
#pragma unroll
                    for (int r = 0; r < 3; r++) { wo[r] = rho1 * info[r]; q[r] = (info[r] * err[r]) * rho1; }
#pragma unroll
                    for (int i = 0; i < 6; i++)
#pragma unroll
                        for (int j = 0; j <= i; j++) {
                            double h = 0;
#pragma unroll
                            for (int r = 0; r < 3; r++) h += (J[r][i] * wo[r]) * J[r][j];
                            row[1 + i * (i + 1) / 2 + j] = h;
                        }
#pragma unroll
                    for (int i = 0; i < 6; i++) {
                        double sb = 0;
                        if (binary) {
#pragma unroll
                            for (int r = 0; r < 3; r++) sb += J[r][i] * q[r];
                        } else {
#pragma unroll
                            for (int r = 0; r < 3; r++) sb += ((rho1 * J[r][i]) * info[r]) * err[r];
                        }
                        row[22 + i] = -sb;
                    }
                };
                auto stage_zero = [&]() __attribute__((always_inline)) {
#pragma unroll
                    for (int k = 0; k < kRed; k++) S.stage[t][k] = 0.0;
                };
                // value k of the 28 is chained by lane k / 4 of wave k % 4
                const int ck = lane * kWaves + (t >> 6);
                const bool chainer = lane * kWaves < kRed;
                double achain = 0;
                for (int base = 0; base < np; base += kStage) {
                    const int e = base + t;
                    if (e < np && !pout[e]) {
                        double info[3], delta, err[3] = {0, 0, 0}, J[3][6];
                        edge_info(e, info, &delta);
                        V3 pc;
                        error_at(e, T, err, &pc);
                        const double x = pc.x, y = pc.y, invz = 1.0 / pc.z, invz_2 = invz * invz;
                        J[0][0] = x * y * invz_2 * cam.fx; J[0][1] = -(1 + (x * x * invz_2)) * cam.fx;
                        J[0][2] = y * invz * cam.fx; J[0][3] = -invz * cam.fx; J[0][4] = 0;
                        J[0][5] = x * invz_2 * cam.fx;
                        J[1][0] = (1 + y * y * invz_2) * cam.fy; J[1][1] = -x * y * invz_2 * cam.fy;
                        J[1][2] = -x * invz * cam.fy; J[1][3] = 0; J[1][4] = -invz * cam.fy;
                        J[1][5] = y * invz_2 * cam.fy;
                        if (pts[e].ur >= 0) {
                            J[2][0] = J[0][0] - cam.bf * y * invz_2; J[2][1] = J[0][1] + cam.bf * x * invz_2;
                            J[2][2] = J[0][2]; J[2][3] = J[0][3]; J[2][4] = 0; J[2][5] = J[0][5] - cam.bf * invz_2;
                        } else {
#pragma unroll
                            for (int d = 0; d < 6; d++) J[2][d] = 0;
                        }
                        stage_terms(J, err, info, delta, false);
                    } else {
                        stage_zero();
                    }
                    __syncthreads();
                    if (chainer) chain_add(achain, &S.stage[0][ck], min(kStage, np - base));
                    __syncthreads();
                }
                PROF_MARK(1);  // pass A point edges
                // plane edges: numeric central differences, delta 1e-9 (base_binary_edge.hpp:130-205); the 13
                // evaluations of a chunk's edges (12 perturbed poses exp(+-1e-9 e_d) * T, and T) run on
                // 13 x chunk threads, then thread j stages the chunk's edge j
                // after an accepted trial the errors at T are the ones pass B evaluated at that trial pose
                // (kept in perrT when the plane edges fit one chunk): 12 evaluations per edge instead of 13
                const bool haveT = tValid && nl <= kPlaneChunk;
                const int nev = haveT ? 12 : 13;
                for (int base = 0; base < nl; base += kPlaneChunk) {
                    const int cnt = min(kPlaneChunk, nl - base);
                    for (int w = t; w < cnt * nev; w += kThreads) {
                        const int j = w / nev, q = w - j * nev, e = np + base + j;
                        double err[3] = {0, 0, 0};
                        if (!plout[e - np]) {
                            const SE3 Tp = se3_mul(S.Eadd[q < 12 ? q : 0], T);
                            const bool pt = q < 12;
                            SE3 Tq;  // field-wise select: one inlined error evaluation for both cases
                            Tq.r.w = pt ? Tp.r.w : T.r.w; Tq.r.x = pt ? Tp.r.x : T.r.x;
                            Tq.r.y = pt ? Tp.r.y : T.r.y; Tq.r.z = pt ? Tp.r.z : T.r.z;
                            Tq.t.x = pt ? Tp.t.x : T.t.x; Tq.t.y = pt ? Tp.t.y : T.t.y; Tq.t.z = pt ? Tp.t.z : T.t.z;
                            error_at(e, Tq, err, nullptr);
                        }
                        S.perr[j][q][0] = err[0]; S.perr[j][q][1] = err[1]; S.perr[j][q][2] = err[2];
                    }
                    __syncthreads();
                    if (t < cnt) {
                        const int e = np + base + t;
                        if (!plout[e - np]) {
                            double info[3], delta, J[3][6];
                            edge_info(e, info, &delta);
                            const double err[3] = {haveT ? S.perrT[t][0] : S.perr[t][12][0],
                                                   haveT ? S.perrT[t][1] : S.perr[t][12][1],
                                                   haveT ? S.perrT[t][2] : S.perr[t][12][2]};
                            const double scalar = 1.0 / (2 * 1e-9);
#pragma unroll
                            for (int d = 0; d < 6; d++)
#pragma unroll
                                for (int r = 0; r < 3; r++)
                                    J[r][d] = scalar * (S.perr[t][2 * d][r] - S.perr[t][2 * d + 1][r]);
                            stage_terms(J, err, info, delta, true);
                        } else {
                            stage_zero();
                        }
                    }
                    __syncthreads();
                    if (chainer) chain_add(achain, &S.stage[0][ck], cnt);
                    __syncthreads();  // stage / perr reuse
                }
                PROF_MARK(2);  // pass A plane edges
                if (chainer) S.tot[ck] = achain;
                __syncthreads();
                double currentChi = S.tot[0];
                const double iniChi = currentChi;
                // H and b wait in LDS for the trial passes: kept in registers they would stay live across pass B
                const double* hbw = S.hb;
                if (t < kRed) S.hb[t] = S.tot[t];
                if (it == 0) {
                    double md = 0;
#pragma unroll
                    for (int j = 0; j < 6; j++) md = fmax(fabs(S.tot[1 + j * (j + 1) / 2 + j]), md);
                    lambda = 1e-5 * md;
                    ni = 2;
                    lmBad = 0;
                }
                __syncthreads();
                PROF_MARK(3);  // reduce A + iteration setup
                // ---- damping trials, kSpec per pass over the edges
                double rho = 0;
                int qmax = 0;
                bool more = true;
                while (more) {
                    // trial q's damping if trials 0..q-1 are rejected: lambda_{q+1} = lambda_q * ni_q, ni *= 2
                    double lam = lambda, nq = ni;
                    const int myq = lane % kSpec;
                    for (int q = 0; q < myq; q++) { lam *= nq; nq *= 2; }
                    double H[6][6], b[6];
                    {
                        int k = 1;
#pragma unroll
                        for (int i = 0; i < 6; i++)
#pragma unroll
                            for (int j = 0; j <= i; j++, k++) H[i][j] = H[j][i] = hbw[k];
#pragma unroll
                        for (int i = 0; i < 6; i++) b[i] = hbw[22 + i];
                    }
                    double x[6] = {0, 0, 0, 0, 0, 0};  // a failed LDLT leaves x unwritten (rejected step)
                    const bool ok = ldlt_solve(H, lam, b, x);
                    const SE3 Tt = se3_mul(se3_exp(x), T);
                    double scale = 0;  // OptimizationAlgorithmLevenberg::computeScale + 1e-3
#pragma unroll
                    for (int j = 0; j < 6; j++) scale += x[j] * (lam * x[j] + b[j]);
                    scale += 1e-3;
                    SE3 Tq[kSpec];
                    double sc[kSpec];
                    bool okq[kSpec];
#pragma unroll
                    for (int q = 0; q < kSpec; q++) {
                        Tq[q] = readlane_se3(Tt, q);
                        sc[q] = readlane_d(scale, q);
                        okq[q] = __builtin_amdgcn_readlane((int)ok, q) != 0;
                    }
                    PROF_MARK(4);  // solves + exp + broadcast
                    PROF_COUNT(10);
                    // robust chi2 of every active edge at each trial pose, chained in edge order by lane 0 of
                    // wave q.  A plane error costs far more than a point error, so the (plane edge, trial)
                    // pairs are evaluated one per thread first (into perr's space).
                    double* prho = &S.perr[0][0][0];
                    constexpr int kPairPlanes = kPlaneChunk * 13 * 3 / kSpec;  // plane edges per prho round
                    auto pairs = [&](int pb) __attribute__((always_inline)) {
                        const int cnt = min(kPairPlanes, nl - pb);
                        for (int w = t; w < cnt * kSpec; w += kThreads) {
                            const int j = pb + w / kSpec, q = w % kSpec;
                            double r0 = 0;
                            if (!plout[j]) {
                                double info[3], delta, err[3] = {0, 0, 0}, rho1;
                                edge_info(np + j, info, &delta);
                                SE3 Tv = Tq[0];  // uniform poses: select by q without dynamic indexing
#pragma unroll
                                for (int k = 1; k < kSpec; k++)
                                    if (q == k) Tv = Tq[k];
                                error_at(np + j, Tv, err, nullptr);
                                huber(chi2_of(err, info), delta, robust, &r0, &rho1);
                                if (nl <= kPlaneChunk) {
                                    S.perrB[j][q][0] = err[0]; S.perrB[j][q][1] = err[1]; S.perrB[j][q][2] = err[2];
                                }
                            }
                            prho[w] = r0;
                        }
                    };
                    pairs(0);
                    double cq = 0;
                    const bool qchainer = lane == 0 && (t >> 6) < kSpec;
                    for (int base = 0; base < np; base += kStage) {
                        const int e = base + t;
                        double r[kSpec];
#pragma unroll
                        for (int q = 0; q < kSpec; q++) r[q] = 0;
                        if (e < np && !pout[e]) {
                            double info[3], delta;
                            edge_info(e, info, &delta);
#pragma unroll
                            for (int q = 0; q < kSpec; q++) {
                                double err[3] = {0, 0, 0}, rho1;
                                error_at(e, Tq[q], err, nullptr);
                                huber(chi2_of(err, info), delta, robust, &r[q], &rho1);
                            }
                        }
#pragma unroll
                        for (int q = 0; q < kSpec; q++) S.stage[t][q] = r[q];
                        __syncthreads();
                        if (qchainer) chain_add(cq, &S.stage[0][t >> 6], min(kStage, np - base));
                        __syncthreads();
                    }
                    for (int pb = 0; pb < nl; pb += kPairPlanes) {
                        if (pb > 0) pairs(pb);  // prho's previous round was chained (the loop's last barrier)
                        __syncthreads();
                        const int cntp = min(kPairPlanes, nl - pb);
                        for (int sb = 0; sb < cntp; sb += kStage) {
#pragma unroll
                            for (int q = 0; q < kSpec; q++) S.stage[t][q] = sb + t < cntp ? prho[(sb + t) * kSpec + q] : 0.0;
                            __syncthreads();
                            if (qchainer) chain_add(cq, &S.stage[0][t >> 6], min(kStage, cntp - sb));
                            __syncthreads();
                        }
                    }
                    if (qchainer) S.tot[t >> 6] = cq;
                    PROF_MARK(5);  // pass B (trial chi2)
                    __syncthreads();
                    double c[kSpec];
#pragma unroll
                    for (int q = 0; q < kSpec; q++) c[q] = S.tot[q];
                // the reference's accept / reject sequence over the evaluated trials
                    int acc = -1, lastq = 0;
#pragma unroll
                    for (int q = 0; q < kSpec; q++) {
                        if (more) {
                            lastq = q;  // the last computeActiveErrors
                            const double tempChi = okq[q] ? c[q] : 1.7976931348623157e308;
                            double r = currentChi - tempChi;
                            r /= sc[q];
                            if (r > 0 && isfinite(tempChi)) {
                                double alpha = 1. - libm64cr::cube_(2 * r - 1);
                                alpha = fmin(alpha, 2. / 3.);
                                lambda *= fmax(1. / 3., alpha);
                                ni = 2;
                                currentChi = tempChi;
                                T = Tq[q];
                                acc = q;
                            } else {
                                lambda *= ni;
                                ni *= 2;
                            }
                            rho = r;
                            qmax++;
                            more = rho < 0 && qmax < kMaxTrials;
                        }
                    }
                    if (lane == 0) {
                        SE3 tl = Tq[0];
#pragma unroll
                        for (int q = 1; q < kSpec; q++)
                            if (q == lastq) tl = Tq[q];
                        S.tlast[t >> 6] = tl;
                    }
                    tValid = tValid || acc >= 0;
                    if (acc >= 0 && t < nl && nl <= kPlaneChunk) {  // thread t reads perrT[t] in the next pass A
#pragma unroll
                        for (int q = 0; q < kSpec; q++)
                            if (q == acc) {
                                S.perrT[t][0] = S.perrB[t][q][0];
                                S.perrT[t][1] = S.perrB[t][q][1];
                                S.perrT[t][2] = S.perrB[t][q][2];
                            }
                    }
                    PROF_MARK(6);  // reduce B + decide
                }
                total_its++;
                if (qmax == kMaxTrials || rho == 0) break;
                if ((iniChi - currentChi) * 1e3 < iniChi) lmBad++;
                else lmBad = 0;
                PROF_MARK(7);  // stop test
                PROF_COUNT(11);
                if (lmBad >= 3) break;
            }
        }
        // ---- relabel (:925-1140): active edges keep the errors of the last trial pose, outliers are
        // recomputed at the optimized pose
        // (with no active edge every edge takes T and tlast is not read)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const SE3 Tlast = S.tlast[t >> 6];
        double bad = 0;
        for (int e = t; e < ne; e += kThreads) {
            double info[3], delta, err[3] = {0, 0, 0};
            edge_info(e, info, &delta);
            const bool was_out = is_outlier(e);
            SE3 Te;  // field-wise select (a selected reference would put both poses in scratch memory)
            Te.r.w = was_out ? T.r.w : Tlast.r.w; Te.r.x = was_out ? T.r.x : Tlast.r.x;
            Te.r.y = was_out ? T.r.y : Tlast.r.y; Te.r.z = was_out ? T.r.z : Tlast.r.z;
            Te.t.x = was_out ? T.t.x : Tlast.t.x; Te.t.y = was_out ? T.t.y : Tlast.t.y; Te.t.z = was_out ? T.t.z : Tlast.t.z;
            error_at(e, Te, err, nullptr);
            const float chi2 = (float)chi2_of(err, info);
            bool bd;
            if (e < np) bd = pts[e].ur < 0 ? chi2 > 5.991f : chi2 > 7.815f;
            else bd = pls[e - np].kind == 0 ? (double)chi2 > K.plane_chi : (double)chi2 > K.vp_chi;
            bad += bd ? 1.0 : 0.0;
            if (e < np) pout[e] = bd;
            else plout[e - np] = bd;
        }
        double cb[1] = {bad};
        wg_sum(cb, S, buf);  // small integers: exact
        nBad = (int)cb[0];
        PROF_MARK(8);  // relabel
        if (round == 2) robust = false;
        if (ne < 10) break;
    }
    if (t == 0) {
        const M3 R = q_to_rot(T.r);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) res->Tcw[4 * i + j] = (float)R.a[3 * i + j];
        res->Tcw[3] = (float)T.t.x; res->Tcw[7] = (float)T.t.y; res->Tcw[11] = (float)T.t.z;
        res->Tcw[12] = 0.f; res->Tcw[13] = 0.f; res->Tcw[14] = 0.f; res->Tcw[15] = 1.f;
        res->n_inliers = ne - nBad;
        res->lm_iterations = total_its;
    }
#ifdef SPSLAM_POSE_PROF
    PROF_MARK(9);  // outputs
    if (t == 0)
        for (int k = 0; k < 12; k++) atomicAdd(&g_pose_prof[k], prof_acc[k]);
#endif
}


// test hook (spslam_debug_libm64): the correctly rounded routines as the pose / LBA kernels run them
__global__ void libm64_debug_kernel(int kind, const double* __restrict__ a, const double* __restrict__ b, int n,
                                    double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = a[i];
    double r;
    if (kind == 0) r = libm64cr::sin_(x);
    else if (kind == 1) r = libm64cr::cos_(x);
    else if (kind == 2) r = libm64cr::atan2_(x, b[i]);
    else r = libm64cr::cube_(x);
    out[i] = r;
}

hipError_t libm64_debug_launch(int kind, const double* a, const double* b, int n, double* out, hipStream_t s) {
    if (n < 1) return hipSuccess;
    hipLaunchKernelGGL(libm64_debug_kernel, dim3((n + 255) / 256), dim3(256), 0, s, kind, a, b, n, out);
    return hipGetLastError();
}

PoseConsts make_pose_consts(const spslam_plane_config& c) {
    PoseConsts K;
    K.delta_mono = (double)(float)sqrt(5.991);
    K.delta_stereo = (double)(float)sqrt(7.815);
    K.angle_info = 3282.8 / (c.angle_info * c.angle_info);
    K.dis_info = c.distance_info * c.distance_info;
    K.par_info = 3282.8 / (c.parallel_info * c.parallel_info);
    K.ver_info = 3282.8 / (c.vertical_info * c.vertical_info);
    K.plane_chi = c.chi;
    K.vp_chi = c.vp_chi;
    K.delta_plane = (double)(float)sqrt(c.chi);
    K.delta_vp = (double)(float)sqrt(c.vp_chi);
    return K;
}

hipError_t pose_launch(int n, const spslam_pose_problem* probs, const spslam_point_obs* pts,
                       const spslam_plane_obs* pls, const PoseConsts& K, const spslam_pose_result* init_from,
                       spslam_pose_result* res, uint8_t* pout, uint8_t* plout, hipStream_t s) {
    static const int spec = [] {
        const char* e = std::getenv("SPSLAM_POSE_SPEC");  // measurement knob: damping trials per edge pass
        return e ? std::atoi(e) : 4;
    }();
    if (spec <= 1)
        hipLaunchKernelGGL(pose_kernel<1>, dim3(n), dim3(kThreads), 0, s, probs, pts, pls, K, init_from, res, pout, plout);
    else if (spec == 2)
        hipLaunchKernelGGL(pose_kernel<2>, dim3(n), dim3(kThreads), 0, s, probs, pts, pls, K, init_from, res, pout, plout);
    else
        hipLaunchKernelGGL(pose_kernel<4>, dim3(n), dim3(kThreads), 0, s, probs, pts, pls, K, init_from, res, pout, plout);
    return hipGetLastError();
}

}  // namespace spslam

#ifdef SPSLAM_POSE_PROF
// Diagnostic build only: the accumulated phase ticks / counters (12 u64), optionally reset.
extern "C" int spslam_pose_prof_read(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pose_prof), 12 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pose_prof), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
