// gfx950 PoseOptimization (reference: src/Optimizer.cc:519-1152 on the
// vendored g2o Levenberg-Marquardt + g2oAddition plane edges).
//
// One 256-thread workgroup per frame problem runs all 4 rounds x <= 10 LM
// iterations (x <= 10 trials) with no host round trip.  Per LM iteration:
//   pass A  (all threads)  per-edge error, Huber weight and Jacobian, local
//                          sums of robust chi2, J^T W J (21 terms), J^T W e (6)
//   reduce                 wave shuffles + LDS, fp64
//   solve   (thread 0)     (H + lambda I) x = b by LDLT with diagonal pivoting
//                          (Eigen::LDLT, solvers/linear_solver_dense.h:103-110)
//   pass B  (all threads)  robust chi2 at exp(x) * T, accept/reject, lambda
// Outlier relabeling after each round reproduces the reference's use of the
// errors cached by the LAST computeActiveErrors (which may belong to a
// rejected trial): those errors are recomputed at that trial pose.
// All arithmetic is fp64 like g2o/Eigen; reductions are tree-ordered, so the
// result matches the reference to rounding, not bitwise.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "wave_priority.h"

#include "../../include/spslam_gpu.h"
#include "g2o_device.h"
#include "pose_launch.h"

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
        for (int j = 0; j < n; j++) m[i][j] = H[i][j] + (i == j ? lambda : 0.0);
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
constexpr int kRed = 28;  // robust chi2, 21 upper-triangle H terms, 6 b terms
constexpr int kPlaneChunk = 64;  // plane edges whose 12 perturbed errors are evaluated together

struct Shared {
    double red[kThreads / 64][kRed];
    SE3 Eadd[12];                    // exp(+-1e-9 e_d), d = 0..5 (numeric Jacobian steps)
    SE3 Tp[12];                      // exp(+-1e-9 e_d) * T for the current iterate
    double perr[kPlaneChunk][13][3]; // plane errors at the 12 perturbed poses and at T
    double H[6][6], b[6], x[6];
    double lambda, ni, currentChi, iniChi, tempChi;
    SE3 T, T0, Ttrial, Tlast;
    int nBad, stop, active_any;
    int count[kThreads / 64];
};

// Block reduction of NV doubles per thread (v[0..NV)) into S.red[0][0..NV).  The
// NV butterfly chains are unrolled together so their shuffle latencies overlap.
template <int NV>
__device__ void block_reduce(double (&v)[NV], Shared& S) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double x[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) x[k] = v[k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int k = 0; k < NV; k++) x[k] += __shfl_xor(x[k], off);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; k++) S.red[w][k] = x[k];
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        double s = 0;
        for (int j = 0; j < kThreads / 64; j++) s += S.red[j][threadIdx.x];
        S.red[0][threadIdx.x] = s;
    }
    __syncthreads();
}

__device__ __forceinline__ void huber(double chi, double delta, bool on, double* rho0, double* rho1) {
    const double dsqr = delta * delta;
    if (!on || chi <= dsqr) { *rho0 = chi; *rho1 = 1.0; return; }
    const double s = sqrt(chi);
    *rho0 = 2 * s * delta - dsqr;
    *rho1 = delta / s;
}

}  // namespace pose

using namespace pose;

// kMinWaves: waves per SIMD the register allocation must leave room for (launch-bounds occupancy).  At 1 the
// kernel takes 256 VGPRs + AGPRs, so a workgroup only starts on a CU whose four SIMDs are nearly empty --
// inside the pipelined step that waits for the extraction kernels' waves to drain.
template <int kMinWaves>
__global__ __launch_bounds__(kThreads, kMinWaves) void pose_kernel(const spslam_pose_problem* __restrict__ probs,
                                                   const spslam_point_obs* __restrict__ pts_all,
                                                   const spslam_plane_obs* __restrict__ pls_all, PoseConsts K,
                                                   const spslam_pose_result* __restrict__ init_from,
                                                   spslam_pose_result* __restrict__ results,
                                                   uint8_t* __restrict__ pout_all, uint8_t* __restrict__ plout_all) {
    tail_wave_priority();
    __shared__ Shared S;
    const int t = threadIdx.x;
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
    if (t == 0) {
        M3 R;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R.a[3 * i + j] = Tin[4 * i + j];
        S.T0.r = q_from_rot(R);
        S.T0.t = V3{Tin[3], Tin[7], Tin[11]};
        q_normalize(S.T0.r);
    }
    __syncthreads();

    // edge e < np: point e; else plane e - np.  Per-edge info/delta:
    auto edge_info = [&](int e, double* info, double* delta, int* dim) __attribute__((always_inline)) {
        if (e < np) {
            const spslam_point_obs& o = pts[e];
            info[0] = info[1] = info[2] = (double)o.inv_sigma2;
            *dim = o.ur < 0 ? 2 : 3;
            *delta = o.ur < 0 ? K.delta_mono : K.delta_stereo;
        } else {
            const int kind = pls[e - np].kind;
            if (kind == 0) { info[0] = info[1] = K.angle_info; info[2] = K.dis_info; *delta = K.delta_plane; *dim = 3; }
            else { info[0] = info[1] = kind == 1 ? K.par_info : K.ver_info; info[2] = 0; *delta = K.delta_vp; *dim = 2; }
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
    auto is_outlier = [&](int e) __attribute__((always_inline)) -> bool { return e < np ? pout[e] != 0 : plout[e - np] != 0; };

    bool robust = true;
    int nBad = 0, total_its = 0;
    for (int round = 0; round < 4; round++) {
        if (t == 0) S.T = S.T0;
        // any active edge?
        int act = 0;
        for (int e = t; e < ne; e += kThreads) act |= !is_outlier(e);
        act = __syncthreads_or(act);
        if (act) {
            for (int it = 0; it < 10; it++) {
                // ---- pass A: errors, robust chi2, quadratic form at T
                double v[kRed];
#pragma unroll
                for (int k = 0; k < kRed; k++) v[k] = 0;
                const SE3 T = S.T;
                // accumulate one edge's robust chi2, J^T W J and -J^T W e
                auto accumulate = [&](const double (&J)[3][6], const double* err, const double* info, int dim,
                                      double delta) {
                    // rows beyond dim carry zero error and Jacobian: their terms add exact zeros
                    (void)dim;
                    double chi = 0;
                    chi = (err[0] * info[0] * err[0] + err[1] * info[1] * err[1]) + err[2] * info[2] * err[2];
                    double rho0, rho1;
                    huber(chi, delta, robust, &rho0, &rho1);
                    v[0] += rho0;
#pragma unroll
                    for (int i = 0; i < 6; i++)
#pragma unroll
                        for (int j = i; j < 6; j++) {
                            double s = 0;
#pragma unroll
                            for (int r = 0; r < 3; r++) s += J[r][i] * (rho1 * info[r]) * J[r][j];
                            v[1 + i * 6 - i * (i - 1) / 2 + (j - i)] += s;
                        }
#pragma unroll
                    for (int i = 0; i < 6; i++) {
                        double s = 0;
#pragma unroll
                        for (int r = 0; r < 3; r++) s += rho1 * J[r][i] * (info[r] * err[r]);
                        v[22 + i] -= s;
                    }
                };
                for (int e = t; e < np; e += kThreads) {
                    if (pout[e]) continue;
                    double info[3], delta, err[3] = {0, 0, 0}, J[3][6];
                    int dim;
                    edge_info(e, info, &delta, &dim);
                    V3 pc;
                    error_at(e, T, err, &pc);
                    const double x = pc.x, y = pc.y, invz = 1.0 / pc.z, invz_2 = invz * invz;
                    J[0][0] = x * y * invz_2 * cam.fx; J[0][1] = -(1 + (x * x * invz_2)) * cam.fx;
                    J[0][2] = y * invz * cam.fx; J[0][3] = -invz * cam.fx; J[0][4] = 0;
                    J[0][5] = x * invz_2 * cam.fx;
                    J[1][0] = (1 + y * y * invz_2) * cam.fy; J[1][1] = -x * y * invz_2 * cam.fy;
                    J[1][2] = -x * invz * cam.fy; J[1][3] = 0; J[1][4] = -invz * cam.fy;
                    J[1][5] = y * invz_2 * cam.fy;
                    if (dim == 3) {
                        J[2][0] = J[0][0] - cam.bf * y * invz_2; J[2][1] = J[0][1] + cam.bf * x * invz_2;
                        J[2][2] = J[0][2]; J[2][3] = J[0][3]; J[2][4] = 0; J[2][5] = J[0][5] - cam.bf * invz_2;
                    } else {
#pragma unroll
                        for (int d = 0; d < 6; d++) J[2][d] = 0;
                    }
                    accumulate(J, err, info, dim, delta);
                }
                // plane edges: numeric central differences, delta 1e-9 (base_binary_edge.hpp:130-205);
                // the 12 perturbed evaluations of each edge run on 12 threads
                if (nl > 0) {
                    if (t < 12) S.Tp[t] = se3_mul(S.Eadd[t], T);
                    __syncthreads();
                    for (int base = 0; base < nl; base += kPlaneChunk) {
                        const int cnt = min(kPlaneChunk, nl - base);
                        // 13 evaluations per edge in parallel: the 12 perturbed poses and T itself (the
                        // error the edge's own accumulation needs -- no second serial evaluation after the sync)
                        for (int w = t; w < cnt * 13; w += kThreads) {
                            const int j = w / 13, q = w - j * 13, e = np + base + j;
                            double err[3] = {0, 0, 0};
                            if (!plout[e - np]) {
                                const SE3& P = S.Tp[q < 12 ? q : 0];
                                const bool pt = q < 12;
                                SE3 Tq;  // field-wise select keeps both poses in registers
                                Tq.r.w = pt ? P.r.w : T.r.w; Tq.r.x = pt ? P.r.x : T.r.x;
                                Tq.r.y = pt ? P.r.y : T.r.y; Tq.r.z = pt ? P.r.z : T.r.z;
                                Tq.t.x = pt ? P.t.x : T.t.x; Tq.t.y = pt ? P.t.y : T.t.y; Tq.t.z = pt ? P.t.z : T.t.z;
                                error_at(e, Tq, err, nullptr);
                            }
                            S.perr[j][q][0] = err[0]; S.perr[j][q][1] = err[1]; S.perr[j][q][2] = err[2];
                        }
                        __syncthreads();
                        for (int j = t; j < cnt; j += kThreads) {
                            const int e = np + base + j;
                            if (plout[e - np]) continue;
                            double info[3], delta, J[3][6];
                            int dim;
                            edge_info(e, info, &delta, &dim);
                            const double err[3] = {S.perr[j][12][0], S.perr[j][12][1], S.perr[j][12][2]};
                            const double scalar = 1.0 / (2 * 1e-9);
#pragma unroll
                            for (int d = 0; d < 6; d++)
#pragma unroll
                                for (int r = 0; r < 3; r++)
                                    J[r][d] = scalar * (S.perr[j][2 * d][r] - S.perr[j][2 * d + 1][r]);
                            accumulate(J, err, info, dim, delta);
                        }
                        __syncthreads();
                    }
                }
                block_reduce(v, S);
                if (t == 0) {
                    S.Tlast = S.T;
                    S.currentChi = S.red[0][0];
                    S.iniChi = S.currentChi;
                    int k = 1;
                    for (int i = 0; i < 6; i++)
                        for (int j = i; j < 6; j++, k++) S.H[i][j] = S.H[j][i] = S.red[0][k];
                    for (int i = 0; i < 6; i++) S.b[i] = S.red[0][22 + i];
                    if (it == 0) {
                        double md = 0;
                        for (int j = 0; j < 6; j++) md = fmax(fabs(S.H[j][j]), md);
                        S.lambda = 1e-5 * md;
                        S.ni = 2;
                        S.nBad = 0;
                    }
                    for (int j = 0; j < 6; j++) S.x[j] = 0;
                }
                __syncthreads();
                // ---- trials
                double rho = 0;
                int qmax = 0;
                bool ok2 = true;
                do {
                    if (t == 0) {
                        double x[6] = {0, 0, 0, 0, 0, 0};  // a failed LDLT leaves x unwritten
                        S.stop = ldlt_solve(S.H, S.lambda, S.b, x) ? 1 : 0;
                        for (int j = 0; j < 6; j++) S.x[j] = x[j];
                        S.Ttrial = se3_mul(se3_exp(x), S.T);
                    }
                    __syncthreads();
                    ok2 = S.stop != 0;
                    const SE3 Tt = S.Ttrial;
                    double c[1] = {0};
                    for (int e = t; e < ne; e += kThreads) {
                        if (is_outlier(e)) continue;
                        double info[3], delta, err[3] = {0, 0, 0};
                        int dim;
                        edge_info(e, info, &delta, &dim);
                        error_at(e, Tt, err, nullptr);
                        double chi = 0;
                        // rows beyond dim hold a zero error: their +0 terms leave chi unchanged
                        chi = (err[0] * info[0] * err[0] + err[1] * info[1] * err[1]) + err[2] * info[2] * err[2];
                        double rho0, rho1;
                        huber(chi, delta, robust, &rho0, &rho1);
                        c[0] += rho0;
                    }
                    block_reduce(c, S);
                    if (t == 0) {
                        S.Tlast = S.Ttrial;
                        double tempChi = S.red[0][0];
                        if (!ok2) tempChi = 1.7976931348623157e308;
                        double r = S.currentChi - tempChi;
                        double scale = 0;
                        for (int j = 0; j < 6; j++) scale += S.x[j] * (S.lambda * S.x[j] + S.b[j]);
                        scale += 1e-3;
                        r /= scale;
                        if (r > 0 && isfinite(tempChi)) {
                            const double r21 = 2 * r - 1;  // pow(2r - 1, 3) as two products (an ocml pow is ~200 serial fp64 ops)
                            double alpha = 1. - r21 * r21 * r21;
                            alpha = fmin(alpha, 2. / 3.);
                            S.lambda *= fmax(1. / 3., alpha);
                            S.ni = 2;
                            S.currentChi = tempChi;
                            S.T = S.Ttrial;
                        } else {
                            S.lambda *= S.ni;
                            S.ni *= 2;
                        }
                        S.tempChi = r;  // broadcast rho
                    }
                    __syncthreads();
                    rho = S.tempChi;
                    qmax++;
                } while (rho < 0 && qmax < 10);
                total_its++;
                if (qmax == 10 || rho == 0) break;
                int stop = 0;
                if (t == 0) {
                    if ((S.iniChi - S.currentChi) * 1e3 < S.iniChi) S.nBad++;
                    else S.nBad = 0;
                    S.stop = S.nBad >= 3;
                }
                __syncthreads();
                stop = S.stop;
                __syncthreads();
                if (stop) break;
            }
        }
        // ---- relabel (:925-1140)
        const SE3 T = S.T, Tl = S.Tlast;
        int bad = 0;
        for (int e = t; e < ne; e += kThreads) {
            double info[3], delta, err[3] = {0, 0, 0};
            int dim;
            edge_info(e, info, &delta, &dim);
            const bool was_out = is_outlier(e);
            SE3 Te;  // field-wise select (a selected reference would put both poses in scratch memory)
            Te.r.w = was_out ? T.r.w : Tl.r.w; Te.r.x = was_out ? T.r.x : Tl.r.x;
            Te.r.y = was_out ? T.r.y : Tl.r.y; Te.r.z = was_out ? T.r.z : Tl.r.z;
            Te.t.x = was_out ? T.t.x : Tl.t.x; Te.t.y = was_out ? T.t.y : Tl.t.y; Te.t.z = was_out ? T.t.z : Tl.t.z;
            error_at(e, Te, err, nullptr);
            double chi = 0;
            // rows beyond dim hold a zero error: their +0 terms leave chi unchanged
                        chi = (err[0] * info[0] * err[0] + err[1] * info[1] * err[1]) + err[2] * info[2] * err[2];
            const float chi2 = (float)chi;
            bool b;
            if (e < np) b = pts[e].ur < 0 ? chi2 > 5.991f : chi2 > 7.815f;
            else b = pls[e - np].kind == 0 ? (double)chi2 > K.plane_chi : (double)chi2 > K.vp_chi;
            bad += b;
            if (e < np) pout[e] = b;
            else plout[e - np] = b;
        }
        // wave-sum then LDS
        for (int off = 32; off >= 1; off >>= 1) bad += __shfl_xor(bad, off);
        if ((t & 63) == 0) S.count[t >> 6] = bad;
        __syncthreads();
        nBad = 0;
#pragma unroll
        for (int w = 0; w < kThreads / 64; w++) nBad += S.count[w];
        __syncthreads();
        if (round == 2) robust = false;
        if (ne < 10) break;
    }
    if (t == 0) {
        const M3 R = q_to_rot(S.T.r);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) res->Tcw[4 * i + j] = (float)R.a[3 * i + j];
        res->Tcw[3] = (float)S.T.t.x; res->Tcw[7] = (float)S.T.t.y; res->Tcw[11] = (float)S.T.t.z;
        res->Tcw[12] = 0.f; res->Tcw[13] = 0.f; res->Tcw[14] = 0.f; res->Tcw[15] = 1.f;
        res->n_inliers = ne - nBad;
        res->lm_iterations = total_its;
    }
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
    static const int occ = [] {
        const char* e = std::getenv("SPSLAM_POSE_OCCUPANCY");  // measurement knob: 1, 2 or 4
        return e ? std::atoi(e) : 1;
    }();
    if (occ >= 4)
        hipLaunchKernelGGL(pose_kernel<4>, dim3(n), dim3(kThreads), 0, s, probs, pts, pls, K, init_from, res, pout, plout);
    else if (occ >= 2)
        hipLaunchKernelGGL(pose_kernel<2>, dim3(n), dim3(kThreads), 0, s, probs, pts, pls, K, init_from, res, pout, plout);
    else
        hipLaunchKernelGGL(pose_kernel<1>, dim3(n), dim3(kThreads), 0, s, probs, pts, pls, K, init_from, res, pout, plout);
    return hipGetLastError();
}

}  // namespace spslam
