// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// CPU restatement of Optimizer::PoseOptimization (src/Optimizer.cc:519-1152)
// on top of a minimal restatement of the vendored g2o pieces it uses:
//   SparseOptimizer::initializeOptimization/optimize/activeRobustChi2
//     (Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:100-114,199-267,354-420)
//   OptimizationAlgorithmLevenberg::solve / computeLambdaInit / computeScale
//     (core/optimization_algorithm_levenberg.cpp:61-189)
//   BlockSolver::buildSystem/setLambda (core/block_solver.hpp:502-590),
//   LinearSolverDense (Eigen LDLT, solvers/linear_solver_dense.h:65-115)
//   RobustKernelHuber (core/robust_kernel_impl.cpp:78-91), robustInformation
//     (core/base_edge.h:96-102), quadratic forms (base_unary_edge.hpp:43-72,
//     base_binary_edge.hpp:55-120), numeric Jacobian (base_binary_edge.hpp:130-205)
//   SE3Quat / VertexSE3Expmap (types/se3quat.h, types_six_dof_expmap.h:73-76)
//   EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose
//     (types_six_dof_expmap.h:143-202, .cpp:266-364)
//   g2oAddition Plane3D / EdgePlane / EdgeParallelPlane / EdgeVerticalPlane
// and the Eigen 3 routines they call (Quaternion(Matrix3), toRotationMatrix,
// quaternion product and vector rotation, AngleAxis, LDLT with diagonal
// pivoting).  All arithmetic is double, like the reference.
//
// Two summation orders (oracle_set_pose_order):
//   0  g2o's: edge by edge in insertion order (BlockSolver::buildSystem,
//      activeRobustChi2), glibc sin / cos / atan2 / pow -- the default;
//   1  the GPU kernel's: the sums of sp-slam_amd/csrc/pose_kernels.hip wg_sum
//      (256 lane-strided partials, xor butterflies over 64 lanes, four wave
//      totals) and its per-edge term order, with libm64_restated.h's sin / cos /
//      atan2 / cube.  The kernel must then agree bit for bit.
// Both run the same LM algorithm; they differ only by the rounding of the sums.
#include <array>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "../include/spslam_gpu.h"
#include "g2o_restated.h"

namespace oracle {
namespace {

using namespace g2o_math;

struct Edge {
    int type;   // 0 mono, 1 stereo, 2 plane, 3 parallel, 4 vertical
    int dim;
    int level = 0;
    Huber rk;
    double info[3];   // diagonal information
    double meas[3];   // point measurements
    V3 Xw;
    Plane world, mplane;
    double err[3] = {0, 0, 0};
    double chi2() const { double s = 0; for (int i = 0; i < dim; i++) s += err[i] * info[i] * err[i]; return s; }
};

struct Cam { double fx, fy, cx, cy, bf; };

void compute_error(Edge& e, const SE3& T, const Cam& c) {
    if (e.type == 0) {
        V3 p = T.map(e.Xw);
        double px = p.x / p.z, py = p.y / p.z;
        e.err[0] = e.meas[0] - (px * c.fx + c.cx);
        e.err[1] = e.meas[1] - (py * c.fy + c.cy);
    } else if (e.type == 1) {
        V3 p = T.map(e.Xw);
        const float invz = (float)(1.0f / p.z);
        double r0 = p.x * invz * c.fx + c.cx, r1 = p.y * invz * c.fy + c.cy, r2 = r0 - c.bf * invz;
        e.err[0] = e.meas[0] - r0; e.err[1] = e.meas[1] - r1; e.err[2] = e.meas[2] - r2;
    } else {
        Plane local = transform(T, e.world);
        if (e.type == 2) ominus(local, e.mplane, e.err);
        else if (e.type == 3) ominus_par(local, e.mplane, e.err);
        else ominus_ver(local, e.mplane, e.err);
    }
}

// Jacobian wrt the pose update (rows = e.dim, cols 6).
void jacobian(Edge& e, const SE3& T, const Cam& c, double J[3][6]) {
    if (e.type <= 1) {
        V3 p = T.map(e.Xw);
        double x = p.x, y = p.y, invz = 1.0 / p.z, invz_2 = invz * invz;
        J[0][0] = x * y * invz_2 * c.fx; J[0][1] = -(1 + (x * x * invz_2)) * c.fx; J[0][2] = y * invz * c.fx;
        J[0][3] = -invz * c.fx; J[0][4] = 0; J[0][5] = x * invz_2 * c.fx;
        J[1][0] = (1 + y * y * invz_2) * c.fy; J[1][1] = -x * y * invz_2 * c.fy; J[1][2] = -x * invz * c.fy;
        J[1][3] = 0; J[1][4] = -invz * c.fy; J[1][5] = y * invz_2 * c.fy;
        if (e.type == 1) {
            J[2][0] = J[0][0] - c.bf * y * invz_2; J[2][1] = J[0][1] + c.bf * x * invz_2; J[2][2] = J[0][2];
            J[2][3] = J[0][3]; J[2][4] = 0; J[2][5] = J[0][5] - c.bf * invz_2;
        }
        return;
    }
    // numeric central differences, delta 1e-9 (base_binary_edge.hpp:130-205)
    const double delta = 1e-9, scalar = 1.0 / (2 * delta);
    double bak[3], save[3];
    std::memcpy(save, e.err, sizeof save);
    for (int d = 0; d < 6; d++) {
        double add[6] = {0, 0, 0, 0, 0, 0};
        add[d] = delta;
        SE3 Tp = SE3::exp(add) * T;
        compute_error(e, Tp, c);
        for (int i = 0; i < e.dim; i++) bak[i] = e.err[i];
        add[d] = -delta;
        SE3 Tm = SE3::exp(add) * T;
        compute_error(e, Tm, c);
        for (int i = 0; i < e.dim; i++) J[i][d] = scalar * (bak[i] - e.err[i]);
    }
    std::memcpy(e.err, save, sizeof save);
}

// Eigen::LDLT<MatrixXd> compute (diagonal pivoting, lower storage) + solve.
bool ldlt_solve(double A[6][6], const double b[6], double x[6]) {
    const int n = 6;
    double m[6][6];
    std::memcpy(m, A, sizeof m);
    int tr[6];
    int sign = 0;  // 0 zero, 1 possemidef, 2 negsemidef, 3 indefinite
    bool ret = true, found_zero = false;
    double temp[6];
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = std::fabs(m[k][k]);
        for (int i = k + 1; i < n; i++)
            if (std::fabs(m[i][i]) > bv) { bv = std::fabs(m[i][i]); big = i; }
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; j++) std::swap(m[k][j], m[big][j]);
            for (int i = big + 1; i < n; i++) std::swap(m[i][k], m[i][big]);
            std::swap(m[k][k], m[big][big]);
            for (int i = k + 1; i < big; ++i) { double t = m[i][k]; m[i][k] = m[big][i]; m[big][i] = t; }
        }
        const int rs = n - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; j++) temp[j] = m[j][j] * m[k][j];
            double s = 0;
            for (int j = 0; j < k; j++) s += m[k][j] * temp[j];
            m[k][k] -= s;
            for (int i = k + 1; i < n; i++) {
                double t = 0;
                for (int j = 0; j < k; j++) t += m[i][j] * temp[j];
                m[i][k] -= t;
            }
        }
        const double akk = m[k][k];
        const bool valid = std::fabs(akk) > 0;
        if (k == 0 && !valid) { sign = 0; return false; }
        if (rs > 0 && valid)
            for (int i = k + 1; i < n; i++) m[i][k] /= akk;
        if (found_zero && valid) ret = false;
        else if (!valid) found_zero = true;
        if (sign == 1) { if (akk < 0) sign = 3; }
        else if (sign == 2) { if (akk > 0) sign = 3; }
        else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
    }
    (void)ret;
    const bool positive = sign == 1 || sign == 0;
    if (!positive) return false;
    // solve: P b, L y = Pb, D z = y (pseudo-inverse), L^T w = z, x = P^T w
    double y[6];
    std::memcpy(y, b, sizeof y);
    for (int k = 0; k < n; k++) std::swap(y[k], y[tr[k]]);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < i; j++) y[i] -= m[i][j] * y[j];
    double maxd = 0;
    for (int i = 0; i < n; i++) maxd = std::max(maxd, std::fabs(m[i][i]));
    const double tol = std::numeric_limits<double>::min();  // Eigen: RealScalar(1)/NumTraits::highest()
    (void)maxd;
    for (int i = 0; i < n; i++) y[i] = std::fabs(m[i][i]) > tol ? y[i] / m[i][i] : 0.0;
    for (int i = n - 1; i >= 0; i--)
        for (int j = i + 1; j < n; j++) y[i] -= m[j][i] * y[j];
    for (int k = n - 1; k >= 0; k--) std::swap(y[k], y[tr[k]]);
    std::memcpy(x, y, sizeof y);
    return true;
}

struct LM {
    double lambda = -1, ni = 2;
    int nBad = 0;
};

double robust_chi2(const std::vector<Edge*>& active) {
    double chi = 0;
    for (Edge* e : active) {
        if (e->rk.on) { double rho[3]; e->rk.robustify(e->chi2(), rho); chi += rho[0]; }
        else chi += e->chi2();
    }
    return chi;
}

// SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg.
int optimize(std::vector<Edge*>& active, SE3& T, const Cam& c, int iterations) {
    LM lm;
    int its = 0;
    for (int it = 0; it < iterations; it++) {
        for (Edge* e : active) compute_error(*e, T, c);
        double currentChi = robust_chi2(active), tempChi = currentChi, iniChi = currentChi;
        // buildSystem
        double H[6][6] = {}, b[6] = {};
        for (Edge* e : active) {
            double J[3][6];
            jacobian(*e, T, c, J);
            double w = 1.0;
            if (e->rk.on) { double rho[3]; e->rk.robustify(e->chi2(), rho); w = rho[1]; }
            for (int r = 0; r < e->dim; r++) {
                const double oe = e->info[r] * e->err[r];
                for (int i = 0; i < 6; i++) {
                    b[i] -= w * J[r][i] * oe;
                    for (int j = 0; j < 6; j++) H[i][j] += J[r][i] * (w * e->info[r]) * J[r][j];
                }
            }
        }
        if (it == 0) {
            double maxDiag = 0;
            for (int j = 0; j < 6; j++) maxDiag = std::max(std::fabs(H[j][j]), maxDiag);
            lm.lambda = 1e-5 * maxDiag;
            lm.ni = 2;
            lm.nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            SE3 backup = T;
            double Hl[6][6];
            std::memcpy(Hl, H, sizeof Hl);
            for (int j = 0; j < 6; j++) Hl[j][j] += lm.lambda;
            double x[6] = {0, 0, 0, 0, 0, 0};  // a failed LDLT leaves x unwritten (rejected step)
            bool ok2 = ldlt_solve(Hl, b, x);
            T = SE3::exp(x) * T;
            for (Edge* e : active) compute_error(*e, T, c);
            tempChi = robust_chi2(active);
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = 0;
            for (int j = 0; j < 6; j++) scale += x[j] * (lm.lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - o_cube(2 * rho - 1);
                alpha = std::min(alpha, 2. / 3.);
                double sf = std::max(1. / 3., alpha);
                lm.lambda *= sf;
                lm.ni = 2;
                currentChi = tempChi;
            } else {
                lm.lambda *= lm.ni;
                lm.ni *= 2;
                T = backup;
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        its++;
        if (qmax == 10 || rho == 0) break;
        if ((iniChi - currentChi) * 1e3 < iniChi) lm.nBad++;
        else lm.nBad = 0;
        if (lm.nBad >= 3) break;
    }
    return its;
}


// ---- device-order mode -------------------------------------------------------
constexpr int kLanes = 256, kWaveLanes = 64;

// wg_sum (pose_kernels.hip): per-thread partials -> xor butterfly per wave -> ((0 + w0) + w1) + w2) + w3
template <size_t NV>
void tree_total(const std::vector<std::array<double, NV>>& part, double* out) {
    for (size_t k = 0; k < NV; k++) {
        double s = 0;
        for (int w = 0; w < kLanes / kWaveLanes; w++) {
            double x[kWaveLanes], y[kWaveLanes];
            for (int l = 0; l < kWaveLanes; l++) x[l] = part[w * kWaveLanes + l][k];
            for (int off = kWaveLanes / 2; off >= 1; off >>= 1) {
                for (int l = 0; l < kWaveLanes; l++) y[l] = x[l] + x[l ^ off];
                std::memcpy(x, y, sizeof x);
            }
            s += x[0];
        }
        out[k] = s;
    }
}

double huber_rho(const Edge& e, double chi, double* rho1) {
    if (!e.rk.on || chi <= e.rk.dsqr) { *rho1 = 1.0; return chi; }
    const double s = std::sqrt(chi);
    *rho1 = e.rk.delta / s;
    return 2 * s * e.rk.delta - e.rk.dsqr;
}

// 3-row error / Jacobian as the kernel holds them (rows beyond the edge's dimension are zero)
void jacobian3(Edge& e, const SE3& T, const Cam& c, double J[3][6]) {
    for (int r = 0; r < 3; r++)
        for (int d = 0; d < 6; d++) J[r][d] = 0;
    jacobian(e, T, c, J);
}

// the kernel's per-edge contribution (pose_kernels.hip accumulate)
void accumulate_dev(const Edge& e, const double J[3][6], std::array<double, 28>& v) {
    const double chi = (e.err[0] * e.info[0] * e.err[0] + e.err[1] * e.info[1] * e.err[1]) + e.err[2] * e.info[2] * e.err[2];
    double rho1;
    v[0] += huber_rho(e, chi, &rho1);
    for (int i = 0; i < 6; i++)
        for (int j = i; j < 6; j++) {
            double s = 0;
            for (int r = 0; r < 3; r++) s += J[r][i] * (rho1 * e.info[r]) * J[r][j];
            v[1 + i * 6 - i * (i - 1) / 2 + (j - i)] += s;
        }
    for (int i = 0; i < 6; i++) {
        double s = 0;
        for (int r = 0; r < 3; r++) s += rho1 * J[r][i] * (e.info[r] * e.err[r]);
        v[22 + i] -= s;
    }
}

double robust_chi2_dev(Edge* edges, int ne, const std::vector<uint8_t>& active) {
    std::vector<std::array<double, 1>> part(kLanes, {0.0});
    for (int k = 0; k < ne; k++) {
        if (!active[k]) continue;
        const Edge& e = edges[k];
        const double chi = (e.err[0] * e.info[0] * e.err[0] + e.err[1] * e.info[1] * e.err[1]) + e.err[2] * e.info[2] * e.err[2];
        double rho1;
        part[k % kLanes][0] += huber_rho(e, chi, &rho1);
    }
    double out;
    tree_total(part, &out);
    return out;
}

// SparseOptimizer::optimize with the kernel's summation order (edges[0..np) points, then planes)
int optimize_dev(Edge* edges, int np, int ne, const std::vector<uint8_t>& active, SE3& T, const Cam& c,
                 int iterations) {
    LM lm;
    int its = 0;
    for (int it = 0; it < iterations; it++) {
        for (int k = 0; k < ne; k++)
            if (active[k]) compute_error(edges[k], T, c);
        // pass A: point edge k on lane k % 256, then plane edge j on lane j % 64
        std::vector<std::array<double, 28>> part(kLanes);
        for (auto& p : part) p.fill(0.0);
        for (int k = 0; k < ne; k++) {
            if (!active[k]) continue;
            double J[3][6];
            jacobian3(edges[k], T, c, J);
            accumulate_dev(edges[k], J, part[k < np ? k % kLanes : (k - np) % kWaveLanes]);
        }
        double tot[28];
        tree_total(part, tot);
        double currentChi = tot[0];
        const double iniChi = currentChi;
        double H[6][6], b[6];
        for (int i = 0, k = 1; i < 6; i++)
            for (int j = i; j < 6; j++, k++) H[i][j] = H[j][i] = tot[k];
        for (int i = 0; i < 6; i++) b[i] = tot[22 + i];
        if (it == 0) {
            double maxDiag = 0;
            for (int j = 0; j < 6; j++) maxDiag = std::max(std::fabs(H[j][j]), maxDiag);
            lm.lambda = 1e-5 * maxDiag;
            lm.ni = 2;
            lm.nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            SE3 backup = T;
            double Hl[6][6];
            std::memcpy(Hl, H, sizeof Hl);
            for (int j = 0; j < 6; j++) Hl[j][j] += lm.lambda;
            double x[6] = {0, 0, 0, 0, 0, 0};
            bool ok2 = ldlt_solve(Hl, b, x);
            T = SE3::exp(x) * T;
            for (int k = 0; k < ne; k++)
                if (active[k]) compute_error(edges[k], T, c);
            double tempChi = robust_chi2_dev(edges, ne, active);
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = 0;
            for (int j = 0; j < 6; j++) scale += x[j] * (lm.lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - o_cube(2 * rho - 1);
                alpha = std::min(alpha, 2. / 3.);
                lm.lambda *= std::max(1. / 3., alpha);
                lm.ni = 2;
                currentChi = tempChi;
            } else {
                lm.lambda *= lm.ni;
                lm.ni *= 2;
                T = backup;
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        its++;
        if (qmax == 10 || rho == 0) break;
        if ((iniChi - currentChi) * 1e3 < iniChi) lm.nBad++;
        else lm.nBad = 0;
        if (lm.nBad >= 3) break;
    }
    return its;
}

thread_local int g_pose_order = 0;  // per thread: concurrent oracle sequences may differ

struct DeviceMathScope {  // switches this thread's g2o_math elementary functions for one call
    bool prev;
    explicit DeviceMathScope(bool on) : prev(device_math()) { device_math() = on; }
    ~DeviceMathScope() { device_math() = prev; }
};

}  // namespace
}  // namespace oracle

using namespace oracle;

extern "C" void oracle_set_pose_order(int mode) { g_pose_order = mode; }
extern "C" int oracle_get_pose_order() { return g_pose_order; }

extern "C" int oracle_pose_optimize(const spslam_pose_problem* P, const spslam_point_obs* pts,
                                    const spslam_plane_obs* pls, const spslam_plane_config* cfg,
                                    spslam_pose_result* out, uint8_t* pout, uint8_t* plout) {
    const bool dev = g_pose_order == 1;
    DeviceMathScope math_scope(dev);
    M3 R;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R.m[i][j] = P->Tcw[4 * i + j];
    const SE3 T0 = SE3::from_Rt(R, {P->Tcw[3], P->Tcw[7], P->Tcw[11]});
    const Cam cam{P->fx, P->fy, P->cx, P->cy, P->bf};
    const float deltaMono = std::sqrt(5.991), deltaStereo = std::sqrt(7.815);
    std::vector<Edge> edges;
    edges.reserve(P->n_points + P->n_planes);
    int nInitial = 0;
    for (int i = 0; i < P->n_points; i++) {
        const spslam_point_obs& o = pts[i];
        Edge e;
        e.Xw = {o.xw[0], o.xw[1], o.xw[2]};
        e.meas[0] = o.u; e.meas[1] = o.v;
        if (o.ur < 0) { e.type = 0; e.dim = 2; e.rk.set(deltaMono); }
        else { e.type = 1; e.dim = 3; e.meas[2] = o.ur; e.rk.set(deltaStereo); }
        for (int k = 0; k < 3; k++) e.info[k] = (double)o.inv_sigma2;
        edges.push_back(e);
        nInitial++;
        pout[i] = 0;
    }
    std::memcpy(out->Tcw, P->Tcw, sizeof out->Tcw);
    out->lm_iterations = 0;
    if (nInitial < 3) { out->n_inliers = 0; for (int i = 0; i < P->n_planes; i++) plout[i] = 0; return 0; }
    const double angleInfo = 3282.8 / (cfg->angle_info * cfg->angle_info);
    const double disInfo = cfg->distance_info * cfg->distance_info;
    const double parInfo = 3282.8 / (cfg->parallel_info * cfg->parallel_info);
    const double verInfo = 3282.8 / (cfg->vertical_info * cfg->vertical_info);
    const double planeChi = cfg->chi, VPplaneChi = cfg->vp_chi;
    const float deltaPlane = std::sqrt(planeChi), VPdeltaPlane = std::sqrt(VPplaneChi);
    for (int i = 0; i < P->n_planes; i++) {
        const spslam_plane_obs& o = pls[i];
        Edge e;
        e.type = 2 + o.kind;
        e.dim = o.kind == 0 ? 3 : 2;
        double w[4], m[4];
        for (int k = 0; k < 4; k++) { w[k] = o.world[k]; m[k] = o.meas[k]; }
        if (o.world[3] < 0.0f) for (double& v : w) v = -v;   // Converter::toPlane3D
        if (o.meas[3] < 0.0f) for (double& v : m) v = -v;
        e.world = Plane::from(w);
        e.mplane = Plane::from(m);
        if (o.kind == 0) { e.info[0] = e.info[1] = angleInfo; e.info[2] = disInfo; e.rk.set(deltaPlane); }
        else { const double inf = o.kind == 1 ? parInfo : verInfo; e.info[0] = e.info[1] = inf; e.info[2] = 0; e.rk.set(VPdeltaPlane); }
        edges.push_back(e);
        nInitial++;
        plout[i] = 0;
    }
    SE3 T = T0;
    int nBad = 0, total_its = 0;
    for (int it = 0; it < 4; it++) {
        T = T0;
        if (dev) {
            std::vector<uint8_t> act(edges.size());
            bool any = false;
            for (size_t k = 0; k < edges.size(); k++) any |= (act[k] = edges[k].level == 0) != 0;
            if (any) total_its += optimize_dev(edges.data(), P->n_points, (int)edges.size(), act, T, cam, 10);
        } else {
            std::vector<Edge*> active;
            for (Edge& e : edges)
                if (e.level == 0) active.push_back(&e);
            total_its += optimize(active, T, cam, 10);
        }
        nBad = 0;
        for (size_t k = 0; k < edges.size(); k++) {
            Edge& e = edges[k];
            const bool is_point = e.type <= 1;
            uint8_t& flag = is_point ? pout[k] : plout[k - P->n_points];
            if (flag) compute_error(e, T, cam);
            const float chi2 = (float)e.chi2();
            bool bad;
            if (e.type == 0) bad = chi2 > 5.991f;
            else if (e.type == 1) bad = chi2 > 7.815f;
            else if (e.type == 2) bad = chi2 > planeChi;
            else bad = chi2 > VPplaneChi;
            flag = bad ? 1 : 0;
            e.level = bad ? 1 : 0;
            nBad += bad;
            if (it == 2) e.rk.on = false;
        }
        if (edges.size() < 10) break;
    }
    // Converter::toCvMat(SE3Quat): to_homogeneous_matrix -> float
    M3 Rr = quat_to_rot(T.r);
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) out->Tcw[4 * i + j] = (float)Rr.m[i][j];
    }
    out->Tcw[3] = (float)T.t.x; out->Tcw[7] = (float)T.t.y; out->Tcw[11] = (float)T.t.z;
    out->Tcw[12] = 0.f; out->Tcw[13] = 0.f; out->Tcw[14] = 0.f; out->Tcw[15] = 1.f;
    out->n_inliers = nInitial - nBad;
    out->lm_iterations = total_its;
    return out->n_inliers;
}
