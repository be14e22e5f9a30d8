// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// CPU restatement of Optimizer::LocalBundleAdjustment (src/Optimizer.cc:
// 1154-1977) from the point where the graph is known (the caller flattens the
// local / fixed keyframes, local map points and map planes with their
// observations, in the reference's insertion order -- include/spslam_gpu.h):
//   vertices  VertexSE3Expmap (local KFs, KF id 0 fixed; fixed cameras),
//             VertexSBAPointXYZ (marginalized), g2oAddition VertexPlane
//             (marginalized), ids mnId / mnId+maxKFid+1 / mnId+maxPointid+1;
//   edges     EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ (types_six_dof_
//             expmap.cpp:103-234, Huber sqrt(5.991) / sqrt(7.815)), EdgePlane /
//             EdgeVerticalPlane / EdgeParallelPlane (binary, numeric Jacobians
//             for both vertices, base_binary_edge.hpp:130-205; Huber sqrt(Chi) /
//             sqrt(VPChi)); the not-seen branches are dead (SURVEY.md 8 notes);
//   solver    SparseOptimizer::initializeOptimization(level) (active edges,
//             vertices with active edges, poses then landmarks by id,
//             sparse_optimizer.cpp), OptimizationAlgorithmLevenberg::solve,
//             BlockSolver_6_3 buildStructure / buildSystem / setLambda / Schur
//             solve in g2o's own order (block_solver.hpp:130-590): every edge's
//             quadratic form added to its vertex blocks in edge-insertion order
//             (Eigen's expression for each robust / non-robust branch,
//             base_binary_edge.hpp:55-120), chi2 summed edge by edge
//             (sparse_optimizer.cpp:100-114), the Schur complement formed
//             landmark by landmark in landmark-index order (Hi1i2 -= BDinv Bj^T,
//             Bb += Bi db, Eigen 3x3 cofactor inverse), the reduced system's
//             pattern = g2o's Hschur pattern (pose pairs over ALL edges of each
//             active landmark, outliers included), factorised by Eigen's
//             SimplicialLDLT after its AMD ordering (eigen_simplicial_restated.h);
//   schedule  optimize(5); relabel (chi2 > 5.991 / 7.815 or depth <= 0 for
//             points, > Chi / VPChi for planes) with the errors cached by the
//             last computeActiveErrors, drop every robust kernel;
//             initializeOptimization(0); optimize(10); outlier observations
//             (vToErase); write back poses (local KFs), points and planes.
// Eigen's reductions inside the fixed-size products (3-term dots, A^T x) are restated left to right, the
// convention of the pose path.  A failed factorisation leaves g2o's x vector
// stale (linear_solver_eigen.h:96-101) before the rejected trial is popped; here x is zero (the trial is
// rejected either way; only computeScale of that rejected trial could differ).
// Parity: unpinned against the reference binary (g2o needs Eigen, absent).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "../include/spslam_gpu.h"
#include "eigen_simplicial_restated.h"
#include "g2o_restated.h"

extern "C" unsigned oracle_get_solve_fail_mask();  // pose_oracle.cpp (test hook)

namespace ORACLE_NS {
namespace lba {

using namespace g2o_math;

struct Vtx {
    int kind;          // 0 pose, 1 point, 2 plane
    long long id;      // g2o vertex id
    bool fixed = false;
    SE3 T;
    V3 X{0, 0, 0};
    Plane P{};
    int hidx = -1;     // index among the active non-fixed poses / landmarks
    SE3 Tb;
    V3 Xb{0, 0, 0};
    Plane Pb{};
};

struct Edge {
    int type;          // 0 mono, 1 stereo, 2 plane, 3 parallel, 4 vertical
    int dim;
    int lm, kf;        // vertex indices (vertex 0 = landmark, vertex 1 = pose)
    int level = 0;
    Huber rk;
    double info[3];
    double meas[3];
    Plane mplane{};
    double fx, fy, cx, cy, bf;
    double err[3] = {0, 0, 0};
    double chi2() const {  // _error.dot(information() * _error), Omega diagonal
        double s = 0;
        for (int i = 0; i < dim; i++) s += err[i] * (info[i] * err[i]);
        return s;
    }
};

struct Graph {
    std::vector<Vtx> v;
    std::vector<Edge> e;
};

void compute_error(Edge& e, const Graph& G) {
    const Vtx& L = G.v[e.lm];
    const SE3& T = G.v[e.kf].T;
    if (e.type <= 1) {
        const V3 p = T.map(L.X);
        if (e.type == 0) {
            e.err[0] = e.meas[0] - (p.x / p.z * e.fx + e.cx);
            e.err[1] = e.meas[1] - (p.y / p.z * e.fy + e.cy);
        } else {
            const float invz = (float)(1.0f / p.z);
            const float bf = (float)e.bf;  // cam_project(..., const float& bf)
            const double r0 = p.x * invz * e.fx + e.cx, r1 = p.y * invz * e.fy + e.cy;
            const double r2 = r0 - (double)(bf * invz);
            e.err[0] = e.meas[0] - r0;
            e.err[1] = e.meas[1] - r1;
            e.err[2] = e.meas[2] - r2;
        }
        return;
    }
    const Plane local = transform(T, L.P);
    if (e.type == 2) ominus(local, e.mplane, e.err);
    else if (e.type == 3) ominus_par(local, e.mplane, e.err);
    else ominus_ver(local, e.mplane, e.err);
}

bool depth_positive(const Edge& e, const Graph& G) {
    const SE3& T = G.v[e.kf].T;
    if (e.type <= 1) return T.map(G.v[e.lm].X).z > 0.0;
    return transform(T, G.v[e.lm].P).distance() > 0;
}

// Jacobians: A (dim x 3, landmark), B (dim x 6, pose).  Fixed vertices are skipped.
void linearize(Edge& e, Graph& G, double A[3][3], double B[3][6]) {
    Vtx& L = G.v[e.lm];
    Vtx& P = G.v[e.kf];
    if (e.type <= 1) {
        const SE3& T = P.T;
        const V3 p = T.map(L.X);
        const double x = p.x, y = p.y, z = p.z, z_2 = z * z;
        const M3 R = quat_to_rot(T.r);
        if (e.type == 0) {
            const double tmp[2][3] = {{e.fx, 0, -x / z * e.fx}, {0, e.fy, -y / z * e.fy}};
            const double s = -1. / z;
            for (int r = 0; r < 2; r++) {
                const double t0 = s * tmp[r][0], t1 = s * tmp[r][1], t2 = s * tmp[r][2];
                for (int c = 0; c < 3; c++) A[r][c] = t0 * R.m[0][c] + t1 * R.m[1][c] + t2 * R.m[2][c];
            }
        } else {
            for (int c = 0; c < 3; c++) {
                A[0][c] = -e.fx * R.m[0][c] / z + e.fx * x * R.m[2][c] / z_2;
                A[1][c] = -e.fy * R.m[1][c] / z + e.fy * y * R.m[2][c] / z_2;
                A[2][c] = A[0][c] - e.bf * R.m[2][c] / z_2;
            }
        }
        B[0][0] = x * y / z_2 * e.fx; B[0][1] = -(1 + (x * x / z_2)) * e.fx; B[0][2] = y / z * e.fx;
        B[0][3] = -1. / z * e.fx; B[0][4] = 0; B[0][5] = x / z_2 * e.fx;
        B[1][0] = (1 + y * y / z_2) * e.fy; B[1][1] = -x * y / z_2 * e.fy; B[1][2] = -x / z * e.fy;
        B[1][3] = 0; B[1][4] = -1. / z * e.fy; B[1][5] = y / z_2 * e.fy;
        if (e.type == 1) {
            B[2][0] = B[0][0] - e.bf * y / z_2; B[2][1] = B[0][1] + e.bf * x / z_2; B[2][2] = B[0][2];
            B[2][3] = B[0][3]; B[2][4] = 0; B[2][5] = B[0][5] - e.bf / z_2;
        }
        return;
    }
    // BaseBinaryEdge numeric Jacobians, delta 1e-9
    const double delta = 1e-9, scalar = 1.0 / (2 * delta);
    double save[3], bak[3];
    std::memcpy(save, e.err, sizeof save);
    if (!L.fixed) {
        const Plane keep = L.P;
        for (int d = 0; d < 3; d++) {
            double add[3] = {0, 0, 0};
            add[d] = delta;
            plane_oplus(L.P, add);
            compute_error(e, G);
            for (int i = 0; i < e.dim; i++) bak[i] = e.err[i];
            L.P = keep;
            add[d] = -delta;
            plane_oplus(L.P, add);
            compute_error(e, G);
            for (int i = 0; i < e.dim; i++) A[i][d] = scalar * (bak[i] - e.err[i]);
            L.P = keep;
        }
    }
    if (!P.fixed) {
        const SE3 keep = P.T;
        for (int d = 0; d < 6; d++) {
            double add[6] = {0, 0, 0, 0, 0, 0};
            add[d] = delta;
            P.T = SE3::exp(add) * keep;
            compute_error(e, G);
            for (int i = 0; i < e.dim; i++) bak[i] = e.err[i];
            add[d] = -delta;
            P.T = SE3::exp(add) * keep;
            compute_error(e, G);
            for (int i = 0; i < e.dim; i++) B[i][d] = scalar * (bak[i] - e.err[i]);
            P.T = keep;
        }
    }
    std::memcpy(e.err, save, sizeof save);
}

// Eigen compute_inverse<Matrix3d> (cofactors, Eigen/src/LU/InverseImpl.h).
void inverse3(const double m[3][3], double r[3][3]) {
    auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1];
    };
    const double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    const double det = (c0 * m[0][0] + c1 * m[1][0]) + c2 * m[2][0];
    const double invdet = 1.0 / det;
    r[0][0] = c0 * invdet; r[0][1] = c1 * invdet; r[0][2] = c2 * invdet;
    r[1][0] = cof(0, 1) * invdet; r[1][1] = cof(1, 1) * invdet; r[1][2] = cof(2, 1) * invdet;
    r[2][0] = cof(0, 2) * invdet; r[2][1] = cof(1, 2) * invdet; r[2][2] = cof(2, 2) * invdet;
}

struct Opt {
    Graph& G;
    std::vector<int> active;   // active edge indices (insertion order)
    std::vector<int> poses;    // active non-fixed poses by id
    std::vector<int> lms;      // active landmarks: points by id, then planes by id
    // Hpl (pose x landmark, 6 x 3) blocks per landmark, sorted by pose index (the _HplCCS column)
    struct Block { int pose; double B[6][3]; };
    std::vector<std::vector<Block>> lblocks;
    std::vector<double> Hpp;   // [np][6][6]
    std::vector<double> Hll;   // [nl][3][3]
    std::vector<double> b;     // poses (6 np) then landmarks (3 nl)
    // the reduced system's pattern (buildStructure's Hschur): upper blocks, scalar CCS of their upper triangle
    std::vector<int> Ap, Ai;
    eigen_sparse::SimplicialLDLT ldlt;
    bool analyzed = false;
    int np = 0, nl = 0;
    double lambda = 0, ni = 2;
    int nBad = 0;
    explicit Opt(Graph& g) : G(g) {}

    void initialize(int level) {
        active.clear(); poses.clear(); lms.clear();
        std::vector<char> has(G.v.size(), 0);
        for (size_t k = 0; k < G.e.size(); k++) {
            const Edge& e = G.e[k];
            if (e.level != level) continue;
            if (G.v[e.lm].fixed && G.v[e.kf].fixed) continue;
            active.push_back((int)k);
            has[e.lm] = has[e.kf] = 1;
        }
        std::vector<int> order;
        for (size_t i = 0; i < G.v.size(); i++) { G.v[i].hidx = -1; if (has[i]) order.push_back((int)i); }
        std::sort(order.begin(), order.end(), [&](int a, int c) { return G.v[a].id < G.v[c].id; });
        for (int i : order)
            if (!G.v[i].fixed) {
                if (G.v[i].kind == 0) { G.v[i].hidx = (int)poses.size(); poses.push_back(i); }
            }
        for (int i : order)
            if (!G.v[i].fixed && G.v[i].kind != 0) { G.v[i].hidx = (int)lms.size(); lms.push_back(i); }
        np = (int)poses.size();
        nl = (int)lms.size();
        // buildStructure's Schur pattern: for every active landmark, every pair of Hessian poses among the
        // vertices of ALL its edges (HyperGraph::Vertex::edges(), any level), i1 <= i2; Hpp's diagonal blocks
        std::vector<std::vector<char>> pat((size_t)np, std::vector<char>((size_t)np, 0));
        for (int p = 0; p < np; p++) pat[p][p] = 1;
        std::vector<std::vector<int>> lposes((size_t)nl);
        for (const Edge& e : G.e) {
            const int l = G.v[e.lm].hidx, h = G.v[e.kf].hidx;
            if (l >= 0 && G.v[e.lm].kind != 0 && h >= 0 && G.v[e.kf].kind == 0) lposes[l].push_back(h);
        }
        for (auto& ps : lposes)
            for (int a : ps)
                for (int c : ps) pat[std::min(a, c)][std::max(a, c)] = 1;
        const int n = 6 * np;
        Ap.assign(n + 1, 0);
        Ai.clear();
        for (int c = 0; c < n; c++) {
            const int i2 = c / 6;
            for (int i1 = 0; i1 <= i2; i1++)
                if (pat[i1][i2])
                    for (int rr = 0; rr < 6; rr++)
                        if (6 * i1 + rr <= c) Ai.push_back(6 * i1 + rr);
            Ap[c + 1] = (int)Ai.size();
        }
        analyzed = false;  // LinearSolverEigen::init(): symbolic analysis at the first solve of optimize()
    }
    double robust_chi2() const {
        double chi = 0;
        for (int k : active) {
            const Edge& e = G.e[k];
            if (e.rk.on) { double rho[3]; e.rk.robustify(e.chi2(), rho); chi += rho[0]; }
            else chi += e.chi2();
        }
        return chi;
    }
    void compute_errors() { for (int k : active) compute_error(G.e[k], G); }

    // BlockSolver::buildSystem: linearizeOplus + constructQuadraticForm of every active edge in insertion order
    // (base_binary_edge.hpp:55-120; vertex 0 = landmark, Jacobian A; vertex 1 = pose, Jacobian B; the Hpl block is
    // mapped transposed, _hessianTransposed).  Omega is diagonal, so Eigen's temporaries reduce to:
    //   robust:     W = rho' Omega;  Hll += (A^T W) A;  Hpl += (B^T W) A;  Hpp += (B^T W) B;
    //               omega_r = (-(Omega e)) rho';  bl += A^T omega_r;  bp += B^T omega_r
    //   non-robust: AtO = A^T Omega;  Hll += AtO A;  Hpl += B^T AtO^T;  Hpp += (B^T Omega) B;  omega_r = -Omega e
    void build_system() {
        Hpp.assign((size_t)np * 36, 0.0);
        Hll.assign((size_t)nl * 9, 0.0);
        b.assign((size_t)6 * np + 3 * nl, 0.0);
        lblocks.assign(nl, {});
        for (int k : active) {
            Edge& e = G.e[k];
            double A[3][3] = {}, B[3][6] = {};
            linearize(e, G, A, B);
            const Vtx& L = G.v[e.lm];
            const Vtx& P = G.v[e.kf];
            double w = 1.0;
            if (e.rk.on) { double rho[3]; e.rk.robustify(e.chi2(), rho); w = rho[1]; }
            double W[3], om_r[3];
            for (int r = 0; r < e.dim; r++) {
                W[r] = e.rk.on ? w * e.info[r] : e.info[r];
                om_r[r] = -(e.info[r] * e.err[r]);
                if (e.rk.on) om_r[r] *= w;
            }
            const bool lfree = !L.fixed, pfree = !P.fixed;
            if (lfree) {
                const int li = L.hidx;
                double* bl = &b[6 * np + 3 * li];
                double* H = &Hll[9 * li];
                for (int i = 0; i < 3; i++) {
                    double s = A[0][i] * om_r[0];
                    for (int r = 1; r < e.dim; r++) s += A[r][i] * om_r[r];
                    bl[i] += s;
                    for (int j = 0; j < 3; j++) {
                        double h = (A[0][i] * W[0]) * A[0][j];
                        for (int r = 1; r < e.dim; r++) h += (A[r][i] * W[r]) * A[r][j];
                        H[3 * i + j] += h;
                    }
                }
                if (pfree) {
                    auto& bl_list = lblocks[li];
                    Block* blk = nullptr;
                    for (auto& x : bl_list) if (x.pose == P.hidx) blk = &x;
                    if (!blk) { bl_list.push_back(Block{P.hidx, {}}); blk = &bl_list.back(); }
                    for (int i = 0; i < 6; i++)
                        for (int j = 0; j < 3; j++) {
                            double h;
                            if (e.rk.on) {
                                h = (B[0][i] * W[0]) * A[0][j];
                                for (int r = 1; r < e.dim; r++) h += (B[r][i] * W[r]) * A[r][j];
                            } else {
                                h = B[0][i] * (A[0][j] * e.info[0]);
                                for (int r = 1; r < e.dim; r++) h += B[r][i] * (A[r][j] * e.info[r]);
                            }
                            blk->B[i][j] += h;
                        }
                }
            }
            if (pfree) {
                const int pi = P.hidx;
                double* bp = &b[6 * pi];
                double* H = &Hpp[36 * pi];
                for (int i = 0; i < 6; i++) {
                    double s = B[0][i] * om_r[0];
                    for (int r = 1; r < e.dim; r++) s += B[r][i] * om_r[r];
                    bp[i] += s;
                    for (int j = 0; j < 6; j++) {
                        double h = (B[0][i] * W[0]) * B[0][j];
                        for (int r = 1; r < e.dim; r++) h += (B[r][i] * W[r]) * B[r][j];
                        H[6 * i + j] += h;
                    }
                }
            }
        }
        for (auto& bl : lblocks)
            std::sort(bl.begin(), bl.end(), [](const Block& a, const Block& c) { return a.pose < c.pose; });
    }
    double lambda_init() const {
        double m = 0;
        for (int p = 0; p < np; p++)
            for (int j = 0; j < 6; j++) m = std::max(std::fabs(Hpp[36 * p + 7 * j]), m);
        for (int l = 0; l < nl; l++)
            for (int j = 0; j < 3; j++) m = std::max(std::fabs(Hll[9 * l + 4 * j]), m);
        return 1e-5 * m;
    }
    // BlockSolver::solve with lambda on the diagonals (setLambda): Schur complement landmark by landmark
    // (block_solver.hpp:381-431), LinearSolverEigen on the reduced system, landmark back-substitution (:444-471).
    // x: g2o's solution buffer (Solver::_x), written only by a successful solve.  It persists for the whole call --
    // both optimize() passes, whose layouts may differ (resizeVector keeps the allocation) -- and a failed solve
    // leaves the previous solution in it, which update() and computeScale() then read anyway
    // (optimization_algorithm_levenberg.cpp:110-127); "never written" is pinned to zeros (a fresh allocation).
    bool solve(double lam, std::vector<double>& xbuf) {
        const int n = 6 * np;
        std::vector<double> x((size_t)n + 3 * nl, 0.0);
        // _Hschur->clear(); _Hpp->add(_Hschur)  (whole diagonal blocks, lambda included)
        std::vector<double> S((size_t)n * n, 0.0), coeff((size_t)n, 0.0);
        for (int p = 0; p < np; p++)
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 6; j++) S[(size_t)(6 * p + i) * n + 6 * p + j] = Hpp[36 * p + 6 * i + j] + (i == j ? lam : 0.0);
        std::vector<double> Dinv((size_t)nl * 9);
        for (int l = 0; l < nl; l++) {
            double D[3][3], Di[3][3];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) D[i][j] = Hll[9 * l + 3 * i + j] + (i == j ? lam : 0.0);
            inverse3(D, Di);
            std::memcpy(&Dinv[9 * l], Di, sizeof Di);
            const double* bl = &b[n + 3 * l];
            double db[3];
            for (int i = 0; i < 3; i++) db[i] = (Di[i][0] * bl[0] + Di[i][1] * bl[1]) + Di[i][2] * bl[2];
            const auto& col = lblocks[l];
            for (size_t a = 0; a < col.size(); a++) {
                const int i1 = col[a].pose;
                const double (&Bi)[6][3] = col[a].B;
                double BDinv[6][3];
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 3; c++)
                        BDinv[r][c] = (Bi[r][0] * Di[0][c] + Bi[r][1] * Di[1][c]) + Bi[r][2] * Di[2][c];
                for (int r = 0; r < 6; r++) coeff[6 * i1 + r] += (Bi[r][0] * db[0] + Bi[r][1] * db[1]) + Bi[r][2] * db[2];
                for (size_t c2 = a; c2 < col.size(); c2++) {
                    const int i2 = col[c2].pose;
                    const double (&Bj)[6][3] = col[c2].B;
                    for (int r = 0; r < 6; r++)
                        for (int c = 0; c < 6; c++)
                            S[(size_t)(6 * i1 + r) * n + 6 * i2 + c] -=
                                (BDinv[r][0] * Bj[c][0] + BDinv[r][1] * Bj[c][1]) + BDinv[r][2] * Bj[c][2];
                }
            }
        }
        std::vector<double> bs((size_t)n);
        for (int i = 0; i < n; i++) bs[i] = b[i] - coeff[i];
        if (!analyzed) {
            ldlt.analyze(n, Ap, Ai);
            analyzed = true;
        }
        std::vector<double> Ax(Ai.size());
        for (int c = 0; c < n; c++)
            for (int p = Ap[c]; p < Ap[c + 1]; p++) Ax[p] = S[(size_t)Ai[p] * n + c];
        if (((solve_fail_mask >> (trials & 31)) & 1u) && trials < 32) return false;  // (test hook)
        if (!ldlt.factorize(Ax)) return false;
        ldlt.solve(bs.data(), x.data());
        // landmarks: cl = bl - Hpl^T xp (_HplCCS->rightMultiply with cp = -xp), xl = Dinv cl
        for (int l = 0; l < nl; l++) {
            double cl[3];
            for (int i = 0; i < 3; i++) cl[i] = b[n + 3 * l + i];
            for (const auto& blk : lblocks[l])
                for (int i = 0; i < 3; i++) {
                    double s = 0;
                    for (int j = 0; j < 6; j++) s += blk.B[j][i] * (-x[6 * blk.pose + j]);
                    cl[i] += s;
                }
            const double* Di = &Dinv[9 * l];
            for (int i = 0; i < 3; i++) x[n + 3 * l + i] = (Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1]) + Di[3 * i + 2] * cl[2];
        }
        if (xbuf.size() < x.size()) xbuf.resize(x.size(), 0.0);
        std::copy(x.begin(), x.end(), xbuf.begin());
        return true;
    }
    void push() {
        for (int i : poses) G.v[i].Tb = G.v[i].T;
        for (int i : lms) { G.v[i].Xb = G.v[i].X; G.v[i].Pb = G.v[i].P; }
    }
    void pop() {
        for (int i : poses) G.v[i].T = G.v[i].Tb;
        for (int i : lms) { G.v[i].X = G.v[i].Xb; G.v[i].P = G.v[i].Pb; }
    }
    void update(const std::vector<double>& x) {
        for (int p = 0; p < np; p++) {
            Vtx& V = G.v[poses[p]];
            V.T = SE3::exp(&x[6 * p]) * V.T;
        }
        for (int l = 0; l < nl; l++) {
            Vtx& V = G.v[lms[l]];
            const double* u = &x[6 * np + 3 * l];
            if (V.kind == 1) V.X = V3{V.X.x + u[0], V.X.y + u[1], V.X.z + u[2]};
            else plane_oplus(V.P, u);
        }
    }
    // SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg
    // pbStopFlag emulation: the flag is raised right after trial number stop_after (SparseOptimizer::terminate();
    // stop_after < 0: never).  cut = a check point saw it where the schedule would have continued.
    int trials = 0, stop_after = -1;
    unsigned solve_fail_mask = oracle_get_solve_fail_mask();
    std::vector<double> xbuf;  // g2o's _x (see solve())
    bool cut = false;
    bool terminate() const { return stop_after >= 0 && trials >= stop_after; }
    int optimize(int iterations) {
        if (active.empty() || (np == 0 && nl == 0)) return 0;
        int its = 0;
        for (int it = 0; it < iterations; it++) {
            if (terminate()) {  // for (...; i < iterations && !terminate() && ok; ...)
                cut = true;
                break;
            }
            compute_errors();
            double currentChi = robust_chi2();
            const double iniChi = currentChi;
            build_system();
            if (it == 0) { lambda = lambda_init(); ni = 2; nBad = 0; }
            double rho = 0;
            int qmax = 0;
            bool more;
            const size_t sz = (size_t)6 * np + 3 * nl;  // _solver->vectorSize()
            do {
                push();
                const bool ok = solve(lambda, xbuf);
                if (xbuf.size() < sz) xbuf.resize(sz, 0.0);
                update(xbuf);  // _optimizer->update(_solver->x()), whether or not the solve succeeded
                compute_errors();
                double tempChi = robust_chi2();
                if (!ok) tempChi = std::numeric_limits<double>::max();
                rho = currentChi - tempChi;
                double scale = 0;
                for (size_t j = 0; j < sz; j++) scale += xbuf[j] * (lambda * xbuf[j] + b[j]);
                scale += 1e-3;
                rho /= scale;
                if (rho > 0 && std::isfinite(tempChi)) {
                    double alpha = 1. - o_cube(2 * rho - 1);
                    alpha = std::min(alpha, 2. / 3.);
                    lambda *= std::max(1. / 3., alpha);
                    ni = 2;
                    currentChi = tempChi;
                } else {
                    lambda *= ni;
                    ni *= 2;
                    pop();
                }
                qmax++;
                trials++;
                more = rho < 0 && qmax < 10;
                if (more && terminate()) {  // while (rho < 0 && qmax < max && !terminate())
                    cut = true;
                    more = false;
                }
            } while (more);
            its++;
            if (qmax == 10 || rho == 0) break;
            if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
            else nBad = 0;
            if (nBad >= 3) break;
        }
        return its;
    }
};

}  // namespace lba
}  // namespace oracle

using namespace ORACLE_NS;
using namespace ORACLE_NS::lba;

namespace {
SE3 se3_from_cv(const float* Tcw) {
    M3 R;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R.m[i][j] = Tcw[4 * i + j];
    return SE3::from_Rt(R, {Tcw[3], Tcw[7], Tcw[11]});
}
void se3_to_cv(const SE3& T, float* out) {
    const M3 R = quat_to_rot(T.r);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) out[4 * i + j] = (float)R.m[i][j];
    out[3] = (float)T.t.x; out[7] = (float)T.t.y; out[11] = (float)T.t.z;
    out[12] = 0.f; out[13] = 0.f; out[14] = 0.f; out[15] = 1.f;
}
Plane plane_from_cv(const float* c) {  // Converter::toPlane3D: flip d < 0, then Plane3D(v) normalises
    double v[4] = {c[0], c[1], c[2], c[3]};
    if (c[3] < 0.0f)
        for (double& x : v) x = -x;
    return Plane::from(v);
}
}  // namespace

// stop_after: pbStopFlag raised after that many LM trials (0 = already set at the call: the reference returns
// before initializeOptimization, Optimizer.cc:1757-1759; < 0 = never raised)
#ifndef ORACLE_FMA_VARIANT
extern "C" int oracle_get_g2o_fma();  // pose_oracle.cpp: this thread's FMA diagnostic mode
extern "C" int oracle_lba_optimize_stop_fma(const spslam_lba_problem* P, const spslam_lba_keyframe* kfs,
                                            const spslam_lba_point* pts, const spslam_lba_point_obs* pobs,
                                            const spslam_lba_plane* pls, const spslam_lba_plane_obs* plobs,
                                            const spslam_plane_config* cfg, float* kf_out, float* pt_out,
                                            float* pl_out, uint8_t* pobs_outlier, uint8_t* plobs_outlier,
                                            spslam_lba_result* res, int stop_after);
#endif
extern "C" int ORACLE_ENTRY(oracle_lba_optimize_stop)(const spslam_lba_problem* P, const spslam_lba_keyframe* kfs,
                                                      const spslam_lba_point* pts, const spslam_lba_point_obs* pobs,
                                                      const spslam_lba_plane* pls, const spslam_lba_plane_obs* plobs,
                                                      const spslam_plane_config* cfg, float* kf_out, float* pt_out,
                                                      float* pl_out, uint8_t* pobs_outlier, uint8_t* plobs_outlier,
                                                      spslam_lba_result* res, int stop_after) {
#ifndef ORACLE_FMA_VARIANT
    if (oracle_get_g2o_fma())
        return oracle_lba_optimize_stop_fma(P, kfs, pts, pobs, pls, plobs, cfg, kf_out, pt_out, pl_out, pobs_outlier,
                                            plobs_outlier, res, stop_after);
#endif
    std::memset(res, 0, sizeof *res);
    if (stop_after == 0) {  // if(*pbStopFlag) return;  -- nothing optimised, nothing erased
        for (int k = 0; k < P->n_kf; k++) std::memcpy(kf_out + 16 * k, kfs[k].Tcw, 64);
        for (int i = 0; i < P->n_points; i++) std::memcpy(pt_out + 3 * i, pts[i].xw, 12);
        for (int i = 0; i < P->n_planes; i++) std::memcpy(pl_out + 4 * i, pls[i].world, 16);
        std::memset(pobs_outlier, 0, P->n_point_obs);
        std::memset(plobs_outlier, 0, P->n_plane_obs);
        res->stopped = 1;
        return 0;
    }
    Graph G;
    long long maxKFid = 0, maxPointid = 0;
    for (int k = 0; k < P->n_kf; k++) {
        const spslam_lba_keyframe& K = kfs[k];
        Vtx v;
        v.kind = 0;
        v.id = K.id;
        v.fixed = K.fixed || K.id == 0;
        v.T = se3_from_cv(K.Tcw);
        G.v.push_back(v);
        maxKFid = std::max(maxKFid, (long long)K.id);
    }
    const int v_pt0 = (int)G.v.size();
    for (int i = 0; i < P->n_points; i++) {
        Vtx v;
        v.kind = 1;
        v.id = pts[i].id + maxKFid + 1;
        v.X = V3{pts[i].xw[0], pts[i].xw[1], pts[i].xw[2]};
        maxPointid = std::max(maxPointid, v.id);
        G.v.push_back(v);
    }
    const int v_pl0 = (int)G.v.size();
    for (int i = 0; i < P->n_planes; i++) {
        Vtx v;
        v.kind = 2;
        v.id = pls[i].id + maxPointid + 1;
        v.P = plane_from_cv(pls[i].world);
        G.v.push_back(v);
    }
    const float thMono = std::sqrt(5.991), thStereo = std::sqrt(7.815);
    std::vector<int> pobs_edge, plobs_edge;
    for (int i = 0; i < P->n_points; i++)
        for (int o = pts[i].obs_offset; o < pts[i].obs_offset + pts[i].n_obs; o++) {
            const spslam_lba_point_obs& ob = pobs[o];
            const spslam_lba_keyframe& K = kfs[ob.kf];
            Edge e;
            e.lm = v_pt0 + i;
            e.kf = ob.kf;
            e.meas[0] = ob.u; e.meas[1] = ob.v; e.meas[2] = ob.ur;
            if (ob.ur < 0) { e.type = 0; e.dim = 2; e.rk.set(thMono); }
            else { e.type = 1; e.dim = 3; e.rk.set(thStereo); }
            for (double& x : e.info) x = (double)ob.inv_sigma2;
            e.fx = K.fx; e.fy = K.fy; e.cx = K.cx; e.cy = K.cy; e.bf = K.bf;
            pobs_edge.push_back((int)G.e.size());
            G.e.push_back(e);
        }
    const double angleInfo = 3282.8 / (cfg->angle_info * cfg->angle_info);
    const double disInfo = cfg->distance_info * cfg->distance_info;
    const double parInfo = 3282.8 / (cfg->parallel_info * cfg->parallel_info);
    const double verInfo = 3282.8 / (cfg->vertical_info * cfg->vertical_info);
    const double planeChi = cfg->chi, VPplaneChi = cfg->vp_chi;
    const float deltaPlane = std::sqrt(planeChi), VPdeltaPlane = std::sqrt(VPplaneChi);
    for (int i = 0; i < P->n_planes; i++)
        for (int o = pls[i].obs_offset; o < pls[i].obs_offset + pls[i].n_obs; o++) {
            const spslam_lba_plane_obs& ob = plobs[o];
            Edge e;
            e.lm = v_pl0 + i;
            e.kf = ob.kf;
            e.mplane = plane_from_cv(ob.meas);
            e.fx = e.fy = e.cx = e.cy = e.bf = 0;
            if (ob.kind == SPSLAM_PLANE_EDGE) {
                e.type = 2; e.dim = 3;
                e.info[0] = e.info[1] = angleInfo; e.info[2] = disInfo;
                e.rk.set(deltaPlane);
            } else {
                e.type = ob.kind == SPSLAM_PARALLEL_EDGE ? 3 : 4;
                e.dim = 2;
                e.info[0] = e.info[1] = ob.kind == SPSLAM_PARALLEL_EDGE ? parInfo : verInfo;
                e.info[2] = 0;
                e.rk.set(VPdeltaPlane);
            }
            plobs_edge.push_back((int)G.e.size());
            G.e.push_back(e);
        }
    Opt opt(G);
    opt.stop_after = stop_after;
    res->iterations[0] = res->iterations[1] = 0;
    if (!G.e.empty()) {
        opt.initialize(0);
        res->iterations[0] = opt.optimize(5);
    }
    if (!G.e.empty() && opt.terminate()) {
        opt.cut = true;  // bool bDoMore = !*pbStopFlag (Optimizer.cc:1763-1767): no relabel, no optimize(10)
    } else if (!G.e.empty()) {
        // relabel with the cached errors, drop the robust kernels
        for (Edge& e : G.e) {
            bool bad;
            if (e.type == 0) bad = e.chi2() > 5.991 || !depth_positive(e, G);
            else if (e.type == 1) bad = e.chi2() > 7.815 || !depth_positive(e, G);
            else if (e.type == 2) bad = e.chi2() > planeChi;
            else bad = e.chi2() > VPplaneChi;
            if (bad) e.level = 1;
            e.rk.on = false;
        }
        opt.initialize(0);
        res->iterations[1] = opt.optimize(10);
    }
    int npo = 0, nplo = 0;
    for (size_t k = 0; k < pobs_edge.size(); k++) {
        const Edge& e = G.e[pobs_edge[k]];
        const bool bad = e.chi2() > (e.type == 0 ? 5.991 : 7.815) || !depth_positive(e, G);
        pobs_outlier[k] = bad;
        npo += bad;
    }
    for (size_t k = 0; k < plobs_edge.size(); k++) {
        const Edge& e = G.e[plobs_edge[k]];
        const bool bad = e.type == 2 ? e.chi2() > planeChi : e.chi2() > VPplaneChi;
        plobs_outlier[k] = bad;
        nplo += bad;
    }
    res->n_point_outliers = npo;
    res->n_plane_outliers = nplo;
    res->status = 0;
    res->trials = opt.trials;
    res->stopped = opt.cut ? 2 : 0;
    for (int k = 0; k < P->n_kf; k++) {
        if (!kfs[k].fixed) se3_to_cv(G.v[k].T, kf_out + 16 * k);
        else std::memcpy(kf_out + 16 * k, kfs[k].Tcw, 64);
    }
    for (int i = 0; i < P->n_points; i++) {
        const V3& X = G.v[v_pt0 + i].X;
        pt_out[3 * i] = (float)X.x; pt_out[3 * i + 1] = (float)X.y; pt_out[3 * i + 2] = (float)X.z;
    }
    for (int i = 0; i < P->n_planes; i++)
        for (int j = 0; j < 4; j++) pl_out[4 * i + j] = (float)G.v[v_pl0 + i].P.c[j];
    return 0;
}

extern "C" int ORACLE_ENTRY(oracle_lba_optimize)(const spslam_lba_problem* P, const spslam_lba_keyframe* kfs,
                                                 const spslam_lba_point* pts, const spslam_lba_point_obs* pobs,
                                                 const spslam_lba_plane* pls, const spslam_lba_plane_obs* plobs,
                                                 const spslam_plane_config* cfg, float* kf_out, float* pt_out,
                                                 float* pl_out, uint8_t* pobs_outlier, uint8_t* plobs_outlier,
                                                 spslam_lba_result* res) {
    return ORACLE_ENTRY(oracle_lba_optimize_stop)(P, kfs, pts, pobs, pls, plobs, cfg, kf_out, pt_out, pl_out, pobs_outlier,
                                    plobs_outlier, res, -1);
}

// Test access to the SimplicialLDLT restatement (tests/test_oracle_lba.py): factorise the upper-triangular CCS
// pattern (Ap, Ai) with values Ax, solve A x = b; perm receives the AMD order (Pinv).  Returns 0, or 1 on a
// zero pivot.
extern "C" int ORACLE_ENTRY(oracle_eigen_ldlt)(int n, const int* Ap, const int* Ai, const double* Ax, const double* b, double* x,
                                 int* perm) {
    ORACLE_NS::eigen_sparse::SimplicialLDLT s;
    std::vector<int> ap(Ap, Ap + n + 1), ai(Ai, Ai + Ap[n]);
    s.analyze(n, ap, ai);
    for (int k = 0; k < n; k++) perm[k] = s.Pinv[k];
    if (!s.factorize(std::vector<double>(Ax, Ax + Ap[n]))) return 1;
    s.solve(b, x);
    return 0;
}
