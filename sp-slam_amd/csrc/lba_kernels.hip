// gfx950 LocalBundleAdjustment (reference: src/Optimizer.cc:1154-1977 on the
// vendored g2o BlockSolver_6_3 + Levenberg-Marquardt, g2oAddition plane
// edges).  Semantics: oracle/lba_oracle.cpp.
//
// A batch of local maps (the keyframes of many sequences) is optimised
// together.  Every phase of an LM step is a grid-wide kernel whose
// workgroups cover all problems at once (a (problem, chunk) work table built
// on the host), so one map spreads over many CUs and latency-bound loops run
// with hundreds of waves in flight:
//   structure   per keyframe: active-edge counts and edge lists (stable);
//               per problem: pose Hessian order (by id), landmark pose masks
//               and (landmark, pose) blocks;
//   errors      edge chunks: error + robust chi2, chunk partial sums;
//   edge terms  edge chunks: analytic (points) / central-difference (planes,
//               both vertices) Jacobians and the quadratic-form terms;
//   sums        landmark chunks: Hll, bl, blocks; keyframes: Hpp, bp;
//   Schur       landmark chunks: (Hll + lambda)^-1 (Eigen 3x3 cofactor inverse),
//               Dinv bl, B Dinv; pose-pair tasks: Hpp + lambda - sum B Dinv B^T,
//               bp - sum B Dinv bl (64-bit pose masks, threads over landmarks);
//   factor      per problem: LDL^T of the reduced 6P x 6P system in LDS
//               (right-looking, the oracle's per-entry operation order);
//   update      landmark chunks / keyframes: backup, back-substitution,
//               exp(x) * T, X + x, Plane3D::oplus, step-scale partials;
//   decide      per problem: OptimizationAlgorithmLevenberg's accept / reject,
//               lambda, iteration and schedule bookkeeping (optimize(5),
//               relabel with the cached errors, optimize(10));
//   restore     rejected trials roll back.
// The host enqueues steps and polls a device counter every few steps.
// pbStopFlag (Optimizer.cc:1351-1352, 1757-1767; g2o SparseOptimizer::terminate):
// read by one thread per problem at g2o's check points -- before optimize(5)
// (return, nothing changed), after every trial (the LM do-while), at every
// iteration start (the optimize() loop), between the passes (bDoMore) -- and
// latched; a raised flag ends the schedule where it would have continued.
// All arithmetic is fp64; reductions are tree-ordered, so results match the
// oracle to rounding (north-star bar 1e-4), not bitwise.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "g2o_device.h"
#include "lba_launch.h"

namespace spslam {
namespace lba {

using namespace g2od;

constexpr int kThreads = kLbaChunk, kWaves = kThreads / 64;
constexpr int kStruct = 0, kIter = 1, kTrial = 2, kRelabel = 3, kDone = 4;
constexpr int kFactorLds = 150 * 1024;   // reduced system held in LDS up to n = 140

struct Ctx {
    int K, Np, Nq, E, Ep, L, nEc, nLc;
    const spslam_lba_keyframe* kf;
    const spslam_lba_point* pt;
    const spslam_lba_point_obs* pobs;
    const spslam_lba_plane* pl;
    const spslam_lba_plane_obs* plobs;
    LbaCtl* ctl;
    double *pose, *pose_b, *X, *X_b, *P, *P_b, *err, *con, *lmH, *lmb, *Dinv, *db, *xl, *blkH, *blkBD, *S, *bs, *dd, *y, *S_part,
        *Hpp, *bp, *part_chi, *part_scale, *part_max;
    int *pose_hidx, *hidx_pose, *e_lm, *e_kf, *e_type, *e_level, *e_blk, *e_src, *lm_boff, *lm_nb, *lm_act, *kf_cnt,
        *pe_off, *pe_idx;
    uint64_t* lm_mask;
};

__device__ Ctx make_ctx(const LbaBatch& b, int p) {
    const spslam_lba_problem pb = b.probs[p];
    Ctx c;
    c.K = pb.n_kf; c.Np = pb.n_points; c.Nq = pb.n_planes;
    c.Ep = pb.n_point_obs; c.E = pb.n_point_obs + pb.n_plane_obs; c.L = c.Np + c.Nq;
    c.nEc = lba_chunks(c.E); c.nLc = lba_chunks(c.L);
    c.kf = b.kfs + pb.kf_offset; c.pt = b.pts + pb.point_offset; c.pl = b.pls + pb.plane_offset;
    c.pobs = b.pobs; c.plobs = b.plobs;
    const LbaLayout Ly = lba_layout(c.K, c.Np, c.Nq, c.E);
    uint8_t* base = b.scratch + b.scratch_off[p];
    c.ctl = (LbaCtl*)(base + Ly.ctl);
    c.pose = (double*)(base + Ly.pose); c.pose_b = (double*)(base + Ly.pose_b);
    c.X = (double*)(base + Ly.pt); c.X_b = (double*)(base + Ly.pt_b);
    c.P = (double*)(base + Ly.pl); c.P_b = (double*)(base + Ly.pl_b);
    c.err = (double*)(base + Ly.e_err); c.con = (double*)(base + Ly.e_con);
    c.lmH = (double*)(base + Ly.lm_H); c.lmb = (double*)(base + Ly.lm_b); c.Dinv = (double*)(base + Ly.lm_Dinv);
    c.db = (double*)(base + Ly.lm_db); c.xl = (double*)(base + Ly.lm_x);
    c.blkH = (double*)(base + Ly.blk_H); c.blkBD = (double*)(base + Ly.blk_BD);
    c.S_part = (double*)(base + Ly.S_part);
    c.S = (double*)(base + Ly.S); c.bs = (double*)(base + Ly.bs); c.dd = (double*)(base + Ly.dd);
    c.y = (double*)(base + Ly.y); c.Hpp = (double*)(base + Ly.Hpp); c.bp = (double*)(base + Ly.bp);
    c.part_chi = (double*)(base + Ly.part_chi); c.part_scale = (double*)(base + Ly.part_scale);
    c.part_max = (double*)(base + Ly.part_max);
    c.pose_hidx = (int*)(base + Ly.pose_hidx); c.hidx_pose = (int*)(base + Ly.hidx_pose);
    c.e_lm = (int*)(base + Ly.e_lm); c.e_kf = (int*)(base + Ly.e_kf); c.e_type = (int*)(base + Ly.e_type);
    c.e_level = (int*)(base + Ly.e_level); c.e_blk = (int*)(base + Ly.e_blk); c.e_src = (int*)(base + Ly.e_src);
    c.lm_boff = (int*)(base + Ly.lm_boff); c.lm_nb = (int*)(base + Ly.lm_nb); c.lm_act = (int*)(base + Ly.lm_act);
    c.kf_cnt = (int*)(base + Ly.kf_cnt); c.pe_off = (int*)(base + Ly.pe_off); c.pe_idx = (int*)(base + Ly.pe_idx);
    c.lm_mask = (uint64_t*)(base + Ly.lm_mask);
    return c;
}

__device__ __forceinline__ void wave_sync() {  // LDS written by this wave, visible to this wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ SE3 load_pose(const double* p) { return SE3{Q{p[0], p[1], p[2], p[3]}, V3{p[4], p[5], p[6]}}; }
__device__ __forceinline__ void store_pose(double* p, const SE3& T) {
    p[0] = T.r.w; p[1] = T.r.x; p[2] = T.r.y; p[3] = T.r.z; p[4] = T.t.x; p[5] = T.t.y; p[6] = T.t.z;
}
// SparseOptimizer::terminate(): the caller's flag, read through to memory (it may be host-coherent and
// raised by another thread while the schedule runs), latched once seen
__device__ __forceinline__ bool stop_requested(const LbaBatch& b, int p, LbaCtl& k) {
    if (!k.stop && b.stop) k.stop = __hip_atomic_load(b.stop + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    if (!k.stop && b.stop_after >= 0 && k.trials >= b.stop_after) k.stop = 1;  // spslam_lba_debug_stop_after
    return k.stop != 0;
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

struct Red {
    double v[kWaves][40];
    int wsum[kWaves];
};

// Block-wide sum of NV doubles per thread (tree order); result valid in every thread.
template <int NV>
__device__ void block_sum(double (&v)[NV], Red& R) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; k++) {
        double x = v[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
        if (lane == 0) R.v[w][k] = x;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; k++) {
        double s = 0;
#pragma unroll
        for (int j = 0; j < kWaves; j++) s += R.v[j][k];
        v[k] = s;
    }
    __syncthreads();
}
__device__ double block_max(double v, Red& R) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    if (lane == 0) R.v[w][0] = v;
    __syncthreads();
    double m = 0;
    for (int j = 0; j < kWaves; j++) m = fmax(m, R.v[j][0]);
    __syncthreads();
    return m;
}
// Exclusive block scan of one int per thread; *total = block sum.
__device__ int block_scan(int v, int* total, Red& R) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) R.wsum[w] = x;
    __syncthreads();
    int base = 0, tot = 0;
    for (int j = 0; j < kWaves; j++) {
        if (j < w) base += R.wsum[j];
        tot += R.wsum[j];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

__device__ __forceinline__ int lm_block_base(const Ctx& c, int l) { return c.lm_act[l] - 1; }
// e_blk: the edge's (landmark, pose) block, -1 if none; kBlkShared marks the edges of a landmark with two active
// edges on one block (summed by the landmark's owner in edge order, not stored per edge)
constexpr int kBlkShared = 1 << 30;
__device__ __forceinline__ int edge_block(const Ctx& c, int e) {
    const int v = c.e_blk[e];
    return v < 0 ? -1 : (v & (kBlkShared - 1));
}

// Edge Jacobians: A (landmark, dim x 3), B (pose, dim x 6); fixed vertices skipped.
// kOnly: 0 = any edge, 1 = point edges only, 2 = plane edges only (the caller filtered the type; instances
// without the numeric plane Jacobians need far fewer registers)
template <int kOnly = 0>
__device__ void edge_jacobians(const Ctx& c, int e, bool pose_free, double (&A)[3][3], double (&B)[3][6]) {
    const int t = c.e_type[e], lm = c.e_lm[e];
    const SE3 T = load_pose(c.pose + 7 * c.e_kf[e]);
    if (kOnly != 2 && (kOnly == 1 || t <= 1)) {
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


// ---------------------------------------------------------------- setup
__global__ __launch_bounds__(kThreads) void k_setup(LbaBatch b, int max_it0) {
    __shared__ Red R;
    const int p = blockIdx.x, t = threadIdx.x;
    Ctx c = make_ctx(b, p);
    spslam_lba_result* res = b.res + p;
    if (c.K > kLbaMaxKeyframes) {
        if (t == 0) {
            *res = spslam_lba_result{};
            res->status = -2;
            c.ctl->state = kDone;
        }
        return;
    }
    for (int k = t; k < c.K; k += kThreads) {  // Converter::toSE3Quat
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
        const P4 q = plane_from_f(c.pl[i].world);
        for (int j = 0; j < 4; j++) c.P[4 * i + j] = q.c[j];
    }
    // edges in insertion order: point observations (points in list order), then plane observations
    int base_e = 0;
    for (int ch = 0; ch < c.L; ch += kThreads) {
        const int l = ch + t;
        const int n_obs = l < c.Np ? c.pt[l].n_obs : (l < c.L ? c.pl[l - c.Np].n_obs : 0);
        int tot;
        const int off = block_scan(n_obs, &tot, R) + base_e;
        if (l < c.L) {
            c.lm_boff[l] = off;
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
    if (t == 0) {
        LbaCtl& k = *c.ctl;
        k = LbaCtl{};
        k.state = c.E > 0 ? kStruct : kDone;
        k.phase = 0;
        k.it = 0;
        k.max_it = max_it0;
        k.robust = 1;
        k.restore_step = -1;
        k.t0 = wall_clock64();
        if (stop_requested(b, p, k)) {  // if(*pbStopFlag) return; before initializeOptimization
            k.state = kDone;
            k.stopped = 1;
        }
    }
}

// start of a step: the optimize() loop's terminate() check at an iteration start (and at a pass start)
__global__ void k_step_begin(LbaBatch b) {
    if (threadIdx.x != 0) return;
    Ctx c = make_ctx(b, blockIdx.x);
    LbaCtl& k = *c.ctl;
    if ((k.state != kStruct && k.state != kIter) || !stop_requested(b, blockIdx.x, k)) return;
    k.stopped = k.phase == 0 && k.trials == 0 ? 1 : 2;  // nothing done yet: same as the early return
    k.state = kDone;
}

// ---------------------------------------------------------------- structure
__global__ __launch_bounds__(kThreads) void k_struct_count(LbaBatch b, LbaWork w) {
    __shared__ Red R;
    const int2 task = w.kf_tasks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    if (c.ctl->state != kStruct) return;
    const int k = task.y;
    int n = 0;
    for (int e = threadIdx.x; e < c.E; e += kThreads) n += (c.e_level[e] == 0 && c.e_kf[e] == k);
    int tot;
    block_scan(n, &tot, R);
    if (threadIdx.x == 0) c.kf_cnt[k] = tot;
}

// pose order (non-fixed keyframes with active edges, by id), edge-list offsets, landmark masks / blocks
__global__ __launch_bounds__(kThreads) void k_struct_final(LbaBatch b) {
    __shared__ Red R;
    __shared__ int hidx[kLbaMaxKeyframes];
    const int t = threadIdx.x;
    Ctx c = make_ctx(b, blockIdx.x);
    if (c.ctl->state != kStruct) return;
    if (t == 0) {
        int np = 0, o = 0;
        for (int k = 0; k < c.K; k++) {
            hidx[k] = -1;
            c.pe_off[k] = o;
            o += c.kf_cnt[k];
        }
        c.pe_off[c.K] = o;
        for (int k = 0; k < c.K; k++) {
            const spslam_lba_keyframe& kk = c.kf[k];
            if (!c.kf_cnt[k] || kk.fixed || kk.id == 0) continue;
            int j = np++;
            while (j > 0 && c.kf[c.hidx_pose[j - 1]].id > kk.id) { c.hidx_pose[j] = c.hidx_pose[j - 1]; j--; }
            c.hidx_pose[j] = k;
        }
        for (int j = 0; j < np; j++) hidx[c.hidx_pose[j]] = j;
        for (int k = 0; k < c.K; k++) c.pose_hidx[k] = hidx[k];
        c.ctl->np = np;
    }
    __syncthreads();
    int base = 0;
    for (int ch = 0; ch < c.L; ch += kThreads) {
        const int l = ch + t;
        uint64_t mask = 0;
        bool act = false, dup = false;
        int e_beg = 0, e_end = 0;
        if (l < c.L) {
            e_beg = c.lm_boff[l];
            e_end = e_beg + c.lm_nb[l];
        }
        for (int e = e_beg; e < e_end; e++)
            if (c.e_level[e] == 0) {
                act = true;
                const int h = hidx[c.e_kf[e]];
                if (h >= 0) {
                    dup |= (mask >> h) & 1ull;  // two active edges on one (landmark, pose) block
                    mask |= 1ull << h;
                }
            }
        const int nb = __popcll(mask);
        int tot;
        const int off = block_scan(nb, &tot, R) + base;
        if (l < c.L) {
            c.lm_mask[l] = mask;
            c.lm_act[l] = act ? off + 1 : 0;
            for (int e = e_beg; e < e_end; e++) {
                const int h = hidx[c.e_kf[e]];
                c.e_blk[e] = (c.e_level[e] == 0 && h >= 0)
                                 ? (off + __popcll(mask & ((1ull << h) - 1))) | (dup ? kBlkShared : 0)
                                 : -1;
            }
        }
        base += tot;
    }
}

// stable per-keyframe lists of active edges (insertion order)
__global__ __launch_bounds__(kThreads) void k_struct_fill(LbaBatch b, LbaWork w) {
    __shared__ Red R;
    const int2 task = w.kf_tasks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    if (c.ctl->state != kStruct) return;
    const int k = task.y;
    int o = c.pe_off[k];
    for (int ch = 0; ch < c.E; ch += kThreads) {
        const int e = ch + threadIdx.x;
        const int f = e < c.E && c.e_level[e] == 0 && c.e_kf[e] == k;
        int tot;
        const int r = block_scan(f, &tot, R);
        if (f) c.pe_idx[o + r] = e;
        o += tot;
    }
}

__global__ void k_struct_done(LbaBatch b) {
    if (threadIdx.x != 0) return;
    Ctx c = make_ctx(b, blockIdx.x);
    LbaCtl& k = *c.ctl;
    if (k.state != kStruct) return;
    k.state = kIter;
    k.it = 0;
}

// ---------------------------------------------------------------- errors, edge terms, sums
// mode 0: at the start of an LM iteration (ITER problems); mode 1: after a trial update (TRIAL problems)
__global__ __launch_bounds__(kThreads) void k_errors(LbaBatch b, LbaWork w, LbaConsts C, int mode) {
    __shared__ Red R;
    const int2 task = w.edge_chunks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    const LbaCtl& k = *c.ctl;
    if (k.state != (mode == 0 ? kIter : kTrial)) return;
    // the landmark part of computeLambdaInit's max is gathered by atomic max into part_max[0]; cleared here,
    // before the iteration's sums (every problem that reaches ITER has an edge chunk at task.y == 0)
    if (mode == 0 && task.y == 0 && threadIdx.x == 0) c.part_max[0] = 0.0;
    const int e = task.y + threadIdx.x;
    double acc[1] = {0.0};
    if (e < c.E && c.e_level[e] == 0) {
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
        const int ty = c.e_type[e];
        double r0, r1;
        huber(chi2_of(err, info, edge_dim(ty)), delta_of(C, ty), k.robust, &r0, &r1);
        acc[0] = r0;
    }
    block_sum(acc, R);
    if (threadIdx.x == 0) c.part_chi[task.y / kThreads] = acc[0];
}

// quadratic-form terms of active edge e from its Jacobians (A: landmark, B: pose) and cached error
__device__ __forceinline__ void store_terms(const Ctx& c, const LbaConsts& C, bool robust, int e, int ty, bool pfree,
                                            const double (&A)[3][3], const double (&B)[3][6]) {
    const int dim = edge_dim(ty);
    double info[3];
    info_of(c, C, e, info);
    const double* err = c.err + 3 * e;
    double r0, wgt;
    huber(chi2_of(err, info, dim), delta_of(C, ty), robust, &r0, &wgt);
    double W[3] = {0, 0, 0}, om[3] = {0, 0, 0};
#pragma unroll
    for (int r = 0; r < 3; r++)
        if (r < dim) {
            W[r] = robust ? wgt * info[r] : info[r];
            om[r] = -(info[r] * err[r]);
            if (robust) om[r] *= wgt;
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

// plane / parallel / vertical edges: central differences (base_binary_edge.hpp:130-205), one wave per edge.
// Evaluation q < 6 is the error at the plane perturbed by +-1e-9 along coordinate q >> 1 (Plane3D::oplus),
// 6 <= q < 18 at the pose exp(+-1e-9 e_d) * T, d = (q - 6) >> 1; evaluation q runs on the lane pair (2q, 2q + 1)
// (plane_error_pair: each lane one member of every atan2 / sincos pair), the differences are gathered with
// shuffles (the reference's per-coordinate expression) and lane 0 stores the terms.
#ifndef SPSLAM_LBA_PL_WAVES
#define SPSLAM_LBA_PL_WAVES 3  // waves per SIMD asked of k_plane_terms (3: 130 VGPRs, no spills; 4: 5 spilled)
#endif
__global__ __launch_bounds__(kThreads, SPSLAM_LBA_PL_WAVES) void k_plane_terms(LbaBatch b, LbaWork w, LbaConsts C) {
    const int2 task = w.plane_tasks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    const LbaCtl& k = *c.ctl;
    if (k.state != kIter) return;
    const int lane = threadIdx.x & 63;
    const int e = task.y + (threadIdx.x >> 6);
    if (e >= c.E || c.e_level[e] != 0) return;  // uniform over the wave
    const int ty = c.e_type[e], dim = edge_dim(ty), lm = c.e_lm[e];
    const bool pfree = c.pose_hidx[c.e_kf[e]] >= 0;
    const SE3 T0 = load_pose(c.pose + 7 * c.e_kf[e]);
    const double* pp = c.P + 4 * (lm - c.Np);
    const P4 P0{{pp[0], pp[1], pp[2], pp[3]}};
    const P4 meas = plane_from_f(c.plobs[c.e_src[e]].meas);
    const double delta = 1e-9, scalar = 1.0 / (2 * delta);
    double ev[3] = {0, 0, 0};
    const int q = lane >> 1;  // this lane pair's evaluation
    if (q < 18 && (q < 6 || pfree)) {
        const double sgn = (q & 1) ? -delta : delta;
        SE3 T = T0;
        P4 P = P0;
        if (q < 6) {
            double add[3] = {0, 0, 0};
            add[q >> 1] = sgn;
            p_oplus(P, add);
        } else {
            double add[6] = {0, 0, 0, 0, 0, 0};
            add[(q - 6) >> 1] = sgn;
            T = se3_mul(se3_exp(add), T0);
        }
        const E3 r = plane_error_pair(ty - 2, T, P, meas, (lane & 1) != 0);
        ev[0] = r.e0; ev[1] = r.e1; ev[2] = r.e2;
    }
    double A[3][3] = {}, B[3][6] = {};
#pragma unroll
    for (int d = 0; d < 3; d++)
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const double ep = __shfl(ev[i], 2 * (2 * d)), em = __shfl(ev[i], 2 * (2 * d + 1));
            A[i][d] = i < dim ? scalar * (ep - em) : 0.0;
        }
#pragma unroll
    for (int d = 0; d < 6; d++)
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const double ep = __shfl(ev[i], 2 * (6 + 2 * d)), em = __shfl(ev[i], 2 * (7 + 2 * d));
            B[i][d] = pfree && i < dim ? scalar * (ep - em) : 0.0;
        }
    if (lane == 0) store_terms(c, C, k.robust, e, ty, pfree, A, B);
}

// Point edges and point landmarks in one pass (the point part of k_lm_sums, without a per-edge kernel before
// it): a workgroup computes the quadratic-form terms of 256 consecutive point edges, one edge per thread
// (edge_jacobians<1> and store_terms' formulas).  Each edge's (landmark, pose) block (Hpl, 18) goes straight to
// memory from its thread -- the block's only term -- and its landmark terms (Hll 9, bl 3) to LDS; a landmark's
// edges are consecutive and at most kLbaMaxKeyframes, so the workgroup owns the landmarks whose first edge lies
// in its first w.seg_own edges and finds all their edges in LDS (the remaining rows are the halo).  Each owned
// landmark is summed by the thread of its first edge in insertion order, exactly as k_lm_sums sums the stored
// terms; a landmark with two active edges on one block (kBlkShared) has its blocks summed by the owner in edge
// order from recomputed terms.  Only the pose-side terms (Hpp 21, bp 6) still go to memory, for k_pose_sums.
constexpr int kSegStride = 13;  // odd stride in doubles (12 landmark terms)
#ifndef SPSLAM_LBA_PT_WAVES
#define SPSLAM_LBA_PT_WAVES 3  // waves per SIMD asked of k_point_terms_sums (3: no spills; 4 spills 28 VGPRs)
#endif
__global__ __launch_bounds__(kThreads, SPSLAM_LBA_PT_WAVES) void k_point_terms_sums(LbaBatch b, LbaWork w, LbaConsts C) {
    __shared__ Red R;
    __shared__ double Tm[kThreads * kSegStride];
    __shared__ uint8_t act[kThreads];
    const int2 task = w.seg_chunks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    const LbaCtl& k = *c.ctl;
    if (k.state != kIter) return;
    const int t = threadIdx.x, e = task.y + t;
    // the landmark-side terms of active point edge ee into row[] (12, or all 30 with the block's when full); when
    // own (each edge's by the workgroup that owns it): its pose-side terms (27) and, unless shared, its block
    auto land_terms = [&](int ee, double* row, bool own, bool full) __attribute__((always_inline)) {
        const int ty = c.e_type[ee];
        const bool pfree = c.pose_hidx[c.e_kf[ee]] >= 0;
        double A[3][3] = {}, B[3][6] = {};
        edge_jacobians<1>(c, ee, pfree, A, B);
        const int dim = edge_dim(ty);
        double info[3];
        info_of(c, C, ee, info);
        const double* err = c.err + 3 * ee;
        double r0, wgt;
        huber(chi2_of(err, info, dim), delta_of(C, ty), k.robust, &r0, &wgt);
        double W[3] = {0, 0, 0}, om[3] = {0, 0, 0};
#pragma unroll
        for (int r = 0; r < 3; r++)
            if (r < dim) {
                W[r] = k.robust ? wgt * info[r] : info[r];
                om[r] = -(info[r] * err[r]);
                if (k.robust) om[r] *= wgt;
            }
        const int bkv = c.e_blk[ee];
        const bool blk_here = own && bkv >= 0 && !(bkv & kBlkShared);
        double* hb = c.blkH + (size_t)(bkv & (kBlkShared - 1)) * 18;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            row[9 + i] = (A[0][i] * om[0] + A[1][i] * om[1]) + A[2][i] * om[2];
#pragma unroll
            for (int j = 0; j < 3; j++)
                row[3 * i + j] = ((A[0][i] * W[0]) * A[0][j] + (A[1][i] * W[1]) * A[1][j]) + (A[2][i] * W[2]) * A[2][j];
#pragma unroll
            for (int j = 0; j < 6; j++) {
                const double v = pfree ? ((A[0][i] * W[0]) * B[0][j] + (A[1][i] * W[1]) * B[1][j]) +
                                             (A[2][i] * W[2]) * B[2][j]
                                       : 0.0;
                if (full) row[12 + 6 * i + j] = v;
                if (blk_here) hb[6 * i + j] = v;
            }
        }
        if (pfree && own) {
            double* o = c.con + (size_t)kLbaCon * ee;
            int q = 30;
#pragma unroll
            for (int i = 0; i < 6; i++)
#pragma unroll
                for (int j = i; j < 6; j++)
                    o[q++] = ((B[0][i] * W[0]) * B[0][j] + (B[1][i] * W[1]) * B[1][j]) + (B[2][i] * W[2]) * B[2][j];
#pragma unroll
            for (int i = 0; i < 6; i++) o[51 + i] = (B[0][i] * om[0] + B[1][i] * om[1]) + B[2][i] * om[2];
        }
    };
    const bool a = e < c.Ep && c.e_level[e] == 0;
    if (a) {
        double row[30];
        land_terms(e, row, t < w.seg_own, false);
#pragma unroll
        for (int j = 0; j < 12; j++) Tm[t * kSegStride + j] = row[j];
    }
    act[t] = a;
    __syncthreads();
    double mx = 0.0;
    const int l = t < w.seg_own && e < c.Ep ? c.e_lm[e] : -1;
    if (l >= 0 && c.lm_boff[l] == e && lm_block_base(c, l) >= 0) {
        const int b0 = lm_block_base(c, l), nb = c.lm_nb[l];
        uint64_t written = 0;
        double H[9] = {}, bl[3] = {};
        for (int q = 0; q < nb; q++) {
            const int bkv = c.e_blk[e + q];
            const bool shared = bkv >= 0 && (bkv & kBlkShared);
            // rows past the workgroup's 256 (a landmark with more edges than the halo allows: only if a point
            // has more observations than the batch has keyframes) and the edges of shared blocks are computed here
            double r[30];
            if (t + q >= kThreads || shared) {
                if (c.e_level[e + q] != 0) continue;
                land_terms(e + q, r, false, true);
            } else {
                if (!act[t + q]) continue;
                const double* src = Tm + (t + q) * kSegStride;
#pragma unroll
                for (int j = 0; j < 12; j++) r[j] = src[j];
            }
#pragma unroll
            for (int j = 0; j < 9; j++) H[j] += r[j];
#pragma unroll
            for (int j = 0; j < 3; j++) bl[j] += r[9 + j];
            if (shared) {
                const int bk = bkv & (kBlkShared - 1);
                double* hb = c.blkH + (size_t)bk * 18;
                const uint64_t bit = 1ull << (bk - b0);
                if (written & bit) {
#pragma unroll
                    for (int j = 0; j < 18; j++) hb[j] += r[12 + j];
                } else {
#pragma unroll
                    for (int j = 0; j < 18; j++) hb[j] = r[12 + j];
                }
                written |= bit;
            }
        }
#pragma unroll
        for (int j = 0; j < 9; j++) c.lmH[9 * l + j] = H[j];
#pragma unroll
        for (int j = 0; j < 3; j++) c.lmb[3 * l + j] = bl[j];
        mx = fmax(fabs(H[0]), fmax(fabs(H[4]), fabs(H[8])));
    }
    mx = block_max(mx, R);
    // max |diag| (computeLambdaInit): non-negative doubles order like their bit patterns; k_errors cleared the slot
    if (t == 0 && mx > 0.0) atomicMax((unsigned long long*)c.part_max, (unsigned long long)__double_as_longlong(mx));
}

// Plane landmarks (point landmarks: k_point_terms_sums): Hll, bl and the (landmark, pose) blocks summed over the
// landmark's edges in insertion order from the terms k_plane_terms stored.  One wave per plane landmark, lane j
// < 30 owns term j (the same per-term sequence of adds as one thread summing all 30).
__global__ __launch_bounds__(kThreads) void k_plane_lm_sums(LbaBatch b, LbaWork w) {
    __shared__ Red R;
    const int2 task = w.plm_tasks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    if (c.ctl->state != kIter) return;
    const int lane = threadIdx.x & 63, l = task.y + (threadIdx.x >> 6);
    double acc = 0.0;
    bool have = false;
    if (l < c.L && lm_block_base(c, l) >= 0) {  // uniform over the wave
        have = true;
        const int b0 = lm_block_base(c, l), j = lane < 30 ? lane : 29;
        uint64_t written = 0;
        for (int e = c.lm_boff[l]; e < c.lm_boff[l] + c.lm_nb[l]; e++) {
            if (c.e_level[e] != 0) continue;
            const double v = c.con[(size_t)kLbaCon * e + j];
            const int bk = edge_block(c, e);
            if (lane < 12) acc += v;
            if (bk >= 0) {
                const uint64_t bit = 1ull << (bk - b0);
                double* hb = c.blkH + (size_t)bk * 18;
                if (lane >= 12 && lane < 30) hb[lane - 12] = (written & bit) ? hb[lane - 12] + v : v;
                written |= bit;
            }
        }
        if (lane < 9) c.lmH[9 * l + lane] = acc;
        else if (lane < 12) c.lmb[3 * l + lane - 9] = acc;
    }
    const double d0 = __shfl(acc, 0), d4 = __shfl(acc, 4), d8 = __shfl(acc, 8);
    double mx = have && lane == 0 ? fmax(fabs(d0), fmax(fabs(d4), fabs(d8))) : 0.0;
    mx = block_max(mx, R);
    if (threadIdx.x == 0 && mx > 0.0)
        atomicMax((unsigned long long*)c.part_max, (unsigned long long)__double_as_longlong(mx));
}

// keyframe Hpp, bp over its active edges (free poses only).  Bound by reading the per-edge pose-side terms
// (27 doubles per edge, ~80 MB per C3 call, from the MALL): coalesced 27-lane rows in 8 ordered streams measured
// the same 47 us, and prefetching 32 edge indices per stream slower (74 us)
__global__ __launch_bounds__(kThreads) void k_pose_sums(LbaBatch b, LbaWork w) {
    __shared__ Red R;
    const int2 task = w.kf_tasks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    if (c.ctl->state != kIter) return;
    const int k = task.y, h = c.pose_hidx[k];
    if (h < 0) {
        if (threadIdx.x == 0) c.part_max[c.nLc + k] = 0.0;
        return;
    }
    double acc[27];
#pragma unroll
    for (int j = 0; j < 27; j++) acc[j] = 0.0;
#pragma unroll 2  // the next edge's loads in flight beside this one's adds (same per-thread order)
    for (int i = c.pe_off[k] + threadIdx.x; i < c.pe_off[k + 1]; i += kThreads) {
        const double* o = c.con + (size_t)kLbaCon * c.pe_idx[i] + 30;
#pragma unroll
        for (int j = 0; j < 27; j++) acc[j] += o[j];
    }
    block_sum(acc, R);
    if (threadIdx.x < 36) {
        const int r = threadIdx.x / 6, q = threadIdx.x % 6, i = r < q ? r : q, j = r < q ? q : r;
        const int idx = 6 * i - i * (i - 1) / 2 + (j - i);
        double v = 0.0;
#pragma unroll
        for (int m = 0; m < 21; m++) if (m == idx) v = acc[m];
        c.Hpp[36 * h + threadIdx.x] = v;
    } else if (threadIdx.x < 42) {
        double v = 0.0;
#pragma unroll
        for (int m = 0; m < 6; m++) if (m == threadIdx.x - 36) v = acc[21 + m];
        c.bp[6 * h + threadIdx.x - 36] = v;
    }
    if (threadIdx.x == 0)
        c.part_max[c.nLc + k] = fmax(fmax(fmax(fabs(acc[0]), fabs(acc[6])), fmax(fabs(acc[11]), fabs(acc[15]))),
                                     fmax(fabs(acc[18]), fabs(acc[20])));
}

__global__ void k_iter_begin(LbaBatch b) {
    if (threadIdx.x != 0) return;
    Ctx c = make_ctx(b, blockIdx.x);
    LbaCtl& k = *c.ctl;
    if (k.state != kIter) return;
    double chi = 0.0;
#pragma unroll 8
    for (int i = 0; i < c.nEc; i++) chi += c.part_chi[i];
    k.currentChi = chi;
    k.iniChi = chi;
    if (k.it == 0) {  // computeLambdaInit: tau * max |diag| over the Hessian vertices
        // the landmark maximum is gathered by atomic max into part_max[0]; the pose maxima sit at [nLc, nLc + K)
        double mx = c.part_max[0];
#pragma unroll 8
        for (int i = c.nLc; i < c.nLc + c.K; i++) mx = fmax(mx, c.part_max[i]);
        k.lambda = 1e-5 * mx;
        k.ni = 2;
        k.nBad = 0;
    }
    k.qmax = 0;
    k.state = kTrial;
}

// ---------------------------------------------------------------- Schur complement
// reduced systems of 6 * np <= 80 rows: Schur sums on the matrix cores (k_schur_mfma + k_schur_reduce)
__device__ __forceinline__ bool mfma_schur(const LbaCtl& k) { return 6 * k.np <= 16 * kLbaMfmaTiles; }
__device__ __forceinline__ int mfma_tiles(const LbaCtl& k) { return (6 * k.np + 15) / 16; }

__global__ __launch_bounds__(kThreads) void k_schur_lm(LbaBatch b, LbaWork w) {
    const int2 task = w.lm_chunks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    const LbaCtl& k = *c.ctl;
    if (k.state != kTrial) return;
    const int l = task.y + threadIdx.x;
    if (l >= c.L || lm_block_base(c, l) < 0) return;
    const double lam = k.lambda;
    const int b0 = lm_block_base(c, l);
    double D[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) D[i][j] = c.lmH[9 * l + 3 * i + j] + (i == j ? lam : 0.0);
    double Di[9];
    inverse3(D, Di);
#pragma unroll
    for (int j = 0; j < 9; j++) c.Dinv[9 * l + j] = Di[j];
    const double* bl = c.lmb + 3 * l;
#pragma unroll
    for (int i = 0; i < 3; i++) c.db[3 * l + i] = (Di[3 * i] * bl[0] + Di[3 * i + 1] * bl[1]) + Di[3 * i + 2] * bl[2];
    if (mfma_schur(k)) return;  // k_schur_mfma forms B Dinv on the fly
    const int nb = __popcll(c.lm_mask[l]);
    for (int a = 0; a < nb; a++) {
        const double* H = c.blkH + (size_t)(b0 + a) * 18;  // 3 x 6 (landmark x pose)
        double* BD = c.blkBD + (size_t)(b0 + a) * 18;     // 6 x 3
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int q = 0; q < 3; q++) BD[3 * r + q] = (H[r] * Di[q] + H[6 + r] * Di[3 + q]) + H[12 + r] * Di[6 + q];
    }
}

// sum_l (B Dinv)_l B_l^T over the landmarks on v_mfma_f64_16x16x4: the reduced system (n = 6 np rows, padded
// to NT x 16) is NT x NT output tiles held by each wave; one MFMA per (tile, landmark) takes k = the landmark's
// 3 coordinates (+ one zero slot).  Lane l feeds A[row l & 15][k l >> 4] = (B Dinv)(pose row, k) formed on the
// fly from the landmark's (landmark, pose) block and Dinv (the pose-pair kernel's formula; zero where the pose
// does not observe the landmark) and B[k l >> 4][col l & 15] = the block's H entry.  Each wave takes
// kLbaMfmaLm landmarks of its workgroup's landmark chunk and writes its tiles to S_part; k_schur_reduce sums
// the partial sets in a fixed order.
// per-wave LDS batch (doubles): Dinv of up to kLbaMfmaLm landmarks (9 each), their bl (3 each), then blocks
constexpr int kStageB = 9 * kLbaMfmaLm, kStageH = 12 * kLbaMfmaLm, kStageD = 2048;
constexpr int kStageBlocks = (kStageD - kStageH) / 18;  // 92; the 1 KiB pieces round up within kStageD
static_assert(kStageH + ((18 * kStageBlocks * 8 + 1023) / 1024) * 128 <= kStageD, "block pieces fit the buffer");
static_assert(9 * kLbaMfmaLm * 8 <= 256 * 9 && 3 * kLbaMfmaLm * 8 <= 256 * 3, "Dinv / bl pieces");
template <int NT>
__global__ __launch_bounds__(kThreads) void k_schur_mfma(LbaBatch b, LbaWork w) {
    typedef double d4 __attribute__((ext_vector_type(4)));
    const int2 task = w.lm_chunks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    const LbaCtl& k = *c.ctl;
    if (k.state != kTrial || !mfma_schur(k) || (mfma_tiles(k) > NT) || (NT > 3 && mfma_tiles(k) < NT)) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n = 6 * k.np, kk = lane >> 4, r16 = lane & 15;
    const int grp = blockIdx.y * kWaves + wave;  // landmark group of the chunk (kLbaChunk / kLbaMfmaLm per chunk)
    const int l0 = task.y + grp * kLbaMfmaLm, nl = min(c.L - l0, kLbaMfmaLm);
    if (nl <= 0) return;  // partial sets exist for the first ceil(L / kLbaMfmaLm) landmark groups only
    // the group's pose masks and block bases, one landmark per lane (read back with readlane)
    const uint64_t m_l = lane < nl ? c.lm_mask[l0 + lane] : 0ull;
    const int b_l = lane < nl ? lm_block_base(c, l0 + lane) : -1;
    d4 acc[NT][NT], accb[NT];  // accb: the right-hand side sum_l (B Dinv)_l bl_l (B operand column 0 = bl)
#pragma unroll
    for (int i = 0; i < NT; i++) {
        accb[i] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < NT; j++) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
    }
    // this lane's pose and component in every tile row / column
    int pose_t[NT], comp_t[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int r = 16 * t + r16;
        pose_t[t] = r < n ? r / 6 : 63;
        comp_t[t] = r - 6 * (r / 6);
    }
    // The group's operands are staged in LDS by LDS-DMA (global_load_lds: no VGPRs, every piece in flight at
    // once) in batches of consecutive landmarks whose (landmark, pose) blocks fit the wave's buffer: the blocks of
    // consecutive landmarks are contiguous (k_struct_final), so a batch is one contiguous range of blocks plus the
    // landmarks' Dinv and bl.  The landmark loop then reads LDS (a round trip of ~100 cycles instead of a global
    // load's ~1 us per landmark).
    __shared__ __attribute__((aligned(16))) double stage[kWaves][kStageD];
    double* st = stage[wave];
    const int nb_l = b_l >= 0 ? __popcll(m_l) : 0;  // blocks of this lane's landmark
    int incl = nb_l;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    const int excl = incl - nb_l;
    const uint64_t actv = __ballot(b_l >= 0);
    const int f = actv ? __ffsll((unsigned long long)actv) - 1 : 0;
    const int G = __builtin_amdgcn_readlane(b_l, f) - __builtin_amdgcn_readlane(excl, f);  // the group's first block
    const int kc = kk < 3 ? kk : 0;
    // one landmark's operands from the staged batch (rel = its index in the batch, bx = its first block there)
    struct Ops { double d[3]; double h[NT][3]; double hb[NT]; bool obs[NT]; double bl; };
    auto load = [&](int i, int rel, int bx, Ops& o) __attribute__((always_inline)) {
        const int bl = __builtin_amdgcn_readlane(b_l, i);
        const uint64_t m = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(m_l >> 32), i) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m_l, i);
        const double* Di = st + 9 * rel;
        o.d[0] = Di[kc]; o.d[1] = Di[3 + kc]; o.d[2] = Di[6 + kc];
        o.bl = st[kStageB + 3 * rel + kc];
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const int p = pose_t[t], q = comp_t[t];
            o.obs[t] = bl >= 0 && kk < 3 && p < 64 && ((m >> p) & 1ull);
            const int blk = o.obs[t] ? bx + __popcll(m & ((1ull << p) - 1ull)) : 0;
            const double* H = st + kStageH + 18 * blk;
            o.h[t][0] = H[q]; o.h[t][1] = H[6 + q]; o.h[t][2] = H[12 + q];
            o.hb[t] = H[6 * kc + q];
        }
    };
    typedef __attribute__((address_space(3))) void* lds_ptr;
    int start = 0;
    while (start < nl) {  // wave-uniform
        const int e0 = __builtin_amdgcn_readlane(excl, start);
        const uint64_t fit = __ballot(lane >= start && lane < nl && incl - e0 <= kStageBlocks);
        const int cnt = __popcll(fit), end = start + cnt;  // >= 1: a landmark has at most 64 blocks
        const int nblk = __builtin_amdgcn_readlane(incl, end - 1) - e0;
        const char* gD = (const char*)(c.Dinv + 9 * (size_t)(l0 + start));
        const char* gb = (const char*)(c.lmb + 3 * (size_t)(l0 + start));
        const char* gH = (const char*)(c.blkH + 18 * (size_t)(G + e0));
        char* sD = (char*)st;
        char* sb = (char*)(st + kStageB);
        char* sH = (char*)(st + kStageH);
#pragma unroll
        for (int p = 0; p < 9; p++)  // Dinv: 72 cnt bytes, 256 per piece
            if (256 * p < 72 * cnt && 256 * p + 4 * lane < 72 * cnt)
                __builtin_amdgcn_global_load_lds((const void*)(gD + 256 * p + 4 * lane), (lds_ptr)(sD + 256 * p), 4, 0, 0);
#pragma unroll
        for (int p = 0; p < 3; p++)  // bl: 24 cnt bytes
            if (256 * p < 24 * cnt && 256 * p + 4 * lane < 24 * cnt)
                __builtin_amdgcn_global_load_lds((const void*)(gb + 256 * p + 4 * lane), (lds_ptr)(sb + 256 * p), 4, 0, 0);
#pragma unroll
        for (int p = 0; p < 13; p++)  // blocks: 144 nblk bytes, 1 KiB per piece
            if (1024 * p < 144 * nblk && 1024 * p + 16 * lane < 144 * nblk)
                __builtin_amdgcn_global_load_lds((const void*)(gH + 1024 * p + 16 * lane), (lds_ptr)(sH + 1024 * p), 16, 0, 0);
        __builtin_amdgcn_s_waitcnt(0);  // the pieces have landed
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        Ops cur, nxt;  // the next landmark's LDS reads in flight beside this one's MFMAs
        load(start, 0, 0, cur);
        for (int i = start; i < end; i++) {
            if (i + 1 < end) load(i + 1, i + 1 - start, __builtin_amdgcn_readlane(excl, i + 1) - e0, nxt);
            if (__builtin_amdgcn_readlane(b_l, i) >= 0) {  // landmarks without an active edge add nothing
                // tiles holding a pose that observes the landmark (wave-uniform): a tile pair without one on either
                // side only adds exact zeros, and only the upper tile triangle is formed (the factorization reads
                // the upper triangle of S alone)
                const uint64_t m = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(m_l >> 32), i) << 32) |
                                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m_l, i);
                unsigned tm = 0;
#pragma unroll
                for (int t = 0; t < NT; t++) {
                    const int plo = 16 * t / 6, phi = (16 * t + 15) / 6;
                    if ((m >> plo) & ((2ull << (phi - plo)) - 1ull)) tm |= 1u << t;
                }
                double a[NT], bb[NT];
#pragma unroll
                for (int t = 0; t < NT; t++) {
                    // (B Dinv)(row, kk): the pose-pair kernel's formula
                    a[t] = cur.obs[t] ? (cur.h[t][0] * cur.d[0] + cur.h[t][1] * cur.d[1]) + cur.h[t][2] * cur.d[2] : 0.0;
                    bb[t] = cur.obs[t] ? cur.hb[t] : 0.0;
                }
                const double bv = r16 == 0 && kk < 3 ? cur.bl : 0.0;
#pragma unroll
                for (int ti = 0; ti < NT; ti++) {
#pragma unroll
                    for (int tj = ti; tj < NT; tj++)
                        if ((tm >> ti) & (tm >> tj) & 1u)
                            acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], bb[tj], acc[ti][tj], 0, 0, 0);
                    if ((tm >> ti) & 1u) accb[ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], bv, accb[ti], 0, 0, 0);
                }
            }
            cur = nxt;
        }
        // every LDS read of the batch has returned before the next batch's pieces overwrite the buffer
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        start = end;
    }
    // C/D layout of the f64 16x16x4 form: col = lane & 15, row = (lane >> 4) + 4 * reg
    double* out = c.S_part + (size_t)((task.y / kLbaChunk) * (kLbaChunk / kLbaMfmaLm) + grp) * lba_part_doubles(NT);
#pragma unroll
    for (int i = 0; i < NT; i++) {
#pragma unroll
        for (int j = i; j < NT; j++)
#pragma unroll
            for (int g = 0; g < 4; g++) out[(i * NT + j) * 256 + (kk + 4 * g) * 16 + r16] = acc[i][j][g];
        if (r16 == 0)
#pragma unroll
            for (int g = 0; g < 4; g++) out[NT * NT * 256 + i * 16 + kk + 4 * g] = accb[i][g];
    }
}

// S(r, q) = Hpp + lambda - sum of the partial tile sets (in landmark-group order) for r <= q, and
// bs = bp - sum of the partial right-hand sides.  Grid: (problem, 256-entry slice of the n x n + n entries).
__global__ __launch_bounds__(kThreads) void k_schur_reduce(LbaBatch b) {
    Ctx c = make_ctx(b, blockIdx.x);
    const LbaCtl& k = *c.ctl;
    if (k.state != kTrial || !mfma_schur(k)) return;
    const int np = k.np, n = 6 * np, ntr = mfma_tiles(k);
    const int NT = ntr < 3 ? 3 : ntr;  // the tile count of the k_schur_mfma instance that served this problem
    const int nparts = (c.L + kLbaMfmaLm - 1) / kLbaMfmaLm;
    const int e = blockIdx.y * kThreads + threadIdx.x;
    if (e >= n * n + n) return;
    const bool rhs = e >= n * n;  // entries n^2 .. n^2 + n - 1: the reduced right-hand side bs
    const int r = rhs ? e - n * n : e / n, q = rhs ? 0 : e - r * n;
    const int p1 = r / 6, p2 = q / 6;
    if (!rhs && r > q) return;  // the upper triangle (k_schur_mfma forms the upper tiles; the factorization reads no more)
    const size_t o = rhs ? (size_t)NT * NT * 256 + r : (size_t)((r >> 4) * NT + (q >> 4)) * 256 + (r & 15) * 16 + (q & 15);
    const double* src = c.S_part + o;
    const size_t stride = lba_part_doubles(NT);
    double v = 0.0;
    int s = 0;
    for (; s + 8 <= nparts; s += 8) {  // eight loads in flight, summed in order
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; u++) x[u] = src[(s + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; u++) v += x[u];
    }
    for (; s < nparts; s++) v += src[s * stride];
    if (rhs) {
        c.bs[r] = c.bp[r] - v;
        return;
    }
    const int rr = r - 6 * p1, qq = q - 6 * p2;
    const double base = p1 == p2 ? c.Hpp[36 * p1 + 6 * rr + qq] + (rr == qq ? k.lambda : 0.0) : 0.0;
    c.S[(size_t)r * n + q] = base - v;
}

// pose-pair tasks: S(p1, p2) for p1 <= p2 (task < np(np+1)/2), then bs(p) (next np tasks); problems of the
// MFMA path only run the bs tasks here
__global__ __launch_bounds__(kThreads) void k_schur_pairs(LbaBatch b, LbaWork w) {
    __shared__ Red R;
    const int2 task = w.pair_tasks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    const LbaCtl& k = *c.ctl;
    if (k.state != kTrial) return;
    // task.y >= 0: pose pair task.y (only issued for problems that may exceed the matrix-core path);
    // task.y < 0: the reduced right-hand side of free pose -task.y - 1
    const int np = k.np, n = 6 * np, npairs = np * (np + 1) / 2, tid = task.y;
    if (tid >= npairs || (tid < 0 && -tid - 1 >= np)) return;
    if (mfma_schur(k)) return;  // k_schur_mfma + k_schur_reduce form S and bs
    if (tid >= 0) {
        int p1 = 0, rem = tid;
        while (rem >= np - p1) { rem -= np - p1; p1++; }
        const int p2 = p1 + rem;
        const uint64_t need = (1ull << p1) | (1ull << p2);
        double acc[36];
#pragma unroll
        for (int j = 0; j < 36; j++) acc[j] = 0.0;
#pragma unroll 1
        for (int l = threadIdx.x; l < c.L; l += kThreads) {
            const uint64_t m = c.lm_mask[l];
            if ((m & need) != need) continue;
            const int b0 = lm_block_base(c, l);
            const int ia = b0 + __popcll(m & ((1ull << p1) - 1)), ib = b0 + __popcll(m & ((1ull << p2) - 1));
            const double* BD = c.blkBD + (size_t)ia * 18;
            const double* H = c.blkH + (size_t)ib * 18;
            double bd[18], hh[18];
#pragma unroll
            for (int j = 0; j < 18; j++) { bd[j] = BD[j]; hh[j] = H[j]; }
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int q = 0; q < 6; q++)
                    acc[6 * r + q] += (bd[3 * r] * hh[q] + bd[3 * r + 1] * hh[6 + q]) + bd[3 * r + 2] * hh[12 + q];
        }
        block_sum(acc, R);
        if (threadIdx.x < 36) {
            const int r = threadIdx.x / 6, q = threadIdx.x % 6;
            double v = 0.0;
#pragma unroll
            for (int j = 0; j < 36; j++) if (j == (int)threadIdx.x) v = acc[j];
            const double base = p1 == p2 ? c.Hpp[36 * p1 + threadIdx.x] + (r == q ? k.lambda : 0.0) : 0.0;
            c.S[(size_t)(6 * p1 + r) * n + 6 * p2 + q] = base - v;
        }
    } else {
        const int p = -tid - 1;
        double acc[6] = {0, 0, 0, 0, 0, 0};
        for (int l = threadIdx.x; l < c.L; l += kThreads) {
            const uint64_t m = c.lm_mask[l];
            if (!((m >> p) & 1)) continue;
            const int ia = lm_block_base(c, l) + __popcll(m & ((1ull << p) - 1));
            const double* H = c.blkH + (size_t)ia * 18;
            const double* db = c.db + 3 * l;
#pragma unroll
            for (int r = 0; r < 6; r++) acc[r] += (H[r] * db[0] + H[6 + r] * db[1]) + H[12 + r] * db[2];
        }
        block_sum(acc, R);
        if (threadIdx.x < 6) {
            double v = 0.0;
#pragma unroll
            for (int j = 0; j < 6; j++) if (j == (int)threadIdx.x) v = acc[j];
            c.bs[6 * p + threadIdx.x] = c.bp[6 * p + threadIdx.x] - v;
        }
    }
}

// ---------------------------------------------------------------- reduced system
// One body per storage (LDS or the problem's global scratch), so every access is a ds_* or global_* one
// (a runtime pointer select would make them all flat).
template <bool in_lds>
__device__ __forceinline__ void factor_body(const Ctx& c, LbaCtl& k, double* lds, int n) {
    const int t = threadIdx.x;
    double* A = in_lds ? lds : c.S;
    double* y = in_lds ? lds + (size_t)n * n : c.y;
    double* dd = in_lds ? y + n : c.dd;
    if (in_lds) {
        for (int i = t; i < n * n; i += kThreads) A[i] = c.S[i];
        for (int i = t; i < n; i += kThreads) y[i] = c.bs[i];
    } else {
        for (int i = t; i < n; i += kThreads) y[i] = c.bs[i];
    }
    __syncthreads();
    // LDL^T of the upper triangle, right-looking: entry (r, q), r <= q, loses (L[q][j] d_j) L[r][j] at step j;
    // L[i][j] is kept in the lower triangle
    bool ok = true;
    for (int j = 0; j < n; j++) {
        const double dj = A[(size_t)j * n + j];
        if (dj == 0.0) { ok = false; break; }
        for (int i = j + 1 + t; i < n; i += kThreads) A[(size_t)i * n + j] = A[(size_t)j * n + i] / dj;
        if (t == 0) dd[j] = dj;
        __syncthreads();
        const int m = n - j - 1;
        for (int r = j + 1 + t / 16; r < n; r += kThreads / 16) {
            const double lr = A[(size_t)r * n + j];
            for (int q = r + (t & 15); q < n; q += 16) A[(size_t)r * n + q] -= (A[(size_t)q * n + j] * dj) * lr;
        }
        (void)m;
        __syncthreads();
    }
    if (ok) {
        for (int kk = 0; kk < n; kk++) {  // forward: y[i] -= L[i][k] y[k], k increasing
            const double yk = y[kk];
            __syncthreads();
            for (int i = kk + 1 + t; i < n; i += kThreads) y[i] -= A[(size_t)i * n + kk] * yk;
            __syncthreads();
        }
        for (int i = t; i < n; i += kThreads) y[i] /= dd[i];
        __syncthreads();
        for (int kk = n - 1; kk >= 0; kk--) {  // backward: y[i] -= L[k][i] y[k], k decreasing
            const double yk = y[kk];
            __syncthreads();
            for (int i = t; i < kk; i += kThreads) y[i] -= A[(size_t)kk * n + i] * yk;
            __syncthreads();
        }
        if (in_lds)
            for (int i = t; i < n; i += kThreads) c.y[i] = y[i];
    }
    if (t == 0) k.ok = ok;
}

// Reduced systems of n <= 64 kC rows with the upper triangle in registers: row r on wave r % 4 (register slot
// r / 4), column q on lane q % 64 (column register q / 64).  Column j: the wave holding row j forms
// L(:, j) = A(j, :) / d_j into LDS (column-major LT, the substitutions' L) and d_j; one barrier; every wave
// loads the column once and updates all its rows, A(r, q) -= (L(q, j) d_j) L(r, j) -- the same per-entry
// expression, in the same column order, as factor_body (rows <= j and lanes q < r carry dead values, never
// read).  One barrier and about one LDS round trip per column instead of a chain of LDS read-modify-writes.
// The substitutions run on wave 0, y in registers (lane i, i + 64), y_k broadcast by readlane.
template <int kC>
__device__ __forceinline__ void factor_reg(const Ctx& c, LbaCtl& k, double* lds, int n) {
    constexpr int kR = 16 * kC;  // rows per wave (n <= 64 kC)
    // w through readfirstlane: the compiler then sees every row test as wave-uniform (scalar branches)
    const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
    double* LT = lds;                    // LT[j n + i] = L(i, j), i > j
    double* dd = lds + (size_t)n * n;    // d_j
    double A[kR][kC];
#pragma unroll
    for (int s = 0; s < kR; s++)
#pragma unroll
        for (int cc = 0; cc < kC; cc++) {
            const int r = 4 * s + w, q = 64 * cc + lane;
            A[s][cc] = r < n && q < n ? c.S[(size_t)r * n + q] : 0.0;
        }
    auto rl = [&](double v, int l) __attribute__((always_inline)) {
        const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
        const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
        return __hiloint2double(hi, lo);
    };
    // the wave holding row j: L(:, j) and d_j (row j is final once column j - 1's update is done)
    auto form = [&](int j) __attribute__((always_inline)) {
        if ((j & 3) != w) return;
#pragma unroll
        for (int s = 0; s < kR; s++)
            if (4 * s + w == j) {
                double dj = 0.0;
#pragma unroll
                for (int cc = 0; cc < kC; cc++)
                    if ((j >> 6) == cc) dj = rl(A[s][cc], j & 63);
                if (dj != 0.0)
#pragma unroll
                    for (int cc = 0; cc < kC; cc++) {
                        const int q = 64 * cc + lane;
                        if (q > j && q < n) LT[(size_t)j * n + q] = A[s][cc] / dj;
                    }
                if (lane == 0) dd[j] = dj;
            }
    };
    form(0);
    __syncthreads();
    bool ok = true;
    for (int j = 0; j < n; j++) {
        const double* col = LT + (size_t)j * n;
        // every load of the column first (one LDS round trip, d_j with it), then the updates; all rows and lanes
        // are updated (rows <= j, rows >= n and lanes q < r hold dead values; the loads past the column stay
        // inside the workgroup's LDS)
        double P[kC], lr[kR];
#pragma unroll
        for (int cc = 0; cc < kC; cc++) P[cc] = col[64 * cc + lane];
#pragma unroll
        for (int s = 0; s < kR; s++) lr[s] = col[4 * s + w];
        const double dj = dd[j];
        if (dj == 0.0) { ok = false; break; }
        if (j + 1 == n) break;
#pragma unroll
        for (int cc = 0; cc < kC; cc++) P[cc] = P[cc] * dj;
#pragma unroll
        for (int s = 0; s < kR; s++)
#pragma unroll
            for (int cc = 0; cc < kC; cc++) A[s][cc] = A[s][cc] - P[cc] * lr[s];
        form(j + 1);
        __syncthreads();
    }
    if (t < 64) {
        double y[kC];
#pragma unroll
        for (int m = 0; m < kC; m++) y[m] = 64 * m + lane < n ? c.bs[64 * m + lane] : 0.0;
        if (ok) {
            // forward: y[i] -= L[i][k] y[k], k increasing (column k + 1 loaded during step k)
            double a[kC], an[kC];
#pragma unroll
            for (int m = 0; m < kC; m++) a[m] = 64 * m + lane < n ? LT[64 * m + lane] : 0.0;
#pragma unroll
            for (int mb = 0; mb < kC; mb++)  // y_k lives in register mb of lane k & 63
                for (int kk = 64 * mb; kk < n && kk < 64 * mb + 64; kk++) {
#pragma unroll
                    for (int m = 0; m < kC; m++)
                        an[m] = kk + 1 < n && 64 * m + lane < n ? LT[(size_t)(kk + 1) * n + 64 * m + lane] : 0.0;
                    const double yk = rl(y[mb], kk & 63);
#pragma unroll
                    for (int m = 0; m < kC; m++)
                        if (64 * m + lane > kk && 64 * m + lane < n) y[m] -= a[m] * yk;
#pragma unroll
                    for (int m = 0; m < kC; m++) a[m] = an[m];
                }
#pragma unroll
            for (int m = 0; m < kC; m++)
                if (64 * m + lane < n) y[m] /= dd[64 * m + lane];
            // backward: y[i] -= L[k][i] y[k], k decreasing (L[k][i] = LT[i n + k])
#pragma unroll
            for (int m = 0; m < kC; m++) a[m] = 64 * m + lane < n - 1 ? LT[(size_t)(64 * m + lane) * n + n - 1] : 0.0;
#pragma unroll
            for (int mb = kC - 1; mb >= 0; mb--)
                for (int kk = min(n, 64 * mb + 64) - 1; kk >= 64 * mb; kk--) {
#pragma unroll
                    for (int m = 0; m < kC; m++)
                        an[m] = kk > 0 && 64 * m + lane < kk - 1 ? LT[(size_t)(64 * m + lane) * n + kk - 1] : 0.0;
                    const double yk = rl(y[mb], kk & 63);
#pragma unroll
                    for (int m = 0; m < kC; m++)
                        if (64 * m + lane < kk) y[m] -= a[m] * yk;
#pragma unroll
                    for (int m = 0; m < kC; m++) a[m] = an[m];
                }
#pragma unroll
            for (int m = 0; m < kC; m++)
                if (64 * m + lane < n) c.y[64 * m + lane] = y[m];
        }
        if (t == 0) k.ok = ok;
    }
}

__global__ __launch_bounds__(kThreads) void k_factor(LbaBatch b) {
    extern __shared__ double lds[];
    Ctx c = make_ctx(b, blockIdx.x);
    LbaCtl& k = *c.ctl;
    if (k.state != kTrial) return;
    const int n = 6 * k.np;
    // (measured alone, tools/factor_micro.hip: LDS-resident right-looking updates cost a chain of LDS round
    // trips per column, ~1 us per column; one wave with wave-level synchronisation was slower still)
    if (n <= 64) factor_reg<1>(c, k, lds, n);
    else if (n <= 128) factor_reg<2>(c, k, lds, n);
    else if ((size_t)n * n * 8 + 3 * (size_t)n * 8 <= (size_t)kFactorLds) factor_body<true>(c, k, lds, n);
    else factor_body<false>(c, k, lds, n);
}

// ---------------------------------------------------------------- update / restore
__global__ __launch_bounds__(kThreads) void k_update_lm(LbaBatch b, LbaWork w) {
    __shared__ Red R;
    const int2 task = w.lm_chunks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    const LbaCtl& k = *c.ctl;
    if (k.state != kTrial) return;
    const int l = task.y + threadIdx.x;
    double acc[1] = {0.0};
    if (l < c.L) {
        // push()
        if (l < c.Np) for (int j = 0; j < 3; j++) c.X_b[3 * l + j] = c.X[3 * l + j];
        else for (int j = 0; j < 4; j++) c.P_b[4 * (l - c.Np) + j] = c.P[4 * (l - c.Np) + j];
        const int b0 = lm_block_base(c, l);
        if (k.ok && b0 >= 0) {
            double cl[3] = {c.lmb[3 * l], c.lmb[3 * l + 1], c.lmb[3 * l + 2]};
            uint64_t m = c.lm_mask[l];
            for (int a = 0; m; a++) {
                const int h = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                const double* H = c.blkH + (size_t)(b0 + a) * 18;
#pragma unroll
                for (int i = 0; i < 3; i++) {
                    double s = 0;
#pragma unroll
                    for (int j = 0; j < 6; j++) s += H[6 * i + j] * (-c.y[6 * h + j]);
                    cl[i] += s;
                }
            }
            const double* Di = c.Dinv + 9 * l;
            double x[3];
#pragma unroll
            for (int i = 0; i < 3; i++) x[i] = (Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1]) + Di[3 * i + 2] * cl[2];
#pragma unroll
            for (int i = 0; i < 3; i++) acc[0] += x[i] * (k.lambda * x[i] + c.lmb[3 * l + i]);
            if (l < c.Np) {
                for (int j = 0; j < 3; j++) c.X[3 * l + j] += x[j];
            } else {
                double* pp = c.P + 4 * (l - c.Np);
                P4 P{{pp[0], pp[1], pp[2], pp[3]}};
                p_oplus(P, x);
                for (int j = 0; j < 4; j++) pp[j] = P.c[j];
            }
        }
    }
    block_sum(acc, R);
    if (threadIdx.x == 0) c.part_scale[task.y / kThreads] = acc[0];
}

__global__ void k_update_pose(LbaBatch b, LbaWork w) {
    const int2 task = w.kf_tasks[blockIdx.x];
    if (threadIdx.x != 0) return;
    Ctx c = make_ctx(b, task.x);
    const LbaCtl& k = *c.ctl;
    if (k.state != kTrial) return;
    const int kf = task.y, h = c.pose_hidx[kf];
    for (int j = 0; j < 7; j++) c.pose_b[7 * kf + j] = c.pose[7 * kf + j];
    if (!k.ok || h < 0) return;
    double u[6];
    for (int j = 0; j < 6; j++) u[j] = c.y[6 * h + j];
    store_pose(c.pose + 7 * kf, se3_mul(se3_exp(u), load_pose(c.pose + 7 * kf)));
}

// OptimizationAlgorithmLevenberg accept / reject + iteration / schedule bookkeeping
__global__ void k_decide(LbaBatch b, int step) {
    if (threadIdx.x != 0) return;
    Ctx c = make_ctx(b, blockIdx.x);
    LbaCtl& k = *c.ctl;
    if (k.state != kTrial) return;
    // (serial sums over global partials: unrolled so that 8 loads are in flight per dependent-add group)
    double tempChi = 0.0;
#pragma unroll 8
    for (int i = 0; i < c.nEc; i++) tempChi += c.part_chi[i];
    double scale = 0.0;
    if (k.ok) {
        const int n = 6 * k.np;
#pragma unroll 8
        for (int i = 0; i < n; i++) scale += c.y[i] * (k.lambda * c.y[i] + c.bp[i]);
#pragma unroll 8
        for (int i = 0; i < c.nLc; i++) scale += c.part_scale[i];
    } else {
        tempChi = DBL_MAX;
    }
    double rho = (k.currentChi - tempChi) / (scale + 1e-3);
    if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - libm64cr::cube_(2 * rho - 1);
        alpha = fmin(alpha, 2. / 3.);
        k.lambda *= fmax(1. / 3., alpha);
        k.ni = 2;
        k.currentChi = tempChi;
    } else {
        k.lambda *= k.ni;
        k.ni *= 2;
        k.restore_step = step;  // k_restore_* roll back in this step
    }
    k.qmax++;
    k.trials++;
    const bool stop = stop_requested(b, blockIdx.x, k);
    if (rho < 0 && k.qmax < 10 && !stop) return;  // next trial (do-while ... && !terminate())
    k.its[k.phase]++;
    bool term = k.qmax == 10 || rho == 0;
    if (!term) {
        if ((k.iniChi - k.currentChi) * 1e3 < k.iniChi) k.nBad++;
        else k.nBad = 0;
        term = k.nBad >= 3;
    }
    k.it++;
    if (k.it >= k.max_it) term = true;
    if (term) k.state = k.phase == 0 ? kRelabel : kDone;
    else k.state = kIter;
    if (stop && k.state != kDone) {  // the next iteration or (bDoMore) the second pass does not run
        k.state = kDone;
        k.stopped = 2;
    }
}

__global__ __launch_bounds__(kThreads) void k_restore_lm(LbaBatch b, LbaWork w, int step) {
    const int2 task = w.lm_chunks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    if (c.ctl->restore_step != step) return;
    const int l = task.y + threadIdx.x;
    if (l >= c.L) return;
    if (l < c.Np) for (int j = 0; j < 3; j++) c.X[3 * l + j] = c.X_b[3 * l + j];
    else for (int j = 0; j < 4; j++) c.P[4 * (l - c.Np) + j] = c.P_b[4 * (l - c.Np) + j];
}
__global__ void k_restore_pose(LbaBatch b, LbaWork w, int step) {
    const int2 task = w.kf_tasks[blockIdx.x];
    if (threadIdx.x >= 7) return;
    Ctx c = make_ctx(b, task.x);
    if (c.ctl->restore_step != step) return;
    c.pose[7 * task.y + threadIdx.x] = c.pose_b[7 * task.y + threadIdx.x];
}

// ---------------------------------------------------------------- relabel (between optimize(5) and optimize(10))
__global__ __launch_bounds__(kThreads) void k_relabel(LbaBatch b, LbaWork w, LbaConsts C) {
    const int2 task = w.edge_chunks[blockIdx.x];
    Ctx c = make_ctx(b, task.x);
    if (c.ctl->state != kRelabel) return;
    const int e = task.y + threadIdx.x;
    if (e >= c.E) return;
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
__global__ void k_relabel_done(LbaBatch b, int max_it1) {
    if (threadIdx.x != 0) return;
    Ctx c = make_ctx(b, blockIdx.x);
    LbaCtl& k = *c.ctl;
    if (k.state != kRelabel) return;
    if (stop_requested(b, blockIdx.x, k)) {  // raised after optimize(5) returned: bDoMore = false
        k.state = kDone;
        k.stopped = 2;
        return;
    }
    k.state = kStruct;
    k.phase = 1;
    k.robust = 0;  // setRobustKernel(0) on every edge
    k.it = 0;
    k.max_it = max_it1;
}

__global__ void k_count_active(LbaBatch b) {
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    for (int p = threadIdx.x; p < b.n; p += blockDim.x) {
        Ctx c = make_ctx(b, p);
        if (c.ctl->state != kDone) atomicAdd(&cnt, 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) *b.active = cnt;
}

// ---------------------------------------------------------------- outputs
__global__ __launch_bounds__(kThreads) void k_outputs(LbaBatch b, LbaConsts C) {
    __shared__ Red R;
    const int p = blockIdx.x, t = threadIdx.x;
    Ctx c = make_ctx(b, p);
    const spslam_lba_problem pb = b.probs[p];
    if (c.K > kLbaMaxKeyframes) return;
    if (c.ctl->stopped == 1) {  // returned before optimizing: the map is untouched, nothing is erased
        for (int e = t; e < c.E; e += kThreads) {
            if (e < c.Ep) b.pobs_out[c.e_src[e]] = 0;
            else b.plobs_out[c.e_src[e]] = 0;
        }
        for (int i = t; i < 16 * c.K; i += kThreads) b.kf_out[16 * (size_t)pb.kf_offset + i] = c.kf[i / 16].Tcw[i % 16];
        for (int i = t; i < 3 * c.Np; i += kThreads) b.pt_out[3 * (size_t)pb.point_offset + i] = c.pt[i / 3].xw[i % 3];
        for (int i = t; i < 4 * c.Nq; i += kThreads) b.pl_out[4 * (size_t)pb.plane_offset + i] = c.pl[i / 4].world[i % 4];
        if (t == 0) {
            spslam_lba_result* r = b.res + p;
            *r = spslam_lba_result{};
            r->stopped = 1;
        }
        return;
    }
    int npo = 0, nplo = 0;
    for (int e = t; e < c.E; e += kThreads) {
        double info[3];
        info_of(c, C, e, info);
        const int ty = c.e_type[e];
        const double chi = chi2_of(c.err + 3 * e, info, edge_dim(ty));
        if (ty <= 1) {
            const bool bad = chi > (ty == 0 ? 5.991 : 7.815) || !depth_positive(c, e);
            b.pobs_out[c.e_src[e]] = bad;
            npo += bad;
        } else {
            const bool bad = ty == 2 ? chi > C.plane_chi : chi > C.vp_chi;
            b.plobs_out[c.e_src[e]] = bad;
            nplo += bad;
        }
    }
    double cnt[2] = {(double)npo, (double)nplo};
    block_sum(cnt, R);
    for (int k = t; k < c.K; k += kThreads) {
        float* o = b.kf_out + 16 * ((size_t)pb.kf_offset + k);
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
        for (int j = 0; j < 3; j++) b.pt_out[3 * ((size_t)pb.point_offset + i) + j] = (float)c.X[3 * i + j];
    for (int i = t; i < c.Nq; i += kThreads)
        for (int j = 0; j < 4; j++) b.pl_out[4 * ((size_t)pb.plane_offset + i) + j] = (float)c.P[4 * i + j];
    if (t == 0) {
        const LbaCtl& k = *c.ctl;
        spslam_lba_result* r = b.res + p;
        *r = spslam_lba_result{};
        r->iterations[0] = k.its[0];
        r->iterations[1] = k.its[1];
        r->n_point_outliers = (int)cnt[0];
        r->n_plane_outliers = (int)cnt[1];
        r->status = k.state == kDone ? 0 : -3;
        r->trials = k.trials;
        r->stopped = k.stopped;
        r->phase_us[0] = (float)((wall_clock64() - k.t0) * 0.01);  // 100 MHz ticks: setup to outputs
    }
}

}  // namespace lba

hipError_t lba_run(const LbaBatch& b, const LbaWork& w, const LbaConsts& C, int max_steps, hipStream_t s,
                   KernelTimer* timer, int* steps_out, const volatile uint8_t* stop_src, volatile int32_t* stop_mirror) {
    using namespace lba;
    static const hipError_t lds_attr =
        hipFuncSetAttribute((const void*)k_factor, hipFuncAttributeMaxDynamicSharedMemorySize, kFactorLds);
    (void)lds_attr;
    if (timer) timer->begin(kKindLba, s);
    const dim3 T(kThreads);
    const int P = b.n;
    hipLaunchKernelGGL(k_setup, dim3(P), T, 0, s, b, 5);
    int steps = 0, active = 1;
    while (steps < max_steps) {
        const int st = steps;
        if (b.stop) hipLaunchKernelGGL(k_step_begin, dim3(P), dim3(64), 0, s, b);
        hipLaunchKernelGGL(k_struct_count, dim3(w.n_kf_tasks), T, 0, s, b, w);
        hipLaunchKernelGGL(k_struct_final, dim3(P), T, 0, s, b);
        hipLaunchKernelGGL(k_struct_fill, dim3(w.n_kf_tasks), T, 0, s, b, w);
        hipLaunchKernelGGL(k_struct_done, dim3(P), dim3(64), 0, s, b);
        hipLaunchKernelGGL(k_errors, dim3(w.n_edge_chunks), T, 0, s, b, w, C, 0);
        if (w.n_plane_tasks) hipLaunchKernelGGL(k_plane_terms, dim3(w.n_plane_tasks), T, 0, s, b, w, C);
        if (w.n_seg_chunks) hipLaunchKernelGGL(k_point_terms_sums, dim3(w.n_seg_chunks), T, 0, s, b, w, C);
        if (w.n_plm_tasks) hipLaunchKernelGGL(k_plane_lm_sums, dim3(w.n_plm_tasks), T, 0, s, b, w);
        hipLaunchKernelGGL(k_pose_sums, dim3(w.n_kf_tasks), T, 0, s, b, w);
        hipLaunchKernelGGL(k_iter_begin, dim3(P), dim3(64), 0, s, b);
        hipLaunchKernelGGL(k_schur_lm, dim3(w.n_lm_chunks), T, 0, s, b, w);
        const dim3 G(w.n_lm_chunks, kLbaChunk / (kWaves * kLbaMfmaLm));
        hipLaunchKernelGGL(k_schur_mfma<3>, G, T, 0, s, b, w);
        hipLaunchKernelGGL(k_schur_mfma<4>, G, T, 0, s, b, w);
        hipLaunchKernelGGL(k_schur_mfma<5>, G, T, 0, s, b, w);
        hipLaunchKernelGGL(k_schur_reduce, dim3(P, (80 * 80 + 80 + kThreads - 1) / kThreads), T, 0, s, b);
        if (w.n_pair_tasks) hipLaunchKernelGGL(k_schur_pairs, dim3(w.n_pair_tasks), T, 0, s, b, w);
        hipLaunchKernelGGL(k_factor, dim3(P), T, kFactorLds, s, b);
        hipLaunchKernelGGL(k_update_lm, dim3(w.n_lm_chunks), T, 0, s, b, w);
        hipLaunchKernelGGL(k_update_pose, dim3(w.n_kf_tasks), dim3(64), 0, s, b, w);
        hipLaunchKernelGGL(k_errors, dim3(w.n_edge_chunks), T, 0, s, b, w, C, 1);
        hipLaunchKernelGGL(k_decide, dim3(P), dim3(64), 0, s, b, st);
        hipLaunchKernelGGL(k_restore_lm, dim3(w.n_lm_chunks), T, 0, s, b, w, st);
        hipLaunchKernelGGL(k_restore_pose, dim3(w.n_kf_tasks), dim3(64), 0, s, b, w, st);
        hipLaunchKernelGGL(k_relabel, dim3(w.n_edge_chunks), T, 0, s, b, w, C);
        hipLaunchKernelGGL(k_relabel_done, dim3(P), dim3(64), 0, s, b, 10);
        steps++;
        if (steps % 4 == 0) {
            if (stop_src && *stop_src) *stop_mirror = 1;
            hipLaunchKernelGGL(k_count_active, dim3(1), T, 0, s, b);
            hipError_t e = hipMemcpyAsync(&active, b.active, sizeof(int), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
            if (active == 0) break;
        }
    }
    hipLaunchKernelGGL(k_outputs, dim3(P), T, 0, s, b, C);
    if (timer) timer->end(kKindLba, s);
    if (steps_out) *steps_out = steps;
    return hipGetLastError();
}

}  // namespace spslam
