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
__device__ unsigned long long g_pose_prof[24];  // 0-9 phases (thread 0), 10-11 counts, 12-15 the chain wave, 16-19 sub-phases
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

// kComputeWaves compute waves and one chain wave per problem.  The compute waves evaluate the edges (errors, Jacobians,
// quadratic-form terms, trial chi2) and stage one row per edge in an LDS ring; the chain wave adds the rows in
// edge order as they arrive.  g2o's sums are serial (one dependent fp64 add per edge and value, ~13 ns each on
// gfx950), so the ordered chains set the floor of every pass; with a wave of their own they run beside the
// edge evaluation instead of after it.  (Measured before: one wave per problem frees SIMDs for the pipelined
// extraction but makes the edge passes 4x longer -- a net loss.)
// Seven compute waves: with ~250 VGPRs a SIMD holds 2 waves, so 7 + the chain wave is a full CU.  Against 4
// compute waves (profiles/r05/ab_pose_waves.txt): B = 1 single sequence 654 -> 689 frames/s (the point rounds of
// both passes spread over more lanes; the plane evaluations are one round either way), C2 step 6.40 -> 6.31 ms
// (the workgroup's 158 KB of LDS pinned the CU already; now its waves fill it)
#ifndef SPSLAM_POSE_COMPUTE_WAVES
#define SPSLAM_POSE_COMPUTE_WAVES 7
#endif
constexpr int kComputeWaves = SPSLAM_POSE_COMPUTE_WAVES;
constexpr int kCompute = 64 * kComputeWaves;
constexpr int kThreads = kCompute + 64;
constexpr int kWaves = kThreads / 64;
constexpr int kChainWave = kComputeWaves;
constexpr int kRed = 28;         // robust chi2, 21 lower-triangle H terms, 6 b terms
constexpr int kPlaneChunk = 64;  // plane edges whose trial-pose errors are kept for the next pass A
constexpr int kMaxTrials = 10;   // OptimizationAlgorithmLevenberg: qmax < 10

// Pass A ring: rows of the 28 terms (odd stride: the 64 lanes' row writes spread over the banks).  Pass B reuses
// the same LDS as a ring of kSpec-value rows (trial robust chi2).
#ifndef SPSLAM_POSE_RING
#define SPSLAM_POSE_RING 512  // rows of the pass-A ring; measured in the pipelined C2 step: 128 rows 7.00 ms,
                              // 256 rows 6.97, 512 rows (146 KB of LDS per problem) 6.80 (profiles/r03/ab_ring*)
#endif
constexpr int kRingA = SPSLAM_POSE_RING;
#ifndef SPSLAM_POSE_STRIDE
#define SPSLAM_POSE_STRIDE 29  // doubles per pass-A ring row (28 terms + 1: an odd stride spreads the row writes)
#endif
constexpr int kStrideA = SPSLAM_POSE_STRIDE;
static_assert(kStrideA >= kRed, "a ring row holds the 28 terms (lanes past them read any column: never added)");
#ifndef SPSLAM_POSE_RING_PAD
#define SPSLAM_POSE_RING_PAD 24
#endif
// spare rows past the ring end (chain_seg loads up to 23 rows past a segment; with 0 those loads read the
// fields that follow the ring in Shared -- never added, and inside the workgroup's allocation)
constexpr int kRingPad = SPSLAM_POSE_RING_PAD;
// A smaller footprint (so ORB's level/fast kernels co-reside beside a pose workgroup) did not pay: pipelined C2
// step 6.66 ms (29/24, 146 KB) vs 6.68 (29/0, 143.5 KB) vs 6.69 (28/0, 139.5 KB), 3 rounds each (profiles/r03/ab_lds_*)
// every wait gives up after PoseConsts::spin_cap polls (default 2^20, s_sleep 1 each: ~30 ms; never reached in a
// correct run)

template <int kSpec>
struct RingB {
    static constexpr int kStride = kSpec + 1;
    static constexpr int kRows = [] {
        int r = 1;
        while (2 * r * kStride <= kRingA * kStrideA) r *= 2;
        return r;
    }();
};

template <int kSpec>
struct Shared {
    double ring[(kRingA + kRingPad) * kStrideA];  // pass A: [kRingA][kStrideA]; pass B: [RingB::kRows][kSpec + 1]
    double tot[kRed];                 // the chained totals, for every thread
    double red[2][kWaves][1];         // wave totals of the workgroup sums, double-buffered
    double perr[kComputeWaves][9][13][3];  // per compute wave: plane errors at the 12 perturbed poses and at T
    double perrB[kPlaneChunk][kSpec][3];   // plane errors at the trial poses of the last pass B
    double perrT[kPlaneChunk][3];     // plane errors at the accepted trial pose = the next iteration's T
    double hb[kRed];                  // the iteration's H (lower, 21) and b (6), slot 0 unused
    SE3 tlast[kWaves];                // each wave's copy of the last trial pose (the relabel's active-edge pose)
    SE3 Eadd[12];                     // exp(+-1e-9 e_d), d = 0..5 (numeric Jacobian steps)
    SE3 T0;                           // the input pose (every round restarts from it)
    double xtrial[2][kSpec][6];       // each trial's applied solution, by trial pass parity (read after pass B)
    P4 pw[kPlaneChunk], pm[kPlaneChunk];  // plane edges' world / measured planes, normalized (nl <= kPlaneChunk)
    int done[kComputeWaves];          // rounds each compute wave has staged in the current pass
    int consumed;                     // rows the chain wave has added in the current pass
    int stall;                        // a wait hit spin_cap (reported through lm_iterations)
    int spin_cap;                     // PoseConsts::spin_cap (kSpinCap unless a test lowers it)
};

// Workgroup sum of NV doubles per thread; every thread returns the same totals.  Fixed order: xor butterfly over
// the 64 lanes of each wave, then (((0 + w0) + w1) + ...) from LDS in every thread.  Only the relabel's outlier
// count uses it (small integers: exact in any order).  One barrier; consecutive calls alternate the two buffers.
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

// acc += rows start .. start + cnt - 1 of a ring column (slot = row & (kRows - 1)), one after the other: the
// reference's order.  The rows are added in contiguous segments (the ring wraps at most once), so every group of 8
// loads is one base address plus immediate offsets.  Three register groups of 8 rotate: while one group's
// dependent adds run, the other two groups' loads are in flight, and a group is refilled right after its adds
// (no register moves: a FIFO rotated with moves makes the compiler wait for every outstanding load once per group
// -- a full LDS round trip per 8 adds; the scheduling barriers keep each refill ahead of the next group's adds).
// Rows past a segment's end are loaded and never added (the ring carries kRingPad spare rows for them).
template <int kStride>
__device__ __forceinline__ void chain_seg(double& acc, const double* p, int cnt) {
    auto ld = [&](double (&v)[8], int i) __attribute__((always_inline)) {
        const double* q = p + i * kStride;
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = q[k * kStride];
    };
    auto add = [&](const double (&v)[8], int n) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (k < n) acc += v[k];
    };
    const int full = cnt - cnt % 24;
    double a[8], b[8], c[8];
    ld(a, 0);
    ld(b, 8);
    ld(c, 16);
    for (int i = 0; i < full; i += 24) {
        add(a, 8);
        ld(a, i + 24);
        __builtin_amdgcn_sched_barrier(0);
        add(b, 8);
        ld(b, i + 32);
        __builtin_amdgcn_sched_barrier(0);
        add(c, 8);
        ld(c, i + 40);
        __builtin_amdgcn_sched_barrier(0);
    }
    const int r = cnt - full;  // < 24 left: a, b, c hold rows full .. full + 23
    add(a, r);
    add(b, r - 8);
    add(c, r - 16);
}
template <int kStride, int kRows>
__device__ __forceinline__ void chain_ring(double& acc, const double* col, int start, int cnt) {
    static_assert((kRows & (kRows - 1)) == 0, "ring wrap");
    const int s0 = start & (kRows - 1), n0 = min(cnt, kRows - s0);
    chain_seg<kStride>(acc, col + s0 * kStride, n0);
    if (cnt > n0) chain_seg<kStride>(acc, col, cnt - n0);
}

// The staging schedule of one pass, known to every wave: point rounds of 256 edges (64 per compute wave), then
// plane rounds of 4 * ps edges (ps per compute wave).  Compute wave w stages its share of round k and publishes
// done[w] = k + 1; the rows below available() are staged.
struct Schedule {
    int np, ne, ps, npr, nr;
    __device__ Schedule(int np_, int nl, int ps_) : np(np_), ne(np_ + nl), ps(ps_) {
        npr = (np + kCompute - 1) / kCompute;
        nr = npr + (nl + kComputeWaves * ps - 1) / (kComputeWaves * ps);
    }
    // edge range [lo, hi) of round k and the edges per wave
    __device__ void round(int k, int& lo, int& hi, int& s) const {
        if (k < npr) {
            lo = kCompute * k; hi = min(lo + kCompute, np); s = 64;
        } else {
            lo = np + kComputeWaves * ps * (k - npr); hi = min(lo + kComputeWaves * ps, ne); s = ps;
        }
    }
    // wave w's edges [a, b) of round k (possibly empty)
    __device__ void share(int k, int w, int& a, int& b) const {
        int lo, hi, s;
        round(k, lo, hi, s);
        a = min(lo + w * s, hi);
        b = min(lo + (w + 1) * s, hi);
    }
};

__device__ __forceinline__ int lds_acquire(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_publish(int* p, int v) {  // after this wave's ring writes (every lane fences)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// rows below this are staged (every compute wave's share of every earlier round, and the leading waves' shares
// of the current one)
template <class Sh>
__device__ __forceinline__ int available(Sh& S, const Schedule& G) {
    int d[kComputeWaves], m = 1 << 30;
#pragma unroll
    for (int w = 0; w < kComputeWaves; w++) {
        d[w] = lds_acquire(&S.done[w]);
        m = min(m, d[w]);
    }
    if (m >= G.nr) return G.ne;
    int lo, hi, s;
    G.round(m, lo, hi, s);
    int j = 0;
#pragma unroll
    for (int w = 0; w < kComputeWaves; w++)
        if (j == w && d[w] > m) j = w + 1;
    return min(lo + j * s, hi);
}

// the chain wave: add every staged row of the pass in edge order, column = this lane's value (lanes past nval
// read the padding column), and hand out the ring slots as rows are added
// (diagnostic build: prof[0] += ticks spent adding, prof[1] += ticks spent waiting for rows)
template <int kStride, int kRows, class Sh>
__device__ __forceinline__ double chain_pass(Sh& S, const Schedule& G, const double* ring, int nval,
                                             unsigned long long* prof) {
    const int lane = threadIdx.x & 63;
    const double* col = ring + (lane < nval ? lane : kStride - 1);
    double acc = 0;
    int c = 0;
    while (c < G.ne) {
#ifdef SPSLAM_POSE_PROF
        const unsigned long long w0 = wall_clock64();
#endif
        int a = available(S, G);
        for (int spin = 0; a <= c; spin++) {
            if (spin >= S.spin_cap) { S.stall = 1; a = G.ne; break; }
            __builtin_amdgcn_s_sleep(1);
            a = available(S, G);
        }
#ifdef SPSLAM_POSE_PROF
        const unsigned long long w1 = wall_clock64();
        prof[1] += w1 - w0;
#endif
        chain_ring<kStride, kRows>(acc, col, c, a - c);
        c = a;
        lds_publish(&S.consumed, c);
#ifdef SPSLAM_POSE_PROF
        prof[0] += wall_clock64() - w1;
#endif
    }
    (void)prof;
    return acc;
}

// a compute wave about to overwrite ring slots of rows [b - kRows, ...): wait until the chain wave added them
template <class Sh>
__device__ __forceinline__ void ring_wait(Sh& S, int need) {
    if (need <= 0) return;
    for (int spin = 0; lds_acquire(&S.consumed) < need; spin++) {
        if (spin >= S.spin_cap) { S.stall = 1; return; }
        __builtin_amdgcn_s_sleep(1);
    }
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

// one edge's 28 terms (BaseUnaryEdge / BaseBinaryEdge::constructQuadraticForm in Eigen's order: the temporary
// A^T (rho' Omega) times A) and -s_e with b -= s_e (unary: ((rho' A^T) Omega) e; binary, pose = vertex 1:
// B^T (rho' Omega e)), preceded by the edge's robust chi2
__device__ __forceinline__ void edge_terms(const double (&J)[3][6], const double* err, const double* info, double delta,
                                           bool robust, bool binary, double (&row)[kRed]) {
    double rho0, rho1;
    const double chi = (err[0] * (info[0] * err[0]) + err[1] * (info[1] * err[1])) + err[2] * (info[2] * err[2]);
    huber(chi, delta, robust, &rho0, &rho1);
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
}

}  // namespace pose

using namespace pose;

// Every thread holds the whole LM state (pose, lambda, chi2 values, H, b): the chained totals reach every thread
// through LDS and every decision is computed redundantly from them.  The damping trials of one LM iteration are
// evaluated kSpec at a time: after a rejected trial the reference only multiplies lambda by ni and doubles ni
// (optimization_algorithm_levenberg.cpp:145-160), so trial q's lambda is known in advance; lane q % kSpec of
// every wave solves trial q, the trial poses are broadcast with readlane, one pass over the edges evaluates all
// kSpec robust chi2 sums, and the accept / reject walk then replays the reference's sequence over them.  Results
// do not depend on kSpec.
template <int kSpec>
__global__ __launch_bounds__(kThreads, 1) void pose_kernel(const spslam_pose_problem* __restrict__ probs,
                                                         const spslam_point_obs* __restrict__ pts_all,
                                                         const spslam_plane_obs* __restrict__ pls_all, PoseConsts K,
                                                         const spslam_pose_result* __restrict__ init_from,
                                                         spslam_pose_result* __restrict__ results,
                                                         uint8_t* __restrict__ pout_all, uint8_t* __restrict__ plout_all) {
    tail_wave_priority();
    __shared__ Shared<kSpec> S;
    using RB = RingB<kSpec>;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const bool chain_wave = wv == kChainWave;
#ifdef SPSLAM_POSE_PROF
    unsigned long long prof_acc[24] = {};
    unsigned long long prof_t = wall_clock64();
#endif
    unsigned long long* chain_prof_a = nullptr;  // the chain wave's ticks (diagnostic build only)
    unsigned long long* chain_prof_b = nullptr;
#ifdef SPSLAM_POSE_PROF
    chain_prof_a = prof_acc + 12;
    chain_prof_b = prof_acc + 14;
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
        if (t == 0) { res->n_inliers = 0; res->lm_iterations = 0; res->trial_passes = 0; res->trials = 0; }
        return;
    }
    if (t < 12 && nl > 0) {
        double add[6] = {0, 0, 0, 0, 0, 0};
        add[t >> 1] = (t & 1) ? -1e-9 : 1e-9;
        S.Eadd[t] = se3_exp(add);
    }
    if (t == 0) {  // (spin_cap < 0, a test hook: the problem is reported as stalled whatever its waits do)
        S.stall = K.spin_cap < 0;
        S.spin_cap = K.spin_cap < 0 ? (1 << 20) : K.spin_cap;
    }
    SE3 T0;  // Converter::toSE3Quat: Quaterniond(R) of the float pose, normalized (every thread)
    {
        M3 R;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R.a[3 * i + j] = Tin[4 * i + j];
        T0.r = q_from_rot(R);
        T0.t = V3{Tin[3], Tin[7], Tin[11]};
        q_normalize(T0.r);
        if (t == 0) S.T0 = T0;  // read back at each round start: not held in registers across the rounds
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
    auto plane_of_global = [&](int e, P4& w, P4& m) __attribute__((always_inline)) {
        const spslam_plane_obs& o = pls[e - np];
        for (int k = 0; k < 4; k++) { w.c[k] = o.world[k]; m.c[k] = o.meas[k]; }
        if (o.world[3] < 0.0f) for (int k = 0; k < 4; k++) w.c[k] = -w.c[k];  // Converter::toPlane3D
        if (o.meas[3] < 0.0f) for (int k = 0; k < 4; k++) m.c[k] = -m.c[k];
        p_normalize(w.c);
        p_normalize(m.c);
    };
    const bool plane_cache = nl <= kPlaneChunk;  // the normalized planes wait in LDS (every evaluation reads them)
    auto plane_of = [&](int e, P4& w, P4& m) __attribute__((always_inline)) {
        if (plane_cache) { w = S.pw[e - np]; m = S.pm[e - np]; }
        else plane_of_global(e, w, m);
    };
    // the same for an edge known to be a point (plane) edge: the loops that only visit one kind call these, so
    // the other kind's evaluation is not compiled into them as a dead branch
    auto point_error_at = [&](int e, const SE3& T, double* err, V3* pc) __attribute__((always_inline)) {
        V3 p;
        const E3 r = point_error(pts[e], T, cam, p);
        if (pc) *pc = p;
        err[0] = r.e0; err[1] = r.e1; err[2] = r.e2;
    };
    auto plane_error_at = [&](int e, const SE3& T, double* err) __attribute__((always_inline)) {
        P4 w, m;
        plane_of(e, w, m);
        const E3 r = plane_error3(pls[e - np].kind, T, w, m);
        err[0] = r.e0; err[1] = r.e1; err[2] = r.e2;
    };
    // the same on the lane pair (lane & ~1, lane | 1): both lanes pass the same edge and pose
    auto plane_error_pair_at = [&](int e, const SE3& T, double* err) __attribute__((always_inline)) {
        P4 w, m;
        plane_of(e, w, m);
        const E3 r = plane_error_pair(pls[e - np].kind, T, w, m, (lane & 1) != 0);
        err[0] = r.e0; err[1] = r.e1; err[2] = r.e2;
    };
    auto chi2_of = [](const double* err, const double* info) __attribute__((always_inline)) {
        // e . (Omega e) (base_edge.h chi2); rows beyond the edge's dimension hold a zero error: their +0 terms
        // leave chi unchanged
        return (err[0] * (info[0] * err[0]) + err[1] * (info[1] * err[1])) + err[2] * (info[2] * err[2]);
    };
    auto is_outlier = [&](int e) __attribute__((always_inline)) -> bool { return e < np ? pout[e] != 0 : plout[e - np] != 0; };
    // a new pass: nothing staged, nothing consumed (every wave has passed the previous pass's final barrier)
    auto pass_begin = [&]() __attribute__((always_inline)) {
        if (t < kComputeWaves) S.done[t] = 0;
        if (t == 0) S.consumed = 0;
        __syncthreads();
    };
    double* ringA = S.ring;
    double* ringB = S.ring;
    if (plane_cache && t < nl) {
        P4 w, m;
        plane_of_global(np + t, w, m);
        S.pw[t] = w;
        S.pm[t] = m;
    }
    __syncthreads();

    int buf = 0;
    bool robust = true;
    int nBad = 0, total_its = 0, total_passes = 0, total_trials = 0;
    // g2o's solution buffer (Solver::_x) across the trials and the four optimize(10) calls: written only by a
    // successful LDLT, applied and used in computeScale whether or not the trial's solve succeeded
    // (optimization_algorithm_levenberg.cpp:110-127, linear_solver_dense.h:107-112); never written = zeros
    double xs[6] = {0, 0, 0, 0, 0, 0};
    SE3 T;
    for (int round = 0; round < 4; round++) {
        PROF_MARK(0);  // setup / previous relabel
        T = S.T0;
        // any active edge?
        int act = 0, ea0 = t;
        asm volatile("" : "+v"(ea0));  // (its unrolled bounds, hoisted to the kernel's start, were spilled)
        for (int e = ea0; e < ne; e += kThreads) act |= !is_outlier(e);
        act = __syncthreads_or(act);
        if (act) {
            double lambda = 0, ni = 2;
            int lmBad = 0;
            bool tValid = false;  // perrT holds the plane errors at T (set when a trial is accepted)
            for (int it = 0; it < 10; it++) {
                // ---- pass A: errors, robust chi2, quadratic form at T, chained in edge order.  Plane edges:
                // numeric central differences, delta 1e-9 (base_binary_edge.hpp:130-205) -- the errors at the 12
                // perturbed poses exp(+-1e-9 e_d) * T (and at T unless an accepted trial left them in perrT) are
                // evaluated on nev lanes per edge, ps edges per compute wave and round, then staged by one lane
                const bool haveT = tValid && nl <= kPlaneChunk;
                // full evaluations per edge: the 6 rotation perturbations, ONE translation perturbation (q = 6)
                // and T unless perrT holds it; the other 5 translation perturbations share q = 6's rotation and
                // reference normal bit for bit (exp(+-1e-9 e_d) for d >= 3 is a pure translation: its quaternion
                // is exactly (1, 0, 0, 0), so every Tq.r equals normalize(T.r)), which leaves only the plane
                // distance to recompute -- checked per perturbation, with a full evaluation where it fails
                const int nev = haveT ? 7 : 8, psA = 64 / nev;
                const Schedule GA(np, nl, psA);
                pass_begin();
                if (chain_wave) {
                    const double a = chain_pass<kStrideA, kRingA>(S, GA, ringA, kRed, chain_prof_a);
                    if (lane < kRed) S.tot[lane] = a;
                } else {
                    for (int k = 0; k < GA.npr; k++) {
                        const int e = kCompute * k + t;
                        double row[kRed];
#pragma unroll
                        for (int v = 0; v < kRed; v++) row[v] = 0.0;
                        if (e < np && !pout[e]) {
                            double info[3], delta, err[3] = {0, 0, 0}, J[3][6];
                            edge_info(e, info, &delta);
                            V3 pc;
                            point_error_at(e, T, err, &pc);
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
                            edge_terms(J, err, info, delta, robust, false, row);
                        }
                        int ea, eb;
                        GA.share(k, wv, ea, eb);
                        ring_wait(S, ea < eb ? eb - kRingA : 0);
                        if (e < np) {
                            double* dst = ringA + (e & (kRingA - 1)) * kStrideA;
#pragma unroll
                            for (int v = 0; v < kRed; v++) dst[v] = row[v];
                        }
                        lds_publish(&S.done[wv], k + 1);
                    }
                    PROF_MARK(1);  // pass A point edges (compute wave 0's view)
                    for (int k = GA.npr; k < GA.nr; k++) {
                        int ea, eb;
                        GA.share(k, wv, ea, eb);
                        // evaluation lanes: slot qe < 7 -> perturbation qe, slot 7 -> T (stored as q = 12)
                        const int i = lane / nev, qe = lane - i * nev, q = qe < 7 ? qe : 12, j = ea - np + i;
                        if (i < psA && np + j < eb) {
                            double err[3] = {0, 0, 0};
                            if (!plout[j]) {
                                const SE3 Tp = se3_mul(S.Eadd[q < 12 ? q : 0], T);
                                const bool pt = q < 12;
                                SE3 Tq;  // field-wise select: one inlined error evaluation for both cases
                                Tq.r.w = pt ? Tp.r.w : T.r.w; Tq.r.x = pt ? Tp.r.x : T.r.x;
                                Tq.r.y = pt ? Tp.r.y : T.r.y; Tq.r.z = pt ? Tp.r.z : T.r.z;
                                Tq.t.x = pt ? Tp.t.x : T.t.x; Tq.t.y = pt ? Tp.t.y : T.t.y;
                                Tq.t.z = pt ? Tp.t.z : T.t.z;
                                plane_error_at(np + j, Tq, err);
                            }
                            S.perr[wv][i][q][0] = err[0]; S.perr[wv][i][q][1] = err[1]; S.perr[wv][i][q][2] = err[2];
                        }
                        wave_sync();
                        {   // the other translation perturbations q = 7 .. 11, one lane each
                            const int i2 = lane / 5, q2 = 7 + (lane - i2 * 5), j2 = ea - np + i2;
                            if (i2 < psA && np + j2 < eb) {
                                double err[3] = {0, 0, 0};
                                if (!plout[j2]) {
                                    const SE3 T6 = se3_mul(S.Eadd[6], T), Tk = se3_mul(S.Eadd[q2], T);
                                    P4 w, m;
                                    plane_of(np + j2, w, m);
                                    // plane_error's first steps for both poses (same rotation: same n2)
                                    const V3 n2 = mv(q_to_rot(T6.r), V3{w.c[0], w.c[1], w.c[2]});
                                    const double va = w.c[3] - dot(T6.t, n2), vb = w.c[3] - dot(Tk.t, n2);
                                    const double vf = vb < 0.0 ? -vb : vb;
                                    const double vn = vf * (1. / sqrt(n2.x * n2.x + n2.y * n2.y + n2.z * n2.z));
                                    auto same = [](double a, double b) { return __double_as_longlong(a) == __double_as_longlong(b); };
                                    const bool shared = same(T6.r.w, Tk.r.w) && same(T6.r.x, Tk.r.x) && same(T6.r.y, Tk.r.y) &&
                                                        same(T6.r.z, Tk.r.z) && (va < 0.0) == (vb < 0.0) && !(vn < 0.0);
                                    if (shared) {
                                        err[0] = S.perr[wv][i2][6][0];
                                        err[1] = S.perr[wv][i2][6][1];
                                        err[2] = pls[j2].kind == 0 ? (-vn) - (-m.c[3]) : 0.0;
                                    } else {
                                        plane_error_at(np + j2, Tk, err);
                                    }
                                }
                                S.perr[wv][i2][q2][0] = err[0]; S.perr[wv][i2][q2][1] = err[1]; S.perr[wv][i2][q2][2] = err[2];
                            }
                        }
                        wave_sync();
                        PROF_MARK(16);  // pass A plane evaluations
                        double row[kRed];
#pragma unroll
                        for (int v = 0; v < kRed; v++) row[v] = 0.0;
                        const int js = ea - np + lane;  // staging lane: plane edge js
                        if (lane < psA && np + js < eb && !plout[js]) {
                            double info[3], delta, J[3][6];
                            edge_info(np + js, info, &delta);
                            const double err[3] = {haveT ? S.perrT[js][0] : S.perr[wv][lane][12][0],
                                                   haveT ? S.perrT[js][1] : S.perr[wv][lane][12][1],
                                                   haveT ? S.perrT[js][2] : S.perr[wv][lane][12][2]};
                            const double scalar = 1.0 / (2 * 1e-9);
#pragma unroll
                            for (int d = 0; d < 6; d++)
#pragma unroll
                                for (int r = 0; r < 3; r++)
                                    J[r][d] = scalar * (S.perr[wv][lane][2 * d][r] - S.perr[wv][lane][2 * d + 1][r]);
                            edge_terms(J, err, info, delta, robust, true, row);
                        }
                        ring_wait(S, ea < eb ? eb - kRingA : 0);
                        if (lane < psA && np + js < eb) {
                            double* dst = ringA + ((np + js) & (kRingA - 1)) * kStrideA;
#pragma unroll
                            for (int v = 0; v < kRed; v++) dst[v] = row[v];
                        }
                        lds_publish(&S.done[wv], k + 1);
                        wave_sync();  // perr[wv] is rewritten by the next round
                        PROF_MARK(17);  // pass A plane staging
                    }
                }
                __syncthreads();
                PROF_MARK(2);  // pass A plane edges + the chain's tail
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
                    double xn[6] = {0, 0, 0, 0, 0, 0};
                    const int gq = total_trials + myq;  // this trial's index in the call (test hook)
                    const bool ok = !(gq < 32 && ((K.fail_mask >> gq) & 1u)) && ldlt_solve(H, lam, b, xn);
                    // the solution trial q applies: its own if its solve succeeded, else that of the last earlier trial
                    // of the pass whose solve did, else the buffer carried in (trials q' < q were rejected if q runs)
                    double x[6];
                    {
                        double xe[6];
#pragma unroll
                        for (int j = 0; j < 6; j++) xe[j] = xs[j];
#pragma unroll
                        for (int q = 0; q < kSpec; q++) {
                            const bool okq = __builtin_amdgcn_readlane((int)ok, q) != 0;
#pragma unroll
                            for (int j = 0; j < 6; j++) {
                                const double v = readlane_d(xn[j], q);
                                xe[j] = okq ? v : xe[j];
                            }
#pragma unroll
                            for (int j = 0; j < 6; j++)
                                if (myq == q) x[j] = xe[j];
                        }
                    }
                    // trial q's applied solution waits in LDS until the walk below knows the last trial run (kept in
                    // registers it would stay live across pass B); the parity buffer orders it against the previous
                    // pass's reads without a barrier
                    if (t < kSpec) {
#pragma unroll
                        for (int j = 0; j < 6; j++) S.xtrial[total_passes & 1][t][j] = x[j];
                    }
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
                    total_passes++;
                    // ---- pass B: robust chi2 of every active edge at each trial pose, one ring row of kSpec
                    // values per edge, chained in edge order by lanes 0 .. kSpec-1 of the chain wave.  Plane edges:
                    // one (edge, trial) pair per lane pair (plane_error_pair), 32 / kSpec edges per compute wave
                    // and round
                    constexpr int psB = 32 / kSpec;
                    const Schedule GB(np, nl, psB);
                    pass_begin();
                    if (chain_wave) {
                        const double a = chain_pass<RB::kStride, RB::kRows>(S, GB, ringB, kSpec, chain_prof_b);
                        if (lane < kSpec) S.tot[lane] = a;
                    } else {
                        for (int k = 0; k < GB.npr; k++) {
                            const int e = kCompute * k + t;
                            double r[kSpec];
#pragma unroll
                            for (int q = 0; q < kSpec; q++) r[q] = 0;
                            if (e < np && !pout[e]) {
                                double info[3], delta;
                                edge_info(e, info, &delta);
#pragma unroll
                                for (int q = 0; q < kSpec; q++) {
                                    double err[3] = {0, 0, 0}, rho1;
                                    point_error_at(e, Tq[q], err, nullptr);
                                    huber(chi2_of(err, info), delta, robust, &r[q], &rho1);
                                }
                            }
                            int ea, eb;
                            GB.share(k, wv, ea, eb);
                            ring_wait(S, ea < eb ? eb - RB::kRows : 0);
                            if (e < np) {
                                double* dst = ringB + (e & (RB::kRows - 1)) * RB::kStride;
#pragma unroll
                                for (int q = 0; q < kSpec; q++) dst[q] = r[q];
                            }
                            lds_publish(&S.done[wv], k + 1);
                        }
                        PROF_MARK(18);  // pass B point rounds
                        for (int k = GB.npr; k < GB.nr; k++) {
                            int ea, eb;
                            GB.share(k, wv, ea, eb);
                            const int pr = lane >> 1, i = pr / kSpec, q = pr % kSpec, j = ea - np + i;
                            const bool lead = (lane & 1) == 0;
                            double r0 = 0;
                            if (np + j < eb && !plout[j]) {
                                double info[3], delta, err[3] = {0, 0, 0}, rho1;
                                edge_info(np + j, info, &delta);
                                SE3 Tv = Tq[0];  // uniform poses: select by q without dynamic indexing
#pragma unroll
                                for (int u = 1; u < kSpec; u++)
                                    if (q == u) Tv = Tq[u];
                                plane_error_pair_at(np + j, Tv, err);
                                huber(chi2_of(err, info), delta, robust, &r0, &rho1);
                                if (lead && nl <= kPlaneChunk) {
                                    S.perrB[j][q][0] = err[0]; S.perrB[j][q][1] = err[1]; S.perrB[j][q][2] = err[2];
                                }
                            }
                            ring_wait(S, ea < eb ? eb - RB::kRows : 0);
                            if (lead && np + j < eb) ringB[((np + j) & (RB::kRows - 1)) * RB::kStride + q] = r0;
                            lds_publish(&S.done[wv], k + 1);
                        }
                        PROF_MARK(19);  // pass B plane rounds
                    }
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
                            total_trials++;
                            more = rho < 0 && qmax < kMaxTrials;
                        }
                    }
                    if (lane == 0) {
                        SE3 tl = Tq[0];
#pragma unroll
                        for (int q = 1; q < kSpec; q++)
                            if (q == lastq) tl = Tq[q];
                        S.tlast[wv] = tl;
                    }
#pragma unroll
                    for (int j = 0; j < 6; j++) xs[j] = S.xtrial[(total_passes - 1) & 1][lastq][j];  // the buffer after the last trial run
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
        wave_sync();
        const SE3 Tlast = S.tlast[wv];
        double bad = 0;
        auto relabel_pose = [&](bool was_out) __attribute__((always_inline)) {
            SE3 Te;  // field-wise select (a selected reference would put both poses in scratch memory)
            Te.r.w = was_out ? T.r.w : Tlast.r.w; Te.r.x = was_out ? T.r.x : Tlast.r.x;
            Te.r.y = was_out ? T.r.y : Tlast.r.y; Te.r.z = was_out ? T.r.z : Tlast.r.z;
            Te.t.x = was_out ? T.t.x : Tlast.t.x; Te.t.y = was_out ? T.t.y : Tlast.t.y; Te.t.z = was_out ? T.t.z : Tlast.t.z;
            return Te;
        };
        // the loops' first indices are opaque here: hoisted out of the round loop, their 64-bit edge addresses
        // were the kernel's only scratch spills (2 x 8 bytes per lane at 254 VGPRs, stored once per launch)
        int e0 = t, j0 = t >> 1;
        asm volatile("" : "+v"(e0), "+v"(j0));
        for (int e = e0; e < np; e += kThreads) {
            double info[3], delta, err[3] = {0, 0, 0};
            edge_info(e, info, &delta);
            point_error_at(e, relabel_pose(pout[e] != 0), err, nullptr);
            const float chi2 = (float)chi2_of(err, info);
            const bool bd = pts[e].ur < 0 ? chi2 > 5.991f : chi2 > 7.815f;
            bad += bd ? 1.0 : 0.0;
            pout[e] = bd;
        }
        for (int j = j0; j < nl; j += kThreads / 2) {  // plane edges on lane pairs
            double info[3], delta, err[3] = {0, 0, 0};
            edge_info(np + j, info, &delta);
            plane_error_pair_at(np + j, relabel_pose(plout[j] != 0), err);
            const float chi2 = (float)chi2_of(err, info);
            const bool bd = pls[j].kind == 0 ? (double)chi2 > K.plane_chi : (double)chi2 > K.vp_chi;
            if ((lane & 1) == 0) {
                bad += bd ? 1.0 : 0.0;
                plout[j] = bd;
            }
        }
        double cb[1] = {bad};
        wg_sum(cb, S, buf);  // small integers: exact
        nBad = (int)cb[0];
        PROF_MARK(8);  // relabel
        if (round == 2) robust = false;
        if (ne < 10) break;
    }
    __syncthreads();
    if (S.stall) {  // every outlier flag set: nothing of a failed problem is kept (the tail's discard reads them)
        int e0 = t;
        asm volatile("" : "+v"(e0));  // (no loop bound hoisted to the kernel's start, where it was spilled)
        for (int e = e0; e < np; e += kThreads) pout[e] = 1;
        for (int j = e0; j < nl; j += kThreads) plout[j] = 1;
    }
    if (t == 0 && S.stall) {
        // a bounded wait gave up (never observed): the sums are not valid, so the problem reports failure -- the
        // input pose, no inliers, lm_iterations = -1, every edge flagged -- and callers treat it as a lost frame
        for (int i = 0; i < 16; i++) res->Tcw[i] = Tin[i];
        res->n_inliers = 0;
        res->lm_iterations = -1;
        res->trial_passes = total_passes;
        res->trials = total_trials;
    } else if (t == 0) {
        const M3 R = q_to_rot(T.r);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) res->Tcw[4 * i + j] = (float)R.a[3 * i + j];
        res->Tcw[3] = (float)T.t.x; res->Tcw[7] = (float)T.t.y; res->Tcw[11] = (float)T.t.z;
        res->Tcw[12] = 0.f; res->Tcw[13] = 0.f; res->Tcw[14] = 0.f; res->Tcw[15] = 1.f;
        res->n_inliers = ne - nBad;
        res->lm_iterations = total_its;
        res->trial_passes = total_passes;
        res->trials = total_trials;
    }
#ifdef SPSLAM_POSE_PROF
    PROF_MARK(9);  // outputs
    if (t == 0) {
        for (int k = 0; k < 12; k++) atomicAdd(&g_pose_prof[k], prof_acc[k]);
        for (int k = 16; k < 20; k++) atomicAdd(&g_pose_prof[k], prof_acc[k]);
    }
    if (t == kCompute)
        for (int k = 12; k < 16; k++) atomicAdd(&g_pose_prof[k], prof_acc[k]);
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
    K.spin_cap = 1 << 20;
    K.fail_mask = 0;
    return K;
}

hipError_t pose_launch(int n, const spslam_pose_problem* probs, const spslam_point_obs* pts,
                       const spslam_plane_obs* pls, const PoseConsts& K, const spslam_pose_result* init_from,
                       spslam_pose_result* res, uint8_t* pout, uint8_t* plout, hipStream_t s) {
    static const int spec = [] {
        const char* e = std::getenv("SPSLAM_POSE_SPEC");  // measurement knob: damping trials per edge pass
        return e ? std::atoi(e) : 4;
    }();
    // measurement knob: SPSLAM_POSE_WHOLE_CU=1 pads the workgroup's LDS to the CU's 160 KB, so no other workgroup
    // shares a PoseOptimization CU (the pose runs at its alone speed; the CUs are unavailable to the rest meanwhile)
    static const size_t pad = [] {
        const char* e = std::getenv("SPSLAM_POSE_WHOLE_CU");
        if (!e || e[0] != '1') return (size_t)0;
        hipFuncAttributes a{};
        if (hipFuncGetAttributes(&a, (const void*)pose_kernel<4>) != hipSuccess) return (size_t)0;
        return a.sharedSizeBytes < 160 * 1024 ? 160 * 1024 - a.sharedSizeBytes : (size_t)0;
    }();
    if (spec <= 1)
        hipLaunchKernelGGL(pose_kernel<1>, dim3(n), dim3(kThreads), 0, s, probs, pts, pls, K, init_from, res, pout, plout);
    else if (spec == 2)
        hipLaunchKernelGGL(pose_kernel<2>, dim3(n), dim3(kThreads), 0, s, probs, pts, pls, K, init_from, res, pout, plout);
    else
        hipLaunchKernelGGL(pose_kernel<4>, dim3(n), dim3(kThreads), pad, s, probs, pts, pls, K, init_from, res, pout,
                           plout);
    return hipGetLastError();
}

}  // namespace spslam

#ifdef SPSLAM_POSE_PROF
// Diagnostic build only: the accumulated phase ticks / counters (24 u64), optionally reset.
extern "C" int spslam_pose_prof_read(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pose_prof), 24 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[24] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pose_prof), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
