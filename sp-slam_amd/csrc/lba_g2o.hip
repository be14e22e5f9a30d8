// gfx950 LocalBundleAdjustment in g2o's own arithmetic (reference: src/Optimizer.cc:1154-1977 on the vendored
// g2o SparseOptimizer + OptimizationAlgorithmLevenberg + BlockSolver_6_3 + LinearSolverEigen, g2oAddition plane
// edges).  Semantics: oracle/lba_oracle.cpp, which this reproduces bit for bit.
//
// One persistent 512-thread workgroup per problem runs the whole schedule -- setup, optimize(5), relabel,
// optimize(10), outputs -- with no host round trip and no cross-workgroup hand-off; many problems (the local maps
// of many sequences) run side by side, one per CU.  Every order-sensitive sum follows g2o:
//   chi2          activeRobustChi2: one lane adds the edges' robust chi2 in edge-insertion order (the others
//                 evaluate the errors first; inactive edges contribute an exact +0.0);
//   Hll, bl, Hpl  per landmark, its edges in insertion order (one thread per landmark);
//   Hpp, bp       per free pose and term, its edges in insertion order (one lane per (pose, term) chain);
//   Schur         Hschur = Hpp (+ lambda), then landmark by landmark in landmark-index (vertex-id) order
//                 Hi1i2 -= BDinv Bj^T and Bb += Bi db (block_solver.hpp:381-431): one lane per (block row of a
//                 pattern block, i.e. (i1, i2, r)) holds the row's six entries and subtracts each landmark's
//                 contribution in order;
//   factor/solve  Eigen SimplicialLDLT<Upper> on g2o's Hschur pattern: AMD ordering (the scalar
//                 minimum_degree_ordering, one lane; every scalar dense -> the natural order at once), elimination
//                 tree and L's column patterns as bitsets, each row's topological pattern order from the same
//                 tree walks, then the up-looking factorisation on one wave (y in registers, one lane per row of
//                 the reduced system, the pattern order's steps as readlane broadcasts), Eigen's triangular solves;
//   scale         computeScale: x . (lambda x + b) over poses then landmarks, one lane.
// The quadratic-form terms of every edge (Jacobians: analytic for points, central differences for planes on lane
// pairs), errors and updates run in parallel.  Floating-point expressions are the oracle's (g2o_restated.h,
// eigen_simplicial_restated.h); DESIGN.md section 3.9.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "g2o_device.h"
#include "lba_launch.h"

// Two instances of this file are compiled (itself and lba_g2o_wide.hip): LBG_PW = 1 (pose masks of one 64-bit
// word: up to 64 free poses, n <= 384) and LBG_PW = 2 (two words: up to 128 free poses, n <= 768).  The narrow one is
// the round-5 kernel unchanged in its arithmetic; the host runs the wide one for windows of more than 64 keyframes.
#ifndef LBG_PW
#define LBG_PW 1
#endif
#if LBG_PW == 1
#define LBG_NS lbag
#define LBG_RUN lba_run_g2o_pw1
#else
#define LBG_NS lbag2
#define LBG_RUN lba_run_g2o_pw2
#endif

namespace spslam {
namespace LBG_NS {

using namespace g2od;

constexpr int kT = kLbgThreads, kW = kT / 64;
constexpr int kMaxKF = kLbgMaxKeyframes;  // keyframes (local + fixed)
constexpr int kPW = LBG_PW;               // 64-bit words of a pose mask
constexpr int kMaxK = 64 * kPW;           // free poses (Hessian blocks)
constexpr int kNW = 6 * kPW;              // bitset words for up to 6 * kMaxK scalars
constexpr int kDyn = 136 * 1024;        // dynamic LDS (setup tiles, AMD workspace, the factorisation's L)
constexpr int kDynAlloc = (LBG_PW == 1 ? 154 : 152) * 1024;  // allocated: kDyn plus the Schur phase's staged Bb
                                                              //   terms and block tables (static LDS + this <= 160 KB)
                                        //   (every phase but the Schur one sizes itself against kDyn)
constexpr int kLdsN = LBG_PW == 1 ? 96 : 90;  // reduced systems of n <= kLdsN rows factorised in LDS (L, S packed:
                                               //   133 KB; the wide instance's structure words take more)
constexpr int kSchurLm = 64;            // Schur phase: landmarks per staged chunk (one bit each in a 64-bit mask)
constexpr int kSchurBlk = LBG_PW == 1 ? 412 : 360;  //   and Hpl blocks per chunk (the staging buffer, 16 doubles a
                                                    //   thread, + BDinv; the wide instance's tables take more)

// A set of free poses (Hessian indices) as kPW 64-bit words; with kPW = 1 every operation is the plain uint64_t one.
struct PMask {
    uint64_t w[kPW];
};
__device__ __forceinline__ PMask pm_zero() {
    PMask m;
#pragma unroll
    for (int k = 0; k < kPW; k++) m.w[k] = 0ull;
    return m;
}
__device__ __forceinline__ PMask pm_bit(int i) {
    PMask m;
    if constexpr (kPW == 1) {
        m.w[0] = 1ull << i;
    } else {
#pragma unroll
        for (int k = 0; k < kPW; k++) m.w[k] = (i >> 6) == k ? 1ull << (i & 63) : 0ull;
    }
    return m;
}
__device__ __forceinline__ bool pm_test(const PMask& m, int i) {
    if constexpr (kPW == 1) {
        return (m.w[0] >> i) & 1ull;
    } else {
        uint64_t v = m.w[0];
#pragma unroll
        for (int k = 1; k < kPW; k++) v = (i >> 6) == k ? m.w[k] : v;
        return (v >> (i & 63)) & 1ull;
    }
}
__device__ __forceinline__ void pm_set(PMask& m, int i) {
    if constexpr (kPW == 1) {
        m.w[0] |= 1ull << i;
    } else {
#pragma unroll
        for (int k = 0; k < kPW; k++) m.w[k] |= (i >> 6) == k ? 1ull << (i & 63) : 0ull;
    }
}
__device__ __forceinline__ PMask pm_and(PMask a, const PMask& b) {
#pragma unroll
    for (int k = 0; k < kPW; k++) a.w[k] &= b.w[k];
    return a;
}
__device__ __forceinline__ PMask pm_or(PMask a, const PMask& b) {
#pragma unroll
    for (int k = 0; k < kPW; k++) a.w[k] |= b.w[k];
    return a;
}
__device__ __forceinline__ PMask pm_andnot(PMask a, const PMask& b) {
#pragma unroll
    for (int k = 0; k < kPW; k++) a.w[k] &= ~b.w[k];
    return a;
}
// bits [0, i), 0 <= i < 64 kPW (the narrow instance: (1 << i) - 1, i < 64)
__device__ __forceinline__ PMask pm_below(int i) {
    PMask m;
    if constexpr (kPW == 1) {
        m.w[0] = (1ull << i) - 1ull;
    } else {
#pragma unroll
        for (int k = 0; k < kPW; k++) {
            const int c = i - 64 * k;
            m.w[k] = c >= 64 ? ~0ull : c <= 0 ? 0ull : (1ull << c) - 1ull;
        }
    }
    return m;
}
// bits [0, n), 0 <= n <= 64 kPW
__device__ __forceinline__ PMask pm_first_n(int n) {
    PMask m;
#pragma unroll
    for (int k = 0; k < kPW; k++) {
        const int c = n - 64 * k;
        m.w[k] = c >= 64 ? ~0ull : c <= 0 ? 0ull : (1ull << c) - 1ull;
    }
    return m;
}
__device__ __forceinline__ int pm_popc(const PMask& m) {
    int c = 0;
#pragma unroll
    for (int k = 0; k < kPW; k++) c += __popcll(m.w[k]);
    return c;
}
__device__ __forceinline__ int pm_popc_below(const PMask& m, int i) { return pm_popc(pm_and(m, pm_below(i))); }
__device__ __forceinline__ bool pm_any(const PMask& m) {
    uint64_t v = m.w[0];
#pragma unroll
    for (int k = 1; k < kPW; k++) v |= m.w[k];
    return v != 0ull;
}
__device__ __forceinline__ bool pm_eq(const PMask& a, const PMask& b) {
    bool e = true;
#pragma unroll
    for (int k = 0; k < kPW; k++) e = e && a.w[k] == b.w[k];
    return e;
}
// lowest set bit (the mask must not be empty)
__device__ __forceinline__ int pm_ffs(const PMask& m) {
    if constexpr (kPW == 1) {
        return __ffsll((unsigned long long)m.w[0]) - 1;
    } else {
        int r = -1;
#pragma unroll
        for (int k = kPW - 1; k >= 0; k--)
            if (m.w[k]) r = 64 * k + __ffsll((unsigned long long)m.w[k]) - 1;
        return r;
    }
}
// the mask without its lowest set bit
__device__ __forceinline__ void pm_pop(PMask& m) {
    if constexpr (kPW == 1) {
        m.w[0] &= m.w[0] - 1;
    } else {
        bool done = false;
#pragma unroll
        for (int k = 0; k < kPW; k++)
            if (!done && m.w[k]) {
                m.w[k] &= m.w[k] - 1;
                done = true;
            }
    }
}

struct Sh {
    double red[kW][4];
    int iscan[kW];
    PMask pat[kMaxK];                   // Schur block pattern: row i1, bits i2 >= i1
    short hidx[kMaxKF];                 // keyframe -> free-pose Hessian index (-1: fixed or inactive)
    unsigned char kact[kMaxKF];         // structure: keyframes with an active edge
    int hpose[kMaxK];                   // Hessian index -> keyframe
    int pdeg[kMaxK];                    // poses coupled with each pose (itself included)
    int np, nl, nact, nch, nb, flag, unsup, dense;
    // the team (one workgroup per member, lba_g2o's header): problem, member, size, barrier generation; this
    // member's buildSystem share (landmark-aligned edge range, its free poses)
    int p, m, T, gen, eb0, eb1, npown, bo0, bo1;
    PMask rmask;                        // this member's Schur block rows
    PMask carry;                        // buildSystem: Hpl blocks touched by the landmark continuing into the next step
    double csum[2][12];                 //   and its partial Hll / bl sums (by step parity)
    int pown[kMaxK];
    // LM / schedule state (every member computes it identically between barriers)
    int pass, it, max_it, robust, qmax, nBad, trials, its[2], stop, stopped, ok, need_err, done, accepted, fail;
    double lambda, ni, currentChi, iniChi, tempChi, scale;
    long long ph[8], tlast, tB;  // diagnostics: wall_clock64 ticks per phase (result phase_us[1..7])
    long long dg[14];            // SPSLAM_LBG_DIAG sub-phase ticks
};
// thread 0 charges the time since the previous mark to phase k (called right after a barrier)
#define LBG_MARK(k)                                  \
    if (threadIdx.x == 0) {                          \
        const long long now_ = wall_clock64();       \
        s.ph[k] += now_ - s.tlast;                   \
        s.tlast = now_;                              \
    }

// Global-memory pointers typed with the global address space: G lives in LDS and the phase functions are not
// inlined, so a generic pointer would make every access a FLAT instruction (which also counts against the LDS
// wait counter, so LDS reads would wait for every outstanding global load).
#define GL __attribute__((address_space(1)))
typedef double GL gdouble;
typedef int GL gint;
typedef uint64_t GL guint64;
struct G {
    int K, Np, Nq, L, E, Ep;
    const spslam_lba_keyframe GL* kf;
    const spslam_lba_point GL* pt;
    const spslam_lba_plane GL* pl;
    const spslam_lba_point_obs GL* pobs;
    const spslam_lba_plane_obs GL* plobs;
    gdouble *pose, *pose_b, *X, *X_b, *P, *P_b, *err, *echi, *sc, *terms, *Hll, *bl, *Dinv, *db, *blkB, *Hps,
        *S, *bs, *x, *Ld;
    gint *e_lm, *e_kf, *e_type, *e_level, *e_src, *e_blk, *lm_boff, *lm_nb, *lm_sorted, *lm_hidx, *hidx_lm, *lmh_blk,
        *pe_off, *pe_idx, *Pinv, *Pm, *parent, *rs_off, *rs_idx, *amd_Ci, *amd_W, *sch, *sch_kb,
        *eseg,   // per edge: {RI, landmark hidx, segment end, first block | segment start << 30}
        *bord;   // Schur pattern blocks, longest chain first
    PMask GL *lmh_mask, *lm_amask;
    guint64 *Lbits, *Abits;
    LbgTeam GL* team;
};
// pose masks in global memory (word by word: an address-space-qualified PMask has no copy constructor)
__device__ __forceinline__ PMask pm_ld(const PMask GL* p) {
    const uint64_t GL* q = (const uint64_t GL*)p;
    PMask m;
#pragma unroll
    for (int k = 0; k < kPW; k++) m.w[k] = q[k];
    return m;
}
__device__ __forceinline__ void pm_st(PMask GL* p, const PMask& m) {
    uint64_t GL* q = (uint64_t GL*)p;
#pragma unroll
    for (int k = 0; k < kPW; k++) q[k] = m.w[k];
}

// The workgroup's LDS objects at namespace scope: the phase functions are not inlined, and a pointer or reference
// argument would reach them as a generic (flat) address -- every LDS access a FLAT instruction, which also waits on
// the outstanding global loads.  Referenced by name, they compile to ds_* instructions.
extern __shared__ __attribute__((aligned(16))) unsigned char lbg_dyn[];
__shared__ Sh lbg_s;
__shared__ G lbg_g;
__shared__ LbaConsts lbg_c;

__device__ G make_g(const LbgBatch& b, int p) {
    const spslam_lba_problem pb = b.probs[p];
    G g;
    g.K = pb.n_kf; g.Np = pb.n_points; g.Nq = pb.n_planes;
    g.Ep = pb.n_point_obs; g.E = pb.n_point_obs + pb.n_plane_obs; g.L = g.Np + g.Nq;
    g.kf = (const spslam_lba_keyframe GL*)(b.kfs + pb.kf_offset);
    g.pt = (const spslam_lba_point GL*)(b.pts + pb.point_offset);
    g.pl = (const spslam_lba_plane GL*)(b.pls + pb.plane_offset);
    g.pobs = (const spslam_lba_point_obs GL*)b.pobs;
    g.plobs = (const spslam_lba_plane_obs GL*)b.plobs;
    const LbgLayout Ly = lbg_layout(g.K, g.Np, g.Nq, g.E, kPW);
    uint8_t* base = b.scratch + b.scratch_off[p];
    auto D = [&](size_t o) { return (double GL*)(base + o); };
    auto I = [&](size_t o) { return (int GL*)(base + o); };
    g.pose = D(Ly.pose); g.pose_b = D(Ly.pose_b); g.X = D(Ly.X); g.X_b = D(Ly.X_b); g.P = D(Ly.P); g.P_b = D(Ly.P_b);
    g.err = D(Ly.err); g.echi = D(Ly.echi); g.sc = D(Ly.sc); g.terms = D(Ly.terms); g.Hll = D(Ly.Hll);
    g.bl = D(Ly.bl); g.Dinv = D(Ly.Dinv); g.db = D(Ly.db); g.blkB = D(Ly.blkB);
    g.Hps = D(Ly.Hps); g.S = D(Ly.S); g.bs = D(Ly.bs); g.x = D(Ly.x); g.Ld = D(Ly.Ld);
    g.e_lm = I(Ly.e_lm); g.e_kf = I(Ly.e_kf); g.e_type = I(Ly.e_type); g.e_level = I(Ly.e_level);
    g.e_src = I(Ly.e_src); g.e_blk = I(Ly.e_blk); g.lm_boff = I(Ly.lm_boff); g.lm_nb = I(Ly.lm_nb);
    g.lm_sorted = I(Ly.lm_sorted); g.lm_hidx = I(Ly.lm_hidx); g.hidx_lm = I(Ly.hidx_lm); g.lmh_blk = I(Ly.lmh_blk);
    g.pe_off = I(Ly.pe_off); g.pe_idx = I(Ly.pe_idx); g.Pinv = I(Ly.Pinv); g.Pm = I(Ly.Pm); g.parent = I(Ly.parent);
    g.rs_off = I(Ly.rs_off); g.rs_idx = I(Ly.rs_idx); g.amd_Ci = I(Ly.amd_Ci); g.amd_W = I(Ly.amd_W);
    g.sch = I(Ly.sch); g.sch_kb = I(Ly.sch_kb); g.eseg = I(Ly.eseg); g.bord = I(Ly.bord);
    g.lmh_mask = (PMask GL*)(base + Ly.lmh_mask); g.lm_amask = (PMask GL*)(base + Ly.lm_amask);
    g.Lbits = (uint64_t GL*)(base + Ly.Lbits); g.Abits = (uint64_t GL*)(base + Ly.Abits);
    g.team = (LbgTeam GL*)(base + Ly.team);
    return g;
}

// ---------------------------------------------------------------- the team
// A problem is solved by T workgroups (members; T = b.team), one per CU.  Membership follows arrival: each
// workgroup takes a ticket (ctl[0]) when it starts; tickets p T .. p T + T - 1 form problem p's team, member 0 (the
// leader) being the first.  A member therefore only ever waits for workgroups that already run, or for the next
// workgroup to be dispatched -- never for one queued behind a waiting member -- so teams cannot deadlock however many
// launches share the chip.  Every member runs the same schedule: the serial steps (setup, structure + AMD, the
// factorisation) on the leader, the parallel ones split over the members, the LM control replicated (each member
// computes the same ordered sums from the same global arrays and takes the same decisions).  Phases meet at
// team_sync, the inter-workgroup hand-off of MI355X_MICROARCH.md ("valid forms"): every storing wave drains its
// stores (s_waitcnt vmcnt(0)), a workgroup barrier, one lane releases at agent scope (buffer_wbl2: the XCD's L2
// written back), drains again (the explicit wait the ROCm 7.2 compiler may drop after the release), and adds to the
// team's counter with a relaxed agent atomic; it polls the counter with relaxed agent loads (sc1: L2, not L1), then
// acquires at agent scope (buffer_inv sc1: this CU's L1 invalidated), drains, and a workgroup barrier lets the other
// waves read with plain loads.  The leader also samples the caller's pbStopFlag before it releases; every member
// reads that sample after the barrier, so all members see the flag change at the same barrier.
__device__ __forceinline__ int* team_ctr(const LbgBatch& b, int p) { return b.ctl + 16 * (p + 1); }
__device__ __noinline__ void team_sync(const LbgBatch& b) {
    Sh& s = lbg_s;
    const G& g = lbg_g;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int gen = ++s.gen;  // this barrier's number
        bool seen = false;
        if (s.m == 0 && b.stop && !s.stop)
            seen = __hip_atomic_load(b.stop + s.p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        if (s.T > 1) {
            // the sample is published as the barrier number it belongs to: a member that reads the record late
            // (after the leader has entered a later barrier) still takes the flag at the same barrier as the others
            if (seen) g.team->stop_gen = gen;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            int* ctr = team_ctr(b, s.p);
            __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int target = s.T * gen;
            while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
                __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int sg = g.team->stop_gen;
            seen = sg != 0 && sg <= gen;
        }
        if (seen) s.stop = 1;  // latched (SparseOptimizer::terminate())
    }
    __syncthreads();
}
__device__ __forceinline__ int split_lo(int n, int m, int T) { return (int)(((long long)n * m) / T); }

// ---------------------------------------------------------------- workgroup primitives
__device__ __forceinline__ int block_scan(int v, int* total, Sh& s) {  // exclusive; *total = sum
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s.iscan[w] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < kW; j++) {
        const int q = s.iscan[j];
        if (j < w) base += q;
        tot += q;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}
__device__ __forceinline__ int block_and(int v, Sh& s) {
    const int w = threadIdx.x >> 6;
    const bool all = __all(v != 0);
    if ((threadIdx.x & 63) == 0) s.iscan[w] = all;
    __syncthreads();
    int r = 1;
#pragma unroll
    for (int j = 0; j < kW; j++) r &= s.iscan[j];
    __syncthreads();
    return r;
}
__device__ __forceinline__ double block_max(double v, Sh& s) {  // max of non-negative values
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) s.red[w][0] = v;
    __syncthreads();
    double m = 0.0;
#pragma unroll
    for (int j = 0; j < kW; j++) m = fmax(m, s.red[j][0]);
    __syncthreads();
    return m;
}
__device__ __forceinline__ double rl(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
// value of entry i of a vector spread over the wave (entry 64 m + lane in register m)
template <int kC>
__device__ __forceinline__ double pick(const double (&v)[kC], int i) {
    double r = rl(v[0], i & 63);  // (wave-uniform selects, no branches)
#pragma unroll
    for (int m = 1; m < kC; m++) {
        const double q = rl(v[m], i & 63);
        r = (i >> 6) == m ? q : r;
    }
    return r;
}
__device__ __forceinline__ int4 ld_i4(const gint* p) {  // one 16-byte load (p 16-byte aligned)
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i v = *(const v4i GL*)p;
    return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ---------------------------------------------------------------- edge math (oracle/lba_oracle.cpp)
template <class PD>
__device__ __forceinline__ SE3 load_pose(const PD* p) { return SE3{Q{p[0], p[1], p[2], p[3]}, V3{p[4], p[5], p[6]}}; }
template <class PD>
__device__ __forceinline__ void store_pose(PD* p, const SE3& T) {
    p[0] = T.r.w; p[1] = T.r.x; p[2] = T.r.y; p[3] = T.r.z; p[4] = T.t.x; p[5] = T.t.y; p[6] = T.t.z;
}
template <class PF>
__device__ __forceinline__ P4 plane_from_f(const PF* c) {  // Converter::toPlane3D + Plane3D(v)
    P4 p{{c[0], c[1], c[2], c[3]}};
    if (c[3] < 0.0f)
        for (int i = 0; i < 4; i++) p.c[i] = -p.c[i];
    p_normalize(p.c);
    return p;
}
__device__ __forceinline__ P4 plane_transform(const SE3& T, const P4& w) {
    const M3 R = q_to_rot(T.r);
    const V3 n2 = mv(R, V3{w.c[0], w.c[1], w.c[2]});
    P4 v{{n2.x, n2.y, n2.z, w.c[3] - dot(T.t, n2)}};
    if (v.c[3] < 0.0)
        for (int i = 0; i < 4; i++) v.c[i] = -v.c[i];
    p_normalize(v.c);
    return v;
}
__device__ __forceinline__ int edge_dim(int type) { return type == 0 ? 2 : (type <= 2 ? 3 : 2); }
__device__ __forceinline__ void info_of_src(const G& g, const LbaConsts& C, int src, int t, double* info) {
    if (t <= 1) {
        const double s = (double)g.pobs[src].inv_sigma2;
        info[0] = info[1] = info[2] = s;
    } else if (t == 2) {
        info[0] = info[1] = C.angle_info; info[2] = C.dis_info;
    } else {
        info[0] = info[1] = t == 3 ? C.par_info : C.ver_info;
        info[2] = 0;
    }
}
__device__ __forceinline__ void info_of(const G& g, const LbaConsts& C, int e, int t, double* info) {
    info_of_src(g, C, t <= 1 ? g.e_src[e] : 0, t, info);
}
template <class PE>
__device__ __forceinline__ double chi2_of(const PE* err, const double* info, int dim) {  // e . (Omega e)
    double s = 0;
    for (int i = 0; i < dim; i++) s += err[i] * (info[i] * err[i]);
    return s;
}
__device__ __forceinline__ double delta_of(const LbaConsts& C, int t) {
    return t == 0 ? C.delta_mono : t == 1 ? C.delta_stereo : t == 2 ? C.delta_plane : C.delta_vp;
}
// RobustKernelHuber::robustify; rho0 / rho1 (non-robust: chi2, 1)
__device__ __forceinline__ void huber(double chi, double delta, bool on, double* rho0, double* rho1) {
    const double dsqr = delta * delta;
    if (!on || chi <= dsqr) { *rho0 = chi; *rho1 = 1.0; return; }
    const double s = sqrt(chi);
    *rho0 = 2 * s * delta - dsqr;
    *rho1 = delta / s;
}
// A point edge's operands, loaded together (errors() gathers several edges' before evaluating any)
struct PointIn {
    SE3 T;
    double X[3];
    float u, v, ur, isg, fx, fy, cx, cy, bf;
};
__device__ __forceinline__ PointIn point_in(const G& g, int kf, int lm, int src) {
    PointIn a;
    a.T = load_pose(g.pose + 7 * kf);
    for (int i = 0; i < 3; i++) a.X[i] = g.X[3 * lm + i];
    const auto& o = g.pobs[src];
    a.u = o.u; a.v = o.v; a.ur = o.ur; a.isg = o.inv_sigma2;
    const auto& k = g.kf[kf];
    a.fx = k.fx; a.fy = k.fy; a.cx = k.cx; a.cy = k.cy; a.bf = k.bf;
    return a;
}
__device__ __forceinline__ void point_error_v(int t, const PointIn& a, double* err) {
    const V3 p = q_rot(a.T.r, V3{a.X[0], a.X[1], a.X[2]}) + a.T.t;
    if (t == 0) {
        err[0] = (double)a.u - (p.x / p.z * (double)a.fx + (double)a.cx);
        err[1] = (double)a.v - (p.y / p.z * (double)a.fy + (double)a.cy);
        err[2] = 0.0;
    } else {
        const float invz = (float)(1.0f / p.z);
        const double r0 = p.x * invz * (double)a.fx + (double)a.cx, r1 = p.y * invz * (double)a.fy + (double)a.cy;
        const double r2 = r0 - (double)(a.bf * invz);  // cam_project(..., const float& bf)
        err[0] = (double)a.u - r0;
        err[1] = (double)a.v - r1;
        err[2] = (double)a.ur - r2;
    }
}
__device__ bool depth_positive(const G& g, int e) {
    const SE3 T = load_pose(g.pose + 7 * g.e_kf[e]);
    const int lm = g.e_lm[e];
    if (g.e_type[e] <= 1) {
        auto X = g.X + 3 * lm;
        return (q_rot(T.r, V3{X[0], X[1], X[2]}) + T.t).z > 0.0;
    }
    auto pp = g.P + 4 * (lm - g.Np);
    return -plane_transform(T, P4{{pp[0], pp[1], pp[2], pp[3]}}).c[3] > 0;
}
// EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ::linearizeOplus (types_six_dof_expmap.cpp:103-234)
// needA false (a uniform branch): only B (the pose side's Jacobian) is formed
// (edge of keyframe kf and landmark lm)
__device__ __forceinline__ void point_jacobians(const G& g, int kf, int lm, int t, double (&A)[3][3], double (&B)[3][6],
                                                bool needA = true) {
    const SE3 T = load_pose(g.pose + 7 * kf);
    const auto& k = g.kf[kf];
    const double fx = k.fx, fy = k.fy, bf = k.bf;
    auto X = g.X + 3 * lm;
    const V3 p = q_rot(T.r, V3{X[0], X[1], X[2]}) + T.t;
    const double x = p.x, y = p.y, z = p.z, z_2 = z * z;
    if (!needA) {
    } else if (t == 0) {
        const M3 R = q_to_rot(T.r);
        const double tmp[2][3] = {{fx, 0, -x / z * fx}, {0, fy, -y / z * fy}};
        const double s = -1. / z;
        for (int r = 0; r < 2; r++) {
            const double t0 = s * tmp[r][0], t1 = s * tmp[r][1], t2 = s * tmp[r][2];
            for (int q = 0; q < 3; q++) A[r][q] = t0 * R.a[q] + t1 * R.a[3 + q] + t2 * R.a[6 + q];
        }
        A[2][0] = A[2][1] = A[2][2] = 0.0;
    } else {
        const M3 R = q_to_rot(T.r);
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
    } else {
        for (int q = 0; q < 6; q++) B[2][q] = 0.0;
    }
}
// Eigen compute_inverse<Matrix3d> (cofactors), r row-major
__device__ __forceinline__ void inverse3(const double (&m)[3][3], double* r) {
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

__device__ __forceinline__ constexpr int upper_idx(int r, int c) { return 6 * r - r * (r - 1) / 2 + (c - r); }  // r <= c < 6

// One edge's quadratic-form terms (BaseBinaryEdge::constructQuadraticForm as Eigen evaluates it, Omega diagonal):
//   Hll += (A^T W) A;  bl += A^T omega_r;  Hpl (6 x 3, pose-major) += (B^T W) A (robust) | B^T (A^T Omega)^T
//   (non-robust);  Hpp upper (r <= c) += (B^T W) B;  bp += B^T omega_r
// W = rho' Omega (robust) or Omega; omega_r = (-(Omega e)) rho' or -(Omega e) (terms_land / terms_pose below).

// SparseOptimizer::terminate(): the caller's flag as the leader sampled it at the last team_sync (latched in s.stop),
// or the deterministic test hook (spslam_lba_debug_stop_after) on the replicated trial count
__device__ __forceinline__ bool stop_requested(const LbgBatch& b, Sh& s) {
    if (!s.stop && b.stop_after >= 0 && s.trials >= b.stop_after) s.stop = 1;
    return s.stop != 0;
}

// ---------------------------------------------------------------- setup (once)
__device__ __noinline__ void setup() {
    const G& g = lbg_g;
    Sh& s = lbg_s;
    int* dyn_i = (int*)lbg_dyn;
    const int t = threadIdx.x;
    for (int k = t; k < g.K; k += kT) {  // Converter::toSE3Quat
        const auto* T = g.kf[k].Tcw;
        M3 Rm;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) Rm.a[3 * i + j] = T[4 * i + j];
        SE3 q;
        q.r = q_from_rot(Rm);
        q.t = V3{T[3], T[7], T[11]};
        q_normalize(q.r);
        store_pose(g.pose + 7 * k, q);
    }
    for (int i = t; i < g.Np; i += kT)
        for (int j = 0; j < 3; j++) g.X[3 * i + j] = g.pt[i].xw[j];
    for (int i = t; i < g.Nq; i += kT) {
        const P4 q = plane_from_f(g.pl[i].world);
        for (int j = 0; j < 4; j++) g.P[4 * i + j] = q.c[j];
    }
    // edges in insertion order: point observations (points in list order), then plane observations
    int base_e = 0;
    for (int ch = 0; ch < g.L; ch += kT) {
        const int l = ch + t;
        const int n_obs = l < g.Np ? g.pt[l].n_obs : (l < g.L ? g.pl[l - g.Np].n_obs : 0);
        int tot;
        const int off = block_scan(n_obs, &tot, s) + base_e;
        if (l < g.L) {
            g.lm_boff[l] = off;
            g.lm_nb[l] = n_obs;
            const int src0 = l < g.Np ? g.pt[l].obs_offset : g.pl[l - g.Np].obs_offset;
            for (int o = 0; o < n_obs; o++) {
                const int e = off + o;
                g.e_lm[e] = l;
                g.e_src[e] = src0 + o;
                g.e_level[e] = 0;
                if (l < g.Np) {
                    const auto& ob = g.pobs[src0 + o];
                    g.e_kf[e] = ob.kf;
                    g.e_type[e] = ob.ur < 0 ? 0 : 1;
                } else {
                    const auto& ob = g.plobs[src0 + o];
                    g.e_kf[e] = ob.kf;
                    g.e_type[e] = ob.kind == SPSLAM_PLANE_EDGE ? 2 : (ob.kind == SPSLAM_PARALLEL_EDGE ? 3 : 4);
                }
            }
        }
        base_e += tot;
    }
    for (int e = g.E + t; e < lbg_pad32(g.E); e += kT) g.echi[e] = 0.0;
    // g2o's solution buffer (Solver::_x): written only by successful solves and read by every update, so a failed
    // solve re-applies the previous solution; never written = zeros (update())
    for (int j = t; j < lbg_pad32(6 * lbg_free_cap(g.K, kPW) + 3 * g.L); j += kT) g.x[j] = 0.0;
    // landmark (vertex-id) order: points by id (ids mnId + maxKFid + 1), then planes by id (mnId + maxPointid + 1,
    // above every point id); stable ranks (id, list index)
    for (int grp = 0; grp < 2; grp++) {
        const int n0 = grp ? g.Np : 0, cnt = grp ? g.Nq : g.Np;
        auto id_of = [&](int i) { return grp ? g.pl[i].id : g.pt[i].id; };
        int ok = 1;
        for (int i = t; i + 1 < cnt; i += kT) ok &= id_of(i) <= id_of(i + 1);
        if (block_and(ok, s)) {
            for (int i = t; i < cnt; i += kT) g.lm_sorted[n0 + i] = n0 + i;
            continue;
        }
        // rank counting over LDS tiles of ids; ranks accumulate in lm_hidx (free until the structure phase)
        for (int i = t; i < cnt; i += kT) g.lm_hidx[n0 + i] = 0;
        constexpr int kTile = kDyn / 4;
        for (int b0 = 0; b0 < cnt; b0 += kTile) {
            const int nt = min(kTile, cnt - b0);
            __syncthreads();
            for (int j = t; j < nt; j += kT) dyn_i[j] = id_of(b0 + j);
            __syncthreads();
            for (int i = t; i < cnt; i += kT) {
                const int id = id_of(i);
                int r = 0;
                for (int j = 0; j < nt; j++) {
                    const int v = dyn_i[j];
                    r += v < id || (v == id && b0 + j < i);
                }
                g.lm_hidx[n0 + i] += r;
            }
        }
        __syncthreads();
        for (int i = t; i < cnt; i += kT) g.lm_sorted[n0 + g.lm_hidx[n0 + i]] = n0 + i;
        __syncthreads();
    }
    __syncthreads();
}

// ---------------------------------------------------------------- AMD (one lane)
// Eigen::internal::minimum_degree_ordering (oracle/eigen_simplicial_restated.h), workspace Ci (t ints, the full
// symmetric pattern in its first Cp[n] entries), W (8 (n + 1) ints), perm (n + 1 ints; perm[k] = k-th pivot).
__device__ int amd_flip(int i) { return -i - 2; }
__device__ int amd_wclear(int mark, int lemax, int* w, int n) {
    if (mark < 2 || (mark + lemax < 0)) {
        for (int k = 0; k < n; k++)
            if (w[k] != 0) w[k] = 1;
        mark = 2;
    }
    return mark;
}
__device__ __noinline__ void amd_order(int n, int* Cp, int* Ci, int t, int* W, int* perm) {
    int d, dk, dext, lemax = 0, e, elenk, eln, i, j, k, k1, k2, k3, jlast, ln, dense, nzmax, mindeg = 0, nvi, nvj,
                     nvk, mark, wnvi, ok, nel = 0, p, p1, p2, p3, p4, pj, pk, pk1, pk2, pn, q, h;
    dense = max(16, (int)(10 * sqrt((double)n)));
    dense = min(n - 2, dense);
    int cnz = Cp[n];
    int* len = W;
    int* nv = W + (n + 1);
    int* next = W + 2 * (n + 1);
    int* head = W + 3 * (n + 1);
    int* elen = W + 4 * (n + 1);
    int* degree = W + 5 * (n + 1);
    int* w = W + 6 * (n + 1);
    int* hhead = W + 7 * (n + 1);
    int* last = perm;
    for (k = 0; k < n; k++) len[k] = Cp[k + 1] - Cp[k];
    len[n] = 0;
    nzmax = t;
    for (i = 0; i <= n; i++) {
        head[i] = -1; last[i] = -1; next[i] = -1; hhead[i] = -1;
        nv[i] = 1; w[i] = 1; elen[i] = 0; degree[i] = len[i];
    }
    mark = amd_wclear(0, 0, w, n);
    for (i = 0; i < n; i++) {  // every column holds its diagonal (the pose's own block)
        d = degree[i];
        if (d == 1) {
            elen[i] = -2; nel++; Cp[i] = -1; w[i] = 0;
        } else if (d > dense) {
            nv[i] = 0; elen[i] = -1; nel++; Cp[i] = amd_flip(n); nv[n]++;
        } else {
            if (head[d] != -1) last[head[d]] = i;
            next[i] = head[d];
            head[d] = i;
        }
    }
    elen[n] = -2; Cp[n] = -1; w[n] = 0;
    while (nel < n) {
        for (k = -1; mindeg < n && (k = head[mindeg]) == -1; mindeg++) {
        }
        if (next[k] != -1) last[next[k]] = -1;
        head[mindeg] = next[k];
        elenk = elen[k];
        nvk = nv[k];
        nel += nvk;
        if (elenk > 0 && cnz + mindeg >= nzmax) {
            for (j = 0; j < n; j++)
                if ((p = Cp[j]) >= 0) { Cp[j] = Ci[p]; Ci[p] = amd_flip(j); }
            for (q = 0, p = 0; p < cnz;) {
                if ((j = amd_flip(Ci[p++])) >= 0) {
                    Ci[q] = Cp[j];
                    Cp[j] = q++;
                    for (k3 = 0; k3 < len[j] - 1; k3++) Ci[q++] = Ci[p++];
                }
            }
            cnz = q;
        }
        dk = 0;
        nv[k] = -nvk;
        p = Cp[k];
        pk1 = (elenk == 0) ? p : cnz;
        pk2 = pk1;
        for (k1 = 1; k1 <= elenk + 1; k1++) {
            if (k1 > elenk) { e = k; pj = p; ln = len[k] - elenk; }
            else { e = Ci[p++]; pj = Cp[e]; ln = len[e]; }
            for (k2 = 1; k2 <= ln; k2++) {
                i = Ci[pj++];
                if ((nvi = nv[i]) <= 0) continue;
                dk += nvi;
                nv[i] = -nvi;
                Ci[pk2++] = i;
                if (next[i] != -1) last[next[i]] = last[i];
                if (last[i] != -1) next[last[i]] = next[i];
                else head[degree[i]] = next[i];
            }
            if (e != k) { Cp[e] = amd_flip(k); w[e] = 0; }
        }
        if (elenk != 0) cnz = pk2;
        degree[k] = dk;
        Cp[k] = pk1;
        len[k] = pk2 - pk1;
        elen[k] = -2;
        mark = amd_wclear(mark, lemax, w, n);
        for (pk = pk1; pk < pk2; pk++) {
            i = Ci[pk];
            if ((eln = elen[i]) <= 0) continue;
            nvi = -nv[i];
            wnvi = mark - nvi;
            for (p = Cp[i]; p <= Cp[i] + eln - 1; p++) {
                e = Ci[p];
                if (w[e] >= mark) w[e] -= nvi;
                else if (w[e] != 0) w[e] = degree[e] + wnvi;
            }
        }
        for (pk = pk1; pk < pk2; pk++) {
            i = Ci[pk];
            p1 = Cp[i];
            p2 = p1 + elen[i] - 1;
            pn = p1;
            for (h = 0, d = 0, p = p1; p <= p2; p++) {
                e = Ci[p];
                if (w[e] != 0) {
                    dext = w[e] - mark;
                    if (dext > 0) { d += dext; Ci[pn++] = e; h += e; }
                    else { Cp[e] = amd_flip(k); w[e] = 0; }
                }
            }
            elen[i] = pn - p1 + 1;
            p3 = pn;
            p4 = p1 + len[i];
            for (p = p2 + 1; p < p4; p++) {
                j = Ci[p];
                if ((nvj = nv[j]) <= 0) continue;
                d += nvj;
                Ci[pn++] = j;
                h += j;
            }
            if (d == 0) {
                Cp[i] = amd_flip(k);
                nvi = -nv[i];
                dk -= nvi; nvk += nvi; nel += nvi;
                nv[i] = 0; elen[i] = -1;
            } else {
                degree[i] = min(degree[i], d);
                Ci[pn] = Ci[p3];
                Ci[p3] = Ci[p1];
                Ci[p1] = k;
                len[i] = pn - p1 + 1;
                h %= n;
                next[i] = hhead[h];
                hhead[h] = i;
                last[i] = h;
            }
        }
        degree[k] = dk;
        lemax = max(lemax, dk);
        mark = amd_wclear(mark + lemax, lemax, w, n);
        for (pk = pk1; pk < pk2; pk++) {
            i = Ci[pk];
            if (nv[i] >= 0) continue;
            h = last[i];
            i = hhead[h];
            hhead[h] = -1;
            for (; i != -1 && next[i] != -1; i = next[i], mark++) {
                ln = len[i];
                eln = elen[i];
                for (p = Cp[i] + 1; p <= Cp[i] + ln - 1; p++) w[Ci[p]] = mark;
                jlast = i;
                for (j = next[i]; j != -1;) {
                    ok = (len[j] == ln) && (elen[j] == eln);
                    for (p = Cp[j] + 1; ok && p <= Cp[j] + ln - 1; p++)
                        if (w[Ci[p]] != mark) ok = 0;
                    if (ok) {
                        Cp[j] = amd_flip(i);
                        nv[i] += nv[j];
                        nv[j] = 0;
                        elen[j] = -1;
                        j = next[j];
                        next[jlast] = j;
                    } else {
                        jlast = j;
                        j = next[j];
                    }
                }
            }
        }
        for (p = pk1, pk = pk1; pk < pk2; pk++) {
            i = Ci[pk];
            if ((nvi = -nv[i]) <= 0) continue;
            nv[i] = nvi;
            d = degree[i] + dk - nvi;
            d = min(d, n - nel - nvi);
            if (head[d] != -1) last[head[d]] = i;
            next[i] = head[d];
            last[i] = -1;
            head[d] = i;
            mindeg = min(mindeg, d);
            degree[i] = d;
            Ci[p++] = i;
        }
        nv[k] = nvk;
        if ((len[k] = p - pk1) == 0) { Cp[k] = -1; w[k] = 0; }
        if (elenk != 0) cnz = p;
    }
    for (i = 0; i < n; i++) Cp[i] = amd_flip(Cp[i]);
    for (j = 0; j <= n; j++) head[j] = -1;
    for (j = n; j >= 0; j--) {
        if (nv[j] > 0) continue;
        next[j] = head[Cp[j]];
        head[Cp[j]] = j;
    }
    for (e = n; e >= 0; e--) {
        if (nv[e] <= 0) continue;
        if (Cp[e] != -1) { next[e] = head[Cp[e]]; head[Cp[e]] = e; }
    }
    int* stack = w;
    for (k = 0, i = 0; i <= n; i++) {
        if (Cp[i] != -1) continue;
        int top = 0;
        stack[0] = i;
        while (top >= 0) {
            const int pp = stack[top];
            const int ii = head[pp];
            if (ii == -1) { top--; perm[k++] = pp; }
            else { head[pp] = next[ii]; stack[++top] = ii; }
        }
    }
}

__device__ __forceinline__ bool coupled(const Sh& s, int q1, int q2) {  // pose blocks (q1, q2) in the Schur pattern
    return q1 <= q2 ? pm_test(s.pat[q1], q2) : pm_test(s.pat[q2], q1);
}
template <class PU>
__device__ __forceinline__ bool bit_of(const PU* bits, int i) { return (bits[i >> 6] >> (i & 63)) & 1ull; }

// ---------------------------------------------------------------- the members' shares (leader, per pass)
// Published in the team record with the structure state the members copy (load_team):
//  * the Schur complement by block rows: every pattern block's chain length (the landmarks whose active edges see
//    both of its poses), the rows (pose i1 with its blocks (i1, i2 >= i1)) dealt to the members by work, largest
//    first to the least loaded (LPT), each member's blocks longest first in g.bord[bo[m] .. bo[m + 1]) -- a member
//    then forms BDinv only for its own rows (schur());
//  * buildSystem: the landmarks in list order -- their edges are one contiguous range -- cut into T runs of about
//    equal work (a plane edge weighs kPlaneW point edges: the Jacobians of its landmark side and of its pose side are
//    read back from the numeric-differentiation pass), and the free poses dealt by edge count, largest first,
//    snaking (build_system()).
constexpr int kPlaneW = 4;
__device__ __forceinline__ int snake_pick(int j, int m, int T) { return j * T + ((j & 1) ? T - 1 - m : m); }
__device__ __noinline__ void team_plan() {
    const G& g = lbg_g;
    Sh& s = lbg_s;
    const int t = threadIdx.x;
    const int np = s.np, nl = s.nl, T = s.T;
    LbgTeam GL* R = g.team;
    int* len = (int*)lbg_dyn;                        // [nb]
    int* brow = len + kMaxK * (kMaxK + 1) / 2;       // [nb] block -> its row i1
    int* rowoff = brow + kMaxK * (kMaxK + 1) / 2;    // [np]
    int* prank = rowoff + kMaxK;                     // [np] free poses by edge count
    int* rw = prank + kMaxK;                         // [np] row work
    int* rmem = rw + kMaxK;                          // [np] row -> member
    if (t == 0) {  // block ids: (i, i) -> i; (i1 < i2) -> rowoff[i1] + rank of i2 among row i1's bits above i1
        int o = np;
        for (int a = 0; a < np; a++) {
            rowoff[a] = o;
            o += pm_popc(s.pat[a]) - 1;
        }
        s.nb = o;
    }
    __syncthreads();
    const int nb = s.nb;
    for (int i = t; i < nb; i += kT) len[i] = 0;
    if (t < np) {
        brow[t] = t;
        for (int j = rowoff[t]; j < rowoff[t] + pm_popc(s.pat[t]) - 1; j++) brow[j] = t;
    }
    __syncthreads();
    for (int h = t; h < nl; h += kT) {
        PMask a = pm_ld(g.lmh_mask + h);
        while (pm_any(a)) {
            const int i1 = pm_ffs(a);
            pm_pop(a);
            atomicAdd(&len[i1], 1);
            const PMask row = pm_andnot(s.pat[i1], pm_bit(i1));
            PMask b2 = a;
            while (pm_any(b2)) {
                const int i2 = pm_ffs(b2);
                pm_pop(b2);
                atomicAdd(&len[rowoff[i1] + pm_popc_below(row, i2)], 1);
            }
        }
    }
    if (t < np) {
        const int c = g.pe_off[t + 1] - g.pe_off[t];
        int r = 0;
        for (int q = 0; q < np; q++) {
            const int v = g.pe_off[q + 1] - g.pe_off[q];
            r += v > c || (v == c && q < t);
        }
        prank[r] = t;
    }
    __syncthreads();
    if (t < np) {  // a row's work: its blocks' chains (+1 each: the block's own cost)
        int w = len[t] + 1;
        for (int j = rowoff[t]; j < rowoff[t] + pm_popc(s.pat[t]) - 1; j++) w += len[j] + 1;
        rw[t] = w;
    }
    __syncthreads();
    if (t == 0) {  // LPT: rows by work, each to the least loaded member
        long long load[kLbgTeamMax];
        PMask rm[kLbgTeamMax];
        for (int mm = 0; mm < T; mm++) { load[mm] = 0; rm[mm] = pm_zero(); }
        PMask done = pm_zero();
        for (int q = 0; q < np; q++) {
            int best = -1;
            for (int a = 0; a < np; a++)
                if (!pm_test(done, a) && (best < 0 || rw[a] > rw[best])) best = a;
            pm_set(done, best);
            int mm = 0;
            for (int u = 1; u < T; u++)
                if (load[u] < load[mm]) mm = u;
            load[mm] += rw[best];
            pm_set(rm[mm], best);
            rmem[best] = mm;
        }
        int o = 0;
        for (int mm = 0; mm < T; mm++) {  // blocks per member -> the members' segments of bord
            R->bo[mm] = o;
            for (int k = 0; k < kPW; k++) R->rmask[mm * kPW + k] = rm[mm].w[k];
            for (int a = 0; a < np; a++)
                if (pm_test(rm[mm], a)) o += pm_popc(s.pat[a]);
        }
        R->bo[T] = o;
    }
    __syncthreads();
    for (int i = t; i < nb; i += kT) {  // each member's blocks longest first (ties: block id)
        const int w = len[i], mi = rmem[brow[i]];
        int r = 0;
        for (int j = 0; j < nb; j++) {
            const int v = len[j];
            r += rmem[brow[j]] == mi && (v > w || (v == w && j < i));
        }
        g.bord[R->bo[mi] + r] = i;
    }
    // landmark runs: exclusive prefix of the edge weights in list order; run m ends after the landmark whose weight
    // interval holds W m / T
    int Wt = 0;
    {
        int tot = 0;
        for (int ch = 0; ch < g.L; ch += kT) {
            int tt;
            block_scan(ch + t < g.L ? g.lm_nb[ch + t] * (ch + t < g.Np ? 1 : kPlaneW) : 0, &tt, s);
            tot += tt;
        }
        Wt = tot;
    }
    if (t <= T) R->eb[t] = t == 0 ? 0 : g.E;
    __syncthreads();
    {
        int base = 0;
        for (int ch = 0; ch < g.L; ch += kT) {
            const int l = ch + t;
            const int w = l < g.L ? g.lm_nb[l] * (l < g.Np ? 1 : kPlaneW) : 0;
            int tt;
            const int ex = block_scan(w, &tt, s) + base;
            for (int mm = 1; mm < T; mm++) {
                const long long tgt = ((long long)Wt * mm) / T;
                if (w > 0 && ex < tgt && tgt <= ex + w) R->eb[mm] = g.lm_boff[l] + g.lm_nb[l];
            }
            base += tt;
        }
    }
    if (t == 0) {
        int o = 0;
        for (int mm = 0; mm < T; mm++) {
            R->npo[mm] = o;
            for (int j = 0; j * T < np; j++) {
                const int r = snake_pick(j, mm, T);
                if (r < np) R->pown[o++] = prank[r];
            }
        }
        R->npo[T] = o;
        R->np = np; R->nl = nl; R->nact = s.nact; R->nch = s.nch; R->nb = nb; R->unsup = 0;
    }
    if (t < kMaxK)
        for (int k = 0; k < kPW; k++) R->pat[t * kPW + k] = t < np ? s.pat[t].w[k] : 0ull;
    for (int k = t; k < g.K; k += kT) R->hidx[k] = s.hidx[k];
    __syncthreads();
}

// every member (after the team_sync that follows the leader's structure pass): the shared structure state into LDS,
// and this member's shares
__device__ __noinline__ void load_team() {
    const G& g = lbg_g;
    Sh& s = lbg_s;
    const int t = threadIdx.x;
    const LbgTeam GL* R = g.team;
    if (s.m != 0) {
        if (t == 0) {
            s.unsup = R->unsup;
            s.np = R->np; s.nl = R->nl; s.nact = R->nact; s.nch = R->nch; s.nb = R->nb;
        }
        for (int k = t; k < g.K; k += kT) s.hidx[k] = R->hidx[k];
        if (t < kMaxK)
            for (int k = 0; k < kPW; k++) s.pat[t].w[k] = R->pat[t * kPW + k];
    }
    const int o0 = R->npo[s.m], o1 = R->npo[s.m + 1];
    if (t == 0) {
        s.eb0 = R->eb[s.m];
        s.eb1 = R->eb[s.m + 1];
        s.npown = o1 - o0;
        s.bo0 = R->bo[s.m];
        s.bo1 = R->bo[s.m + 1];
        for (int k = 0; k < kPW; k++) s.rmask.w[k] = R->rmask[s.m * kPW + k];
    }
    if (t < o1 - o0) s.pown[t] = R->pown[o0 + t];
    __syncthreads();
}

// ---------------------------------------------------------------- structure (per optimize() pass)
// initializeOptimization(0) + buildStructure + LinearSolverEigen's symbolic analysis
__device__ __noinline__ void structure() {
    const G& g = lbg_g;
    Sh& s = lbg_s;
    unsigned char* dyn = lbg_dyn;
    const int t = threadIdx.x, lane = t & 63;
    for (int k = t; k < g.K; k += kT) {
        s.kact[k] = 0;
        s.hidx[k] = -1;
    }
    __syncthreads();
    int na = 0;
    for (int e = t; e < g.E; e += kT)
        if (g.e_level[e] == 0) {
            s.kact[g.e_kf[e]] = 1;  // (every writer stores the same value)
            na++;
        }
    int nact;
    block_scan(na, &nact, s);
    if (t == 0) s.nact = nact;
    __syncthreads();
    if (t == 0) {  // free poses with an active edge, by id (buildIndexMapping over the id-sorted active vertices)
        int np = 0;
        for (int k = 0; k < g.K; k++) {
            const auto& kk = g.kf[k];
            if (!s.kact[k] || kk.fixed || kk.id == 0) continue;
            if (np == kMaxK) { np++; break; }  // more free poses than the pose masks hold: status -2
            int j = np++;
            while (j > 0 && g.kf[s.hpose[j - 1]].id > kk.id) { s.hpose[j] = s.hpose[j - 1]; j--; }
            s.hpose[j] = k;
        }
        s.unsup = np > kMaxK;
        s.dense = 0;
        if (!s.unsup)
            for (int j = 0; j < np; j++) s.hidx[s.hpose[j]] = (short)j;
        s.np = s.unsup ? 0 : np;
    }
    __syncthreads();
    if (s.unsup) return;
    const int np = s.np;
    // landmarks with an active edge in id order; pose masks of their active edges (the Hpl blocks) and of all
    // their edges (buildStructure's Schur pattern walks v->edges(), any level)
    int base = 0;
    for (int ch = 0; ch < g.L; ch += kT) {
        const int j = ch + t;
        const int l = j < g.L ? g.lm_sorted[j] : -1;
        int act = 0;
        PMask mask = pm_zero(), amask = pm_zero();
        if (l >= 0)
            for (int e = g.lm_boff[l]; e < g.lm_boff[l] + g.lm_nb[l]; e++) {
                const int h = s.hidx[g.e_kf[e]];
                if (h >= 0) pm_set(amask, h);
                if (g.e_level[e] == 0) {
                    act = 1;
                    if (h >= 0) pm_set(mask, h);
                }
            }
        int tot;
        const int off = block_scan(act, &tot, s) + base;
        if (l >= 0) {
            g.lm_hidx[l] = act ? off : -1;
            pm_st(g.lm_amask + l, amask);
            if (act) {
                g.hidx_lm[off] = l;
                pm_st(g.lmh_mask + off, mask);
            }
        }
        base += tot;
    }
    const int nl = base;
    if (t == 0) s.nl = nl;
    // Hpl blocks of landmark h at lmh_blk[h] .. (pose order), contiguous in landmark order
    base = 0;
    for (int ch = 0; ch < nl; ch += kT) {
        const int h = ch + t;
        const int c = h < nl ? pm_popc(pm_ld(g.lmh_mask + h)) : 0;
        int tot;
        const int off = block_scan(c, &tot, s) + base;
        if (h < nl) g.lmh_blk[h] = off;
        base += tot;
    }
    if (t == 0) g.lmh_blk[nl] = base;
    __syncthreads();
    // the Schur phase's landmark chunks: groups of kSchurLm landmarks, split greedily where a group's Hpl blocks
    // exceed kSchurBlk (a landmark has at most 64 blocks); sch[c] = first landmark of chunk c, sch_kb its first block
    {
        int nc = 0;
        const int ng = (nl + kSchurLm - 1) / kSchurLm;
        for (int pass2 = 0; pass2 < 2; pass2++) {
            int base2 = 0;
            for (int ch = 0; ch < ng; ch += kT) {
                const int gi = ch + t;
                int cntc = 0;
                if (gi < ng) {
                    const int h0 = gi * kSchurLm, h1 = min(nl, h0 + kSchurLm);
                    int k0 = g.lmh_blk[h0];
                    cntc = 1;
                    for (int h = h0 + 1; h < h1; h++) {
                        const int kh = g.lmh_blk[h + 1];
                        if (kh - k0 > kSchurBlk) { k0 = g.lmh_blk[h]; cntc++; }
                    }
                }
                int tot;
                const int off = block_scan(cntc, &tot, s) + base2;
                if (pass2 == 1 && gi < ng) {
                    const int h0 = gi * kSchurLm, h1 = min(nl, h0 + kSchurLm);
                    int k0 = g.lmh_blk[h0], o = off;
                    g.sch[o] = h0;
                    g.sch_kb[o++] = k0;
                    for (int h = h0 + 1; h < h1; h++) {
                        const int kh = g.lmh_blk[h + 1];
                        if (kh - k0 > kSchurBlk) { k0 = g.lmh_blk[h]; g.sch[o] = h; g.sch_kb[o++] = k0; }
                    }
                }
                base2 += tot;
            }
            nc = base2;
        }
        if (t == 0) {
            g.sch[nc] = nl;
            g.sch_kb[nc] = g.lmh_blk[nl];
            s.nch = nc;
        }
    }
    if (t < np) s.pat[t] = pm_bit(t);
    __syncthreads();
    for (int l = t; l < g.L; l += kT) {
        const int h = g.lm_hidx[l];
        const PMask mask = h >= 0 ? pm_ld(g.lmh_mask + h) : pm_zero();
        const int b0 = g.lm_boff[l], e1 = b0 + g.lm_nb[l], kb = h >= 0 ? g.lmh_blk[h] : 0;
        for (int e = b0; e < e1; e++) {
            int eb = -1;
            const int ph = s.hidx[g.e_kf[e]];
            const bool on = g.e_level[e] == 0;
            if (h >= 0 && on && ph >= 0) eb = kb + pm_popc_below(mask, ph);
            g.e_blk[e] = eb;
            // build_system's row record: RI (the edge's Hpl block, -1 none, -2 inactive), the landmark's segment
            g.eseg[4 * e] = on ? eb : -2;
            g.eseg[4 * e + 1] = h;
            g.eseg[4 * e + 2] = e1;
            g.eseg[4 * e + 3] = kb | (e == b0 ? 1 << 30 : 0);
        }
        if (h >= 0) {
            const PMask am0 = pm_ld(g.lm_amask + l);
            PMask am = am0;
            while (pm_any(am)) {
                const int i1 = pm_ffs(am);
                const PMask row = pm_andnot(am0, pm_below(i1));
                for (int k = 0; k < kPW; k++)
                    if (row.w[k]) atomicOr((unsigned long long*)&s.pat[i1].w[k], (unsigned long long)row.w[k]);
                pm_pop(am);
            }
        }
    }
    // per free pose, its active edges in insertion order: a stable bucketing in one pass over the edges (round 5 ran
    // a block scan over all edges per pose: np x E / 512 scans).  Counts per pose, their prefix = pe_off; then per
    // chunk of kT edges each edge's rank among the chunk's earlier edges of its pose -- within its wave from the
    // lanes that share the pose (one ballot per distinct pose of the wave), across waves from the per-wave counts
    // taken in wave order -- after the edges of earlier chunks (run).
    {
        int* cnt = (int*)dyn;          // [kW][kMaxK] this chunk's per-wave counts
        int* run = cnt + kW * kMaxK;   // [kMaxK] edges placed so far, then (first) the totals
        const int wv = t >> 6;
        auto pose_of = [&](int e) { return e < g.E && g.e_level[e] == 0 ? (int)s.hidx[g.e_kf[e]] : -1; };
        for (int k = t; k < kMaxK; k += kT) run[k] = 0;
        __syncthreads();
        for (int e = t; e < g.E; e += kT) {
            const int h = pose_of(e);
            if (h >= 0) atomicAdd(&run[h], 1);
        }
        __syncthreads();
        if (t == 0) {
            int o = 0;
            for (int hh = 0; hh < np; hh++) {
                g.pe_off[hh] = o;
                o += run[hh];
            }
            g.pe_off[np] = o;
        }
        __syncthreads();
        for (int k = t; k < kMaxK; k += kT) run[k] = 0;
        for (int ch = 0; ch < g.E; ch += kT) {
            for (int k = t; k < kW * kMaxK; k += kT) cnt[k] = 0;
            __syncthreads();
            const int e = ch + t, h = pose_of(e);
            int rank = 0;
            uint64_t rem = __ballot(h >= 0);
            while (rem) {
                const int hq = __builtin_amdgcn_readlane(h, __builtin_ctzll(rem));
                const uint64_t m = __ballot(h == hq);
                if (h == hq) rank = __popcll(m & (lane == 0 ? 0ull : ~0ull >> (64 - lane)));
                if (lane == 0) cnt[wv * kMaxK + hq] = __popcll(m);
                rem &= ~m;
            }
            __syncthreads();
            if (h >= 0) {
                int base = g.pe_off[h] + run[h] + rank;
                for (int w = 0; w < wv; w++) base += cnt[w * kMaxK + h];
                g.pe_idx[base] = e;
            }
            __syncthreads();
            for (int k = t; k < np; k += kT) {
                int a = 0;
                for (int w = 0; w < kW; w++) a += cnt[w * kMaxK + k];
                run[k] += a;
            }
            __syncthreads();  // (the next chunk clears cnt)
        }
    }
    team_plan();
    // ---- LinearSolverEigen::computeSymbolicDecomposition (analyzePattern, Eigen's AMD)
    const int n = 6 * np;
    if (n == 0) {
        if (t == 0) g.rs_off[0] = 0;
        __syncthreads();
        return;
    }
    if (t < np) {
        int c = 0;
        for (int q = 0; q < np; q++) c += coupled(s, t, q);
        s.pdeg[t] = c;
    }
    __syncthreads();
    const int dense = min(n - 2, max(16, (int)(10 * sqrt((double)n))));
    int alld = 1;
    for (int q = t; q < np; q += kT) alld &= 6 * s.pdeg[q] > dense;
    int full = 1;  // every pose coupled with every other
    for (int q = t; q < np; q += kT) full &= pm_eq(s.pat[q], pm_andnot(pm_first_n(np), pm_below(q)));
    full = block_and(full, s);
    if (block_and(alld, s)) {
        if (t == 0) s.dense = full;
        for (int k = t; k < n; k += kT) g.Pinv[k] = k;  // every scalar dense: absorbed in index order (natural)
    } else {
        // full symmetric pattern (diagonal kept), columns sorted; cs_amd's elbow room
        int cnz = 0;
        for (int q = 0; q < np; q++) cnz += 36 * s.pdeg[q];
        const int tcap = cnz + cnz / 5 + 2 * n;
        const bool in_lds = (size_t)(tcap + 10 * (n + 1)) * 4 <= (size_t)kDyn;
        int* Ci = in_lds ? (int*)dyn : (int*)g.amd_Ci;
        int* W = in_lds ? Ci + tcap : (int*)g.amd_W;
        int* perm = W + 8 * (n + 1);
        int* Cp = perm + (n + 1);
        for (int tt = t; tt < n; tt += kT) {
            const int q2 = tt / 6;
            int c0 = 0;
            for (int q = 0; q < q2; q++) c0 += 6 * s.pdeg[q];
            c0 *= 6;
            c0 += (tt - 6 * q2) * 6 * s.pdeg[q2];
            Cp[tt] = c0;
            int c = c0;
            for (int q = 0; q < np; q++)
                if (coupled(s, q, q2))
                    for (int rr = 0; rr < 6; rr++) Ci[c++] = 6 * q + rr;
        }
        if (t == 0) Cp[n] = cnz;
        __syncthreads();
        if (t == 0) amd_order(n, Cp, Ci, tcap, W, perm);
        __syncthreads();
        for (int k = t; k < n; k += kT) g.Pinv[k] = perm[k];
        __syncthreads();
    }
    for (int k = t; k < n; k += kT) g.Pm[g.Pinv[k]] = k;
    __syncthreads();
    // lower structure of each column j of ap = P a P^T: Abits[j] = {i > j : (Pinv j, Pinv i) in the pattern}
    for (int tt = t; tt < n; tt += kT) {
        const int qj = g.Pinv[tt] / 6;
        uint64_t wv[kNW] = {};
        for (int i = tt + 1; i < n; i++)
            if (coupled(s, qj, g.Pinv[i] / 6)) wv[i >> 6] |= 1ull << (i & 63);
#pragma unroll
        for (int w = 0; w < kNW; w++) g.Abits[tt * kNW + w] = wv[w];
    }
    __syncthreads();
    // elimination tree and L's column structures: struct L(:, j) = Abits[j] U (children's structures \ {j});
    // one lane per bitset word
    if (t < 64) {
        uint64_t* acc = (uint64_t*)dyn;  // n x kNW
        for (int i = lane; i < n * kNW; i += 64) acc[i] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int j = 0; j < n; j++) {
            uint64_t S = 0;
            if (lane < kNW) S = g.Abits[j * kNW + lane] | acc[j * kNW + lane];
            const uint64_t nz = __ballot(lane < kNW && S != 0);
            int par = -1;
            if (nz) {
                const int fw = __ffsll((unsigned long long)nz) - 1;
                const uint64_t wv = rl64(S, fw);
                par = 64 * fw + __ffsll((unsigned long long)wv) - 1;
            }
            if (lane < kNW) {
                g.Lbits[j * kNW + lane] = S;
                if (par >= 0) {
                    const uint64_t keep = (par >> 6) == lane ? ~(1ull << (par & 63)) : ~0ull;
                    acc[par * kNW + lane] |= S & keep;
                }
            }
            if (lane == 0) g.parent[j] = par;  // (each lane reads and writes its own word of acc only)
        }
        // the factorisation's masked-step structure words (a ring step past a piece's end reads row n's kC words:
        // all of them zero, not only the first -- the rest would be whatever an earlier call left in the scratch)
        if (lane < kNW) g.Lbits[n * kNW + lane] = 0;
    }
    __syncthreads();
    // each row k of L: its pattern {i : k in struct L(:, i)} in factorize_preordered's order -- ap's column k
    // entries in source order (original index ascending), an elimination-tree walk from each, the walks' paths
    // stacked so that the last path comes first, each path from its start upwards
    int rs_base = 0;
    for (int k0 = 0; k0 < n; k0 += kT) {  // rows k0 .. k0 + kT - 1 (one pass for n <= kT)
        const int k = k0 + t;
        int cnt = 0;
        if (k < n)
            for (int i = 0; i < k; i++) cnt += bit_of(g.Lbits + i * kNW, k);
        int tot;
        const int off = block_scan(cnt, &tot, s) + rs_base;
        rs_base += tot;
        if (k < n) g.rs_off[k] = off;
        if (k0 + kT >= n && t == 0) g.rs_off[n] = rs_base;
        if (k < n && cnt > 0) {
            const int ok = g.Pinv[k];
            uint64_t vis[kNW] = {};
            vis[k >> 6] |= 1ull << (k & 63);
            auto seg = g.rs_idx + off;
            int wpos = 0;
            for (int o2 = 0; o2 < n; o2++) {
                const int r = g.Pm[o2];
                if (r >= k || !coupled(s, o2 / 6, ok / 6)) continue;
                int i = r;
                while (!((vis[i >> 6] >> (i & 63)) & 1ull)) {
                    vis[i >> 6] |= 1ull << (i & 63);
                    seg[wpos++] = i;
                    i = g.parent[i];
                }
            }
            // paths were written in discovery order: reverse the whole row, then each path back to start-upwards
            for (int a = 0, b2 = cnt - 1; a < b2; a++, b2--) {
                const int v = seg[a];
                seg[a] = seg[b2];
                seg[b2] = v;
            }
            int a = 0;
            while (a < cnt) {  // a reversed path: consecutive entries (prev, next) with parent[next] == prev
                int b2 = a;
                while (b2 + 1 < cnt && g.parent[seg[b2 + 1]] == seg[b2]) b2++;
                for (int x = a, y = b2; x < y; x++, y--) {
                    const int v = seg[x];
                    seg[x] = seg[y];
                    seg[y] = v;
                }
                a = b2 + 1;
            }
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------- errors + robust chi2
// computeActiveErrors: err of every active edge, its robust chi2 (activeRobustChi2's terms) in echi (+0.0 for
// inactive edges: an exact no-op in the ordered sum)
__device__ __noinline__ void errors() {
    const LbaConsts& C = lbg_c;
    const G& g = lbg_g;
    const Sh& s = lbg_s;
    const int t = threadIdx.x;
    const bool robust = s.robust;
    // this member's share: point edges [p0, p1), plane edges [Ep + q0, Ep + q1)
    const int p0 = split_lo(g.Ep, s.m, s.T), p1 = split_lo(g.Ep, s.m + 1, s.T);
    const int npl = g.E - g.Ep, q0 = split_lo(npl, s.m, s.T), q1 = split_lo(npl, s.m + 1, s.T);
    // point edges, kEU per thread at a time: every edge's records, then every edge's operands, are loaded before
    // any is evaluated (a dependent load chain per group instead of per edge)
    constexpr int kEU = 3;
    for (int e0 = p0 + t; e0 < p1; e0 += kEU * kT) {
        int lv[kEU], ty[kEU], kf[kEU], lm[kEU], src[kEU];
#pragma unroll
        for (int u = 0; u < kEU; u++) {
            const int e = e0 + u * kT, ec = e < p1 ? e : e0;
            lv[u] = e < p1 ? g.e_level[ec] : 1;
            ty[u] = g.e_type[ec];
            kf[u] = g.e_kf[ec];
            lm[u] = g.e_lm[ec];
            src[u] = g.e_src[ec];
        }
        PointIn in[kEU];
#pragma unroll
        for (int u = 0; u < kEU; u++) in[u] = point_in(g, kf[u], lm[u], src[u]);
#pragma unroll
        for (int u = 0; u < kEU; u++) {
            const int e = e0 + u * kT;
            if (e >= p1) break;
            double chi = 0.0;
            if (lv[u] == 0) {
                double err[3];
                point_error_v(ty[u], in[u], err);
                for (int i = 0; i < 3; i++) g.err[3 * e + i] = err[i];
                const double info[3] = {(double)in[u].isg, (double)in[u].isg, (double)in[u].isg};  // info_of, t <= 1
                double r1;
                huber(chi2_of(err, info, edge_dim(ty[u])), delta_of(C, ty[u]), robust, &chi, &r1);
            }
            g.echi[e] = chi;
        }
    }
    // plane edges: one lane pair per edge (plane_error_pair)
    for (int q = q0 + (t >> 1); q < q0 + ((q1 - q0 + kT / 2 - 1) / (kT / 2)) * (kT / 2); q += kT / 2) {
        const int e = g.Ep + q;
        const bool act = q < q1 && g.e_level[e] == 0;
        E3 r{0, 0, 0};
        if (__any(act)) {
            const int ee = act ? e : g.Ep + (q < q1 ? q : q0);
            if (q < q1) {
                const int ty = g.e_type[ee];
                auto pp = g.P + 4 * (g.e_lm[ee] - g.Np);
                r = plane_error_pair(ty - 2, load_pose(g.pose + 7 * g.e_kf[ee]), P4{{pp[0], pp[1], pp[2], pp[3]}},
                                     plane_from_f(g.plobs[g.e_src[ee]].meas), (t & 1) != 0);
            }
        }
        if (q < q1 && (t & 1) == 0) {
            double chi = 0.0;
            if (act) {
                const int ty = g.e_type[e];
                const double err[3] = {r.e0, r.e1, r.e2};
                for (int i = 0; i < 3; i++) g.err[3 * e + i] = err[i];
                double info[3], r1;
                info_of(g, C, e, ty, info);
                huber(chi2_of(err, info, edge_dim(ty)), delta_of(C, ty), robust, &chi, &r1);
            }
            g.echi[e] = chi;
        }
    }
}

// one lane: sum of v[0 .. n32) in index order (n32 a multiple of 32; two 16-load batches in flight)
template <class PD>
__device__ __forceinline__ double ordered_sum(const PD* v, int n32) {
    double acc = 0.0;
    double A[16], B[16];
#pragma unroll
    for (int u = 0; u < 16; u++) A[u] = n32 > 0 ? v[u] : 0.0;
    for (int e = 0; e < n32; e += 32) {
#pragma unroll
        for (int u = 0; u < 16; u++) B[u] = v[e + 16 + u];
#pragma unroll
        for (int u = 0; u < 16; u++) acc += A[u];
        const bool more = e + 32 < n32;
#pragma unroll
        for (int u = 0; u < 16; u++) A[u] = more ? v[e + 32 + u] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; u++) acc += B[u];
    }
    return acc;
}

// the same over LDS, 16-byte reads: 8 loads per batch of 16 values, so the wait for one batch can leave the next
// batch in flight (the LDS counter holds at most 15 outstanding loads; 16 single loads would force a full wait)
__device__ __forceinline__ double ordered_sum_lds(const double* v, int n32, double acc = 0.0) {
    const double2* w = (const double2*)v;
    double2 A[8], B[8];
    const double2 z = make_double2(0.0, 0.0);
#pragma unroll
    for (int u = 0; u < 8; u++) A[u] = n32 > 0 ? w[u] : z;
    for (int e = 0; e < n32; e += 32) {
        const int q = e >> 1;
#pragma unroll
        for (int u = 0; u < 8; u++) B[u] = w[q + 8 + u];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            acc += A[u].x;
            acc += A[u].y;
        }
        const bool more = e + 32 < n32;
#pragma unroll
        for (int u = 0; u < 8; u++) A[u] = more ? w[q + 16 + u] : z;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            acc += B[u].x;
            acc += B[u].y;
        }
    }
    return acc;
}

// the ordered sums of a computeActiveErrors (activeRobustChi2: the edges' chi2 in edge order) and, for a trial
// (nS > 0), of its scale (x . (lambda x + b), entry order): the operands staged in LDS by the whole workgroup
// (coalesced), then one lane per sum -- the dependent add chains read LDS instead of global memory.  nS == 0:
// currentChi, else tempChi and scale.
__device__ __noinline__ void sums_staged(int nE, int nS) {
    const G& g = lbg_g;
    Sh& s = lbg_s;
    const int t = threadIdx.x;
    double* V = (double*)lbg_dyn;
    if ((size_t)(nE + nS) * 8 <= (size_t)kDyn) {
        for (int i = t; i < nE; i += kT) V[i] = g.echi[i];
        for (int i = t; i < nS; i += kT) V[nE + i] = g.sc[i];
        __syncthreads();
        if (t == 0) {
            const double c = ordered_sum_lds(V, nE);
            if (nS > 0) s.tempChi = c; else s.currentChi = c;
        }
        if (t == 64 && nS > 0) s.scale = ordered_sum_lds(V + nE, nS);
    } else {
        // larger graphs: chunks of kHalf values through two LDS buffers, wave 0's lane 0 adding one chunk (the chain
        // carried across chunks: the same sequence of additions) while the other waves stage the next
        constexpr int kHalf = kDyn / 16;
        auto chain = [&](auto src, int n) __attribute__((always_inline)) {
            double acc = 0.0;
            for (int i = t; i < min(kHalf, n); i += kT) V[i] = src[i];
            __syncthreads();
            for (int c = 0; c * kHalf < n; c++) {
                const int b0 = c * kHalf, nb = min(kHalf, n - b0), n0 = b0 + kHalf, nn = max(0, min(kHalf, n - n0));
                double* nxt = V + ((c + 1) & 1) * kHalf;
                if (t == 0) acc = ordered_sum_lds(V + (c & 1) * kHalf, nb, acc);
                else if (t >= 64)
                    for (int i = t - 64; i < nn; i += kT - 64) nxt[i] = src[n0 + i];
                __syncthreads();
            }
            return acc;
        };
        const double c = chain(g.echi, nE);
        if (t == 0) {
            if (nS > 0) s.tempChi = c; else s.currentChi = c;
        }
        if (nS > 0) {
            const double sc = chain(g.sc, nS);
            if (t == 0) s.scale = sc;
        }
    }
}

// ---------------------------------------------------------------- per iteration: quadratic forms and sums
// BlockSolver::buildSystem in chunks of kCh consecutive edges: (A) every edge's quadratic-form terms into LDS rows
// (every edge on two threads of different waves -- both evaluate the Jacobians, one the landmark side, the other the
// pose side; the plane edges' numeric Jacobians from plane_jacobians); (B) the sums, in edge order: each
// landmark's segment in the chunk as (segment, component) chains (continuing the landmark's partial sums when it
// started in an earlier chunk), each (free pose, term) chain by its own lane over the chunk's edges of that pose
// (LDS bitmasks), the chains' accumulators carried in registers from chunk to chunk.
constexpr int kCh = 256;                    // edges per chunk
constexpr int kSL = 13, kSP = 27, kSB = 19;  // LDS row strides (doubles): Hll + bl (12), Hpp + bp (27), Hpl (18)
constexpr int kPoseSlots = (27 * kMaxK + kT - 1) / kT;

struct EdgeW {  // Omega, robust weights and omega_r of one edge
    int dim;
    double W[3], om[3], info[3];
};
__device__ __forceinline__ EdgeW edge_weights(const LbaConsts& C, bool robust, int ty, const double* err, const double* info) {
    EdgeW w;
    w.dim = edge_dim(ty);
    double r0, wgt;
    huber(chi2_of(err, info, w.dim), delta_of(C, ty), robust, &r0, &wgt);
#pragma unroll
    for (int r = 0; r < 3; r++) {
        w.info[r] = info[r];
        w.W[r] = robust ? wgt * info[r] : info[r];
        w.om[r] = -(info[r] * err[r]);
        if (robust) w.om[r] *= wgt;
    }
    return w;
}
// landmark side: Hll 9, bl 3 (L), Hpl 18 (Bk); see edge_terms
__device__ __forceinline__ void terms_land(const EdgeW& w, bool robust, const double (&A)[3][3], const double (&B)[3][6],
                                           bool pfree, double* L, double* Bk) {
    const bool d3 = w.dim == 3;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double s = A[0][i] * w.om[0] + A[1][i] * w.om[1];
        if (d3) s += A[2][i] * w.om[2];
        L[9 + i] = s;
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double h = (A[0][i] * w.W[0]) * A[0][j] + (A[1][i] * w.W[1]) * A[1][j];
            if (d3) h += (A[2][i] * w.W[2]) * A[2][j];
            L[3 * i + j] = h;
        }
    }
    if (!pfree) return;
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double h;
            if (robust) {
                h = (B[0][i] * w.W[0]) * A[0][j] + (B[1][i] * w.W[1]) * A[1][j];
                if (d3) h += (B[2][i] * w.W[2]) * A[2][j];
            } else {
                h = B[0][i] * (A[0][j] * w.info[0]) + B[1][i] * (A[1][j] * w.info[1]);
                if (d3) h += B[2][i] * (A[2][j] * w.info[2]);
            }
            Bk[3 * i + j] = h;
        }
}
// pose side: Hpp upper 21, bp 6
__device__ __forceinline__ void terms_pose(const EdgeW& w, const double (&B)[3][6], double* P) {
    const bool d3 = w.dim == 3;
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = i; j < 6; j++) {
            double h = (B[0][i] * w.W[0]) * B[0][j] + (B[1][i] * w.W[1]) * B[1][j];
            if (d3) h += (B[2][i] * w.W[2]) * B[2][j];
            P[upper_idx(i, j)] = h;
        }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double s = B[0][i] * w.om[0] + B[1][i] * w.om[1];
        if (d3) s += B[2][i] * w.om[2];
        P[21 + i] = s;
    }
}

// plane / parallel / vertical edges: numeric Jacobians (base_binary_edge.hpp:130-205) into g.terms (A 3x3, then
// B 3x6, per edge), kPJ edges at a time: one lane pair per (edge, evaluation q) -- q < 6: plane perturbed by
// +-1e-9 along q >> 1 (Plane3D::oplus); 6 <= q < 18: pose exp(+-1e-9 e_d) * T, d = (q - 6) >> 1 (free poses
// only) -- the errors into LDS, then one thread per Jacobian entry: (e(+) - e(-)) / 2e-9
// Run by the errors phase on the member's plane edges [e_lo, e_hi): the Jacobians at the state whose errors it
// computes -- the linearisation point of the next buildSystem whenever one follows (a rejected trial's are never
// read: the state is popped and the errors recomputed before the next build).
constexpr int kPJ = 128;
__device__ __noinline__ void plane_jacobians(int e_lo, int e_hi) {
    const G& g = lbg_g;
    const Sh& s = lbg_s;
    double* EV = (double*)lbg_dyn;  // [kPJ][18][3]
    const int t = threadIdx.x, pr = t >> 1;
    const bool half = (t & 1) != 0;
    const double delta = 1e-9, scalar = 1.0 / (2 * delta);
    __syncthreads();  // the previous phase's LDS use is over
    for (int e0 = e_lo; e0 < e_hi; e0 += kPJ) {
        const int cnt = min(kPJ, e_hi - e0);
        for (int task = pr; task < cnt * 18; task += kT / 2) {  // (both lanes of a pair: the same task)
            const int le = task / 18, q = task - 18 * le, pe = e0 + le;
            if (g.e_level[pe] != 0) continue;
            const bool pfree = s.hidx[g.e_kf[pe]] >= 0;
            if (q >= 6 && !pfree) continue;
            const int ty = g.e_type[pe], lm = g.e_lm[pe];
            SE3 T = load_pose(g.pose + 7 * g.e_kf[pe]);
            auto pp = g.P + 4 * (lm - g.Np);
            P4 P{{pp[0], pp[1], pp[2], pp[3]}};
            const P4 meas = plane_from_f(g.plobs[g.e_src[pe]].meas);
            const double sgn = (q & 1) ? -delta : delta;
            if (q < 6) {
                double add[3] = {0, 0, 0};
                add[q >> 1] = sgn;
                p_oplus(P, add);
            } else {
                double add[6] = {0, 0, 0, 0, 0, 0};
                add[(q - 6) >> 1] = sgn;
                T = se3_mul(se3_exp(add), T);
            }
            const E3 r = plane_error_pair(ty - 2, T, P, meas, half);
            if (!half) {
                double* o = EV + 3 * (18 * le + q);
                o[0] = r.e0; o[1] = r.e1; o[2] = r.e2;
            }
        }
        __syncthreads();
        for (int i = t; i < cnt * 27; i += kT) {
            const int le = i / 27, j = i - 27 * le, pe = e0 + le;
            if (g.e_level[pe] != 0) continue;
            const int dim = edge_dim(g.e_type[pe]);
            const bool pfree = s.hidx[g.e_kf[pe]] >= 0;
            const double* ev = EV + 54 * le;
            double v;
            if (j < 9) {  // A[ii][d]: the plane's evaluations 2d, 2d + 1
                const int ii = j / 3, d = j - 3 * ii;
                v = ii < dim ? scalar * (ev[3 * (2 * d) + ii] - ev[3 * (2 * d + 1) + ii]) : 0.0;
            } else {      // B[ii][d]: the pose's evaluations 6 + 2d, 7 + 2d
                const int ii = (j - 9) / 6, d = (j - 9) - 6 * ii;
                v = pfree && ii < dim ? scalar * (ev[3 * (6 + 2 * d) + ii] - ev[3 * (7 + 2 * d) + ii]) : 0.0;
            }
            g.terms[27 * (size_t)pe + j] = v;
        }
        __syncthreads();
    }
}

// This member's buildSystem share, in steps of kCh rows per side:
//  * the landmark side of the edges [eb0, eb1) (whole landmarks): every edge's Hll / bl / Hpl terms into LDS rows on
//    threads 0 .. kCh - 1, then (B) each landmark's segment summed in edge order as (segment, component) chains
//    (continuing the landmark's partial sums across steps), each Hpl block stored as 0 + its first term and its
//    later terms added in edge order;
//  * the pose side of this member's free poses: R = kCh / P rows of each pose's active edges (in insertion order,
//    g.pe_idx) per step, their Hpp / bp terms into LDS rows on threads kCh .. 2 kCh - 1, then each (pose, term)
//    chain adds its pose's rows of the step in order (one lane per chain, the accumulators in registers across
//    steps).
// Both sides read the plane edges' Jacobians of the errors phase (plane_jacobians).  The partial sums never leave
// their member before they are complete, so every sum keeps g2o's order (sparse_optimizer.cpp:100-114,
// block_solver.hpp:502-561).  Returns this member's largest |diagonal| of Hll and Hpp (computeLambdaInit) in the team
// record.
__device__ __noinline__ void build_system() {
    const LbaConsts& C = lbg_c;
    const G& g = lbg_g;
    Sh& s = lbg_s;
    unsigned char* dyn = lbg_dyn;
    long long tb0 = wall_clock64(), tA = 0, tB = 0;  // diagnostics
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const bool robust = s.robust;
    const int e0 = s.eb0, e1 = s.eb1, P = s.npown;
    const int R = P > 0 ? kCh / P : kCh;  // rows of each owned pose per step
    double* TL = (double*)dyn;
    double* TP = TL + kCh * kSL;
    double* TB = TP + kCh * kSP;
    int* RI = (int*)(TB + kCh * kSB);  // [kCh] per landmark-side row: its Hpl block, -1 none, -2 inactive edge
    // the step's landmark segments, compacted per wave: (first row, end row, landmark, first block | continuing
    // << 30 | complete << 31); per row the Hpl term's kind (0 none, 1 the block's first term: a plain store, 2 a
    // later term of the same block: an addition)
    int4* SG = (int4*)(RI + kCh);                    // [kCh]
    unsigned char* RF = (unsigned char*)(SG + kCh);  // [kCh]
    int* NSW = (int*)(RF + kCh);                     // [kW] segments per wave, [kW]: any addition rows
    int* PS = NSW + kW + 1;                          // [kMaxK] owned pose a: first entry of its edge list in pe_idx
    int* PC = PS + kMaxK;                            //   and its length
    int* NST = PC + kMaxK;                           // steps
    static_assert((size_t)kCh * (kSL + kSP + kSB) * 8 + kCh * (4 + 16 + 1) + 4 * (kW + 2 + 2 * kMaxK) <= (size_t)kDyn,
                  "LDS");
    if (t < P) {
        const int hh = s.pown[t];
        PS[t] = g.pe_off[hh];
        PC[t] = g.pe_off[hh + 1] - g.pe_off[hh];
    }
    __syncthreads();
    if (t == 0) {
        int ns = (e1 - e0 + kCh - 1) / kCh;
        for (int a = 0; a < P; a++) ns = max(ns, (PC[a] + R - 1) / R);
        *NST = ns;
    }
    double acc[kPoseSlots];
    int task[kPoseSlots];
#pragma unroll
    for (int k = 0; k < kPoseSlots; k++) {
        acc[k] = 0.0;
        task[k] = t + k * kT < 27 * P ? t + k * kT : -1;
    }
    double mx = 0.0;
    // this thread's row: landmark side (t < kCh) row t of the step's landmark chunk, pose side (t >= kCh) row i of
    // owned pose a.  Its records (level, type, keyframe, landmark, observation) and, landmark side, its structure
    // record (eseg) are loaded for the next step during the current step's (B)
    const bool land = t < kCh;
    const int q = t - kCh, pa = land ? 0 : q / R, pi = land ? 0 : q - pa * R;
    const bool prow = !land && pa < P;
    auto edge_of = [&](int st) __attribute__((always_inline)) -> int {  // -1: no row
        if (land) {
            const int e = e0 + st * kCh + t;
            return e < e1 ? e : -1;
        }
        if (!prow) return -1;
        const int i = st * R + pi;
        return i < PC[pa] ? g.pe_idx[PS[pa] + i] : -1;
    };
    int nlv = 1, nty = 0, nkf = 0, nlm = 0, nsrc = 0, ne = -1;
    int4 sgn = make_int4(-2, -1, 0, 0);
    auto edge_rec = [&](int e) __attribute__((always_inline)) {
        ne = e;
        if (e >= 0) {
            nlv = g.e_level[e]; nty = g.e_type[e]; nkf = g.e_kf[e]; nlm = g.e_lm[e]; nsrc = g.e_src[e];
            if (land) sgn = ld_i4(g.eseg + 4 * e);
        } else {
            nlv = 1;
        }
    };
    __syncthreads();
    const int nst = *NST;
    edge_rec(edge_of(0));
#ifdef SPSLAM_LBG_DIAG_BUILD
    long long db1 = 0, db2 = 0, db3 = 0;
#endif
    for (int st = 0; st < nst; st++) {
        const int c0 = e0 + st * kCh;
        const int cnt = max(0, min(kCh, e1 - c0));
        const int4 sg = sgn;
        // (B) landmark segments: the rows' Hpl kinds in edge order (head threads), segments compacted per wave
        bool head = false, again = false;
        int end_row = 0, own_h = -1, own_kb = 0;
        PMask touched = pm_zero();
        if (land && t < cnt) {
            RI[t] = sg.x;
            RF[t] = 0;
            const bool first = (sg.w >> 30) & 1;
            if ((first || t == 0) && sg.y >= 0) {
                head = true;
                own_h = sg.y;
                own_kb = sg.w & ((1 << 30) - 1);
                end_row = min(sg.z, c0 + cnt) - c0;
                touched = first ? pm_zero() : s.carry;  // (only row 0 continues a landmark of the previous step)
            }
        }
        {
            const uint64_t hb = __ballot(head);
            if (head) {
                const int li = __popcll(hb & ((1ull << lane) - 1));
                const unsigned fl = (unsigned)own_kb | ((t == 0 && !((sg.w >> 30) & 1)) ? 1u << 30 : 0u) |
                                    (c0 + end_row == sg.z ? 1u << 31 : 0u);
                SG[64 * wv + li] = make_int4(t, end_row, own_h, (int)fl);
            }
            if (lane == 0 && wv < kCh / 64) NSW[wv] = __popcll(hb);
            if (t == 0) NSW[kW] = 0;
        }
        __syncthreads();
        if (head) {
            // (the segment's block indices four at a time: one LDS round trip per four rows, not per row)
            for (int r0 = t; r0 < end_row; r0 += 4) {
                int bkv[4];
#pragma unroll
                for (int u = 0; u < 4; u++) bkv[u] = RI[min(r0 + u, end_row - 1)];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (r0 + u >= end_row) break;
                    const int bk = bkv[u];
                    unsigned char f = 0;
                    if (bk >= 0) {
                        f = pm_test(touched, bk - own_kb) ? 2 : 1;
                        pm_set(touched, bk - own_kb);
                    }
                    RF[r0 + u] = f;
                    again |= f == 2;
                }
            }
            if (c0 + end_row != sg.z) s.carry = touched;  // (the chunk's last segment; read after two barriers)
            if (again) NSW[kW] = 1;
        }
#ifdef SPSLAM_LBG_DIAG_BUILD
        __syncthreads();
        db1 = wall_clock64();
        if (t == 0) s.dg[0] += db1 - tb0;  // segment heads (Hpl kinds, lm_amask)
#endif
        // (A) every row's terms (the plane edges' Jacobians from plane_jacobians)
        {
            const int e = ne;
            const int row = land ? t : q;
            if (e >= 0 && nlv == 0) {
                const int ty = nty;
                const int ph = s.hidx[nkf];
                const bool pfree = ph >= 0;
                double A[3][3], B[3][6], info[3], err[3];
                if (e < g.Ep) {
                    point_jacobians(g, nkf, nlm, ty, A, B, land);
                } else {
                    auto J = g.terms + 27 * (size_t)e;
#pragma unroll
                    for (int i = 0; i < 3; i++) {
#pragma unroll
                        for (int d = 0; d < 3; d++) A[i][d] = J[3 * i + d];
#pragma unroll
                        for (int d = 0; d < 6; d++) B[i][d] = J[9 + 6 * i + d];
                    }
                }
                info_of_src(g, C, nsrc, ty, info);
                for (int i = 0; i < 3; i++) err[i] = g.err[3 * e + i];
                const EdgeW w = edge_weights(C, robust, ty, err, info);
                if (land) terms_land(w, robust, A, B, pfree, TL + kSL * row, TB + kSB * row);
                else terms_pose(w, B, TP + kSP * row);
            }
        }
        __syncthreads();
        const long long tb1 = wall_clock64();
        tA += tb1 - tb0;
#ifdef SPSLAM_LBG_DIAG_BUILD
        if (t == 0) s.dg[1] += tb1 - db1;  // (A) terms
#endif
        edge_rec(edge_of(st + 1));  // the next step's records land during (B)
        // (B) landmark segment chains: Hll (9) and bl (3) in edge order, four rows' loads in flight
        {
            int nseg = 0;
#pragma unroll
            for (int w = 0; w < kCh / 64; w++) nseg += NSW[w];
            for (int tk = t; tk < 12 * nseg; tk += kT) {
                const int si = tk / 12, comp = tk - 12 * si;
                int w = 0, li = si;
                while (li >= NSW[w]) li -= NSW[w++];
                const int4 sgm = SG[64 * w + li];
                const unsigned fl = (unsigned)sgm.w;
                const int h = sgm.z;
                auto dst = comp < 9 ? g.Hll + 9 * h + comp : g.bl + 3 * h + (comp - 9);
                // a landmark continuing from the previous step resumes from its partial sums in LDS
                double a = (fl >> 30) & 1 ? s.csum[st & 1][comp] : 0.0;
                int r = sgm.x;
                for (; r + 4 <= sgm.y; r += 4) {
                    double v[4];
                    bool ok[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        ok[u] = RI[r + u] != -2;
                        v[u] = TL[kSL * (r + u) + comp];
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) a = ok[u] ? a + v[u] : a;
                }
                for (; r < sgm.y; r++)
                    if (RI[r] != -2) a += TL[kSL * r + comp];
                if (fl >> 31) {
                    *dst = a;
                    if (comp == 0 || comp == 4 || comp == 8) mx = fmax(mx, fabs(a));
                } else {
                    s.csum[(st + 1) & 1][comp] = a;
                }
            }
#ifdef SPSLAM_LBG_DIAG_BUILD
            __syncthreads();
            db2 = wall_clock64();
            if (t == 0) s.dg[2] += db2 - tb1;  // landmark chains
#endif
            // each block's first term: 0 + term (one entry per task)
            for (int i = t; i < 18 * cnt; i += kT) {
                const int r = i / 18, c = i - 18 * r;
                if (RF[r] == 1) g.blkB[(size_t)18 * RI[r] + c] = 0.0 + TB[kSB * r + c];
            }
            if (NSW[kW]) {  // (block-uniform) the later terms, after every first term is stored
                __syncthreads();
                if (again) {
                    for (int r = t; r < end_row; r++) {
                        if (RF[r] != 2) continue;
                        auto dst = g.blkB + (size_t)18 * RI[r];
                        const double* rb = TB + kSB * r;
#pragma unroll
                        for (int j = 0; j < 18; j++) dst[j] += rb[j];
                    }
                }
            }
        }
#ifdef SPSLAM_LBG_DIAG_BUILD
        __syncthreads();
        db3 = wall_clock64();
        if (t == 0) s.dg[3] += db3 - db2;  // Hpl blocks
#endif
        // (free pose, term) chains over the step's rows of the pose: four rows' loads in flight, then their four adds
        // in edge order (a missing row: a select keeps the sum)
#pragma unroll
        for (int k = 0; k < kPoseSlots; k++) {
            if (task[k] < 0) continue;
            const int a = task[k] / 27, j = task[k] - 27 * a;
            const int n_a = min(R, PC[a] - st * R);
            const double* rows = TP + kSP * (a * R) + j;
            for (int i = 0; i < n_a; i += 4) {
                double v[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    ok[u] = i + u < n_a;
                    v[u] = rows[kSP * (ok[u] ? i + u : i)];
                }
#pragma unroll
                for (int u = 0; u < 4; u++) acc[k] = ok[u] ? acc[k] + v[u] : acc[k];
            }
        }
        __syncthreads();
        tb0 = wall_clock64();
        tB += tb0 - tb1;
#ifdef SPSLAM_LBG_DIAG_BUILD
        if (t == 0) { s.dg[4] += tb0 - db3; s.dg[5] += 1; }  // pose chains, steps
#endif
    }
    if (t == 0) { s.ph[0] += tA; s.tB += tB; }
#pragma unroll
    for (int k = 0; k < kPoseSlots; k++) {
        if (task[k] < 0) continue;
        const int a = task[k] / 27, j = task[k] - 27 * a;
        g.Hps[27 * s.pown[a] + j] = acc[k];
        if (j == 0 || j == 6 || j == 11 || j == 15 || j == 18 || j == 20) mx = fmax(mx, fabs(acc[k]));
    }
    mx = block_max(mx, s);
    if (t == 0) g.team->mx[s.m] = mx;
}

// ---------------------------------------------------------------- per trial

// setLambda + the Schur complement (block_solver.hpp:367-436), this member's block rows.  Every entry of a pattern
// block (i1, i2) is its own chain in g2o's order: Hschur(6 i1 + r, 6 i2 + c) = 0 + Hpp (+ lambda) then, landmark by
// landmark in landmark (vertex-id) order, -= (BDinv(r, 0) Bj(c, 0) + BDinv(r, 1) Bj(c, 1)) + BDinv(r, 2) Bj(c, 2); and
// Bb(6 i1 + r) = 0 + the landmarks' (Bi db)(r) in the same order.  One wave per block: lane 6 r + c holds entry (r,
// c), lanes 36 + r the diagonal block's Bb(r) (team_plan gives each member whole block rows, each wave up to kBW
// blocks, longest chains dealt first).  Every member stages every landmark in chunks of up to 64: their Hpl blocks
// (one contiguous range, coalesced), masks, Hll and bl -- the chunk's (Hll + lambda)^-1 and Dinv bl formed in place
// (the expressions of update()) -- then BDinv = Bi Dinv and Bi db for the blocks of its own rows (one thread per
// block row) and every free pose's chunk landmarks as a bitmask; then each wave, per block, compacts the chunk's
// landmarks that observe both poses into a list of (BDinv block, Bj block) pairs held one per lane, and walks it with
// the next landmark's operands loading while the current one is subtracted (the list read with v_readlane at the
// loop counter: no load on the chain's critical path).
#ifndef SPSLAM_LBG_SCHUR_BLOCKS
#define SPSLAM_LBG_SCHUR_BLOCKS 8
#endif
constexpr int kBW = SPSLAM_LBG_SCHUR_BLOCKS;  // blocks per wave per round
#ifndef SPSLAM_LBG_SCHUR_TASKS
#define SPSLAM_LBG_SCHUR_TASKS 2
#endif
constexpr int kSchurTasks = SPSLAM_LBG_SCHUR_TASKS;  // schur_rows: chains per lane per round
// (Hll + lambda)^-1 (Eigen's cofactor inverse) and Dinv bl of one landmark
__device__ __forceinline__ void landmark_dinv(const double* H, const double* bv, double lam, double* Di, double* db) {
    double D[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) D[i][j] = H[3 * i + j] + (i == j ? lam : 0.0);
    inverse3(D, Di);
    for (int i = 0; i < 3; i++) db[i] = (Di[3 * i] * bv[0] + Di[3 * i + 1] * bv[1]) + Di[3 * i + 2] * bv[2];
}
__device__ __noinline__ void schur() {
    const G& g = lbg_g;
    Sh& s = lbg_s;
    unsigned char* dyn = lbg_dyn;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int np = s.np, n = 6 * np, nch = s.nch;
    const double lam = s.lambda;
    // LDS: the staged chunk (blocks, Dinv, Dinv bl | masks, block offsets, block -> landmark, block -> pose), its
    // BDinv and Bi db, the poses' landmark masks, the waves' candidate lists
    constexpr int kBufD = kSchurBlk * 18 + kSchurLm * 12;
    double* BUF = (double*)dyn;                          // [kBufD]
    double* SD = BUF + kBufD;                            // [kSchurBlk][18] BDinv
    double* SU = SD + kSchurBlk * 18;                    // [kSchurBlk][6] B row . Dinv bl (Bb's terms)
    PMask* SM = (PMask*)(SU + kSchurBlk * 6);            // [kSchurLm]
    uint64_t* PM = (uint64_t*)(SM + kSchurLm);           // [kMaxK]
    int* SO = (int*)(PM + kMaxK);                        // [kSchurLm + 1]
    unsigned short* OB = (unsigned short*)(SO + kSchurLm + 1);  // [kMaxK][kSchurLm] (pose, landmark) -> its block
    unsigned char* BL = (unsigned char*)(OB + kMaxK * kSchurLm);  // [kSchurBlk] block -> landmark
    unsigned char* BP = BL + kSchurBlk;                  // [kSchurBlk] block -> pose
    using LdsU = __attribute__((address_space(3))) unsigned;
    LdsU* LST = (LdsU*)(unsigned*)(((uintptr_t)(BP + kSchurBlk) + 3) & ~(uintptr_t)3);  // [kW][64]
    const double* SDi = BUF + kSchurBlk * 18;
    const double* Sdb = SDi + kSchurLm * 9;
    static_assert((kBufD + kSchurBlk * 24 + kSchurLm * kPW + kMaxK) * 8 + (kSchurLm + 1) * 4 + kMaxK * kSchurLm * 2 +
                      2 * kSchurBlk + 4 + kW * 64 * 4 <= kDynAlloc, "LDS");
    constexpr int kPer = (kBufD + kT - 1) / kT;          // staged doubles per thread
    const int bo0 = s.bo0, nbm = s.bo1 - s.bo0;
    const PMask rmask = s.rmask;
    // this lane's entry: (r, c) on lanes 0 .. 35, Bb(r) on lanes 36 .. 41 (its operand addresses clamped in range)
    const bool ent = lane < 36;
    const int er = ent ? lane / 6 : min(lane - 36, 5), ec = ent ? lane - 6 * (lane / 6) : 0;
    using LdsD = const __attribute__((address_space(3))) double;
    LdsD* pE = (LdsD*)(SD + 3 * er);   // (LDS address-space pointers: 32-bit address arithmetic, ds_* accesses)
    LdsD* pJ = (LdsD*)(BUF + 3 * ec);
    LdsD* pU = (LdsD*)(SU + er);
    for (int round = 0; round * kW * kBW < nbm; round++) {
        int i1[kBW], i2[kBW];
        double acc[kBW];
#pragma unroll
        for (int k = 0; k < kBW; k++) {
            i1[k] = -1; i2[k] = 0; acc[k] = 0.0;
            const int jb = round * kW * kBW + snake_pick(k, wv, kW);
            if (jb < nbm) {
                const int blk = g.bord[bo0 + jb];
                if (blk < np) {
                    i1[k] = i2[k] = blk;
                } else {
                    int rem = blk - np, a = 0;
                    while (rem >= pm_popc(s.pat[a]) - 1) { rem -= pm_popc(s.pat[a]) - 1; a++; }
                    PMask row = pm_andnot(s.pat[a], pm_bit(a));
                    for (int u = 0; u < rem; u++) pm_pop(row);
                    i1[k] = a;
                    i2[k] = pm_ffs(row);
                }
                i1[k] = uni(i1[k]);
                i2[k] = uni(i2[k]);
                if (i1[k] == i2[k] && ent && ec >= er) {
                    const double h = g.Hps[27 * i1[k] + upper_idx(er, ec)];
                    acc[k] = 0.0 + (ec == er ? h + lam : h);
                }
            }
        }
        // chunk c's records into registers (global loads in flight), later into the staging buffer.  Every load is
        // unconditional (addresses clamped into the chunk; the surplus entries are never read) and nothing loaded is
        // used before the commit, so no wait lands in the chunk loop; the chunk bounds (sch, sch_kb) of the chunk
        // after next load one chunk ahead.
        double pv[kPer];
        PMask pmk = pm_zero();
        int pof = 0, pof1 = 0;
        auto prefetch = [&](int h0, int h1, int kb0, int kb1) __attribute__((always_inline)) {
            const int nbk = kb1 - kb0, nh = h1 - h0;
            const int cb = max(nbk * 18 - 1, 0), ch = max(nh * 9 - 1, 0), cl = max(nh * 3 - 1, 0);
#pragma unroll
            for (int q = 0; q < kPer; q++) {
                const int i = t + q * kT;
                const gdouble* src;
                if ((q + 1) * kT <= kSchurBlk * 18) {  // (compile time) the slice is in the Hpl block range
                    src = g.blkB + (size_t)18 * kb0 + min(i, cb);
                } else {
                    const int j = i - kSchurBlk * 18, j2 = j - kSchurLm * 9;
                    const gdouble* a = g.blkB + (size_t)18 * kb0 + min(i, cb);
                    const gdouble* h = g.Hll + (size_t)9 * h0 + min(max(j, 0), ch);
                    const gdouble* l = g.bl + (size_t)3 * h0 + min(max(j2, 0), cl);
                    src = j < 0 ? a : (j2 < 0 ? h : l);
                }
                pv[q] = *src;
            }
            const int tc = min(t, max(nh - 1, 0));
            pmk = pm_ld(g.lmh_mask + h0 + tc);
            pof = g.lmh_blk[h0 + min(t, nh)];
            pof1 = g.lmh_blk[h0 + tc + 1];
        };
        auto commit = [&](int nh, int kb0) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < kPer; q++)
                if (t + q * kT < kBufD) BUF[t + q * kT] = pv[q];
            if (t < nh) {
                SM[t] = pmk;
                PMask m = pmk;
                for (int bk = pof - kb0; bk < pof1 - kb0; bk++) {  // (the blocks of a landmark are in pose order)
                    BL[bk] = (unsigned char)t;
                    BP[bk] = (unsigned char)pm_ffs(m);
                    pm_pop(m);
                }
            }
            if (t <= nh) SO[t] = pof - kb0;
        };
        __syncthreads();  // the previous phase's LDS use is over
        // chunk bounds: (h0, h1, kb0, kb1) of the current chunk, the next, and the one after (loading)
        int cur_h0 = 0, cur_h1 = 0, cur_k0 = 0, cur_k1 = 0, nx_h1 = 0, nx_k1 = 0, nn_h1 = 0, nn_k1 = 0;
        if (nch > 0) {
            cur_h0 = g.sch[0]; cur_h1 = g.sch[1]; cur_k0 = g.sch_kb[0]; cur_k1 = g.sch_kb[1];
            nx_h1 = g.sch[min(2, nch)]; nx_k1 = g.sch_kb[min(2, nch)];
            prefetch(cur_h0, cur_h1, cur_k0, cur_k1);
            commit(cur_h1 - cur_h0, cur_k0);
            nn_h1 = g.sch[min(3, nch)]; nn_k1 = g.sch_kb[min(3, nch)];
        }
        for (int c = 0; c < nch; c++) {
#ifdef SPSLAM_LBG_DIAG
            long long d0 = wall_clock64();
#endif
            __syncthreads();  // chunk c is staged
#ifdef SPSLAM_LBG_DIAG
            long long d1 = wall_clock64();
            if (t == 0) s.dg[0] += d1 - d0;
#endif
            const int nh = cur_h1 - cur_h0;
            const int nbk = cur_k1 - cur_k0;
            if (t < nh) {  // the staged Hll, bl -> Dinv, Dinv bl, in place
                double* Hd = BUF + kSchurBlk * 18 + 9 * t;
                double* bd = BUF + kSchurBlk * 18 + kSchurLm * 9 + 3 * t;
                double H[9], bv[3], Di[9], db[3];
                for (int j = 0; j < 9; j++) H[j] = Hd[j];
                for (int j = 0; j < 3; j++) bv[j] = bd[j];
                landmark_dinv(H, bv, lam, Di, db);
                for (int j = 0; j < 9; j++) Hd[j] = Di[j];
                for (int j = 0; j < 3; j++) bd[j] = db[j];
            }
            __syncthreads();
            for (int i = t; i < nbk * 6; i += kT) {  // BDinv row by row: (Bi Dinv)(r, q), and Bi(r) . Dinv bl
                const int bk = i / 6, r6 = i - 6 * bk;
                if (!pm_test(rmask, BP[bk])) continue;  // a block row of another member
                const int hb = BL[bk];
                const double* Bi = BUF + 18 * bk + 3 * r6;
                const double* Di = SDi + 9 * hb;
                const double* db = Sdb + 3 * hb;
                double* BD = SD + 18 * bk + 3 * r6;
#pragma unroll
                for (int q = 0; q < 3; q++) BD[q] = (Bi[0] * Di[q] + Bi[1] * Di[3 + q]) + Bi[2] * Di[6 + q];
                SU[i] = (Bi[0] * db[0] + Bi[1] * db[1]) + Bi[2] * db[2];
            }
            for (int i = wv; i < np; i += kW) {  // free pose i's landmarks in the chunk, and their blocks
                const PMask mk = lane < nh ? SM[lane] : pm_zero();
                const bool obs = pm_test(mk, i);
                const uint64_t m = __ballot(obs);
                if (lane == 0) PM[i] = m;
                if (obs) OB[kSchurLm * i + lane] = (unsigned short)(SO[lane] + pm_popc_below(mk, i));
            }
            __syncthreads();
#ifdef SPSLAM_LBG_DIAG
            long long d2 = wall_clock64();
            if (t == 0) s.dg[1] += d2 - d1;
#endif
            if (c + 1 < nch) prefetch(cur_h1, nx_h1, cur_k1, nx_k1);  // lands while chunk c is processed
#ifdef SPSLAM_LBG_DIAG_SCHUR
            const long long wc0 = clock64();
            int wsteps = 0;
#endif
#pragma unroll
            for (int k = 0; k < kBW; k++) {
                if (i1[k] < 0) continue;  // (wave-uniform)
                const uint64_t cand = rl64(PM[i1[k]] & PM[i2[k]], 0);
                if (!cand) continue;
                // the candidates' (BDinv block, Bj block) pairs, compacted in landmark order, one per lane
                const bool in = (cand >> lane) & 1ull;
                const unsigned pos = __builtin_amdgcn_mbcnt_hi((unsigned)(cand >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((unsigned)cand, 0u));
                if (in) LST[64 * wv + pos] = (unsigned)OB[kSchurLm * i1[k] + lane] |
                                             ((unsigned)OB[kSchurLm * i2[k] + lane] << 16);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const unsigned my = LST[64 * wv + lane];
                const int nc = __popcll(cand);

                // operands of list entry q: BDinv row er of its first block, Bj row ec of its second, Bi db (er).  The
                // entry is opaque to the compiler, so the next entry's loads (issued before the current one is
                // subtracted) are not merged with the current one's into loads behind a wait at the loop top.
                auto ld = [&](int q, double (&E)[3], double (&B)[3], double& u) __attribute__((always_inline)) {
                    unsigned bb = __builtin_amdgcn_readlane(my, q);
                    asm volatile("" : "+s"(bb));
                    const unsigned b1 = bb & 0xffffu, b2 = bb >> 16;
                    LdsD* pe = pE + 18 * b1;
                    LdsD* pj = pJ + 18 * b2;
                    LdsD* pu = pU + 6 * b1;
                    E[0] = pe[0]; E[1] = pe[1]; E[2] = pe[2];
                    B[0] = pj[0]; B[1] = pj[1]; B[2] = pj[2];
                    u = pu[0];
                };
                auto step = [&](double a, const double (&E)[3], const double (&B)[3], double u)
                    __attribute__((always_inline)) {
                    const double sub = a - ((E[0] * B[0] + E[1] * B[1]) + E[2] * B[2]);
                    const double add = a + u;
                    return ent ? sub : add;
                };
                double EA[3], BA[3], uA, EB[3], BB[3], uB;
                ld(0, EA, BA, uA);
                double a = acc[k];
                int q = 0;
                for (; q + 2 <= nc; q += 2) {  // two operand sets in turn: one in flight while the other is used
                    ld(q + 1, EB, BB, uB);
                    a = step(a, EA, BA, uA);
                    ld(min(q + 2, nc - 1), EA, BA, uA);
                    a = step(a, EB, BB, uB);
                }
                if (q < nc) a = step(a, EA, BA, uA);
                acc[k] = a;
#ifdef SPSLAM_LBG_DIAG_SCHUR
                wsteps += nc;
#endif
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the list is free again
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
#ifdef SPSLAM_LBG_DIAG_SCHUR  // per wave: chain cycles and steps (summed), the chunk's slowest wave (summed)
            if (lane == 0) {
                const unsigned long long wc = (unsigned long long)(clock64() - wc0);
                atomicAdd((unsigned long long*)&s.dg[10], wc);
                atomicAdd((unsigned long long*)&s.dg[11], (unsigned long long)wsteps);
                atomicMax((unsigned long long*)&s.dg[12], wc);
            }
#endif
            __syncthreads();  // the staging buffer, BDinv and the masks are free again
#ifdef SPSLAM_LBG_DIAG_SCHUR
            if (t == 0) { s.dg[13] += s.dg[12]; s.dg[12] = 0; }
#endif
#ifdef SPSLAM_LBG_DIAG
            long long d3 = wall_clock64();
            if (t == 0) s.dg[2] += d3 - d2;
#endif
            if (c + 1 < nch) commit(nx_h1 - cur_h1, cur_k1);
            // advance the bounds; the chunk after next's load lands during the next chunk
            cur_h0 = cur_h1; cur_h1 = nx_h1; cur_k0 = cur_k1; cur_k1 = nx_k1;
            nx_h1 = nn_h1; nx_k1 = nn_k1;
            nn_h1 = g.sch[min(c + 4, nch)]; nn_k1 = g.sch_kb[min(c + 4, nch)];
#ifdef SPSLAM_LBG_DIAG
            if (t == 0) s.dg[3] += wall_clock64() - d3;
#endif
        }
#pragma unroll
        for (int k = 0; k < kBW; k++) {
            if (i1[k] < 0) continue;
            if (ent) g.S[(size_t)(6 * i1[k] + er) * n + 6 * i2[k] + ec] = acc[k];
            else if (lane < 42 && i1[k] == i2[k]) g.bs[6 * i1[k] + er] = g.Hps[27 * i1[k] + 21 + er] - acc[k];
        }
    }
}

// The same Schur complement with one lane per (block, R rows r0 .. r0 + R - 1) holding those rows' entries (and the
// diagonal block's Bb(r)), each lane walking its own candidate landmarks, TT such tasks per lane: fewer LDS bytes per
// entry than schur()'s lane per entry (a landmark's Bj block is read once for R rows), but a dependent LDS round trip
// per landmark.  The faster of the two when a member holds many blocks (teams of 1 - 4); R and TT are chosen per call
// from the member's block count (schur_rows_pick): every chain keeps g2o's landmark order whatever the split.
template <int R, int TT>
__device__ __noinline__ void schur_rows() {
    constexpr int kG = 6 / R;  // row groups per block
    const G& g = lbg_g;
    Sh& s = lbg_s;
    unsigned char* dyn = lbg_dyn;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int np = s.np, n = 6 * np, nch = s.nch;
    const double lam = s.lambda;
    // LDS: the staged chunk (blocks, Dinv, Dinv bl | masks, block offsets, block -> landmark, block -> pose), its
    // BDinv and Bi db, the poses' landmark masks, the waves' candidate lists
    constexpr int kBufD = kSchurBlk * 18 + kSchurLm * 12;
    double* BUF = (double*)dyn;                          // [kBufD]
    double* SD = BUF + kBufD;                            // [kSchurBlk][18] BDinv
    double* SU = SD + kSchurBlk * 18;                    // [kSchurBlk][6] B row . Dinv bl (Bb's terms)
    PMask* SM = (PMask*)(SU + kSchurBlk * 6);            // [kSchurLm]
    uint64_t* PM = (uint64_t*)(SM + kSchurLm);           // [kMaxK]
    int* SO = (int*)(PM + kMaxK);                        // [kSchurLm + 1]
    unsigned short* OB = (unsigned short*)(SO + kSchurLm + 1);  // [kMaxK][kSchurLm] (pose, landmark) -> its block
    unsigned char* BL = (unsigned char*)(OB + kMaxK * kSchurLm);  // [kSchurBlk] block -> landmark
    unsigned char* BP = BL + kSchurBlk;                  // [kSchurBlk] block -> pose
    const double* SDi = BUF + kSchurBlk * 18;
    const double* Sdb = SDi + kSchurLm * 9;
    static_assert((kBufD + kSchurBlk * 24 + kSchurLm * kPW + kMaxK) * 8 + (kSchurLm + 1) * 4 + kMaxK * kSchurLm * 2 +
                      2 * kSchurBlk + 4 + kW * 64 * 4 <= kDynAlloc, "LDS");
    constexpr int kPer = (kBufD + kT - 1) / kT;          // staged doubles per thread
    const int bo0 = s.bo0, nbm = s.bo1 - s.bo0;
    const PMask rmask = s.rmask;
    using LdsD = const __attribute__((address_space(3))) double;
    for (int round = 0; round * TT * kT < kG * nbm; round++) {
        int i1[TT], i2[TT], rr[TT];
        double acc[TT][R][6], cf[TT][R];
#pragma unroll
        for (int k = 0; k < TT; k++) {
            i1[k] = -1; i2[k] = 0; rr[k] = 0;
            const int task = (round * TT + k) * kT + t;
            if (task < kG * nbm) {
                const int jb = task / kG;
                rr[k] = R * (task - kG * jb);
                const int blk = g.bord[bo0 + jb];
                if (blk < np) {
                    i1[k] = i2[k] = blk;
                } else {
                    int rem = blk - np, a = 0;
                    while (rem >= pm_popc(s.pat[a]) - 1) { rem -= pm_popc(s.pat[a]) - 1; a++; }
                    PMask row = pm_andnot(s.pat[a], pm_bit(a));
                    for (int u = 0; u < rem; u++) pm_pop(row);
                    i1[k] = a;
                    i2[k] = pm_ffs(row);
                }
            }
            const bool diag = i1[k] >= 0 && i1[k] == i2[k];
#pragma unroll
            for (int q = 0; q < R; q++) {
                const int r = rr[k] + q;
#pragma unroll
                for (int c = 0; c < 6; c++) {
                    double base = 0.0;
                    if (diag && c >= r)
                        base = c == r ? g.Hps[27 * i1[k] + upper_idx(r, c)] + lam : g.Hps[27 * i1[k] + upper_idx(r, c)];
                    acc[k][q][c] = 0.0 + base;
                }
                cf[k][q] = 0.0;
            }
        }
        // chunk c's records into registers (global loads in flight), later into the staging buffer.  Every load is
        // unconditional (addresses clamped into the chunk; the surplus entries are never read) and nothing loaded is
        // used before the commit, so no wait lands in the chunk loop; the chunk bounds (sch, sch_kb) of the chunk
        // after next load one chunk ahead.
        double pv[kPer];
        PMask pmk = pm_zero();
        int pof = 0, pof1 = 0;
        auto prefetch = [&](int h0, int h1, int kb0, int kb1) __attribute__((always_inline)) {
            const int nbk = kb1 - kb0, nh = h1 - h0;
            const int cb = max(nbk * 18 - 1, 0), ch = max(nh * 9 - 1, 0), cl = max(nh * 3 - 1, 0);
#pragma unroll
            for (int q = 0; q < kPer; q++) {
                const int i = t + q * kT;
                const gdouble* src;
                if ((q + 1) * kT <= kSchurBlk * 18) {  // (compile time) the slice is in the Hpl block range
                    src = g.blkB + (size_t)18 * kb0 + min(i, cb);
                } else {
                    const int j = i - kSchurBlk * 18, j2 = j - kSchurLm * 9;
                    const gdouble* a = g.blkB + (size_t)18 * kb0 + min(i, cb);
                    const gdouble* h = g.Hll + (size_t)9 * h0 + min(max(j, 0), ch);
                    const gdouble* l = g.bl + (size_t)3 * h0 + min(max(j2, 0), cl);
                    src = j < 0 ? a : (j2 < 0 ? h : l);
                }
                pv[q] = *src;
            }
            const int tc = min(t, max(nh - 1, 0));
            pmk = pm_ld(g.lmh_mask + h0 + tc);
            pof = g.lmh_blk[h0 + min(t, nh)];
            pof1 = g.lmh_blk[h0 + tc + 1];
        };
        auto commit = [&](int nh, int kb0) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < kPer; q++)
                if (t + q * kT < kBufD) BUF[t + q * kT] = pv[q];
            if (t < nh) {
                SM[t] = pmk;
                PMask m = pmk;
                for (int bk = pof - kb0; bk < pof1 - kb0; bk++) {  // (the blocks of a landmark are in pose order)
                    BL[bk] = (unsigned char)t;
                    BP[bk] = (unsigned char)pm_ffs(m);
                    pm_pop(m);
                }
            }
            if (t <= nh) SO[t] = pof - kb0;
        };
        __syncthreads();  // the previous phase's LDS use is over
        // chunk bounds: (h0, h1, kb0, kb1) of the current chunk, the next, and the one after (loading)
        int cur_h0 = 0, cur_h1 = 0, cur_k0 = 0, cur_k1 = 0, nx_h1 = 0, nx_k1 = 0, nn_h1 = 0, nn_k1 = 0;
        if (nch > 0) {
            cur_h0 = g.sch[0]; cur_h1 = g.sch[1]; cur_k0 = g.sch_kb[0]; cur_k1 = g.sch_kb[1];
            nx_h1 = g.sch[min(2, nch)]; nx_k1 = g.sch_kb[min(2, nch)];
            prefetch(cur_h0, cur_h1, cur_k0, cur_k1);
            commit(cur_h1 - cur_h0, cur_k0);
            nn_h1 = g.sch[min(3, nch)]; nn_k1 = g.sch_kb[min(3, nch)];
        }
        for (int c = 0; c < nch; c++) {
#ifdef SPSLAM_LBG_DIAG
            long long d0 = wall_clock64();
#endif
            __syncthreads();  // chunk c is staged
#ifdef SPSLAM_LBG_DIAG
            long long d1 = wall_clock64();
            if (t == 0) s.dg[0] += d1 - d0;
#endif
            const int nh = cur_h1 - cur_h0;
            const int nbk = cur_k1 - cur_k0;
            if (t < nh) {  // the staged Hll, bl -> Dinv, Dinv bl, in place
                double* Hd = BUF + kSchurBlk * 18 + 9 * t;
                double* bd = BUF + kSchurBlk * 18 + kSchurLm * 9 + 3 * t;
                double H[9], bv[3], Di[9], db[3];
                for (int j = 0; j < 9; j++) H[j] = Hd[j];
                for (int j = 0; j < 3; j++) bv[j] = bd[j];
                landmark_dinv(H, bv, lam, Di, db);
                for (int j = 0; j < 9; j++) Hd[j] = Di[j];
                for (int j = 0; j < 3; j++) bd[j] = db[j];
            }
            __syncthreads();
            for (int i = t; i < nbk * 6; i += kT) {  // BDinv row by row: (Bi Dinv)(r, q), and Bi(r) . Dinv bl
                const int bk = i / 6, r6 = i - 6 * bk;
                if (!pm_test(rmask, BP[bk])) continue;  // a block row of another member
                const int hb = BL[bk];
                const double* Bi = BUF + 18 * bk + 3 * r6;
                const double* Di = SDi + 9 * hb;
                const double* db = Sdb + 3 * hb;
                double* BD = SD + 18 * bk + 3 * r6;
#pragma unroll
                for (int q = 0; q < 3; q++) BD[q] = (Bi[0] * Di[q] + Bi[1] * Di[3 + q]) + Bi[2] * Di[6 + q];
                SU[i] = (Bi[0] * db[0] + Bi[1] * db[1]) + Bi[2] * db[2];
            }
            for (int i = wv; i < np; i += kW) {  // free pose i's landmarks in the chunk, and their blocks
                const PMask mk = lane < nh ? SM[lane] : pm_zero();
                const bool obs = pm_test(mk, i);
                const uint64_t m = __ballot(obs);
                if (lane == 0) PM[i] = m;
                if (obs) OB[kSchurLm * i + lane] = (unsigned short)(SO[lane] + pm_popc_below(mk, i));
            }
            __syncthreads();
#ifdef SPSLAM_LBG_DIAG
            long long d2 = wall_clock64();
            if (t == 0) s.dg[1] += d2 - d1;
#endif
            if (c + 1 < nch) prefetch(cur_h1, nx_h1, cur_k1, nx_k1);  // lands while chunk c is processed
#pragma unroll
            for (int k = 0; k < TT; k++) {
                if (i1[k] < 0) continue;
                const int r = rr[k];
                uint64_t cand = PM[i1[k]] & PM[i2[k]];
                // one LDS round trip per landmark: the next landmark's blocks (the chunk's (pose, landmark) block
                // table) load while this one's are subtracted, and the diagonal lanes' Bb term comes staged (SU)
                // with the blocks instead of through a dependent load of Dinv bl
                if (cand) {
                    using LdsU16 = const __attribute__((address_space(3))) unsigned short;
                    LdsU16* O1 = (LdsU16*)(OB + kSchurLm * i1[k]);
                    LdsU16* O2 = (LdsU16*)(OB + kSchurLm * i2[k]);
                    LdsD* SDr = (LdsD*)(SD + 3 * r);
                    LdsD* SUr = (LdsD*)(SU + r);
                    LdsD* BUFl = (LdsD*)BUF;
                    int hl = __ffsll((unsigned long long)cand) - 1;
                    cand &= cand - 1;
                    int b1 = O1[hl], b2 = O2[hl];
                    // (opaque here: otherwise the first landmark's loads and the loop's next-landmark loads are
                    // merged into one load at the top of the loop, behind a wait -- the round trip this loop avoids)
                    asm volatile("" : "+v"(b1), "+v"(b2));
                    for (;;) {
                        LdsD* BD = SDr + __umul24(b1, 18);  // (24-bit products: full-rate multiplies)
                        LdsD* Bj = BUFl + __umul24(b2, 18);
                        double e[3 * R];
#pragma unroll
                        for (int q = 0; q < 3 * R; q++) e[q] = BD[q];  // BDinv rows r .. r + R - 1
                        double bj[18];
#pragma unroll
                        for (int q = 0; q < 18; q++) bj[q] = Bj[q];
                        double u[R];
#pragma unroll
                        for (int q = 0; q < R; q++) u[q] = SUr[__umul24(b1, 6) + q];  // (b1 = b2 on the diagonal)
                        const bool more = cand != 0;
                        const int hn = more ? __ffsll((unsigned long long)cand) - 1 : hl;
                        cand &= cand - 1;
                        const int b1n = O1[hn], b2n = O2[hn];
#pragma unroll
                        for (int q = 0; q < R; q++)
#pragma unroll
                            for (int cc = 0; cc < 6; cc++)
                                acc[k][q][cc] -= (e[3 * q] * bj[3 * cc] + e[3 * q + 1] * bj[3 * cc + 1]) +
                                                 e[3 * q + 2] * bj[3 * cc + 2];
#pragma unroll
                        for (int q = 0; q < R; q++)
                            cf[k][q] += u[q];  // (kept for the diagonal lanes only: unconditional, so the load is not
                                               // sunk into a branch that waits for the next landmark's loads too)
                        if (!more) break;
                        hl = hn;
                        b1 = b1n;
                        b2 = b2n;
                    }
                }
            }
            __syncthreads();  // the staging buffer, BDinv and the masks are free again
#ifdef SPSLAM_LBG_DIAG
            long long d3 = wall_clock64();
            if (t == 0) s.dg[2] += d3 - d2;
#endif
            if (c + 1 < nch) commit(nx_h1 - cur_h1, cur_k1);
            // advance the bounds; the chunk after next's load lands during the next chunk
            cur_h0 = cur_h1; cur_h1 = nx_h1; cur_k0 = cur_k1; cur_k1 = nx_k1;
            nx_h1 = nn_h1; nx_k1 = nn_k1;
            nn_h1 = g.sch[min(c + 4, nch)]; nn_k1 = g.sch_kb[min(c + 4, nch)];
#ifdef SPSLAM_LBG_DIAG
            if (t == 0) s.dg[3] += wall_clock64() - d3;
#endif
        }
#pragma unroll
        for (int k = 0; k < TT; k++) {
            if (i1[k] < 0) continue;
#pragma unroll
            for (int q = 0; q < R; q++) {
                const int r = rr[k] + q;
#pragma unroll
                for (int cc = 0; cc < 6; cc++) g.S[(size_t)(6 * i1[k] + r) * n + 6 * i2[k] + cc] = acc[k][q][cc];
                if (i1[k] == i2[k]) g.bs[6 * i1[k] + r] = g.Hps[27 * i1[k] + 21 + r] - cf[k][q];
            }
        }
    }
}
// the row-group layout for this member's nbm blocks: fewest passes over the landmark chunks first (each pass stages
// every chunk again), then the least time per landmark step -- the largest of one lane's dependent step (an LDS
// round trip, ~120 clocks, then its fp64 work: 4 clocks per wave instruction, 6 per entry + 1 per Bb term), the
// busiest SIMD's fp64 issue and the waves' LDS reads (bytes / 128 per clock).  Measured: 55 blocks per member
// (12-keyframe maps) run fastest with one row per task, 325 (25 free poses) with two rows and two tasks per lane.
__device__ __forceinline__ int schur_rows_pick(int nbm) {
    const int R[4] = {6, 3, 2, 1}, TT[4] = {1, 1, 2, 2};
    int best = 3;
    long long best_cost = -1;
    for (int v = 0; v < 4; v++) {
        const long long tasks = (long long)(6 / R[v]) * nbm, slots = (long long)kT * TT[v];
        const long long rounds = (tasks + slots - 1) / slots;
        const long long per_round = (tasks + rounds - 1) / max(rounds, 1ll);
        const long long waves = (per_round + 64 * TT[v] - 1) / (64 * TT[v]);
        const long long lds = waves * 64 * TT[v] * (4 * R[v] + 18) * 8 / 128;
        const long long step = (long long)TT[v] * (37 * R[v]) * 4;
        const long long issue = (waves + 3) / 4 * step;
        const long long cost = rounds * 1000000 + rounds * max(max(lds, issue), 120 + step);
        if (best_cost < 0 || cost < best_cost) { best_cost = cost; best = v; }
    }
    return best;
}
__device__ __forceinline__ void schur_rows_any() {
    switch (schur_rows_pick(lbg_s.bo1 - lbg_s.bo0)) {
        case 0: schur_rows<6, 1>(); break;
        case 1: schur_rows<3, 1>(); break;
        case 2: schur_rows<2, 2>(); break;
        default: schur_rows<1, kSchurTasks>(); break;
    }
}

// LinearSolverEigen::solve: SimplicialLDLT::factorize + solve on wave 0.  Row r of the permuted system lives in
// lane r & 63, register r >> 6.  LD: L column-major (LD[i n + r] = L(r, i)), LB: L's column structures (bitsets),
// RS / RO: the rows' pattern orders, PI: Pinv.
// SP: the reduced system's upper triangle, packed column by column (SP[c (c + 1) / 2 + r] = S(r, c), r <= c) when
// kPacked, else g.S (dense, row-major)
template <int kC, bool kPacked, class PD, class PU, class PI_, class PS>
__device__ __forceinline__ void factor_body(PD* LD, const PU* LB, const PI_* RO, const PI_* RS, const PI_* PI,
                                            const PS* SP, double* PR /* LDS, 64 doubles */,
                                            const double* Dpre = nullptr /* factorised already (factor_dense) */) {
    const G& g = lbg_g;
    Sh& s = lbg_s;
    const int lane = threadIdx.x & 63;
    const int n = 6 * s.np;
    double Dg[kC];
#pragma unroll
    for (int m = 0; m < kC; m++) Dg[m] = 0.0;
    bool ok = true;
    if (Dpre) {  // L and D from factor_dense; s.ok set there
#pragma unroll
        for (int m = 0; m < kC; m++)
            if (64 * m + lane < n) Dg[m] = Dpre[64 * m + lane];
        ok = s.ok;
    }
    for (int k = 0; k < (Dpre ? 0 : n); k++) {
        const int ok_ = PI[k], qk = ok_ / 6;
        double y[kC];
#pragma unroll
        for (int m = 0; m < kC; m++) {
            const int r = 64 * m + lane;
            y[m] = 0.0;
            if (r <= k) {
                const int orr = PI[r];
                if (coupled(s, orr / 6, qk)) {
                    const int lo = min(orr, ok_), hi = max(orr, ok_);
                    y[m] = 0.0 + (kPacked ? SP[(hi * (hi + 1)) / 2 + lo] : SP[(size_t)lo * n + hi]);
                }
            }
        }
        double d = pick(y, k) * 1.0 + 0.0;
        const int t0 = RO[k], t1 = RO[k + 1];
        // The row's pattern order 64 entries at a time in registers (lane q: entry q of the piece), with each
        // entry's LDS byte offsets of its L column and structure word and its lane / register in y precomputed
        // per lane: a step reads them with v_readlane at a loop-counter lane and uses them only in vector
        // address arithmetic and as readlane lane selects, so no scalar instruction waits on a vector result
        // inside the chain.  The columns of L and the structure words of the next kRing steps are in flight
        // while a step runs (a ring of operand sets, each written only by its fetch and read only by its step).
        // Past the piece's end the entries repeat its last one with the structure word LB[n kNW] (zero): masked
        // steps.  A column's rows past n read the next one's (in the LDS layout; unused: masked by r < k).
        // (a divisor of 64: a piece's last ring round ends at step 63 -- with 6, a full piece of 64 entries ran two
        // steps past it, on entry 63's operands refetched and entry 0's lane select).  Global-memory pieces are L2
        // latency bound: a deeper ring where the registers allow it (kC <= 3: 8 operand sets, kC <= 6: 4)
        constexpr int kRing = kPacked ? 8 : kC <= 3 ? 8 : kC <= 6 ? 4 : 2;
        const char* LDc = (const char*)LD;
        const char* LBc = (const char*)LB;
        // rows r < k of register m as a lane mask: a step's update condition is one bit test (a select, no
        // exec-mask branch)
        uint64_t km[kC];
#pragma unroll
        for (int m = 0; m < kC; m++) {
            const int c = k - 64 * m;
            km[m] = c >= 64 ? ~0ull : c <= 0 ? 0ull : (1ull << c) - 1ull;
        }
        auto stepf = [&](int lsel, int rsel, const double (&v)[kC], const uint64_t (&wr)[kC]) __attribute__((always_inline)) {
            // (the structure words opaque until here: otherwise the compiler masks each one as soon as its load is
            // issued -- a wait for the LDS read every step, which defeats the ring)
            uint64_t w[kC];
#pragma unroll
            for (int m = 0; m < kC; m++) {
                w[m] = wr[m];
                asm volatile("" : "+v"(w[m]));
            }
            double yi = rl(y[0], lsel);
#pragma unroll
            for (int m = 1; m < kC; m++) {
                const double q = rl(y[m], lsel);
                yi = rsel == m ? q : yi;
            }
#pragma unroll
            for (int m = 0; m < kC; m++) {
                const double nv = y[m] - v[m] * yi;
                y[m] = (((w[m] & km[m]) >> lane) & 1ull) ? nv : y[m];
            }
        };
#ifdef SPSLAM_LBG_DIAG
        const long long c0 = clock64();
#endif
        for (int p0 = t0; p0 < t1; p0 += 64) {
            const int ns = min(64, t1 - p0);
            const int rsv = RS[p0 + min(lane, ns - 1)];
            const int cofs = rsv * n * 8;                                   // L column, bytes
            const int wofs = (lane < ns ? rsv : n) * (kNW * 8);             // structure words (past the end: zero)
            const int lsel = rsv & 63, rsel = rsv >> 6;                    // y's lane / register of the entry
            auto fetch = [&](int j, double (&v)[kC], uint64_t (&w)[kC]) __attribute__((always_inline)) {
                const int co = __builtin_amdgcn_readlane(cofs, j);
                int wo = __builtin_amdgcn_readlane(wofs, j);
                asm volatile("v_mov_b32 %0, %1" : "=v"(wo) : "s"(wo));  // the address sum in a vector op
#pragma unroll
                for (int m = 0; m < kC; m++) {
                    const int r = 64 * m + lane;
                    v[m] = (kPacked || r < n) ? *(const PD*)(LDc + co + 8 * r) : 0.0;
                    w[m] = *(const PU*)(LBc + wo + 8 * m);
                }
            };
            double v[kRing][kC];
            uint64_t w[kRing][kC];
#pragma unroll
            for (int q = 0; q < kRing; q++) fetch(min(q, 63), v[q], w[q]);
            for (int j = 0; j < ns; j += kRing) {
#pragma unroll
                for (int q = 0; q < kRing; q++) {
                    stepf(__builtin_amdgcn_readlane(lsel, j + q), __builtin_amdgcn_readlane(rsel, j + q), v[q], w[q]);
                    fetch(min(j + q + kRing, 63), v[q], w[q]);
                }
            }
        }
#ifdef SPSLAM_LBG_DIAG
        const long long c1 = clock64();
        if (lane == 0) { s.dg[6] += c1 - c0; s.dg[8] += t1 - t0; }
#endif
        double pr[kC];
#pragma unroll
        for (int m = 0; m < kC; m++) {
            const int r = 64 * m + lane;
            pr[m] = 0.0;
            if (r < k && bit_of(LB + (size_t)r * kNW, k)) {
                const double l = y[m] / Dg[m];
                LD[(size_t)r * n + k] = l;
                pr[m] = l * y[m];
            }
        }
        // d -= l_ki y_i in pattern order: the piece's terms gathered into pattern order across the lanes
        // (ds_bpermute), then subtracted lane by lane (loop-counter readlanes, off the dependent chain)
        for (int p0 = t0; p0 < t1; p0 += 64) {
            const int ns = min(64, t1 - p0);
            const int rsv = RS[p0 + min(lane, ns - 1)];
            const int src = (rsv & 63) * 4;
            double pv = 0.0;
#pragma unroll
            for (int m = 0; m < kC; m++) {
                const int lo = __builtin_amdgcn_ds_bpermute(src, __double2loint(pr[m]));
                const int hi = __builtin_amdgcn_ds_bpermute(src, __double2hiint(pr[m]));
                pv = (rsv >> 6) == m ? __hiloint2double(hi, lo) : pv;
            }
            // lane q's term into LDS slot q, then every lane subtracts the slots in order (broadcast reads:
            // no cross-lane register moves on the chain)
            PR[lane] = pv;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            int j = 0;
            for (; j + 8 <= ns; j += 8) {
                double a[8];
#pragma unroll
                for (int q = 0; q < 8; q++) a[q] = PR[j + q];
#pragma unroll
                for (int q = 0; q < 8; q++) d -= a[q];
            }
            for (; j < ns; j++) d -= PR[j];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#ifdef SPSLAM_LBG_DIAG
        if (lane == 0) s.dg[7] += clock64() - c1;
#endif
#pragma unroll
        for (int m = 0; m < kC; m++)
            if (64 * m + lane == k) Dg[m] = d;
        if (d == 0.0) {
            ok = false;
            break;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0 && !Dpre) s.ok = ok;
#ifdef SPSLAM_LBG_DIAG
    if (lane == 0) s.dg[4] = wall_clock64();
#endif
    if (!ok) return;
    // x = P b; L x = x; x = D^-1 x; L^T x = x; x = P^-1 x
    const bool haveL = RO[n] > 0;
    double tv[kC];
#pragma unroll
    for (int m = 0; m < kC; m++) {
        const int r = 64 * m + lane;
        tv[m] = r < n ? g.bs[PI[r]] : 0.0;
    }
    if (haveL)
        for (int i = 0; i < n; i++) {
            const double tmp = pick(tv, i);
            if (tmp != 0.0) {
                const auto* cb = LB + (size_t)i * kNW;
#pragma unroll
                for (int m = 0; m < kC; m++) {
                    const int r = 64 * m + lane;
                    if ((cb[m] >> lane) & 1ull) tv[m] = tv[m] - tmp * LD[(size_t)i * n + r];
                }
            }
        }
#pragma unroll
    for (int m = 0; m < kC; m++)
        if (64 * m + lane < n) tv[m] = (1.0 / Dg[m]) * tv[m];
    if (haveL)
        for (int i = n - 1; i >= 0; i--) {
            const auto* cb = LB + (size_t)i * kNW;
            double pr[kC];
#pragma unroll
            for (int m = 0; m < kC; m++) {
                const int r = 64 * m + lane;
                pr[m] = ((cb[m] >> lane) & 1ull) ? LD[(size_t)i * n + r] * tv[m] : 0.0;
            }
            double tmp = pick(tv, i);
#pragma unroll
            for (int m = 0; m < kC; m++) {
                uint64_t bits = (uint64_t)(uint32_t)uni((int)(uint32_t)cb[m]) | ((uint64_t)(uint32_t)uni((int)(cb[m] >> 32)) << 32);
                while (bits) {
                    const int r = __ffsll((unsigned long long)bits) - 1;
                    tmp -= rl(pr[m], r);
                    bits &= bits - 1;
                }
            }
#pragma unroll
            for (int m = 0; m < kC; m++)
                if (64 * m + lane == i) tv[m] = tmp;
        }
#pragma unroll
    for (int m = 0; m < kC; m++) {
        const int r = 64 * m + lane;
        if (r < n) g.x[PI[r]] = tv[m];
    }
}

// byte offsets of the factorisation's LDS copy (n <= kLdsN): L, its column structures, the rows' pattern orders
// (offsets, indices), P^-1, S packed
// (and factor_dense's pivots D and per-row progress PG, + a failure flag)
struct FactorLds { size_t LB, RO, RS, PI, SP, PR, D, PG, end; };
__device__ __forceinline__ FactorLds factor_lds(int n) {
    FactorLds f;
    f.LB = (size_t)n * n * 8;
    f.RO = f.LB + (size_t)(n + 1) * kNW * 8;  // row n: LB[n kNW ..] = 0
    f.RS = f.RO + (size_t)(n + 1) * 4;
    f.PI = f.RS + (size_t)((n * (n + 1)) / 2 + 1) * 4;
    f.SP = (f.PI + (size_t)n * 4 + 7) & ~(size_t)7;
    f.PR = f.SP + (size_t)((n * (n + 1)) / 2) * 8;
    f.D = f.PR + 64 * 8;
    f.PG = f.D + (size_t)n * 8;
    f.end = f.PG + (size_t)(n + 1) * 4;
    return f;
}
static_assert((size_t)kLdsN * kLdsN * 8 + ((kLdsN + 1) * kNW) * 8 + (kLdsN + 1) * 4 + (kLdsN * (kLdsN + 1) / 2 + 1) * 4 +
                  kLdsN * 4 + 8 + (kLdsN * (kLdsN + 1) / 2) * 8 + 64 * 8 + kLdsN * 8 + (kLdsN + 1) * 4 <= (size_t)kDyn,
              "the factorisation's LDS copy");

// SimplicialLDLT::factorize for a fully dense reduced system in the natural order (every pose coupled with every
// other; AMD then returns the identity and the elimination tree is a chain, so row k's pattern order is 0 .. k - 1
// and column i's structure every row below i), pipelined over the workgroup's waves: row k on wave k mod kW.  Row k
// runs Eigen's up-looking steps exactly as factor_body does -- for i = 0 .. k - 1: y_i read, y_r -= L(r, i) y_i for
// i < r < k, then l_ki = y_i / D_i and d -= l_ki y_i (the same pivot-update order as factor_body's pattern-order
// chain) -- and publishes L(k, i) at its step i and D_k when it ends.  Its step i needs L(r, i) for every r < k: row
// k - 1 has passed step i (PG[k - 1] > i) only after row k - 2 had, and so on, so one progress word per row orders
// them.  Same arithmetic, same order, rows overlapped.
template <int kC>
__device__ __noinline__ void factor_dense() {
    Sh& s = lbg_s;
    const int n = 6 * s.np;
    const FactorLds f = factor_lds(n);
    double* LD = (double*)lbg_dyn;
    const double* SP = (const double*)(lbg_dyn + f.SP);
    double* D = (double*)(lbg_dyn + f.D);
    volatile int* PG = (volatile int*)(lbg_dyn + f.PG);
    volatile int* FL = PG + n;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int k = t; k <= n; k += kT) PG[k] = 0;  // (PG[n] = FL)
    __syncthreads();
    for (int k = w; k < n; k += kW) {
        double y[kC];
#pragma unroll
        for (int m = 0; m < kC; m++) {
            const int r = 64 * m + lane;
            y[m] = r <= k ? 0.0 + SP[(k * (k + 1)) / 2 + r] : 0.0;
        }
        double d = pick(y, k) * 1.0 + 0.0;
        int seen = 0;
        bool failed = false;
        for (int i = 0; i < k; i++) {
            while (seen <= i) {  // row k - 1 has published L(k - 1, i)
                seen = __builtin_amdgcn_readfirstlane(PG[k - 1]);
                if (seen <= i) {
                    if (*FL) { failed = true; break; }
                    __builtin_amdgcn_s_sleep(0);
                }
            }
            if (failed) break;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const double yi = pick(y, i);
            const double Di = D[i];
            double v[kC];
#pragma unroll
            for (int m = 0; m < kC; m++) v[m] = LD[(size_t)i * n + 64 * m + lane];  // L(r, i), rows r < k published
            const double l = yi / Di;
#pragma unroll
            for (int m = 0; m < kC; m++) {
                const int r = 64 * m + lane;
                const double nv = y[m] - v[m] * yi;
                y[m] = (r > i && r < k) ? nv : y[m];
            }
            d -= l * yi;
            if (lane == 0) LD[(size_t)i * n + k] = l;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) PG[k] = i + 1;
        }
        if (failed) break;
        if (d == 0.0) {  // Eigen stops at a zero pivot (ok = false); the other rows see the flag and stop
            if (lane == 0) *FL = 1;
            break;
        }
        if (lane == 0) D[k] = d;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) PG[k] = k + 1;
    }
    __syncthreads();
    if (t == 0) s.ok = *FL == 0;
    __syncthreads();
}

// The same pipelined factorisation for dense systems too large for factor_dense's LDS copy (kLdsN < n <= kPackN,
// e.g. a window of 25 free poses, n = 150): L packed column by column in LDS (column i's rows i + 1 .. n - 1, a guard
// in front so that the masked reads of rows <= i stay in range), S read from global memory once per row, D and the
// progress words in LDS.  Then the solve (factor_body's order with every column's structure "all rows below").
constexpr int kPackN = 180;
__host__ __device__ constexpr int pk_col(int i, int n) { return (i * (2 * n - i - 1)) / 2 - i - 1 + n; }  // L(r, i) at + r
__host__ __device__ constexpr size_t pk_words(int n, int kC) { return (size_t)n + (size_t)n * (n - 1) / 2 + 64 * kC; }
static_assert((pk_words(kPackN, 3) + kPackN) * 8 + (kPackN + 1) * 4 <= (size_t)kDyn, "packed dense factorisation");
template <int kC>
__device__ __noinline__ void factor_dense_packed() {
    const G& g = lbg_g;
    Sh& s = lbg_s;
    const int n = 6 * s.np;
    double* LP = (double*)lbg_dyn;
    double* D = LP + pk_words(n, kC);
    volatile int* PG = (volatile int*)(D + n);
    volatile int* FL = PG + n;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int k = t; k <= n; k += kT) PG[k] = 0;  // (PG[n] = FL)
    __syncthreads();
    for (int k = w; k < n; k += kW) {
        double y[kC];
#pragma unroll
        for (int m = 0; m < kC; m++) {
            const int r = 64 * m + lane;
            y[m] = r <= k ? 0.0 + g.S[(size_t)r * n + k] : 0.0;
        }
        double d = pick(y, k) * 1.0 + 0.0;
        int seen = 0;
        bool failed = false;
        for (int i = 0; i < k; i++) {
            while (seen <= i) {  // row k - 1 has published L(k - 1, i)
                seen = __builtin_amdgcn_readfirstlane(PG[k - 1]);
                if (seen <= i) {
                    if (*FL) { failed = true; break; }
                    __builtin_amdgcn_s_sleep(0);
                }
            }
            if (failed) break;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const double yi = pick(y, i);
            const double Di = D[i];
            const double* col = LP + pk_col(i, n);
            double v[kC];
#pragma unroll
            for (int m = 0; m < kC; m++) v[m] = col[64 * m + lane];  // L(r, i): rows i < r < k published
            const double l = yi / Di;
#pragma unroll
            for (int m = 0; m < kC; m++) {
                const int r = 64 * m + lane;
                const double nv = y[m] - v[m] * yi;
                y[m] = (r > i && r < k) ? nv : y[m];
            }
            d -= l * yi;
            if (lane == 0) LP[pk_col(i, n) + k] = l;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) PG[k] = i + 1;
        }
        if (failed) break;
        if (d == 0.0) {  // Eigen stops at a zero pivot (ok = false); the other rows see the flag and stop
            if (lane == 0) *FL = 1;
            break;
        }
        if (lane == 0) D[k] = d;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) PG[k] = k + 1;
    }
    __syncthreads();
    if (t == 0) s.ok = *FL == 0;
    __syncthreads();
}
// x = P b; L x = x; x = D^-1 x; L^T x = x; x = P^-1 x (factor_body's solve, every column's structure the rows below it);
// one wave
template <int kC>
__device__ __noinline__ void solve_dense_packed() {
    const G& g = lbg_g;
    const Sh& s = lbg_s;
    if (!s.ok) return;
    const int n = 6 * s.np, lane = threadIdx.x & 63;
    const double* LP = (const double*)lbg_dyn;
    const double* D = LP + pk_words(n, kC);
    double tv[kC], Dg[kC];
#pragma unroll
    for (int m = 0; m < kC; m++) {
        const int r = 64 * m + lane;
        tv[m] = r < n ? g.bs[g.Pinv[r]] : 0.0;
        Dg[m] = r < n ? D[r] : 0.0;
    }
    if (n > 1)
        for (int i = 0; i < n; i++) {
            const double tmp = pick(tv, i);
            if (tmp != 0.0) {
                const double* col = LP + pk_col(i, n);
#pragma unroll
                for (int m = 0; m < kC; m++) {
                    const int r = 64 * m + lane;
                    if (r > i && r < n) tv[m] = tv[m] - tmp * col[r];
                }
            }
        }
#pragma unroll
    for (int m = 0; m < kC; m++)
        if (64 * m + lane < n) tv[m] = (1.0 / Dg[m]) * tv[m];
    if (n > 1)
        for (int i = n - 1; i >= 0; i--) {
            const double* col = LP + pk_col(i, n);
            double pr[kC];
#pragma unroll
            for (int m = 0; m < kC; m++) {
                const int r = 64 * m + lane;
                pr[m] = (r > i && r < n) ? col[r] * tv[m] : 0.0;
            }
            double tmp = pick(tv, i);
#pragma unroll
            for (int m = 0; m < kC; m++) {
                const int lo = max(i + 1 - 64 * m, 0), hi = min(n - 64 * m, 64);  // lanes of rows i < r < n
                for (int q = lo; q < hi; q++) tmp -= rl(pr[m], q);
            }
#pragma unroll
            for (int m = 0; m < kC; m++)
                if (64 * m + lane == i) tv[m] = tmp;
        }
#pragma unroll
    for (int m = 0; m < kC; m++) {
        const int r = 64 * m + lane;
        if (r < n) g.x[g.Pinv[r]] = tv[m];
    }
}

template <int kC, bool kLds, bool kPre = false>
__device__ __noinline__ void factor_solve() {
    const int n = 6 * lbg_s.np;
    if (kLds) {  // the layout of k_lba_g2o's copy in LDS
        const FactorLds f = factor_lds(n);
        factor_body<kC, true>((double*)lbg_dyn, (const uint64_t*)(lbg_dyn + f.LB), (const int*)(lbg_dyn + f.RO),
                              (const int*)(lbg_dyn + f.RS), (const int*)(lbg_dyn + f.PI),
                              (const double*)(lbg_dyn + f.SP), (double*)(lbg_dyn + f.PR),
                              kPre ? (const double*)(lbg_dyn + f.D) : nullptr);
    } else {
        const G& g = lbg_g;
        factor_body<kC, false>(g.Ld, g.Lbits, g.rs_off, g.rs_idx, g.Pinv, g.S, (double*)lbg_dyn);  // (LDS unused)
    }
}

// this member's landmarks [h0, h1) (Hessian order) and keyframes [k0, k1)
struct Share { int h0, h1, k0, k1; };
__device__ __forceinline__ Share my_share(const Sh& s, int K) {
    return Share{split_lo(s.nl, s.m, s.T), split_lo(s.nl, s.m + 1, s.T), split_lo(K, s.m, s.T), split_lo(K, s.m + 1, s.T)};
}
// landmark increments (xl = Dinv (bl - Hpl^T xp), Dinv as the Schur phase formed it), push, update
// (block_solver.hpp:444-471, oplus); this member's landmarks and keyframes.  After a failed solve nothing of x was
// written (block_solver.hpp:447-457: the landmark part is formed only after a successful pose solve) and g2o still
// applies it: every vertex moves by the previous solution (optimization_algorithm_levenberg.cpp:110-115).
__device__ __noinline__ void update() {
    const G& g = lbg_g;
    const Sh& s = lbg_s;
    const int t = threadIdx.x;
    const int np = s.np, n = 6 * np;
    const bool ok = s.ok;
    const double lam = s.lambda;
    const Share sh = my_share(s, g.K);
    for (int h = sh.h0 + t; h < sh.h1; h += kT) {
        const int l = g.hidx_lm[h];
        if (l < g.Np) for (int j = 0; j < 3; j++) g.X_b[3 * l + j] = g.X[3 * l + j];
        else for (int j = 0; j < 4; j++) g.P_b[4 * (l - g.Np) + j] = g.P[4 * (l - g.Np) + j];
        double xl[3];
        if (ok) {
            double cl[3] = {g.bl[3 * h], g.bl[3 * h + 1], g.bl[3 * h + 2]};
            PMask m = pm_ld(g.lmh_mask + h);
            int bk = g.lmh_blk[h];
            while (pm_any(m)) {
                const int p = pm_ffs(m);
                pm_pop(m);
                auto B = g.blkB + (size_t)18 * bk++;
                for (int i = 0; i < 3; i++) {
                    double sm = 0;
                    for (int r = 0; r < 6; r++) sm += B[3 * r + i] * (-g.x[6 * p + r]);
                    cl[i] += sm;
                }
            }
            double H[9], Di[9], db[3];
            for (int j = 0; j < 9; j++) H[j] = g.Hll[9 * h + j];
            landmark_dinv(H, cl, lam, Di, db);  // (db unused)
            for (int i = 0; i < 3; i++) xl[i] = (Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1]) + Di[3 * i + 2] * cl[2];
            for (int j = 0; j < 3; j++) g.x[n + 3 * h + j] = xl[j];
        } else {
            for (int j = 0; j < 3; j++) xl[j] = g.x[n + 3 * h + j];
        }
        if (l < g.Np) {
            for (int j = 0; j < 3; j++) g.X[3 * l + j] += xl[j];
        } else {
            auto pp = g.P + 4 * (l - g.Np);
            P4 P{{pp[0], pp[1], pp[2], pp[3]}};
            p_oplus(P, xl);
            for (int j = 0; j < 4; j++) pp[j] = P.c[j];
        }
    }
    for (int k = sh.k0 + t; k < sh.k1; k += kT) {
        for (int j = 0; j < 7; j++) g.pose_b[7 * k + j] = g.pose[7 * k + j];
        const int h = s.hidx[k];
        if (h < 0) continue;
        double u[6];
        for (int j = 0; j < 6; j++) u[j] = g.x[6 * h + j];
        store_pose(g.pose + 7 * k, se3_mul(se3_exp(u), load_pose(g.pose + 7 * k)));
    }
}

__device__ __noinline__ void restore() {  // pop(): this member's landmarks and keyframes
    const G& g = lbg_g;
    const Sh& s = lbg_s;
    const int t = threadIdx.x;
    const Share sh = my_share(s, g.K);
    for (int h = sh.h0 + t; h < sh.h1; h += kT) {
        const int l = g.hidx_lm[h];
        if (l < g.Np) for (int j = 0; j < 3; j++) g.X[3 * l + j] = g.X_b[3 * l + j];
        else for (int j = 0; j < 4; j++) g.P[4 * (l - g.Np) + j] = g.P_b[4 * (l - g.Np) + j];
    }
    for (int k = sh.k0 + t; k < sh.k1; k += kT)
        for (int j = 0; j < 7; j++) g.pose[7 * k + j] = g.pose_b[7 * k + j];
}

// computeScale terms x_j (lambda x_j + b_j), poses then landmarks (Hessian order), zero-padded to 32; this member's
// share of the entries
__device__ __noinline__ void scale_terms() {
    const G& g = lbg_g;
    const Sh& s = lbg_s;
    const int t = threadIdx.x;
    const int n = 6 * s.np, tot = n + 3 * s.nl, pad = lbg_pad32(tot);
    const double lam = s.lambda;
    for (int j = split_lo(pad, s.m, s.T) + t; j < split_lo(pad, s.m + 1, s.T); j += kT) {
        double v = 0.0;
        if (j < tot) {  // (x as update() applied it: after a failed solve, the previous solution)
            const double b = j < n ? g.Hps[27 * (j / 6) + 21 + j % 6] : g.bl[j - n];
            const double x = g.x[j];
            v = x * (lam * x + b);
        }
        g.sc[j] = v;
    }
}

// relabel between the passes with the errors cached by the last computeActiveErrors (Optimizer.cc:1815-1851); this
// member's edges
__device__ __noinline__ void relabel() {
    const LbaConsts& C = lbg_c;
    const G& g = lbg_g;
    const Sh& s = lbg_s;
    for (int e = split_lo(g.E, s.m, s.T) + threadIdx.x; e < split_lo(g.E, s.m + 1, s.T); e += kT) {
        double info[3];
        const int ty = g.e_type[e];
        info_of(g, C, e, ty, info);
        const double chi = chi2_of(g.err + 3 * e, info, edge_dim(ty));
        bool bad;
        if (ty == 0) bad = chi > 5.991 || !depth_positive(g, e);
        else if (ty == 1) bad = chi > 7.815 || !depth_positive(g, e);
        else if (ty == 2) bad = chi > C.plane_chi;
        else bad = chi > C.vp_chi;
        if (bad) g.e_level[e] = 1;
    }
}

// computeActiveErrors (+ the plane edges' Jacobians at the same state): this member's edges
__device__ __noinline__ void errors_phase() {
    const G& g = lbg_g;
    const Sh& s = lbg_s;
    errors();
    const int npl = g.E - g.Ep;
    plane_jacobians(g.Ep + split_lo(npl, s.m, s.T), g.Ep + split_lo(npl, s.m + 1, s.T));
}

// ---------------------------------------------------------------- outputs
__device__ __noinline__ void outputs(const LbgBatch& b, int p) {
    const LbaConsts& C = lbg_c;
    const G& g = lbg_g;
    Sh& s = lbg_s;
    const int t = threadIdx.x;
    const spslam_lba_problem pb = b.probs[p];
    if (s.stopped == 1) {  // returned before optimizing: the map is untouched, nothing is erased
        // (setup did not run: the observations are addressed through the input records)
        for (int i = t; i < g.Np; i += kT)
            for (int o = g.pt[i].obs_offset; o < g.pt[i].obs_offset + g.pt[i].n_obs; o++) b.pobs_out[o] = 0;
        for (int i = t; i < g.Nq; i += kT)
            for (int o = g.pl[i].obs_offset; o < g.pl[i].obs_offset + g.pl[i].n_obs; o++) b.plobs_out[o] = 0;
        for (int i = t; i < 16 * g.K; i += kT) b.kf_out[16 * (size_t)pb.kf_offset + i] = g.kf[i / 16].Tcw[i % 16];
        for (int i = t; i < 3 * g.Np; i += kT) b.pt_out[3 * (size_t)pb.point_offset + i] = g.pt[i / 3].xw[i % 3];
        for (int i = t; i < 4 * g.Nq; i += kT) b.pl_out[4 * (size_t)pb.plane_offset + i] = g.pl[i / 4].world[i % 4];
        if (t == 0) {
            spslam_lba_result* r = b.res + p;
            *r = spslam_lba_result{};
            r->stopped = 1;
        }
        return;
    }
    int cnt[2] = {0, 0};
    for (int e = t; e < g.E; e += kT) {
        double info[3];
        const int ty = g.e_type[e];
        info_of(g, C, e, ty, info);
        const double chi = chi2_of(g.err + 3 * e, info, edge_dim(ty));
        if (ty <= 1) {
            const bool bad = chi > (ty == 0 ? 5.991 : 7.815) || !depth_positive(g, e);
            b.pobs_out[g.e_src[e]] = bad;
            cnt[0] += bad;
        } else {
            const bool bad = ty == 2 ? chi > C.plane_chi : chi > C.vp_chi;
            b.plobs_out[g.e_src[e]] = bad;
            cnt[1] += bad;
        }
    }
    int tot0, tot1;
    block_scan(cnt[0], &tot0, s);
    block_scan(cnt[1], &tot1, s);
    for (int k = t; k < g.K; k += kT) {
        float* o = b.kf_out + 16 * ((size_t)pb.kf_offset + k);
        if (g.kf[k].fixed) {
            for (int j = 0; j < 16; j++) o[j] = g.kf[k].Tcw[j];
            continue;
        }
        const SE3 T = load_pose(g.pose + 7 * k);
        const M3 Rm = q_to_rot(T.r);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) o[4 * i + j] = (float)Rm.a[3 * i + j];
        o[3] = (float)T.t.x; o[7] = (float)T.t.y; o[11] = (float)T.t.z;
        o[12] = 0.f; o[13] = 0.f; o[14] = 0.f; o[15] = 1.f;
    }
    for (int i = t; i < g.Np; i += kT)
        for (int j = 0; j < 3; j++) b.pt_out[3 * ((size_t)pb.point_offset + i) + j] = (float)g.X[3 * i + j];
    for (int i = t; i < g.Nq; i += kT)
        for (int j = 0; j < 4; j++) b.pl_out[4 * ((size_t)pb.plane_offset + i) + j] = (float)g.P[4 * i + j];
    if (t == 0) {
        spslam_lba_result* r = b.res + p;
        *r = spslam_lba_result{};
        r->iterations[0] = s.its[0];
        r->iterations[1] = s.its[1];
        r->n_point_outliers = tot0;
        r->n_plane_outliers = tot1;
        r->status = s.fail ? -3 : 0;
        r->trials = s.trials;
        r->stopped = s.stopped;
    }
}

// ---------------------------------------------------------------- the schedule
__global__ __launch_bounds__(kT) void k_lba_g2o(LbgBatch b, LbaConsts C) {
    unsigned char* dyn = lbg_dyn;
    Sh& s = lbg_s;
    const int t = threadIdx.x;
    if (t == 0) {  // the team ticket (lba_g2o's header: membership by arrival)
        const int T = b.team;
        const int slot = __hip_atomic_fetch_add(b.ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s.p = slot / T;
        s.m = slot - s.p * T;
        s.T = T;
        s.gen = 0;
        lbg_g = make_g(b, s.p);
        lbg_c = C;
    }
    __syncthreads();
    const int p = s.p;
    const bool lead = s.m == 0;
    const G& g = lbg_g;
    const long long t0 = wall_clock64();
    if (g.K > kMaxKF) {  // (every member leaves here)
        if (lead && t == 0) {
            b.res[p] = spslam_lba_result{};
            b.res[p].status = -2;
        }
        return;
    }
    if (t == 0) {
        s.stop = 0; s.stopped = 0; s.trials = 0; s.its[0] = s.its[1] = 0; s.fail = 0; s.robust = 1; s.done = 0;
        s.unsup = 0;
        for (int i = 0; i < 8; i++) s.ph[i] = 0;
        for (int i = 0; i < 14; i++) s.dg[i] = 0;
        s.tB = 0;
        s.tlast = t0;
        if (lead) g.team->stop_gen = 0;
    }
    team_sync(b);  // the leader's first sample of pbStopFlag
    if (t == 0 && stop_requested(b, s)) {  // if(*pbStopFlag) return; before initializeOptimization
        s.stopped = 1;
        s.done = 1;
    }
    __syncthreads();
#ifdef SPSLAM_LBG_PROBE  // diagnostic: the cost of the building blocks of the ordered chains inside this kernel
    double probe[4] = {0, 0, 0, 0};
    if (t < 64) {
        const double a = (double)g.E * 1e-9;
        const int lane = t & 63;
        double x = 1.0, yv = (double)lane * 1e-3, z = 0.0;
        long long c0 = clock64();
        for (int i = 0; i < 4096; i++) x = x + a;  // (1) dependent v_add_f64
        long long c1 = clock64();
        for (int i = 0; i < 4096; i++) z = z + rl(yv, i & 63);  // (2) + a v_readlane operand
        long long c2 = clock64();
        int k = lane;
        for (int i = 0; i < 4096; i++) k = __builtin_amdgcn_readlane(k, (k + i) & 63) & 63;  // (3) readlane -> lane select
        long long c3 = clock64();
        probe[0] = (double)(c1 - c0) / 4096;
        probe[1] = (double)(c2 - c1) / 4096;
        probe[2] = (double)(c3 - c2) / 4096;
        probe[3] = x + z + k;
    }
#endif
    if (!s.done && lead) setup();  // (the members wait at the structure pass's team_sync)
    if (t == 0 && g.E == 0) s.done = 1;  // no edges: nothing to optimise, the map goes back through the converters
    __syncthreads();
    for (int pass = 0; pass < 2 && !s.done; pass++) {
        if (lead) {
            structure();
            if (t == 0) g.team->unsup = s.unsup;
        }
        team_sync(b);
        load_team();
        if (s.unsup) break;
        LBG_MARK(1);
        const int n = 6 * s.np;
        // the factorisation's operands in LDS for n <= kLdsN: L, its column structures, the rows' pattern orders, P
        const bool lds = n <= kLdsN;
        const FactorLds fl = factor_lds(n);  // (used when lds)
        uint64_t* LB = (uint64_t*)(dyn + fl.LB);
        int* RO = (int*)(dyn + fl.RO);
        int* RS = (int*)(dyn + fl.RS);
        int* PI = (int*)(dyn + fl.PI);
        if (t == 0) {
            s.it = 0; s.max_it = pass ? 10 : 5; s.need_err = 1;
        }
        __syncthreads();
        // SparseOptimizer::optimize on a graph without active edges (every edge relabelled): nothing to do
        const bool empty = s.nact == 0 || (s.np == 0 && s.nl == 0);
        // SparseOptimizer::optimize(max_it) with OptimizationAlgorithmLevenberg
        for (int it = 0; it < (empty ? 0 : pass ? 10 : 5); it++) {
            if (t == 0 && stop_requested(b, s)) {  // for (...; !terminate(); ...)
                s.stopped = pass == 0 && s.trials == 0 ? 1 : 2;
                s.done = 1;
            }
            __syncthreads();
            if (s.done) break;
            if (s.need_err) {
                LBG_MARK(1);
                errors_phase();
                team_sync(b);
                LBG_MARK(2);
                sums_staged(lbg_pad32(g.E), 0);
                __syncthreads();
                LBG_MARK(3);
            }
            if (t == 0) s.iniChi = s.currentChi;
            build_system();
            team_sync(b);
            LBG_MARK(4);
            if (t == 0) {
                double mx = 0.0;  // computeLambdaInit: the members' maxima
                for (int q = 0; q < s.T; q++) mx = fmax(mx, g.team->mx[q]);
                if (it == 0) { s.lambda = 1e-5 * mx; s.ni = 2; s.nBad = 0; }
                s.qmax = 0;
            }
            __syncthreads();
            double rho = 0.0;
            bool more = true;
            while (more) {
                LBG_MARK(1);
                // the row-group layout for teams of up to 4, and for any member with 16 or more blocks: it reads ~3x
                // fewer LDS bytes per block step than schur()'s lane per entry, which wins when the LDS is busy;
                // schur() splits a block's chain over 36 lanes, which wins for a few short chains (measured:
                // profiles/r06/schur_layouts.txt)
                if (s.T <= b.rows_max_team || s.bo1 - s.bo0 >= 16) schur_rows_any();
                else schur();
                team_sync(b);
                LBG_MARK(5);
                const bool forced = s.trials < 32 && ((b.fail_mask >> s.trials) & 1u);  // (test hook)
                if (lead && forced) {
                    if (t == 0) { s.ok = 0; g.team->ok = 0; }
                } else if (lead) {
                    if (lds) {  // the factorisation's symbolic data into LDS (the other phases use the same LDS)
                        for (int i = t; i < (n + 1) * kNW; i += kT) LB[i] = i < n * kNW ? g.Lbits[i] : 0ull;
                        for (int i = t; i <= n; i += kT) RO[i] = g.rs_off[i];
                        const int nz = g.rs_off[n];
                        for (int i = t; i < nz; i += kT) RS[i] = g.rs_idx[i];
                        for (int i = t; i < n; i += kT) PI[i] = g.Pinv[i];
                        double* SP = (double*)(dyn + fl.SP);  // S, packed upper
                        for (int i = t; i < n * n; i += kT) {
                            const int r = i / n, c = i - r * n;
                            if (r <= c) SP[(c * (c + 1)) / 2 + r] = g.S[i];
                        }
                        __syncthreads();
                    }
#ifdef SPSLAM_LBG_DIAG
                    const long long f0 = wall_clock64();
#endif
                    if (lds && s.dense) {  // every pose coupled, natural order: the rows pipelined over the waves
                        if (n <= 64) factor_dense<1>();
                        else factor_dense<2>();
                        if (t < 64) {
                            if (n <= 64) factor_solve<1, true, true>();
                            else factor_solve<2, true, true>();
                        }
                    } else if (s.dense && n <= kPackN) {  // dense, past the LDS copy: L packed in LDS
                        if (n <= 128) factor_dense_packed<2>();
                        else factor_dense_packed<3>();
                        if (t < 64) {
                            if (n <= 128) solve_dense_packed<2>();
                            else solve_dense_packed<3>();
                        }
                    } else if (t < 64) {
                        if (n <= 64) factor_solve<1, true>();
                        else if (n <= kLdsN) factor_solve<2, true>();
                        else if (n <= 128) factor_solve<2, false>();
                        else if (n <= 192) factor_solve<3, false>();
                        else if (n <= 256) factor_solve<4, false>();
                        else if (kPW == 1 || n <= 384) factor_solve<6, false>();
#if LBG_PW > 1
                        else if (n <= 512) factor_solve<8, false>();
                        else factor_solve<12, false>();
#endif
                    }
                    if (n == 0 && t == 0) s.ok = 1;
#ifdef SPSLAM_LBG_DIAG
                    if (t == 0) s.dg[5] += s.dg[4] - f0;
#endif
                    __syncthreads();
                    if (t == 0) g.team->ok = s.ok;
                }
                team_sync(b);
                if (!lead && t == 0) s.ok = g.team->ok;
                __syncthreads();
                LBG_MARK(6);
                update();
                team_sync(b);
                LBG_MARK(1);
                errors_phase();
                scale_terms();
                team_sync(b);
                LBG_MARK(2);
                sums_staged(lbg_pad32(g.E), lbg_pad32(n + 3 * s.nl));
                __syncthreads();
                LBG_MARK(3);
                if (t == 0) {
                    double tempChi = s.ok ? s.tempChi : DBL_MAX;
                    double r = s.currentChi - tempChi;
                    double scale = s.scale;
                    scale += 1e-3;
                    r /= scale;
                    if (r > 0 && isfinite(tempChi)) {
                        double alpha = 1. - libm64cr::cube_(2 * r - 1);
                        alpha = fmin(alpha, 2. / 3.);
                        s.lambda *= fmax(1. / 3., alpha);
                        s.ni = 2;
                        s.currentChi = tempChi;
                        s.accepted = 1;
                    } else {
                        s.lambda *= s.ni;
                        s.ni *= 2;
                        s.accepted = 0;
                    }
                    s.qmax++;
                    s.trials++;
                    s.red[0][2] = r;
                    const bool stop = stop_requested(b, s);
                    s.flag = r < 0 && s.qmax < 10 && !stop;  // do { ... } while (rho < 0 && qmax < max && !terminate())
                }
                __syncthreads();
                if (!s.accepted) {
                    restore();
                    team_sync(b);
                }
                rho = s.red[0][2];
                more = s.flag;
            }
            if (t == 0) {
                s.need_err = !s.accepted;  // an accepted trial's errors are the new state's (same operands, same bits)
                s.its[pass]++;
                bool term = s.qmax == 10 || rho == 0;
                if (!term) {
                    if ((s.iniChi - s.currentChi) * 1e3 < s.iniChi) s.nBad++;
                    else s.nBad = 0;
                    term = s.nBad >= 3;
                }
                s.flag = term;
                if (s.stop && !term && it + 1 < (pass ? 10 : 5)) {  // the next iteration's terminate() check
                    s.stopped = 2;
                    s.done = 1;
                }
            }
            __syncthreads();
            if (s.flag || s.done) break;
        }
        if (s.done) break;
        if (pass == 0) {
            if (t == 0 && stop_requested(b, s)) {  // bDoMore = !*pbStopFlag
                s.stopped = 2;
                s.done = 1;
            }
            __syncthreads();
            if (s.done) break;
            // relabel with the errors cached by the last computeActiveErrors, drop the robust kernels
            relabel();
            if (t == 0) s.robust = 0;
            team_sync(b);
        }
    }
    team_sync(b);  // every member's writes are in before the leader's outputs
    if (!lead) return;
    if (s.unsup) {  // more free poses than kMaxK: nothing written but the status
        if (t == 0) {
            b.res[p] = spslam_lba_result{};
            b.res[p].status = -2;
        }
        return;
    }
    outputs(b, p);
    if (t == 0) {  // setup / structure / update / decide, errors, ordered chains, terms, Schur, factor + solve, sums
        b.res[p].phase_us[0] = (float)((wall_clock64() - t0) * 0.01);
        for (int i = 1; i < 8; i++) b.res[p].phase_us[i] = (float)(s.ph[i] * 0.01);
        b.res[p].pad = (int)(s.tB * 0.01);  // diagnostic: build phase (B) us
#ifdef SPSLAM_LBG_DIAG_BUILD  // buildSystem: heads, (A) terms, landmark chains, Hpl blocks, pose chains (us); steps
        for (int i = 0; i < 5; i++) b.res[p].phase_us[1 + i] = (float)(s.dg[i] * 0.01);
        b.res[p].pad = (int)s.dg[5];
#endif
#ifdef SPSLAM_LBG_DIAG  // Schur: staging wait, BDinv, chains, commit; factor-only
        for (int i = 0; i < 4; i++) b.res[p].phase_us[1 + i] = (float)(s.dg[i] * 0.01);
        b.res[p].phase_us[5] = (float)(s.dg[6] * 1e-3);  // factor: step-loop shader kcycles,
        b.res[p].phase_us[6] = (float)(s.dg[7] * 1e-3);  //   pivot-update kcycles,
        b.res[p].pad = (int)s.dg[8];                     //   steps
        b.res[p].phase_us[7] = (float)(s.dg[5] * 0.01);
#endif
#ifdef SPSLAM_LBG_DIAG_SCHUR  // Schur chains: kcycles summed over waves, steps, cycles per step, sum of chunk maxima
        b.res[p].phase_us[1] = (float)(s.dg[10] * 1e-3);
        b.res[p].phase_us[2] = (float)s.dg[11];
        b.res[p].phase_us[3] = (float)s.dg[10] / (float)max(1ll, s.dg[11]);
        b.res[p].phase_us[4] = (float)(s.dg[13] * 1e-3);
#endif
#ifdef SPSLAM_LBG_PROBE  // shader-clock ticks per (1) add, (2) add of a readlane, (3) readlane chain
        for (int i = 0; i < 3; i++) b.res[p].phase_us[1 + i] = (float)probe[i];
        if (probe[3] == 12345.0) b.res[p].pad = 1;
#endif
    }
}

}  // namespace LBG_NS

hipError_t LBG_RUN(const LbgBatch& b, const LbaConsts& C, hipStream_t s, KernelTimer* timer) {
    using namespace LBG_NS;
    static const hipError_t attr =
        hipFuncSetAttribute((const void*)k_lba_g2o, hipFuncAttributeMaxDynamicSharedMemorySize, kDynAlloc);
    if (attr != hipSuccess) return attr;
    if (b.team < 1 || b.team > kLbgTeamMax) return hipErrorInvalidValue;
    const hipError_t z = hipMemsetAsync(b.ctl, 0, lbg_ctl_ints(b.n) * sizeof(int), s);
    if (z != hipSuccess) return z;
    if (timer) timer->begin(kKindLba, s);
    hipLaunchKernelGGL(k_lba_g2o, dim3(b.n * b.team), dim3(kT), kDynAlloc, s, b, C);
    if (timer) timer->end(kKindLba, s);
    return hipGetLastError();
}

}  // namespace spslam

#if LBG_PW == 1
namespace spslam {
// the instance of a batch: LbgBatch::pw (lbg_pw_for of its largest window)
hipError_t lba_run_g2o(const LbgBatch& b, const LbaConsts& C, hipStream_t s, KernelTimer* timer) {
    return b.pw == 1 ? lba_run_g2o_pw1(b, C, s, timer) : lba_run_g2o_pw2(b, C, s, timer);
}
}  // namespace spslam
#endif
