// Host-side entry points of lba_kernels.hip (Optimizer::LocalBundleAdjustment).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"

namespace spslam {

constexpr int kLbaMaxKeyframes = 64;   // local + fixed keyframes per problem (pose masks are 64-bit)
constexpr int kLbaChunk = 256;         // edges / landmarks per workgroup in the grid-wide phases
constexpr int kLbaCon = 57;            // per-edge terms: Hll 9, bl 3, Hpl 18 (3x6), Hpp upper 21, bp 6
// Schur complement on the matrix cores (v_mfma_f64_16x16x4): reduced systems of up to kLbaMfmaTiles x 16 rows
// (6 * free poses <= 80); larger ones use the pose-pair kernel.  One partial 16x16-tile set per 64 landmarks.
constexpr int kLbaMfmaTiles = 5;
constexpr int kLbaMfmaLm = 32;  // landmarks per k_schur_mfma wave (per partial tile set)

// LM / schedule state of one problem (device, in its scratch); see lba_kernels.hip.
struct LbaCtl {
    int state;        // 0 STRUCT, 1 ITER, 2 TRIAL, 3 RELABEL, 4 DONE
    int phase, it, max_it, robust, qmax, nBad, np, ok, restore_step, trials, its[2];
    int stop;         // pbStopFlag seen (latched)
    int stopped;      // 1 = before optimize(5) (nothing changed), 2 = schedule cut short
    double lambda, ni, currentChi, iniChi;
    long long t0;     // wall_clock64 at setup (diagnostics)
};

// Per-problem scratch layout (bytes), computed identically on host and device.
struct LbaLayout {
    size_t ctl;
    size_t pose, pose_b, pt, pt_b, pl, pl_b, e_err, e_con, lm_H, lm_b, lm_Dinv, lm_db, lm_x, blk_H, blk_BD, S, bs,
        dd, y, Hpp, bp, part_chi, part_scale, part_max, S_part;                            // double arrays
    size_t pose_hidx, hidx_pose, e_lm, e_kf, e_type, e_level, e_blk, e_src, lm_boff, lm_nb, lm_act, kf_cnt, pe_off,
        pe_idx;                                                                            // int arrays
    size_t lm_mask;                                                                        // uint64
    size_t bytes;
};

__host__ __device__ inline int lba_chunks(int n) { return (n + kLbaChunk - 1) / kLbaChunk; }
// one k_schur_mfma partial set: NT x NT tiles of 16 x 16 (the upper ones written) + the right-hand side (16 NT)
__host__ __device__ inline size_t lba_part_doubles(int nt) { return (size_t)nt * nt * 256 + (size_t)nt * 16; }

__host__ __device__ inline LbaLayout lba_layout(int K, int Np, int Nq, int E) {
    LbaLayout L{};
    const size_t Lm = (size_t)Np + Nq, n6 = 6 * (size_t)K;
    const size_t nEc = lba_chunks(E), nLc = lba_chunks((int)Lm);
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t r = o; o += (bytes + 255) & ~(size_t)255; return r; };
    L.ctl = take(sizeof(LbaCtl));
    L.pose = take(K * 7 * 8); L.pose_b = take(K * 7 * 8);
    L.pt = take(Np * 3 * 8); L.pt_b = take(Np * 3 * 8);
    L.pl = take(Nq * 4 * 8); L.pl_b = take(Nq * 4 * 8);
    L.e_err = take((size_t)E * 3 * 8); L.e_con = take((size_t)E * kLbaCon * 8);
    L.lm_H = take(Lm * 9 * 8); L.lm_b = take(Lm * 3 * 8); L.lm_Dinv = take(Lm * 9 * 8);
    L.lm_db = take(Lm * 3 * 8); L.lm_x = take(Lm * 3 * 8);
    L.blk_H = take((size_t)E * 18 * 8); L.blk_BD = take((size_t)E * 18 * 8);
    L.S = take(n6 * n6 * 8); L.bs = take(n6 * 8); L.dd = take(n6 * 8); L.y = take(n6 * 8);
    L.Hpp = take(K * 36 * 8); L.bp = take(K * 6 * 8);
    L.part_chi = take(nEc * 8); L.part_scale = take(nLc * 8); L.part_max = take((nLc + K) * 8);
    // partial tile sets of k_schur_mfma: NT = max(3, ceil(6 np / 16)) <= kLbaMfmaTiles tiles per dimension,
    // np <= K free poses
    size_t nt = (n6 + 15) / 16;
    nt = nt < 3 ? 3 : (nt > (size_t)kLbaMfmaTiles ? (size_t)kLbaMfmaTiles : nt);
    L.S_part = take(((Lm + kLbaMfmaLm - 1) / kLbaMfmaLm) * lba_part_doubles((int)nt) * 8);
    L.pose_hidx = take(K * 4); L.hidx_pose = take(K * 4);
    L.e_lm = take((size_t)E * 4); L.e_kf = take((size_t)E * 4); L.e_type = take((size_t)E * 4);
    L.e_level = take((size_t)E * 4); L.e_blk = take((size_t)E * 4); L.e_src = take((size_t)E * 4);
    L.lm_boff = take(Lm * 4); L.lm_nb = take(Lm * 4); L.lm_act = take(Lm * 4);
    L.kf_cnt = take(K * 4); L.pe_off = take((K + 1) * 4); L.pe_idx = take((size_t)E * 4);
    L.lm_mask = take(Lm * 8);
    L.bytes = o;
    return L;
}

struct LbaConsts {
    double angle_info, dis_info, par_info, ver_info, plane_chi, vp_chi;  // Optimizer.cc:1489-1500
    double delta_mono, delta_stereo, delta_plane, delta_vp;             // Huber deltas (float sqrt, as g2o gets them)
};

// Work tables of a batch (host-built, device copies): (problem, first index) per workgroup.
struct LbaWork {
    const int2* edge_chunks; int n_edge_chunks;
    const int2* lm_chunks; int n_lm_chunks;
    const int2* kf_tasks; int n_kf_tasks;
    const int2* pair_tasks; int n_pair_tasks;
    const int2* plane_tasks; int n_plane_tasks;  // (problem, first plane edge) per kLbaPlaneEdgesPerTask edges
    const int2* seg_chunks; int n_seg_chunks;    // (problem, first point edge) per seg_own point edges
    const int2* plm_tasks; int n_plm_tasks;      // (problem, first plane landmark) per kLbaChunk / 64 planes
    int seg_own;  // point edges owned per k_point_terms_sums workgroup: kLbaChunk - (most keyframes of a problem
                  // - 1), so the rest of the 256 rows (the halo) holds any landmark's remaining edges
};
// a point has at most one observation per keyframe (MapPoint::mObservations is a map keyed by KeyFrame*)
inline int lba_seg_own(int max_kf) { return kLbaChunk - (max_kf > 1 ? max_kf - 1 : 0); }
constexpr int kLbaPlaneEdgesPerTask = kLbaChunk / 64;  // one wave per plane edge

struct LbaBatch {
    int n;
    const spslam_lba_problem* probs;
    const long long* scratch_off;
    uint8_t* scratch;
    const spslam_lba_keyframe* kfs;
    const spslam_lba_point* pts;
    const spslam_lba_point_obs* pobs;
    const spslam_lba_plane* pls;
    const spslam_lba_plane_obs* plobs;
    float *kf_out, *pt_out, *pl_out;
    uint8_t *pobs_out, *plobs_out;
    spslam_lba_result* res;
    int* active;      // problems not DONE (polled by the host)
    const int32_t* stop;  // per problem pbStopFlag (device-visible; NULL = no flag)
    int stop_after;       // test hook: the flag counts as raised once a problem has run this many trials (-1 off)
};

// ---------------------------------------------------------------------------------------------------------------
// g2o-order LocalBundleAdjustment (lba_g2o.hip, the default): a team of persistent workgroups per problem (one CU
// each) runs the whole schedule with every sum in g2o's order.  Per-problem scratch, computed identically on host and
// device.
constexpr int kLbgThreads = 512;
constexpr int kLbgMaxKeyframes = 1024;  // local + fixed keyframes per problem
constexpr int kLbgMaxFree = 64;         // free (local) poses with an active edge, narrow instance: 64-bit pose masks,
                                        //   n <= 384
constexpr int kLbgMaxFreeWide = 128;    // the wide instance (lba_g2o_wide.hip): two-word pose masks, n <= 768
constexpr int kLbgTeamMax = 16;         // workgroups per problem
// What the team's leader publishes for its members after each structure pass (lba_g2o.hip load_team).
struct LbgTeam {
    int np, nl, nact, nch, nb, ok, unsup;
    int stop_gen;               // the team barrier at which the leader first saw pbStopFlag raised (0: not yet)
    int eb[kLbgTeamMax + 1];    // buildSystem: member m sums the landmarks whose edges are [eb[m], eb[m + 1])
    int npo[kLbgTeamMax + 1];   //   and the (free pose, term) chains of poses pown[npo[m] .. npo[m + 1])
    int pown[kLbgMaxFreeWide];
    int bo[kLbgTeamMax + 1];    // Schur: member m's pattern blocks bord[bo[m] .. bo[m + 1]), the block rows rmask[m]
    uint64_t rmask[2 * kLbgTeamMax];  //   (pw words per member)
    double mx[2 * kLbgTeamMax];  // computeLambdaInit: each member's largest |diagonal| (landmarks, poses)
    uint64_t pat[2 * kLbgMaxFreeWide];  // the Schur pattern's rows (pw words per row)
    short hidx[kLbgMaxKeyframes];
};
// pw: 64-bit words of the instance's pose masks (1: narrow, 2: wide)
__host__ __device__ inline int lbg_free_cap(int K, int pw) { return K < 64 * pw ? K : 64 * pw; }
// the instance a batch runs: wide when a window holds more keyframes than the narrow one's free poses
__host__ __device__ inline int lbg_pw_for(int max_kf) { return max_kf <= kLbgMaxFree ? 1 : 2; }
struct LbgLayout {
    size_t pose, pose_b, X, X_b, P, P_b, err, echi, sc, terms, Hll, bl, Dinv, db, blkB, Hps, S, bs, x, Ld;  // double
    size_t e_lm, e_kf, e_type, e_level, e_src, e_blk, lm_boff, lm_nb, lm_sorted, lm_hidx, hidx_lm, lmh_blk, pe_off,
        pe_idx, Pinv, Pm, parent, rs_off, rs_idx, amd_Ci, amd_W, sch, sch_kb, eseg, bord;                  // int
    size_t lmh_mask, lm_amask, Lbits, Abits;                                                                // uint64
    size_t team;                                                                                            // LbgTeam
    size_t bytes;
};
__host__ __device__ inline int lbg_pad32(int n) { return (n + 31) & ~31; }
// K keyframes (<= kLbgMaxKeyframes), the Hessian-sized arrays for at most lbg_free_cap(K, pw) free poses
__host__ __device__ inline LbgLayout lbg_layout(int K, int Np, int Nq, int E, int pw) {
    LbgLayout Ly{};
    const int Kf = lbg_free_cap(K, pw);
    const size_t L = (size_t)Np + Nq, n = 6 * (size_t)Kf, Ep = lbg_pad32(E), Xn = lbg_pad32((int)(n + 3 * L));
    const size_t nC = n * n + n * n / 5 + 2 * n;  // cs_amd's elbow room over the full symmetric pattern
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t r = o; o += (bytes + 255) & ~(size_t)255; return r; };
    Ly.team = take(sizeof(LbgTeam));
    Ly.pose = take(K * 7 * 8); Ly.pose_b = take(K * 7 * 8);
    Ly.X = take(Np * 3 * 8); Ly.X_b = take(Np * 3 * 8);
    Ly.P = take(Nq * 4 * 8); Ly.P_b = take(Nq * 4 * 8);
    Ly.err = take((size_t)E * 3 * 8); Ly.echi = take(Ep * 8); Ly.sc = take(Xn * 8);
    Ly.terms = take((size_t)E * kLbaCon * 8);
    Ly.Hll = take(L * 9 * 8); Ly.bl = take(L * 3 * 8); Ly.Dinv = take(L * 9 * 8); Ly.db = take(L * 3 * 8);
    Ly.blkB = take((size_t)E * 18 * 8);
    Ly.Hps = take(Kf * 27 * 8); Ly.S = take(n * n * 8); Ly.bs = take(n * 8); Ly.x = take(Xn * 8);
    Ly.Ld = take(n * n * 8);
    Ly.e_lm = take((size_t)E * 4); Ly.e_kf = take((size_t)E * 4); Ly.e_type = take((size_t)E * 4);
    Ly.e_level = take((size_t)E * 4); Ly.e_src = take((size_t)E * 4); Ly.e_blk = take((size_t)E * 4);
    Ly.lm_boff = take(L * 4); Ly.lm_nb = take(L * 4); Ly.lm_sorted = take(L * 4); Ly.lm_hidx = take(L * 4);
    Ly.hidx_lm = take(L * 4); Ly.lmh_blk = take((L + 1) * 4); Ly.pe_off = take((Kf + 1) * 4);
    Ly.pe_idx = take((size_t)E * 4);
    Ly.Pinv = take(n * 4); Ly.Pm = take(n * 4); Ly.parent = take(n * 4); Ly.rs_off = take((n + 1) * 4);
    Ly.rs_idx = take((n * (n + 1) / 2 + 1) * 4);
    Ly.amd_Ci = take((nC + 1) * 4); Ly.amd_W = take(10 * (n + 1) * 4);
    Ly.sch = take((L + 2) * 4); Ly.sch_kb = take((L + 2) * 4); Ly.eseg = take((size_t)E * 16);
    Ly.bord = take(((size_t)Kf * (Kf + 1) / 2 + 1) * 4);
    Ly.lmh_mask = take(L * 8 * pw); Ly.lm_amask = take(L * 8 * pw);
    Ly.Lbits = take((n + 1) * 6 * pw * 8); Ly.Abits = take(n * 6 * pw * 8);
    Ly.bytes = o;
    return Ly;
}
struct LbgBatch {
    int n;
    const spslam_lba_problem* probs;
    const long long* scratch_off;
    uint8_t* scratch;
    const spslam_lba_keyframe* kfs;
    const spslam_lba_point* pts;
    const spslam_lba_point_obs* pobs;
    const spslam_lba_plane* pls;
    const spslam_lba_plane_obs* plobs;
    float *kf_out, *pt_out, *pl_out;
    uint8_t *pobs_out, *plobs_out;
    spslam_lba_result* res;
    const int32_t* stop;  // per problem pbStopFlag (device-visible; NULL = no flag)
    int stop_after;       // test hook: the flag counts as raised once a problem has run this many trials (-1 off)
    int team;             // workgroups per problem (1 .. kLbgTeamMax); the grid is n * team
    unsigned fail_mask;   // test hook: bit q = LM trial q's solve reports failure (spslam_debug_force_solve_failures)
    int* ctl;             // lbg_ctl_ints(n) ints, zeroed before the launch: [0] the workgroups' arrival ticket,
                          //   [16 (p + 1)] problem p's team barrier counter (one 64-byte line each)
    int pw;               // the instance: pose-mask words (lbg_pw_for; the scratch laid out with lbg_layout(..., pw))
    int rows_max_team;    // teams up to this size use the row-group Schur layout (SPSLAM_LBG_ROWS_MAX_TEAM, default 4)
};
__host__ __device__ inline size_t lbg_ctl_ints(int n) { return 16 * ((size_t)n + 1); }
// One launch: the whole optimize(5) / relabel / optimize(10) schedule of every problem, no host round trip.  The
// ctl block is cleared on `s` first.
hipError_t lba_run_g2o(const LbgBatch& b, const LbaConsts& C, hipStream_t s, KernelTimer* timer);
hipError_t lba_run_g2o_pw1(const LbgBatch& b, const LbaConsts& C, hipStream_t s, KernelTimer* timer);
hipError_t lba_run_g2o_pw2(const LbgBatch& b, const LbaConsts& C, hipStream_t s, KernelTimer* timer);

// Runs the whole LocalBundleAdjustment schedule of a batch: enqueues the phase
// kernels step by step on `s` and polls the device every few steps until
// every problem is DONE (so it returns after the work completed).
// stop_src / stop_mirror: a host bool (pbStopFlag of the host-buffer entry point) copied into the
// device-visible flag at every poll (NULL = none).
hipError_t lba_run(const LbaBatch& b, const LbaWork& w, const LbaConsts& C, int max_steps, hipStream_t s,
                   KernelTimer* timer, int* steps_out, const volatile uint8_t* stop_src = nullptr,
                   volatile int32_t* stop_mirror = nullptr);

}  // namespace spslam
