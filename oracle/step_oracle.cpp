// ORACLE -- TEST INFRASTRUCTURE ONLY (bench.py cpu_baseline, tests).
//
// One frame of the benchmarked step in C++, the whole chain of
// oracle/oracle_step.py with no Python between the stages, and a timed loop
// over frames on 1..T threads (one independent frame stream per thread):
//   GrabImageRGBD (src/Tracking.cc:208-229: cvtColor RGB2GRAY + convertTo)
//   -> ORBextractor::operator() + ComputePlanesFromOrganizedPointCloud +
//      GeneratePlanesFromBoundries + the RGB-D Frame keypoint steps
//   -> TrackWithMotionModel (Tracking.cc:951-1000): SearchByProjection,
//      AssociatePlanesByBoundary, the PoseOptimization graph, outlier discard
//   -> TrackLocalMap (Tracking.cc:1055-1068): SearchLocalPoints (seen points
//      skipped), the surviving plane associations re-associated, the graph,
//      PoseOptimization
//   (+ LocalBundleAdjustment every lba_every frames for C3).
// Each stage calls the oracle restatement the Python checker uses (same
// parameters as oracle_step.run), so the result equals oracle_step.run on the
// same inputs (tests/test_oracle_step_cpp.py).
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../include/spslam_gpu.h"

extern "C" {
void* oracle_orb_new(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
void oracle_orb_free(void* h);
int oracle_orb_extract(void* h, const uint8_t* gray, int w, int hgt, int stride, spslam_keypoint* kps, uint8_t* desc,
                       int cap, int* n);
void* oracle_planes_new();
void oracle_planes_free(void* h);
int oracle_planes_extract(void* h, const float* depth, int w, int hgt, int stride, float fx, float fy, float cx,
                          float cy, int cloud_dis, int min_size, float angle_th, float dist_th);
int oracle_planes_dims(void* h, int* W, int* H, int* n_models);
void oracle_planes_cloud(void* h, float* xyz);
void oracle_planes_model(void* h, int i, float* coef, int* n_inliers, int* n_contour);
void oracle_planes_model_contour(void* h, int i, int* out);
int oracle_planes_kept(void* h, int k, float* coef);
void* oracle_supposed_new();
void oracle_supposed_free(void* h);
int oracle_supposed_generate(void* h, const float* depth, int w, int hgt, int stride, const float* cloud_xyz,
                             float fx, float fy, float cx, float cy, int n_planes, const float* coefs,
                             const int* con_off, const int* con_n, const int* contours, double line_ratio,
                             float dis_th, const float* bounds);
int oracle_supposed_plane(void* h, int k, float* coef);
void oracle_frame_rgbd(const float* params10, const float* kxy, int n, const float* depth, int w, int h, int stride,
                       float* un, float* dep, float* ur, int* cell, int* grid_off, int* grid_idx, float* bounds);
int oracle_search_by_projection(const void* frame, const void* points, const void* keys_un, const uint8_t* desc,
                                const float* uright, int n_kp, const int32_t* grid_off, const int32_t* grid_idx,
                                const float* geometry, const void* params, int32_t* match, int* passes);
int oracle_search_local_points(const void* frame, const void* points, const void* keys_un, const uint8_t* desc,
                               const float* uright, int n_kp, const int32_t* grid_off, const int32_t* grid_idx,
                               const float* geometry, const void* params, const uint8_t* taken, int32_t* match,
                               uint8_t* in_view);
int oracle_planes_associate(const float* Tcw, const float* coefs, int n_planes, const void* map_planes, int n_map,
                            const float* boundary_xyz, const float* params, int32_t* match, int32_t* parallel,
                            int32_t* vertical, float* world, double* dist, int carry);
int oracle_pose_optimize(const spslam_pose_problem* P, const spslam_point_obs* pts, const spslam_plane_obs* pls,
                         const spslam_plane_config* cfg, spslam_pose_result* out, uint8_t* pout, uint8_t* plout);
int oracle_lba_optimize(const spslam_lba_problem* P, const spslam_lba_keyframe* kfs, const spslam_lba_point* pts,
                        const spslam_lba_point_obs* pobs, const spslam_lba_plane* pls,
                        const spslam_lba_plane_obs* plobs, const spslam_plane_config* cfg, float* kf_out,
                        float* pt_out, float* pl_out, uint8_t* pobs_outlier, uint8_t* plobs_outlier,
                        spslam_lba_result* res);
}

// Everything one frame reads (host pointers, caller-owned).
struct oracle_step_frame {
    const uint8_t* rgb;            // H x W x 3, R G B (GrabImageRGBD with mbRGB = 1)
    const uint16_t* depth_raw;     // H x W
    int32_t w, h;
    float depth_scale;             // mDepthMapFactor as stored (1 / DepthMapFactor)
    float cam[5];                  // fx fy cx cy bf
    const float* geometry;         // 19 floats (oracle_match geometry)
    const float* inv_sigma2;       // mvInvLevelSigma2 (8)
    const spslam_proj_frame* proj_frame;
    const spslam_proj_point* proj_points;
    const spslam_local_frame* local_frame;
    const spslam_local_point* local_points;
    const spslam_map_plane* map_planes;
    int32_t n_map;
    int32_t min_size;              // Plane.MinSize
    const float* boundary_xyz;
    const spslam_plane_config* pose_cfg;
    int32_t local_seen;            // SearchLocalPoints skips the map points the motion model matched
    int32_t supp_cap;              // supposed planes kept (the GPU path's capacity), < 0 = all
};

// Per-frame outputs of interest (checks and the CPU reference trajectory).
struct oracle_step_out {
    float Tcw1[16], Tcw2[16];
    int32_t n_kps, n_planes, n_supposed, nmatches, local_nmatches, inliers1, inliers2, pad;
};

struct oracle_lba_set {            // C3: the local maps LocalMapping optimises (one per lba_every frames)
    int32_t n, lba_every;
    const spslam_lba_problem* const* prob;
    const spslam_lba_keyframe* const* kfs;
    const spslam_lba_point* const* pts;
    const spslam_lba_point_obs* const* pobs;
    const spslam_lba_plane* const* pls;
    const spslam_lba_plane_obs* const* plobs;
    const spslam_plane_config* cfg;
};

namespace {

constexpr int kCells = 64 * 48, kKpCap = 20000;
constexpr float kAssocParams[4] = {0.2f, 0.8f, 0.08716f, 0.9962f};  // oracle_assoc.ASSOC_PARAMS

struct Worker {
    void* orb;
    void* planes;
    void* supp;
    std::vector<uint8_t> gray, desc, taken;
    std::vector<float> depth, cloud, coefs, kxy, un, dep, ur, bounds;
    std::vector<spslam_keypoint> kps, kun;
    std::vector<int> cell, grid_off, grid_idx, con_off, con_n, con, edge;
    std::vector<int32_t> match, lmatch, lmatch_s, a0[3], a1[3];
    std::vector<uint8_t> in_view, po, plo;
    std::vector<spslam_point_obs> pts;
    std::vector<spslam_plane_obs> pls;
    std::vector<spslam_local_point> lsub;
    std::vector<int> lidx;
    std::vector<float> lba_kf, lba_pt, lba_pl;
    std::vector<uint8_t> lba_po, lba_plo;
    explicit Worker(int nfeatures)
        : orb(oracle_orb_new(nfeatures, 1.2f, 8, 20, 7)), planes(oracle_planes_new()), supp(oracle_supposed_new()) {}
    ~Worker() {
        oracle_orb_free(orb);
        oracle_planes_free(planes);
        oracle_supposed_free(supp);
    }
    Worker(const Worker&) = delete;
    Worker& operator=(const Worker&) = delete;
};

// Optimizer.cc:681-860 edge order: plane edges over the frame planes, then parallel, then vertical
void plane_edges(const float* coefs, int n, const std::vector<int32_t>* a, const spslam_map_plane* M,
                 std::vector<spslam_plane_obs>& out) {
    out.clear();
    for (int kind = 0; kind < 3; kind++)
        for (int i = 0; i < n; i++) {
            const int m = a[kind][i];
            if (m < 0) continue;
            spslam_plane_obs o{};
            std::memcpy(o.meas, coefs + 4 * i, 16);
            std::memcpy(o.world, M[m].world, 16);
            o.kind = kind;
            o.plane_index = i;
            o.map_plane_id = M[m].id;
            out.push_back(o);
        }
}

spslam_pose_problem problem(const float* Tcw, const float* cam, int np, int nq) {
    spslam_pose_problem p{};
    std::memcpy(p.Tcw, Tcw, 64);
    p.fx = cam[0]; p.fy = cam[1]; p.cx = cam[2]; p.cy = cam[3]; p.bf = cam[4];
    p.n_points = np;
    p.n_planes = nq;
    return p;
}

void step_frame(Worker& W, const oracle_step_frame& F, oracle_step_out* out) {
    const int w = F.w, h = F.h, npx = w * h;
    const float fx = F.cam[0], fy = F.cam[1], cx = F.cam[2], cy = F.cam[3], bf = F.cam[4];
    // --- GrabImageRGBD: cvtColor RGB2GRAY (8U fixed point) + convertTo(CV_32F, mDepthMapFactor)
    W.gray.resize(npx);
    W.depth.resize(npx);
    for (int i = 0; i < npx; i++) {
        const uint8_t* c = F.rgb + 3 * (size_t)i;
        W.gray[i] = (uint8_t)((c[0] * 4899 + c[1] * 9617 + c[2] * 1868 + (1 << 13)) >> 14);
        W.depth[i] = (float)F.depth_raw[i] * F.depth_scale;
    }
    // --- ORB
    W.kps.resize(kKpCap);
    W.desc.resize((size_t)kKpCap * 32);
    int n = 0;
    oracle_orb_extract(W.orb, W.gray.data(), w, h, w, W.kps.data(), W.desc.data(), kKpCap, &n);
    // --- planes + supposed planes
    const int n_pl = oracle_planes_extract(W.planes, W.depth.data(), w, h, w, fx, fy, cx, cy, 3, F.min_size, 3.0f,
                                           0.05f);
    int cW, cH, nmod;
    oracle_planes_dims(W.planes, &cW, &cH, &nmod);
    W.cloud.resize((size_t)cW * cH * 3);
    oracle_planes_cloud(W.planes, W.cloud.data());
    W.coefs.assign((size_t)4 * n_pl, 0.f);
    W.con_off.assign(n_pl, 0);
    W.con_n.assign(n_pl, 0);
    W.con.clear();
    for (int k = 0; k < n_pl; k++) {
        const int m = oracle_planes_kept(W.planes, k, &W.coefs[4 * k]);
        float mc[4];
        int ninl, ncon;
        oracle_planes_model(W.planes, m, mc, &ninl, &ncon);
        W.con_off[k] = (int)W.con.size();
        W.con_n[k] = ncon;
        W.con.resize(W.con.size() + ncon);
        if (ncon) oracle_planes_model_contour(W.planes, m, W.con.data() + W.con_off[k]);
    }
    if (W.con.empty()) W.con.push_back(0);
    int n_supp = oracle_supposed_generate(W.supp, W.depth.data(), w, h, w, W.cloud.data(), fx, fy, cx, cy, n_pl,
                                          W.coefs.data(), W.con_off.data(), W.con_n.data(), W.con.data(), 0.2, 0.01f,
                                          nullptr);
    if (F.supp_cap >= 0 && n_supp > F.supp_cap) n_supp = F.supp_cap;
    const int nc = n_pl + n_supp;
    W.coefs.resize((size_t)4 * nc);
    for (int k = 0; k < n_supp; k++) oracle_supposed_plane(W.supp, k, &W.coefs[4 * (n_pl + k)]);
    // --- RGB-D Frame keypoint steps (no distortion, as oracle_step.run)
    W.kxy.resize(2 * (size_t)std::max(n, 1));
    for (int i = 0; i < n; i++) { W.kxy[2 * i] = W.kps[i].x; W.kxy[2 * i + 1] = W.kps[i].y; }
    const float p10[10] = {fx, fy, cx, cy, 0.f, 0.f, 0.f, 0.f, 0.f, bf};
    const size_t n1 = std::max(n, 1);
    W.un.resize(2 * n1); W.dep.resize(n1); W.ur.resize(n1); W.cell.resize(n1); W.grid_idx.resize(n1);
    W.grid_off.resize(kCells + 1); W.bounds.resize(4);
    oracle_frame_rgbd(p10, W.kxy.data(), n, W.depth.data(), w, h, w, W.un.data(), W.dep.data(), W.ur.data(),
                      W.cell.data(), W.grid_off.data(), W.grid_idx.data(), W.bounds.data());
    W.kun.assign(W.kps.begin(), W.kps.begin() + n);
    for (int i = 0; i < n; i++) { W.kun[i].x = W.un[2 * i]; W.kun[i].y = W.un[2 * i + 1]; }
    if (W.kun.empty()) W.kun.resize(1);
    // --- TrackWithMotionModel
    const spslam_proj_frame& PF = *F.proj_frame;
    const spslam_proj_point* P = F.proj_points;
    W.match.assign(n1, -1);
    int32_t prm[4];
    const float th = 15.0f;
    std::memcpy(&prm[0], &th, 4);
    prm[1] = 0; prm[2] = 1; prm[3] = 20;
    int passes = 0;
    const int nm = oracle_search_by_projection(&PF, PF.n_points ? P : nullptr, W.kun.data(), W.desc.data(),
                                               W.ur.data(), n, W.grid_off.data(), W.grid_idx.data(), F.geometry, prm,
                                               W.match.data(), &passes);
    const size_t nc1 = std::max(nc, 1);
    for (int k = 0; k < 3; k++) W.a0[k].assign(nc1, -1);
    oracle_planes_associate(PF.Tcw, W.coefs.data(), nc, F.n_map ? F.map_planes : nullptr, F.n_map, F.boundary_xyz,
                            kAssocParams, W.a0[0].data(), W.a0[1].data(), W.a0[2].data(), nullptr, nullptr, 0);
    W.pts.clear();
    W.edge.assign(n1, -1);
    for (int i = 0; i < n; i++) {  // Optimizer.cc:561-640, keypoint order
        const int m = W.match[i];
        if (m < 0) continue;
        spslam_point_obs o{};
        o.u = W.kun[i].x; o.v = W.kun[i].y; o.ur = W.ur[i]; o.inv_sigma2 = F.inv_sigma2[W.kun[i].octave];
        std::memcpy(o.xw, P[m].xw, 12);
        o.kp_index = i;
        W.edge[i] = (int)W.pts.size();
        W.pts.push_back(o);
    }
    plane_edges(W.coefs.data(), nc, W.a0, F.map_planes, W.pls);
    spslam_pose_problem pb1 = problem(PF.Tcw, F.cam, (int)W.pts.size(), (int)W.pls.size());
    spslam_pose_result r1{};
    W.po.assign(std::max<size_t>(W.pts.size(), 1), 0);
    W.plo.assign(std::max<size_t>(W.pls.size(), 1), 0);
    oracle_pose_optimize(&pb1, W.pts.data(), W.pls.data(), F.pose_cfg, &r1, W.po.data(), W.plo.data());
    // discard (Tracking.cc:986-1000) + the taken test of SearchLocalPoints (ORBmatcher.cc:95-97)
    W.taken.assign(n1, 0);
    std::vector<uint8_t> keep(n1, 0);
    for (int i = 0; i < n; i++) {
        const int e = W.edge[i];
        if (e >= 0 && !W.po[e]) {
            keep[i] = 1;
            W.taken[i] = P[W.match[i]].n_obs > 0;
        }
    }
    // --- TrackLocalMap: SearchLocalPoints at the first optimised pose
    spslam_local_frame LF = *F.local_frame;
    std::memcpy(LF.Tcw, r1.Tcw, 64);
    const float lsf = std::log(1.2f);  // Frame::mfLogScaleFactor (glibc logf)
    int32_t lprm[8] = {0, 0, 0, 0, 8, 0, 0, 0};
    const float lp[4] = {3.0f, 0.8f, 0.5f, lsf};
    std::memcpy(lprm, lp, 16);
    W.lmatch.assign(n1, -1);
    int nlm;
    if (F.local_seen) {  // mnLastFrameSeen: the points this frame's motion-model matches hold are skipped
        std::unordered_set<int> seen;
        for (int i = 0; i < n; i++)
            if (W.match[i] >= 0) seen.insert(P[W.match[i]].id);
        W.lsub.clear();
        W.lidx.clear();
        for (int j = 0; j < LF.n_points; j++)
            if (!seen.count(F.local_points[j].id)) {
                W.lsub.push_back(F.local_points[j]);
                W.lidx.push_back(j);
            }
        spslam_local_frame LS = LF;
        LS.n_points = (int)W.lsub.size();
        W.in_view.assign(std::max<size_t>(W.lsub.size(), 1), 0);
        W.lmatch_s.assign(n1, -1);
        nlm = oracle_search_local_points(&LS, W.lsub.empty() ? nullptr : W.lsub.data(), W.kun.data(), W.desc.data(),
                                         W.ur.data(), n, W.grid_off.data(), W.grid_idx.data(), F.geometry, lprm,
                                         W.taken.data(), W.lmatch_s.data(), W.in_view.data());
        for (int i = 0; i < n; i++) W.lmatch[i] = W.lmatch_s[i] >= 0 ? W.lidx[W.lmatch_s[i]] : -1;
    } else {
        W.in_view.assign(std::max(LF.n_points, 1), 0);
        nlm = oracle_search_local_points(&LF, LF.n_points ? F.local_points : nullptr, W.kun.data(), W.desc.data(),
                                         W.ur.data(), n, W.grid_off.data(), W.grid_idx.data(), F.geometry, lprm,
                                         W.taken.data(), W.lmatch.data(), W.in_view.data());
    }
    // the second association starts from the first one's survivors (Tracking.cc:1004-1028, Map.cc:230-252)
    int e = 0;
    for (int k = 0; k < 3; k++) {
        W.a1[k] = W.a0[k];
        for (int i = 0; i < nc; i++)
            if (W.a1[k][i] >= 0) {
                if (W.plo[e]) W.a1[k][i] = -1;
                e++;
            }
    }
    oracle_planes_associate(r1.Tcw, W.coefs.data(), nc, F.n_map ? F.map_planes : nullptr, F.n_map, F.boundary_xyz,
                            kAssocParams, W.a1[0].data(), W.a1[1].data(), W.a1[2].data(), nullptr, nullptr, 1);
    W.pts.clear();
    for (int i = 0; i < n; i++) {  // local-map match, else the kept motion-model match
        const float* xw;
        if (W.lmatch[i] >= 0) xw = F.local_points[W.lmatch[i]].xw;
        else if (keep[i]) xw = P[W.match[i]].xw;
        else continue;
        spslam_point_obs o{};
        o.u = W.kun[i].x; o.v = W.kun[i].y; o.ur = W.ur[i]; o.inv_sigma2 = F.inv_sigma2[W.kun[i].octave];
        std::memcpy(o.xw, xw, 12);
        o.kp_index = i;
        W.pts.push_back(o);
    }
    plane_edges(W.coefs.data(), nc, W.a1, F.map_planes, W.pls);
    spslam_pose_problem pb2 = problem(r1.Tcw, F.cam, (int)W.pts.size(), (int)W.pls.size());
    spslam_pose_result r2{};
    W.po.assign(std::max<size_t>(W.pts.size(), 1), 0);
    W.plo.assign(std::max<size_t>(W.pls.size(), 1), 0);
    oracle_pose_optimize(&pb2, W.pts.data(), W.pls.data(), F.pose_cfg, &r2, W.po.data(), W.plo.data());
    if (out) {
        std::memcpy(out->Tcw1, r1.Tcw, 64);
        std::memcpy(out->Tcw2, r2.Tcw, 64);
        out->n_kps = n;
        out->n_planes = n_pl;
        out->n_supposed = n_supp;
        out->nmatches = nm;
        out->local_nmatches = nlm;
        out->inliers1 = r1.n_inliers;
        out->inliers2 = r2.n_inliers;
    }
}

void local_ba(Worker& W, const oracle_lba_set& S, int k) {
    const spslam_lba_problem& p = *S.prob[k];
    W.lba_kf.resize(16 * (size_t)std::max(p.n_kf, 1));
    W.lba_pt.resize(3 * (size_t)std::max(p.n_points, 1));
    W.lba_pl.resize(4 * (size_t)std::max(p.n_planes, 1));
    W.lba_po.resize(std::max(p.n_point_obs, 1));
    W.lba_plo.resize(std::max(p.n_plane_obs, 1));
    spslam_lba_result r{};
    oracle_lba_optimize(&p, S.kfs[k], S.pts[k], S.pobs[k], S.pls[k], S.plobs[k], S.cfg, W.lba_kf.data(),
                        W.lba_pt.data(), W.lba_pl.data(), W.lba_po.data(), W.lba_plo.data(), &r);
}

}  // namespace

extern "C" {

// One frame (the checker of the C++ chain against oracle_step.run).
int oracle_step_frame_run(const oracle_step_frame* F, int nfeatures, oracle_step_out* out) {
    Worker W(nfeatures);
    step_frame(W, *F, out);
    return 0;
}

extern "C" void oracle_set_libm(int mode);  // pose_oracle.cpp: this thread's PoseOptimization / LBA libm

// Timed loop: n_threads workers, each its own frame stream (thread t starts at distinct frame t) running
// `warmup` untimed frames, a barrier, then `timed` frames (+ one LocalBundleAdjustment per lba_every frames when
// lba is given).  elapsed[t] = thread t's timed seconds; outs (may be NULL) = thread 0's outputs of the distinct
// frames, from its warm-up and timed frames (needs warmup + timed >= n_frames to cover them all).  libm: the
// workers' elementary functions (oracle_set_libm: 0 correctly rounded, 1 the host glibc).
int oracle_step_bench(const oracle_step_frame* frames, int n_frames, int nfeatures, int warmup, int timed,
                      int n_threads, const oracle_lba_set* lba, oracle_step_out* outs, double* elapsed, int libm) {
    if (n_frames < 1 || n_threads < 1 || timed < 0 || warmup < 0) return -1;
    std::atomic<int> ready{0};
    std::vector<std::thread> th;
    auto body = [&](int t) {
        oracle_set_libm(libm);
        Worker W(nfeatures);
        oracle_step_out o;
        int k = 0;
        auto frame = [&](int j) {
            const int f = (t + j) % n_frames;
            step_frame(W, frames[f], &o);
            if (t == 0 && outs && j < n_frames) outs[f] = o;
            if (lba && lba->n > 0 && lba->lba_every > 0 && j % lba->lba_every == 0)
                local_ba(W, *lba, (j / lba->lba_every) % lba->n);
        };
        for (; k < warmup; k++) frame(k);
        ready.fetch_add(1);
        while (ready.load() < n_threads) std::this_thread::yield();
        const auto t0 = std::chrono::steady_clock::now();
        for (int j = 0; j < timed; j++, k++) frame(k);
        elapsed[t] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    for (int t = 1; t < n_threads; t++) th.emplace_back(body, t);
    body(0);
    for (auto& x : th) x.join();
    oracle_set_libm(0);
    return 0;
}

}  // extern "C"
