// C ABI (include/spslam_gpu.h) over the gfx950 ORB kernels.
//
// The context owns: the level tables of ORBextractor (src/ORBextractor.cc:
// 410-470), the pyramid geometry, device scratch for `max_batch` frames and a
// HIP stream.  Nothing here falls back to a CPU path: if the HIP runtime or
// the gfx950 code object is unusable every entry point returns SPSLAM_ERR_HIP.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <sstream>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/spslam_gpu.h"
#include "orb_launch.h"
#include "plane_launch.h"
#include "pose_launch.h"
#include "supposed_launch.h"
#include "frame_launch.h"
#include "lba_launch.h"
#include "assoc_launch.h"
#include "bow_launch.h"
#include "match_launch.h"
#include "track_launch.h"
#include "grab_launch.h"

using namespace spslam;

// HIP-event timer per kernel kind; events recorded on the launch stream.
struct EventTimer : KernelTimer {
    struct Pair { int kind; hipEvent_t e0, e1; };
    std::vector<Pair> pending;
    std::vector<hipEvent_t> pool;
    double total_ms[kNumKernelKinds] = {};
    long long count[kNumKernelKinds] = {};
    hipEvent_t cur[kNumKernelKinds] = {};
    hipEvent_t get() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
    void begin(int kind, hipStream_t s) override { cur[kind] = get(); (void)hipEventRecord(cur[kind], s); }
    void end(int kind, hipStream_t s) override {
        hipEvent_t e1 = get();
        (void)hipEventRecord(e1, s);
        pending.push_back(Pair{kind, cur[kind], e1});
    }
    void collect() {
        for (auto& p : pending) {
            float ms = 0.f;
            if (hipEventSynchronize(p.e1) == hipSuccess && hipEventElapsedTime(&ms, p.e0, p.e1) == hipSuccess) {
                total_ms[p.kind] += ms;
                count[p.kind] += 1;
            }
            pool.push_back(p.e0);
            pool.push_back(p.e1);
        }
        pending.clear();
    }
    void reset() { collect(); for (int k = 0; k < kNumKernelKinds; k++) { total_ms[k] = 0; count[k] = 0; } }
    ~EventTimer() override {
        for (auto& p : pending) { (void)hipEventDestroy(p.e0); (void)hipEventDestroy(p.e1); }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

struct spslam_ctx {
    int device = 0;
    int num_cus = 256;  // compute units of the device (spslam_create)
    hipStream_t stream = nullptr;
    spslam_orb_params p{};
    std::string err;
    // ORBextractor tables
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> nfeat;
    int umax[16]{};
    OrbGeom geom{};
    long long pyr_frame_stride = 0, blur_frame_stride = 0;
    int max_kp = 0;
    // device buffers
    uint8_t* d_pyr = nullptr;
    uint8_t* d_blur = nullptr;
    uint8_t* d_score = nullptr;
    OrbBuffers b{};
    uint8_t* d_in = nullptr;
    spslam_keypoint* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int* d_cnt = nullptr;
    // last call (debug stage access)
    const uint8_t* last_gray = nullptr;
    size_t last_frame_stride = 0;
    int last_stride = 0, last_frames = 0;
    EventTimer* timer = nullptr;
    // drop-in PoseOptimization staging
    uint8_t* d_pose_scratch = nullptr;
    size_t pose_scratch_bytes = 0;
    // plane stage
    bool planes_ready = false;
    PlaneGeom pg{};
    PlaneBuffers pb{};
    float* plane_cloud[2] = {nullptr, nullptr};  // organized-cloud sets (spslam_planes_select_cloud_set)
    int cloud_set = 0;
    // the depth output whose cloud a fused grab wrote into each set (spslam_grab_fuse_cloud); null = none
    struct CloudTag { const float* depth = nullptr; int n = 0; } cloud_tag[2];
    bool grab_cloud = [] { const char* e = getenv("SPSLAM_GRAB_CLOUD"); return e && e[0] == '1'; }();
    void* d_plane_scratch = nullptr;
    float* d_depth_in = nullptr;
    spslam_plane* d_planes1 = nullptr;
    int* d_plane_cnt1 = nullptr;
    int32_t* d_inl1 = nullptr;
    int32_t* d_con1 = nullptr;
    int plane_last_frames = 0;
    // supposed-plane stage (GeneratePlanesFromBoundries)
    SuppParams sp{};
    SuppBuffers sb{};
    void* d_supp_scratch = nullptr;
    spslam_supposed_plane* d_supp1 = nullptr;
    int* d_supp_cnt1 = nullptr;
    int32_t* d_line1 = nullptr;
    float* d_patch1 = nullptr;
    int supp_last_frames = 0;
    // RGB-D frame stage (UndistortKeyPoints / ComputeStereoFromRGBD / AssignFeaturesToGrid)
    bool frame_ready = false;
    FrameGeom fg{};
    uint8_t* d_frame1 = nullptr;  // single-frame staging: kps, keys_un, depth, uR, grid_off, grid_idx, count
    // LocalBundleAdjustment scratch (grown on demand)
    uint8_t* d_lba_scratch = nullptr;
    size_t lba_scratch_bytes = 0;
    long long* d_lba_off = nullptr;
    hipStream_t orb_aux = nullptr;  // orb_launch's second stream (the small pyramid levels' chain)
    hipEvent_t orb_fork = nullptr, orb_join = nullptr;
    int32_t* h_lba_stop = nullptr;    // host-mapped coherent pbStopFlag mirror of spslam_lba_optimize
    int32_t* d_lba_stop = nullptr;    // its device alias (hipHostGetDevicePointer)
    int lba_stop_after = -1;          // spslam_lba_debug_stop_after
    int lba_order = SPSLAM_LBA_G2O_ORDER;  // spslam_lba_set_order
    int lba_team = 0;                 // spslam_lba_set_team (0: as many workgroups per problem as fill the chip)
    int* d_lba_ctl = nullptr;         // the g2o-order launch's tickets and team barrier counters
    size_t lba_ctl_cap = 0;           //   (ints)
    hipEvent_t lba_done = nullptr;    // recorded after each LBA launch: the next call's stream waits on it before it
                                      //   rewrites the offsets, the ctl block or the scratch (one LBA call in flight
                                      //   per context, whatever the streams)
    int pose_spin_cap = 0;            // spslam_debug_pose_spin_cap (0 = the kernel's default)
    unsigned solve_fail_mask = 0;     // spslam_debug_force_solve_failures
    int lba_off_cap = 0;
    uint8_t* d_lba_stage = nullptr;   // drop-in staging
    size_t lba_stage_bytes = 0;
    int2* d_lba_work = nullptr;       // (problem, first index) work tables + the active counter
    size_t lba_work_cap = 0;
    // plane association: per (frame, frame plane, map plane) boundary distances
    float* d_assoc_dist = nullptr;
    size_t assoc_dist_bytes = 0;
    // projection matching: per (frame, last-frame point) windows + accepted-match lists
    uint8_t* d_match_scratch = nullptr;
    size_t match_scratch_bytes = 0;
    // bag of words: the vocabulary (one HBM blob), per-feature transform scratch, drop-in staging
    uint8_t* d_vocab = nullptr;
    VocabDev vocab{};
    uint8_t* d_bow_scratch = nullptr;
    size_t bow_scratch_bytes = 0;
    uint8_t* d_bow_stage = nullptr;
    size_t bow_stage_bytes = 0;
};

namespace {

int fail(spslam_ctx* c, int code, const char* fmt, const char* what = "") {
    if (c) {
        char buf[512];
        std::snprintf(buf, sizeof buf, fmt, what);
        c->err = buf;
    }
    return code;
}
#define HIP_CHECK(ctx, expr)                                                                  \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(ctx, SPSLAM_ERR_HIP, #expr ": %s", hipGetErrorString(e_)); \
    } while (0)

int cv_round(float v) { return (int)std::nearbyint(v); }

// ORBextractor::ORBextractor tables, src/ORBextractor.cc:415-469.
void build_tables(spslam_ctx* c) {
    const int nl = c->p.nlevels;
    const double scaleFactor = c->p.scale_factor;  // member is double, ctor arg float
    c->scale.assign(nl, 1.f); c->sigma2.assign(nl, 1.f);
    for (int i = 1; i < nl; i++) {
        c->scale[i] = (float)(c->scale[i - 1] * scaleFactor);
        c->sigma2[i] = c->scale[i] * c->scale[i];
    }
    c->inv_scale.resize(nl); c->inv_sigma2.resize(nl);
    for (int i = 0; i < nl; i++) {
        c->inv_scale[i] = 1.0f / c->scale[i];
        c->inv_sigma2[i] = 1.0f / c->sigma2[i];
    }
    c->nfeat.assign(nl, 0);
    float factor = (float)(1.0f / scaleFactor);
    float nDesired = c->p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
    int sum = 0;
    for (int l = 0; l < nl - 1; l++) {
        c->nfeat[l] = cv_round(nDesired);
        sum += c->nfeat[l];
        nDesired *= factor;
    }
    c->nfeat[nl - 1] = std::max(c->p.nfeatures - sum, 0);
    const int HP = 15;
    int v, v0, vmax = (int)std::floor(HP * std::sqrt(2.f) / 2 + 1), vmin = (int)std::ceil(HP * std::sqrt(2.f) / 2);
    const double hp2 = HP * HP;
    for (v = 0; v <= vmax; ++v) c->umax[v] = (int)std::nearbyint(std::sqrt(hp2 - v * v));
    for (v = HP, v0 = 0; v >= vmin; --v) {
        while (c->umax[v0] == c->umax[v0 + 1]) ++v0;
        c->umax[v] = v0;
        ++v0;
    }
}

// Pyramid + FAST-cell geometry (src/ORBextractor.cc:769-787, 1111-1112) and
// scratch layout.  Returns an error string for unsupported shapes.
const char* build_geom(spslam_ctx* c) {
    OrbGeom& g = c->geom;
    std::memset(&g, 0, sizeof g);
    g.nlevels = c->p.nlevels;
    long long pyr = 0, blur = 0;
    int cells = 0, kpb = 0, keyb = 0;
    for (int l = 0; l < g.nlevels; l++) {
        LevelGeom& L = g.lv[l];
        L.w = cv_round((float)c->p.width * c->inv_scale[l]);
        L.h = cv_round((float)c->p.height * c->inv_scale[l]);
        if (L.w > 4095 || L.h > 4095) return "level wider/taller than 4095 px";
        L.maxBorderX = L.w - kEdgeThreshold + 3;
        L.maxBorderY = L.h - kEdgeThreshold + 3;
        const float width = (float)(L.maxBorderX - kMinBorder), height = (float)(L.maxBorderY - kMinBorder);
        L.nCols = (int)(width / 30.f);
        L.nRows = (int)(height / 30.f);
        if (L.nCols < 1 || L.nRows < 1) return "pyramid level smaller than one FAST cell (reference divides by zero)";
        L.wCell = (int)std::ceil(width / L.nCols);
        L.hCell = (int)std::ceil(height / L.nRows);
        if (L.wCell + 6 > kCellWinMax || L.hCell + 6 > kCellWinMax) return "FAST cell window exceeds LDS tile";
        if (((L.wCell + 1) / 2) * ((L.hCell + 1) / 2) > kCellCap) return "FAST cell survivor bound exceeds kCellCap";
        const int nIni = (int)std::round(width / height);
        if (nIni < 1 || 4 * nIni > 64) return "unsupported aspect ratio for DistributeOctTree";
        L.cell_base = cells;
        cells += L.nCols * L.nRows;
        if (L.nCols * L.nRows > 2048) return "too many FAST cells per level";
        L.nfeat = c->nfeat[l];
        L.kp_cap = std::max(L.nfeat + 16, 4 * nIni + 4);
        if (L.kp_cap > kNodeCap) return "nfeatures per level exceeds DistributeOctTree node capacity";
        L.kp_base = kpb;
        kpb += L.kp_cap;
        L.key_base = keyb;
        keyb += L.nCols * L.nRows * kCellCap;
        L.scale = c->scale[l];
        L.patch_size = (int)(31 * c->scale[l]);
        // pitched rows (multiple of 64 bytes): level_kernel writes 4 pixels per dword store, its 64-wide
        // tiles never cross a row's padded end
        L.bpitch = (L.w + kLevelTileW - 1) / kLevelTileW * kLevelTileW;
        if (l > 0) {
            L.stride = L.bpitch;
            L.img = reinterpret_cast<const uint8_t*>(pyr);  // offset, rebased after allocation
            pyr += (long long)L.stride * L.h;
        }
        L.blur = reinterpret_cast<uint8_t*>(blur);
        L.score = reinterpret_cast<uint8_t*>(blur);
        blur += (long long)L.bpitch * L.h;
        L.tiles_x = (L.w + kLevelTileW - 1) / kLevelTileW;
        g.level_tiles[l] = L.tiles_x * ((L.h + kLevelTileH - 1) / kLevelTileH);
        if (l > 0) {
            L.rscale_x = 1. / ((double)L.w / g.lv[l - 1].w);
            L.rscale_y = 1. / ((double)L.h / g.lv[l - 1].h);
        }
    }
    c->pyr_frame_stride = (pyr + 255) / 256 * 256;
    c->blur_frame_stride = (blur + 255) / 256 * 256;
    g.cells_per_frame = cells;
    g.lvl_kp_per_frame = kpb;
    g.keys_per_frame = keyb;
    c->max_kp = kpb;
    return nullptr;
}

void free_all(spslam_ctx* c) {
    void* ptrs[] = {c->d_pyr,    c->d_blur,   c->d_score,         c->b.cand,          c->b.cand_cnt,     c->b.keys,
                    c->b.keynode, c->b.lvl_kp, c->b.lvl_cnt,       c->d_in,           c->d_kps,
                    c->d_desc,   c->d_cnt,    c->d_pose_scratch,  c->d_plane_scratch, c->d_depth_in,
                    c->d_planes1, c->d_plane_cnt1, c->d_inl1,     c->d_con1,   c->d_supp_scratch,
                    c->d_supp1,   c->d_supp_cnt1,  c->d_line1,    c->d_patch1,  c->d_frame1,
                    c->d_lba_scratch, c->d_lba_off, c->d_lba_stage, c->d_lba_work, c->d_assoc_dist, c->d_match_scratch,
                    c->d_vocab, c->d_bow_scratch, c->d_bow_stage, c->d_lba_ctl};
    if (c->lba_done) (void)hipEventSynchronize(c->lba_done);
    for (void* q : ptrs)
        if (q) (void)hipFree(q);
    if (c->lba_done) (void)hipEventDestroy(c->lba_done);
    if (c->h_lba_stop) (void)hipHostFree(c->h_lba_stop);
    if (c->orb_fork) (void)hipEventDestroy(c->orb_fork);
    if (c->orb_join) (void)hipEventDestroy(c->orb_join);
    if (c->orb_aux) (void)hipStreamDestroy(c->orb_aux);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c->timer;
    c->timer = nullptr;
}

// Point level 0 at the caller's frames and levels >= 1 at the context pyramid.
void bind_frames(spslam_ctx* c, const uint8_t* d_gray, size_t frame_stride, int stride) {
    OrbGeom& g = c->geom;
    g.lv[0].img = d_gray;
    g.lv[0].stride = stride;
    g.lv[0].frame_stride = (long long)frame_stride;
}

}  // namespace

extern "C" {

int spslam_create(int device, const spslam_orb_params* params, spslam_ctx** out) {
    if (!params || !out) return SPSLAM_ERR_ARG;
    *out = nullptr;
    spslam_ctx* c = new (std::nothrow) spslam_ctx();
    if (!c) return SPSLAM_ERR_ARG;
    c->device = device;
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            c->num_cus = cus;
    }
    c->p = *params;
    if (c->p.nlevels < 1 || c->p.nlevels > SPSLAM_MAX_LEVELS || c->p.nfeatures < 1 || c->p.scale_factor <= 1.f ||
        c->p.width < 64 || c->p.height < 64 || c->p.max_batch < 1) {
        delete c;
        return SPSLAM_ERR_ARG;
    }
    build_tables(c);
    if (const char* e = build_geom(c)) {
        delete c;
        std::fprintf(stderr, "spslam_create: %s\n", e);
        return SPSLAM_ERR_ARG;
    }
    int rc = SPSLAM_OK;
    auto hip_ok = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == SPSLAM_OK) {
            rc = fail(c, SPSLAM_ERR_HIP, "%s", what);
            c->err += std::string(": ") + hipGetErrorString(e);
        }
        return e == hipSuccess;
    };
    if (!hip_ok(hipSetDevice(device), "hipSetDevice") ||
        !hip_ok(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate") ||
        !hip_ok(orb_upload_tables(c->umax), "upload tables")) {
        std::fprintf(stderr, "spslam_create: %s\n", c->err.c_str());
        free_all(c);
        delete c;
        return SPSLAM_ERR_HIP;
    }
    const size_t B = (size_t)c->p.max_batch;
    const OrbGeom& g = c->geom;
    hip_ok(hipMalloc(&c->d_pyr, B * c->pyr_frame_stride), "alloc pyramid");
    hip_ok(hipMalloc(&c->d_blur, B * c->blur_frame_stride), "alloc blur");
    hip_ok(hipMalloc(&c->d_score, B * c->blur_frame_stride), "alloc FAST scores");
    hip_ok(hipMalloc(&c->b.cand, B * g.cells_per_frame * kCellCap * sizeof(uint32_t)), "alloc cand");
    hip_ok(hipMalloc(&c->b.cand_cnt, B * g.cells_per_frame * sizeof(uint16_t)), "alloc cand_cnt");
    hip_ok(hipMalloc(&c->b.keys, B * g.keys_per_frame * sizeof(uint32_t)), "alloc keys");
    hip_ok(hipMalloc(&c->b.keynode, B * g.keys_per_frame * sizeof(uint16_t)), "alloc keynode");
    hip_ok(hipMalloc(&c->b.lvl_kp, B * g.lvl_kp_per_frame * sizeof(LevelKp)), "alloc lvl_kp");
    hip_ok(hipMalloc(&c->b.lvl_cnt, B * kMaxLevels * sizeof(int)), "alloc lvl_cnt");
    hip_ok(hipMalloc(&c->d_in, (size_t)c->p.width * c->p.height), "alloc input");
    hip_ok(hipMalloc(&c->d_kps, (size_t)c->max_kp * sizeof(spslam_keypoint)), "alloc kps");
    hip_ok(hipMalloc(&c->d_desc, (size_t)c->max_kp * 32), "alloc desc");
    hip_ok(hipMalloc(&c->d_cnt, sizeof(int) * 4), "alloc cnt");
    if (rc != SPSLAM_OK) {
        std::fprintf(stderr, "spslam_create: %s\n", c->err.c_str());
        free_all(c);
        delete c;
        return rc;
    }
    // rebase level offsets onto the allocations
    OrbGeom& gm = c->geom;
    for (int l = 0; l < gm.nlevels; l++) {
        LevelGeom& L = gm.lv[l];
        if (l > 0) {
            L.img = c->d_pyr + reinterpret_cast<long long>(L.img);
            L.frame_stride = c->pyr_frame_stride;
        }
        L.blur = c->d_blur + reinterpret_cast<long long>(L.blur);
        L.score = c->d_score + reinterpret_cast<long long>(L.score);
        L.blur_frame_stride = c->blur_frame_stride;
    }
    *out = c;
    return SPSLAM_OK;
}

void spslam_destroy(spslam_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    free_all(ctx);
    delete ctx;
}

const char* spslam_last_error(const spslam_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int spslam_orb_tables(const spslam_ctx* c, int* nlevels, float* scale, float* inv_scale, float* sigma2,
                      float* inv_sigma2, int* fpl) {
    if (!c) return SPSLAM_ERR_ARG;
    const int nl = c->p.nlevels;
    if (nlevels) *nlevels = nl;
    for (int l = 0; l < nl; l++) {
        if (scale) scale[l] = c->scale[l];
        if (inv_scale) inv_scale[l] = c->inv_scale[l];
        if (sigma2) sigma2[l] = c->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = c->inv_sigma2[l];
        if (fpl) fpl[l] = c->nfeat[l];
    }
    return SPSLAM_OK;
}

int spslam_orb_max_keypoints(const spslam_ctx* c) { return c ? c->max_kp : SPSLAM_ERR_ARG; }

int spslam_orb_level_size(const spslam_ctx* c, int level, int* w, int* h) {
    if (!c || level < 0 || level >= c->p.nlevels) return SPSLAM_ERR_ARG;
    *w = c->geom.lv[level].w;
    *h = c->geom.lv[level].h;
    return SPSLAM_OK;
}

int spslam_orb_extract_batch_device(spslam_ctx* c, const uint8_t* d_gray, int n_frames, size_t frame_stride,
                                    int stride, spslam_keypoint* d_kps, uint8_t* d_desc, int* d_counts,
                                    int cap_per_frame, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (!d_gray || !d_kps || !d_desc || !d_counts || n_frames < 1 || n_frames > c->p.max_batch ||
        stride < c->p.width || (n_frames > 1 && frame_stride < (size_t)stride * c->p.height) || cap_per_frame < 1)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_orb_extract_batch_device");
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the default stream (header)
    bind_frames(c, d_gray, frame_stride, stride);
    if (!c->orb_aux) {  // the small levels' chain (orb_launch)
        HIP_CHECK(c, hipStreamCreateWithFlags(&c->orb_aux, hipStreamNonBlocking));
        HIP_CHECK(c, hipEventCreateWithFlags(&c->orb_fork, hipEventDisableTiming));
        HIP_CHECK(c, hipEventCreateWithFlags(&c->orb_join, hipEventDisableTiming));
    }
    HIP_CHECK(c, orb_launch(c->geom, c->b, n_frames, c->p.ini_th_fast, c->p.min_th_fast, d_kps, d_desc, d_counts,
                            cap_per_frame, s, c->timer, c->orb_aux, c->orb_fork, c->orb_join));
    c->last_gray = d_gray;
    c->last_frame_stride = frame_stride;
    c->last_stride = stride;
    c->last_frames = n_frames;
    return SPSLAM_OK;
}

int spslam_orb_extract(spslam_ctx* c, const uint8_t* gray, int w, int h, int stride, spslam_keypoint* kps,
                       uint8_t* desc, int cap, int* n) {
    if (!c || !n) return SPSLAM_ERR_ARG;
    if (w == 0 || h == 0 || !gray) {  // reference: empty image -> return, outputs untouched
        *n = 0;
        return SPSLAM_OK;
    }
    if (w != c->p.width || h != c->p.height || stride < w)
        return fail(c, SPSLAM_ERR_ARG, "image size does not match the context%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, hipMemcpy2DAsync(c->d_in, w, gray, stride, w, h, hipMemcpyHostToDevice, c->stream));
    int rc = spslam_orb_extract_batch_device(c, c->d_in, 1, (size_t)w * h, w, c->d_kps, c->d_desc, c->d_cnt,
                                             c->max_kp, c->stream);
    if (rc) return rc;
    int cnt = 0;
    HIP_CHECK(c, hipMemcpyAsync(&cnt, c->d_cnt, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    *n = cnt;
    if (cnt > cap) return fail(c, SPSLAM_ERR_CAPACITY, "keypoint buffer too small%s", "");
    if (cnt > 0) {
        if (kps) HIP_CHECK(c, hipMemcpy(kps, c->d_kps, cnt * sizeof(spslam_keypoint), hipMemcpyDeviceToHost));
        if (desc) HIP_CHECK(c, hipMemcpy(desc, c->d_desc, (size_t)cnt * 32, hipMemcpyDeviceToHost));
    }
    return SPSLAM_OK;
}

int spslam_pose_optimize_batch_device(spslam_ctx* c, int n, const spslam_pose_problem* d_problems,
                                      const spslam_point_obs* d_points, const spslam_plane_obs* d_planes,
                                      const spslam_plane_config* cfg, const spslam_pose_result* d_init_from,
                                      spslam_pose_result* d_results, uint8_t* d_point_outlier,
                                      uint8_t* d_plane_outlier, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (n < 0 || !cfg || (n > 0 && (!d_problems || !d_points || !d_results || !d_point_outlier)))
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_pose_optimize_batch_device");
    if (n == 0) return SPSLAM_OK;
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the default stream (header)
    PoseConsts K = make_pose_consts(*cfg);
    if (c->pose_spin_cap != 0) K.spin_cap = c->pose_spin_cap;
    K.fail_mask = c->solve_fail_mask;
    if (c->timer) c->timer->begin(kKindPose, s);
    HIP_CHECK(c, pose_launch(n, d_problems, d_points, d_planes, K, d_init_from, d_results, d_point_outlier,
                             d_plane_outlier, s));
    if (c->timer) c->timer->end(kKindPose, s);
    return SPSLAM_OK;
}

int spslam_pose_optimize(spslam_ctx* c, const spslam_pose_problem* problem, const spslam_point_obs* points,
                         const spslam_plane_obs* planes, const spslam_plane_config* cfg, spslam_pose_result* result,
                         uint8_t* point_outlier, uint8_t* plane_outlier) {
    if (!c || !problem || !cfg || !result) return SPSLAM_ERR_ARG;
    const int np = problem->n_points, nl = problem->n_planes;
    if (np < 0 || nl < 0 || (np && (!points || !point_outlier)) || (nl && (!planes || !plane_outlier)))
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_pose_optimize");
    HIP_CHECK(c, hipSetDevice(c->device));
    const size_t need = sizeof(spslam_pose_problem) + sizeof(spslam_pose_result) +
                        (size_t)np * (sizeof(spslam_point_obs) + 1) + (size_t)nl * (sizeof(spslam_plane_obs) + 1) +
                        256;
    if (need > c->pose_scratch_bytes) {
        if (c->d_pose_scratch) (void)hipFree(c->d_pose_scratch);
        c->d_pose_scratch = nullptr;
        c->pose_scratch_bytes = 0;
        HIP_CHECK(c, hipMalloc(&c->d_pose_scratch, need * 2));
        c->pose_scratch_bytes = need * 2;
    }
    uint8_t* base = c->d_pose_scratch;
    auto carve = [&](size_t bytes) { uint8_t* p = base; base += (bytes + 15) / 16 * 16; return p; };
    auto* d_prob = (spslam_pose_problem*)carve(sizeof(spslam_pose_problem));
    auto* d_res = (spslam_pose_result*)carve(sizeof(spslam_pose_result));
    auto* d_pts = (spslam_point_obs*)carve((size_t)np * sizeof(spslam_point_obs));
    auto* d_pls = (spslam_plane_obs*)carve((size_t)nl * sizeof(spslam_plane_obs));
    auto* d_po = carve((size_t)np + 1);
    auto* d_plo = carve((size_t)nl + 1);
    spslam_pose_problem prob = *problem;
    prob.point_offset = 0;
    prob.plane_offset = 0;
    HIP_CHECK(c, hipMemcpyAsync(d_prob, &prob, sizeof prob, hipMemcpyHostToDevice, c->stream));
    if (np) HIP_CHECK(c, hipMemcpyAsync(d_pts, points, np * sizeof(spslam_point_obs), hipMemcpyHostToDevice, c->stream));
    if (nl) HIP_CHECK(c, hipMemcpyAsync(d_pls, planes, nl * sizeof(spslam_plane_obs), hipMemcpyHostToDevice, c->stream));
    int rc = spslam_pose_optimize_batch_device(c, 1, d_prob, d_pts, d_pls, cfg, nullptr, d_res, d_po, d_plo, c->stream);
    if (rc) return rc;
    HIP_CHECK(c, hipMemcpyAsync(result, d_res, sizeof *result, hipMemcpyDeviceToHost, c->stream));
    if (np) HIP_CHECK(c, hipMemcpyAsync(point_outlier, d_po, np, hipMemcpyDeviceToHost, c->stream));
    if (nl) HIP_CHECK(c, hipMemcpyAsync(plane_outlier, d_plo, nl, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return SPSLAM_OK;
}

}  // extern "C"

namespace {

// GeneratePlanesFromBoundries constants and scratch (supposed_kernels.hip).
hipError_t configure_supposed(spslam_ctx* c, const spslam_plane_params* p) {
    const PlaneGeom& g = c->pg;
    SuppParams& sp = c->sp;
    sp.line_ratio = p->line_ratio;
    // (double)s < (double)th * th  <=>  s <= sqr_th_f
    const double T = (double)p->line_distance_threshold * (double)p->line_distance_threshold;
    float f = (float)T;
    while ((double)f >= T && f > 0.f) f = std::nextafter(f, 0.f);
    while ((double)std::nextafter(f, 1.f) < T) f = std::nextafter(f, 1.f);
    sp.sqr_th_f = f;
    const bool nob = p->image_bounds[0] == 0.f && p->image_bounds[1] == 0.f && p->image_bounds[2] == 0.f &&
                     p->image_bounds[3] == 0.f;
    sp.min_x = nob ? 0.f : p->image_bounds[0];
    sp.max_x = nob ? (float)p->width : p->image_bounds[1];
    sp.min_y = nob ? 0.f : p->image_bounds[2];
    sp.max_y = nob ? (float)p->height : p->image_bounds[3];
    sp.supp_cap = kMaxSuppPerFrame;
    sp.line_cap = g.contour_cap;
    // CaculatePlanes' loop: for (float i = -0.25; i < 0.25;) { ...; i = i + 0.01; } (double step)
    int ns = 0;
    for (float v = -0.25f; v < 0.25f; v = (float)((double)v + 0.01)) {
        if (ns >= kMaxPatchSteps) return hipErrorInvalidValue;
        sp.steps[ns++] = v;
    }
    sp.n_steps = ns;
    const size_t F = (size_t)c->p.max_batch, CC = (size_t)g.contour_cap;
    SuppBuffers& b = c->sb;
    const size_t bytes = (size_t)kSuppRndTable * 4 +
                         F * kMaxPlanesPerFrame * kMaxLinesPerBoundary * sizeof(LineCand) +
                         F * kMaxPlanesPerFrame * sizeof(int) + F * CC * (4 + 16 + 4 + 1) +
                         F * kMaxPlanesPerFrame * 8 * sizeof(long long) + 9 * 256;
    if (c->d_supp_scratch) (void)hipFree(c->d_supp_scratch);
    c->d_supp_scratch = nullptr;
    hipError_t e = hipMalloc(&c->d_supp_scratch, bytes);
    if (e != hipSuccess) return e;
    uint8_t* q = (uint8_t*)c->d_supp_scratch;
    auto carve = [&](size_t n) { uint8_t* r = q; q += (n + 255) / 256 * 256; return r; };
    b.rnd = (const uint32_t*)carve((size_t)kSuppRndTable * 4);
    b.cand = (LineCand*)carve(F * kMaxPlanesPerFrame * kMaxLinesPerBoundary * sizeof(LineCand));
    b.n_cand = (int*)carve(F * kMaxPlanesPerFrame * sizeof(int));
    b.line_idx = (int32_t*)carve(F * CC * 4);
    b.big = (float4*)carve(F * CC * 16);
    b.big_sh = (int*)carve(F * CC * 4);
    b.big_flag = (uint8_t*)carve(F * CC);
    b.prof = (long long*)carve(F * kMaxPlanesPerFrame * 8 * sizeof(long long));
    e = hipMemset(b.prof, 0, F * kMaxPlanesPerFrame * 8 * sizeof(long long));
    if (e != hipSuccess) return e;
    // every SACSegmentation::segment() seeds boost::mt19937(12345u); rnd() = uniform_int<>(0, INT_MAX) = mt() >> 1
    std::vector<uint32_t> tab(kSuppRndTable);
    std::mt19937 mt(12345u);
    for (auto& v : tab) v = (uint32_t)mt() >> 1;
    e = hipMemcpy((void*)b.rnd, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) return e;
    void* olds[] = {c->d_supp1, c->d_supp_cnt1, c->d_line1, c->d_patch1};
    for (void* o : olds)
        if (o) (void)hipFree(o);
    const size_t patch = (size_t)sp.n_steps * sp.n_steps;
    if ((e = hipMalloc(&c->d_supp1, sp.supp_cap * sizeof(spslam_supposed_plane))) != hipSuccess) return e;
    if ((e = hipMalloc(&c->d_supp_cnt1, 16)) != hipSuccess) return e;
    if ((e = hipMalloc(&c->d_line1, CC * 4)) != hipSuccess) return e;
    return hipMalloc(&c->d_patch1, sp.supp_cap * patch * 12);
}

}  // namespace

extern "C" {

int spslam_planes_configure(spslam_ctx* c, const spslam_plane_params* p) {
    if (!c || !p) return SPSLAM_ERR_ARG;
    if (p->cloud_dis < 1 || p->width < 1 || p->height < 1 || p->fx == 0.f || p->fy == 0.f)
        return fail(c, SPSLAM_ERR_ARG, "bad plane parameters%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    PlaneGeom& g = c->pg;
    g.w = p->width;
    g.h = p->height;
    g.ds = p->cloud_dis;
    g.W = (int)std::ceil(p->width / (float)p->cloud_dis);
    g.H = (int)std::ceil(p->height / (float)p->cloud_dis);
    g.N = g.W * g.H;
    if (g.H > 512) return fail(c, SPSLAM_ERR_ARG, "organized cloud taller than 512 rows%s", "");
    if (g.N > 160000) return fail(c, SPSLAM_ERR_ARG, "organized cloud larger than the LDS state map%s", "");
    if (3 * 10 * g.W * 4 > 65536) return fail(c, SPSLAM_ERR_ARG, "organized cloud wider than the LDS row band%s", "");
    g.fx = p->fx; g.fy = p->fy; g.cx = p->cx; g.cy = p->cy;
    g.min_size = p->min_size;
    g.ang_cos = std::cos((float)(0.017453 * p->angle_threshold));  // cosf(static_cast<float>(0.017453*AngTh))
    g.dist_th = p->distance_threshold;
    g.inlier_cap = g.N;
    g.contour_cap = 4 * g.N;
    const long long N = g.N, F = c->p.max_batch, IWH = (long long)(g.W + 1) * (g.H + 1);
    PlaneBuffers& b = c->pb;
    const long long SH = wave_size(g.W, g.H);
    b.cloud_fs = 3 * N; b.wave_fs = SH; b.dist_fs = N; b.integral_fs = 6 * (IWH + g.W + 1); b.normal_fs = 3 * N; b.pd_fs = N;
    b.labels_fs = N; b.work_fs = 4 * N; b.grown_fs = N; b.maps_fs = 2 * N;
    const size_t bytes = F * (sizeof(float) * (2 * b.cloud_fs + b.wave_fs + b.dist_fs + b.normal_fs + b.pd_fs) +
                              sizeof(double) * b.integral_fs + sizeof(uint32_t) * b.labels_fs +
                              sizeof(int) * (b.work_fs + b.grown_fs) + b.maps_fs + 16 * sizeof(long long)) + 8192;
    if (c->d_plane_scratch) (void)hipFree(c->d_plane_scratch);
    c->d_plane_scratch = nullptr;
    HIP_CHECK(c, hipMalloc(&c->d_plane_scratch, bytes));
    uint8_t* q = (uint8_t*)c->d_plane_scratch;
    auto carve = [&](size_t n) { uint8_t* r = q; q += (n + 255) / 256 * 256; return r; };
    b.integral = (double*)carve(F * b.integral_fs * sizeof(double));
    c->plane_cloud[0] = (float*)carve(F * b.cloud_fs * 4);
    c->plane_cloud[1] = (float*)carve(F * b.cloud_fs * 4);
    b.cloud = c->plane_cloud[0];
    c->cloud_set = 0;
    c->cloud_tag[0] = c->cloud_tag[1] = {};
    b.wave = (float*)carve(F * b.wave_fs * 4);
    b.dist = (float*)carve(F * b.dist_fs * 4);
    b.normal = (float*)carve(F * b.normal_fs * 4);
    b.pd = (float*)carve(F * b.pd_fs * 4);
    b.labels = (uint32_t*)carve(F * b.labels_fs * 4);
    b.work = (int*)carve(F * b.work_fs * 4);
    b.grown = (int*)carve(F * b.grown_fs * 4);
    b.maps = (uint8_t*)carve(F * b.maps_fs);
    b.ts = (long long*)carve(F * 16 * sizeof(long long));
    void* olds[] = {c->d_depth_in, c->d_planes1, c->d_plane_cnt1, c->d_inl1, c->d_con1};
    for (void* o : olds)
        if (o) (void)hipFree(o);
    HIP_CHECK(c, hipMalloc(&c->d_depth_in, (size_t)g.w * g.h * sizeof(float)));
    HIP_CHECK(c, hipMalloc(&c->d_planes1, kMaxPlanesPerFrame * sizeof(spslam_plane)));
    HIP_CHECK(c, hipMalloc(&c->d_plane_cnt1, 16));
    HIP_CHECK(c, hipMalloc(&c->d_inl1, (size_t)g.inlier_cap * 4));
    HIP_CHECK(c, hipMalloc(&c->d_con1, (size_t)g.contour_cap * 4));
    HIP_CHECK(c, configure_supposed(c, p));
    c->planes_ready = true;
    return SPSLAM_OK;
}

int spslam_planes_capacity(const spslam_ctx* c, int* planes_cap, int* inlier_cap, int* contour_cap) {
    if (!c || !c->planes_ready) return SPSLAM_ERR_NOT_READY;
    if (planes_cap) *planes_cap = kMaxPlanesPerFrame;
    if (inlier_cap) *inlier_cap = c->pg.inlier_cap;
    if (contour_cap) *contour_cap = c->pg.contour_cap;
    return SPSLAM_OK;
}

int spslam_planes_extract_batch_device(spslam_ctx* c, const float* d_depth, int n_frames, size_t frame_stride,
                                       int stride_floats, spslam_plane* d_planes, int* d_counts,
                                       int32_t* d_inliers, int32_t* d_contours, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (!c->planes_ready) return fail(c, SPSLAM_ERR_NOT_READY, "spslam_planes_configure not called%s", "");
    if (!d_depth || !d_planes || !d_counts || !d_inliers || !d_contours || n_frames < 1 ||
        n_frames > c->p.max_batch || stride_floats < c->pg.w)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_planes_extract_batch_device");
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the default stream (header)
    // a fused grab already wrote this depth's cloud into the selected set (spslam_grab_fuse_cloud)
    auto& tag = c->cloud_tag[c->cloud_set];
    const bool have_cloud = tag.depth == d_depth && n_frames <= tag.n &&
                            frame_stride == (size_t)c->pg.w * c->pg.h && stride_floats == c->pg.w;
    tag = {};
    HIP_CHECK(c, plane_launch(c->pg, c->pb, n_frames, d_depth, (long long)frame_stride, stride_floats, d_planes,
                              d_counts, kMaxPlanesPerFrame, d_inliers, d_contours, s, c->timer, have_cloud));
    c->plane_last_frames = n_frames;
    return SPSLAM_OK;
}

int spslam_planes_extract(spslam_ctx* c, const float* depth, int w, int h, int stride_floats, spslam_plane* planes,
                          int planes_cap, int* n_planes, int32_t* inliers, int32_t* contours) {
    if (!c || !n_planes) return SPSLAM_ERR_ARG;
    if (!c->planes_ready) return fail(c, SPSLAM_ERR_NOT_READY, "spslam_planes_configure not called%s", "");
    if (!depth || w != c->pg.w || h != c->pg.h || stride_floats < w)
        return fail(c, SPSLAM_ERR_ARG, "depth size does not match the plane configuration%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, hipMemcpy2DAsync(c->d_depth_in, (size_t)w * 4, depth, (size_t)stride_floats * 4, (size_t)w * 4, h,
                                  hipMemcpyHostToDevice, c->stream));
    int rc = spslam_planes_extract_batch_device(c, c->d_depth_in, 1, (size_t)w * h, w, c->d_planes1, c->d_plane_cnt1,
                                                c->d_inl1, c->d_con1, c->stream);
    if (rc) return rc;
    int n = 0;
    spslam_plane tmp[kMaxPlanesPerFrame];
    HIP_CHECK(c, hipMemcpyAsync(&n, c->d_plane_cnt1, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(tmp, c->d_planes1, sizeof tmp, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    *n_planes = n;
    if (n > planes_cap) return fail(c, SPSLAM_ERR_CAPACITY, "plane buffer too small%s", "");
    int ni = 0, nc = 0;
    for (int k = 0; k < n; k++) {
        planes[k] = tmp[k];
        ni = std::max(ni, tmp[k].inlier_offset + tmp[k].n_inliers);
        nc = std::max(nc, tmp[k].contour_offset + tmp[k].n_contour);
    }
    if (inliers && ni) HIP_CHECK(c, hipMemcpy(inliers, c->d_inl1, (size_t)ni * 4, hipMemcpyDeviceToHost));
    if (contours && nc) HIP_CHECK(c, hipMemcpy(contours, c->d_con1, (size_t)nc * 4, hipMemcpyDeviceToHost));
    return SPSLAM_OK;
}

int spslam_supposed_capacity(const spslam_ctx* c, int* supp_cap, int* line_cap, int* patch_points) {
    if (!c || !c->planes_ready) return SPSLAM_ERR_NOT_READY;
    if (supp_cap) *supp_cap = c->sp.supp_cap;
    if (line_cap) *line_cap = c->sp.line_cap;
    if (patch_points) *patch_points = c->sp.n_steps * c->sp.n_steps;
    return SPSLAM_OK;
}

int spslam_planes_select_cloud_set(spslam_ctx* c, int set) {
    if (!c) return SPSLAM_ERR_ARG;
    if (!c->planes_ready) return fail(c, SPSLAM_ERR_NOT_READY, "spslam_planes_configure not called%s", "");
    if (set < 0 || set > 1) return fail(c, SPSLAM_ERR_ARG, "cloud set not 0 or 1%s", "");
    c->pb.cloud = c->plane_cloud[set];
    c->cloud_set = set;
    return SPSLAM_OK;
}

int spslam_planes_generate_from_boundaries_batch_device(spslam_ctx* c, const float* d_depth, int n_frames,
                                                        size_t frame_stride, int stride_floats,
                                                        const spslam_plane* d_planes, const int* d_counts,
                                                        const int32_t* d_contours, spslam_supposed_plane* d_out,
                                                        int* d_out_counts, int32_t* d_line_idx, float* d_patch,
                                                        void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (!c->planes_ready) return fail(c, SPSLAM_ERR_NOT_READY, "spslam_planes_configure not called%s", "");
    if (!d_depth || !d_planes || !d_counts || !d_contours || !d_out || !d_out_counts || !d_line_idx || !d_patch ||
        n_frames < 1 || stride_floats < c->pg.w)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_planes_generate_from_boundaries_batch_device");
    if (n_frames > c->plane_last_frames)
        return fail(c, SPSLAM_ERR_NOT_READY, "%s", "more frames than the last plane extraction holds");
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the default stream (header)
    HIP_CHECK(c, supp_launch(c->pg, c->pb, c->sp, c->sb, n_frames, d_depth, (long long)frame_stride, stride_floats,
                             d_planes, d_counts, d_contours, d_out, d_out_counts, d_line_idx, d_patch, s, c->timer));
    c->supp_last_frames = n_frames;
    return SPSLAM_OK;
}

int spslam_planes_generate_from_boundaries(spslam_ctx* c, const float* depth, int w, int h, int stride_floats,
                                           spslam_supposed_plane* out, int cap, int* n, int32_t* line_idx,
                                           float* patch_xyz) {
    if (!c || !n) return SPSLAM_ERR_ARG;
    if (!c->planes_ready) return fail(c, SPSLAM_ERR_NOT_READY, "spslam_planes_configure not called%s", "");
    if (!depth || w != c->pg.w || h != c->pg.h || stride_floats < w)
        return fail(c, SPSLAM_ERR_ARG, "depth size does not match the plane configuration%s", "");
    if (c->plane_last_frames < 1) return fail(c, SPSLAM_ERR_NOT_READY, "%s", "spslam_planes_extract not called");
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, hipMemcpy2DAsync(c->d_depth_in, (size_t)w * 4, depth, (size_t)stride_floats * 4, (size_t)w * 4, h,
                                  hipMemcpyHostToDevice, c->stream));
    int rc = spslam_planes_generate_from_boundaries_batch_device(c, c->d_depth_in, 1, (size_t)w * h, w, c->d_planes1,
                                                                 c->d_plane_cnt1, c->d_con1, c->d_supp1,
                                                                 c->d_supp_cnt1, c->d_line1, c->d_patch1, c->stream);
    if (rc) return rc;
    int m = 0;
    std::vector<spslam_supposed_plane> tmp(c->sp.supp_cap);
    HIP_CHECK(c, hipMemcpyAsync(&m, c->d_supp_cnt1, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(tmp.data(), c->d_supp1, tmp.size() * sizeof(spslam_supposed_plane),
                                hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    *n = m;
    const int stored = std::min(m, c->sp.supp_cap);
    if (m > cap || m > c->sp.supp_cap) return fail(c, SPSLAM_ERR_CAPACITY, "supposed-plane buffer too small%s", "");
    int nl = 0;
    for (int k = 0; k < stored; k++) {
        out[k] = tmp[k];
        nl = std::max(nl, tmp[k].line_offset + tmp[k].n_line);
    }
    const size_t patch = (size_t)c->sp.n_steps * c->sp.n_steps;
    if (line_idx && nl) HIP_CHECK(c, hipMemcpy(line_idx, c->d_line1, (size_t)nl * 4, hipMemcpyDeviceToHost));
    if (patch_xyz && stored)
        HIP_CHECK(c, hipMemcpy(patch_xyz, c->d_patch1, stored * patch * 12, hipMemcpyDeviceToHost));
    return SPSLAM_OK;
}

int spslam_debug_plane_not_seen(spslam_ctx* c, const float* planes, int n_planes, const float* coefs, int n_coefs,
                                int* not_seen) {
    if (!c || n_planes < 0 || n_coefs < 0 || (n_planes && !planes) || (n_coefs && (!coefs || !not_seen)))
        return SPSLAM_ERR_ARG;
    if (!n_coefs) return SPSLAM_OK;
    HIP_CHECK(c, hipSetDevice(c->device));
    const size_t pb = (size_t)std::max(n_planes, 1) * 16, cb = (size_t)n_coefs * 16;
    uint8_t* q = nullptr;
    HIP_CHECK(c, hipMallocAsync((void**)&q, pb + cb + (size_t)n_coefs * 4, c->stream));
    if (n_planes) HIP_CHECK(c, hipMemcpyAsync(q, planes, (size_t)n_planes * 16, hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(q + pb, coefs, cb, hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(c, plane_not_seen_debug_launch((const float*)q, n_planes, (const float*)(q + pb), n_coefs,
                                             (int*)(q + pb + cb), c->stream));
    HIP_CHECK(c, hipMemcpyAsync(not_seen, q + pb + cb, (size_t)n_coefs * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipFreeAsync(q, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return SPSLAM_OK;
}

int spslam_debug_force_solve_failures(spslam_ctx* c, unsigned trial_mask) {
    if (!c) return SPSLAM_ERR_ARG;
    c->solve_fail_mask = trial_mask;
    return SPSLAM_OK;
}

int spslam_debug_pose_spin_cap(spslam_ctx* c, int cap) {
    if (!c || cap < -1) return SPSLAM_ERR_ARG;
    c->pose_spin_cap = cap;
    return SPSLAM_OK;
}

int spslam_debug_plane_labels(spslam_ctx* c, int keep) {
    if (!c) return SPSLAM_ERR_ARG;
    c->pb.keep_labels = keep ? 1 : 0;
    return SPSLAM_OK;
}

int spslam_debug_libm64(spslam_ctx* c, int kind, const double* a, const double* b, int n, double* out) {
    if (!c || n < 0 || kind < 0 || kind > 3 || (n && (!a || !out || (kind == 2 && !b)))) return SPSLAM_ERR_ARG;
    if (!n) return SPSLAM_OK;
    HIP_CHECK(c, hipSetDevice(c->device));
    const size_t nb = (size_t)n * 8;
    uint8_t* q = nullptr;
    HIP_CHECK(c, hipMallocAsync((void**)&q, 3 * nb, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(q, a, nb, hipMemcpyHostToDevice, c->stream));
    if (kind == 2) HIP_CHECK(c, hipMemcpyAsync(q + nb, b, nb, hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(c, libm64_debug_launch(kind, (const double*)q, (const double*)(q + nb), n, (double*)(q + 2 * nb),
                                     c->stream));
    HIP_CHECK(c, hipMemcpyAsync(out, q + 2 * nb, nb, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipFreeAsync(q, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return SPSLAM_OK;
}

int spslam_supposed_debug(spslam_ctx* c, int frame, int plane, spslam_line_candidate* cand, int* n_cand,
                          int32_t* idx, int idx_cap) {
    static_assert(sizeof(spslam_line_candidate) == sizeof(LineCand), "candidate layout");
    if (!c || !cand || !n_cand) return SPSLAM_ERR_ARG;
    if (frame < 0 || frame >= c->supp_last_frames || plane < 0 || plane >= kMaxPlanesPerFrame)
        return fail(c, SPSLAM_ERR_NOT_READY, "no supposed-plane data for that frame%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, hipDeviceSynchronize());
    int nc = 0;
    HIP_CHECK(c, hipMemcpy(&nc, c->sb.n_cand + frame * kMaxPlanesPerFrame + plane, sizeof(int), hipMemcpyDeviceToHost));
    nc = std::min(std::max(nc, 0), kMaxLinesPerBoundary);
    LineCand lc[kMaxLinesPerBoundary];
    if (nc)
        HIP_CHECK(c, hipMemcpy(lc, c->sb.cand + ((size_t)frame * kMaxPlanesPerFrame + plane) * kMaxLinesPerBoundary,
                               nc * sizeof(LineCand), hipMemcpyDeviceToHost));
    *n_cand = nc;
    int lo = 0;
    for (int k = 0; k < nc; k++) {
        std::memcpy(&cand[k], &lc[k], sizeof(LineCand));
        if (lc[k].flags & 1) {
            const int m = lc[k].n_inliers;
            if (idx && lo + m <= idx_cap && m)
                HIP_CHECK(c, hipMemcpy(idx + lo, c->sb.line_idx + (size_t)frame * c->pg.contour_cap + lc[k].idx_off,
                                       (size_t)m * 4, hipMemcpyDeviceToHost));
            cand[k].idx_offset = lo;
            lo += m;
        } else {
            cand[k].idx_offset = -1;
        }
    }
    return lo > idx_cap ? SPSLAM_ERR_CAPACITY : SPSLAM_OK;
}

int spslam_planes_debug(spslam_ctx* c, int frame, int what, void* out, int* n_points) {
    if (!c || !out) return SPSLAM_ERR_ARG;
    if (!c->planes_ready || frame < 0 || frame >= c->plane_last_frames)
        return fail(c, SPSLAM_ERR_NOT_READY, "no plane data for that frame%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, hipDeviceSynchronize());
    const PlaneBuffers& b = c->pb;
    const long long N = c->pg.N;
    if (n_points) *n_points = (int)N;
    if (what == 0 || what == 1) {  // SoA on device -> AoS x,y,z
        const float* src = what == 0 ? b.cloud + frame * b.cloud_fs : b.normal + frame * b.normal_fs;
        std::vector<float> soa(3 * N);
        HIP_CHECK(c, hipMemcpy(soa.data(), src, 3 * N * 4, hipMemcpyDeviceToHost));
        float* o = (float*)out;
        for (long long i = 0; i < N; i++) { o[3 * i] = soa[i]; o[3 * i + 1] = soa[N + i]; o[3 * i + 2] = soa[2 * N + i]; }
        return SPSLAM_OK;
    }
    if (what == 2) {
        HIP_CHECK(c, hipMemcpy(out, b.dist + frame * b.dist_fs, N * 4, hipMemcpyDeviceToHost));
        return SPSLAM_OK;
    }
    if (what == 3) {
        bool in_lds = false;
        plane_segment_lds_bytes(c->pg, &in_lds);
        if (in_lds && !b.keep_labels)
            return fail(c, SPSLAM_ERR_NOT_READY, "labels are kept only after spslam_debug_plane_labels(ctx, 1)%s", "");
        HIP_CHECK(c, hipMemcpy(out, b.labels + frame * b.labels_fs, N * 4, hipMemcpyDeviceToHost));
        return SPSLAM_OK;
    }
    if (what == 4) {
        HIP_CHECK(c, hipMemcpy(out, b.ts + frame * 16, 16 * sizeof(long long), hipMemcpyDeviceToHost));
        return SPSLAM_OK;
    }
    if (what == 5) {  // supp_lines phase clocks (SPSLAM_SUPP_PROF build), [kMaxPlanesPerFrame][8]
        HIP_CHECK(c, hipMemcpy(out, c->sb.prof + (size_t)frame * kMaxPlanesPerFrame * 8,
                               kMaxPlanesPerFrame * 8 * sizeof(long long), hipMemcpyDeviceToHost));
        return SPSLAM_OK;
    }
    return fail(c, SPSLAM_ERR_ARG, "unknown debug stage%s", "");
}

}  // extern "C"

namespace {

// cv::undistortPoints(point, K, D, noArray(), K), OpenCV 3.4 (frame_kernels.hip restates it for the device).
void undistort_host(const FrameGeom& g, float u, float v, float* ou, float* ov) {
    const double fx = g.fx, fy = g.fy, cx = g.cx, cy = g.cy, ifx = 1. / fx, ify = 1. / fy;
    const double k0 = g.dist[0], k1 = g.dist[1], k2 = g.dist[2], k3 = g.dist[3], k4 = g.dist[4];
    const double k5 = 0, k6 = 0, k7 = 0, k8 = 0, k9 = 0, k10 = 0, k11 = 0;
    double x = ((double)u - cx) * ifx, y = ((double)v - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k7 * r2 + k6) * r2 + k5) * r2) / (1 + ((k4 * r2 + k1) * r2 + k0) * r2);
        const double deltaX = 2 * k2 * x * y + k3 * (r2 + 2 * x * x) + k8 * r2 + k9 * r2 * r2;
        const double deltaY = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y + k10 * r2 + k11 * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    *ou = (float)((fx * x + 0. * y + cx) * (1. / (0. * x + 0. * y + 1.)));
    *ov = (float)((0. * x + fy * y + cy) * (1. / (0. * x + 0. * y + 1.)));
}

}  // namespace

extern "C" {

int spslam_frame_configure(spslam_ctx* c, const spslam_frame_params* p, float* bounds, float* grid_inv) {
    if (!c || !p || p->fx == 0.f || p->fy == 0.f || p->width < 1 || p->height < 1) return SPSLAM_ERR_ARG;
    FrameGeom& g = c->fg;
    g.fx = p->fx; g.fy = p->fy; g.cx = p->cx; g.cy = p->cy;
    for (int k = 0; k < 5; k++) g.dist[k] = p->dist[k];
    g.bf = p->bf;
    g.undistort = p->dist[0] != 0.0f;
    // Frame::ComputeImageBounds (Frame.cc:536-564)
    if (g.undistort) {
        float cu[4], cv[4];
        const float px[4] = {0.f, (float)p->width, 0.f, (float)p->width};
        const float py[4] = {0.f, 0.f, (float)p->height, (float)p->height};
        for (int i = 0; i < 4; i++) undistort_host(g, px[i], py[i], &cu[i], &cv[i]);
        g.min_x = std::min(cu[0], cu[2]); g.max_x = std::max(cu[1], cu[3]);
        g.min_y = std::min(cv[0], cv[1]); g.max_y = std::max(cv[2], cv[3]);
    } else {
        g.min_x = 0.f; g.max_x = (float)p->width; g.min_y = 0.f; g.max_y = (float)p->height;
    }
    g.ginv_x = (float)SPSLAM_GRID_COLS / (g.max_x - g.min_x);
    g.ginv_y = (float)SPSLAM_GRID_ROWS / (g.max_y - g.min_y);
    if (bounds) { bounds[0] = g.min_x; bounds[1] = g.max_x; bounds[2] = g.min_y; bounds[3] = g.max_y; }
    if (grid_inv) { grid_inv[0] = g.ginv_x; grid_inv[1] = g.ginv_y; }
    HIP_CHECK(c, hipSetDevice(c->device));
    if (!c->d_frame1) {
        const size_t cap = (size_t)c->max_kp;
        const size_t bytes = cap * (2 * sizeof(spslam_keypoint) + 3 * 4) + (SPSLAM_GRID_COLS * SPSLAM_GRID_ROWS + 1) * 4 +
                             4096;
        HIP_CHECK(c, hipMalloc(&c->d_frame1, bytes));
    }
    c->frame_ready = true;
    return SPSLAM_OK;
}

int spslam_frame_rgbd_batch_device(spslam_ctx* c, const spslam_keypoint* d_kps, const int* d_counts,
                                   int cap_per_frame, const float* d_depth, int n_frames, size_t frame_stride,
                                   int stride_floats, spslam_keypoint* d_keys_un, float* d_mv_depth,
                                   float* d_mv_uright, int32_t* d_grid_off, int32_t* d_grid_idx,
                                   int* d_plane_counts, int* d_supp_counts, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (!c->frame_ready) return fail(c, SPSLAM_ERR_NOT_READY, "spslam_frame_configure not called%s", "");
    if (!d_kps || !d_counts || !d_depth || !d_keys_un || !d_mv_depth || !d_mv_uright || !d_grid_off || !d_grid_idx ||
        n_frames < 1 || cap_per_frame < 1 || cap_per_frame > 32767 || stride_floats < 1)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_frame_rgbd_batch_device");
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the default stream (header)
    HIP_CHECK(c, frame_launch(c->fg, n_frames, d_kps, d_counts, cap_per_frame, d_depth, (long long)frame_stride,
                              stride_floats, d_keys_un, d_mv_depth, d_mv_uright, d_grid_off, d_grid_idx,
                              d_plane_counts, d_supp_counts, s, c->timer));
    return SPSLAM_OK;
}

int spslam_frame_rgbd(spslam_ctx* c, const spslam_keypoint* kps, int n, const float* depth, int w, int h,
                      int stride_floats, spslam_keypoint* keys_un, float* mv_depth, float* mv_uright,
                      int32_t* grid_off, int32_t* grid_idx) {
    if (!c || n < 0 || (n && (!kps || !keys_un || !mv_depth || !mv_uright || !grid_idx)) || !grid_off || !depth ||
        w < 1 || h < 1 || stride_floats < w)
        return SPSLAM_ERR_ARG;
    if (!c->frame_ready) return fail(c, SPSLAM_ERR_NOT_READY, "spslam_frame_configure not called%s", "");
    if (n > c->max_kp) return fail(c, SPSLAM_ERR_CAPACITY, "more keypoints than the context holds%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    const size_t cap = (size_t)std::max(n, 1);
    uint8_t* q = c->d_frame1;
    auto* d_k = (spslam_keypoint*)q; q += (size_t)c->max_kp * sizeof(spslam_keypoint);
    auto* d_u = (spslam_keypoint*)q; q += (size_t)c->max_kp * sizeof(spslam_keypoint);
    auto* d_d = (float*)q; q += (size_t)c->max_kp * 4;
    auto* d_r = (float*)q; q += (size_t)c->max_kp * 4;
    auto* d_gi = (int32_t*)q; q += (size_t)c->max_kp * 4;
    auto* d_go = (int32_t*)q; q += (SPSLAM_GRID_COLS * SPSLAM_GRID_ROWS + 1) * 4;
    auto* d_n = (int*)(((uintptr_t)q + 255) & ~(uintptr_t)255);
    // the depth image is staged in a stream-ordered temporary
    float* d_depth = nullptr;
    HIP_CHECK(c, hipMallocAsync((void**)&d_depth, (size_t)w * h * 4, c->stream));
    HIP_CHECK(c, hipMemcpy2DAsync(d_depth, (size_t)w * 4, depth, (size_t)stride_floats * 4, (size_t)w * 4, h,
                                  hipMemcpyHostToDevice, c->stream));
    if (n) HIP_CHECK(c, hipMemcpyAsync(d_k, kps, n * sizeof(spslam_keypoint), hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(d_n, &n, sizeof(int), hipMemcpyHostToDevice, c->stream));
    int rc = spslam_frame_rgbd_batch_device(c, d_k, d_n, (int)cap, d_depth, 1, (size_t)w * h, w, d_u, d_d, d_r,
                                            d_go, d_gi, nullptr, nullptr, c->stream);
    if (rc) { (void)hipFreeAsync(d_depth, c->stream); return rc; }
    if (n) {
        HIP_CHECK(c, hipMemcpyAsync(keys_un, d_u, n * sizeof(spslam_keypoint), hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(c, hipMemcpyAsync(mv_depth, d_d, n * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(c, hipMemcpyAsync(mv_uright, d_r, n * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_CHECK(c, hipMemcpyAsync(grid_off, d_go, (SPSLAM_GRID_COLS * SPSLAM_GRID_ROWS + 1) * 4, hipMemcpyDeviceToHost,
                                c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    const int ng = grid_off[SPSLAM_GRID_COLS * SPSLAM_GRID_ROWS];
    if (ng) HIP_CHECK(c, hipMemcpy(grid_idx, d_gi, (size_t)ng * 4, hipMemcpyDeviceToHost));
    HIP_CHECK(c, hipFreeAsync(d_depth, c->stream));
    return SPSLAM_OK;
}

namespace {
// the Schur layout's team threshold (measurement knob; the results do not depend on it)
int lba_rows_max_team() {
    static const int v = [] {
        const char* e = getenv("SPSLAM_LBG_ROWS_MAX_TEAM");
        return e ? atoi(e) : 4;
    }();
    return v;
}

int lba_batch(spslam_ctx* c, int n, const spslam_lba_problem* problems, const spslam_lba_problem* d_problems,
              const spslam_lba_keyframe* d_kfs, const spslam_lba_point* d_points,
              const spslam_lba_point_obs* d_point_obs, const spslam_lba_plane* d_planes,
              const spslam_lba_plane_obs* d_plane_obs, const spslam_plane_config* cfg, float* d_kf_out,
              float* d_pt_out, float* d_pl_out, uint8_t* d_point_obs_outlier, uint8_t* d_plane_obs_outlier,
              spslam_lba_result* d_results, const int32_t* d_stop_flags, void* hip_stream,
              const volatile uint8_t* stop_src, volatile int32_t* stop_mirror) {
    if (!c) return SPSLAM_ERR_ARG;
    if (n < 1 || !problems || !d_problems || !d_kfs || !cfg || !d_kf_out || !d_results)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_lba_optimize_batch_device");
    LbaConsts C{};
    C.angle_info = 3282.8 / (cfg->angle_info * cfg->angle_info);
    C.dis_info = cfg->distance_info * cfg->distance_info;
    C.par_info = 3282.8 / (cfg->parallel_info * cfg->parallel_info);
    C.ver_info = 3282.8 / (cfg->vertical_info * cfg->vertical_info);
    C.plane_chi = cfg->chi;
    C.vp_chi = cfg->vp_chi;
    C.delta_mono = (float)std::sqrt(5.991);     // const float thHuberMono = sqrt(5.991)
    C.delta_stereo = (float)std::sqrt(7.815);
    C.delta_plane = (float)std::sqrt(cfg->chi);  // const float deltaPlane = sqrt(planeChi)
    C.delta_vp = (float)std::sqrt(cfg->vp_chi);
    std::vector<long long> off(n);
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the default stream (header)
    if (!c->lba_done) HIP_CHECK(c, hipEventCreateWithFlags(&c->lba_done, hipEventDisableTiming));
    // the previous LBA call of this context (on any stream) has finished reading the offsets, ctl and scratch
    // before this one's copies on `s` rewrite them (recorded below after every launch; a never-recorded event
    // is complete)
    HIP_CHECK(c, hipStreamWaitEvent(s, c->lba_done, 0));
    if (c->lba_order == SPSLAM_LBA_G2O_ORDER) {
        // the instance: pose masks of one word (up to 64 free poses) unless a window has more keyframes than that
        int max_kf = 0;
        for (int i = 0; i < n; i++) max_kf = std::max(max_kf, problems[i].n_kf);
        const int pw = lbg_pw_for(max_kf);
        size_t total = 0;
        for (int i = 0; i < n; i++) {
            const spslam_lba_problem& p = problems[i];
            if (p.n_kf < 0 || p.n_points < 0 || p.n_planes < 0 || p.n_point_obs < 0 || p.n_plane_obs < 0)
                return fail(c, SPSLAM_ERR_ARG, "negative count in LBA problem%s", "");
            if ((p.n_points && (!d_points || !d_point_obs || !d_pt_out || !d_point_obs_outlier)) ||
                (p.n_planes && (!d_planes || !d_plane_obs || !d_pl_out || !d_plane_obs_outlier)))
                return fail(c, SPSLAM_ERR_ARG, "missing LBA buffers%s", "");
            off[i] = (long long)total;
            total += lbg_layout(std::min(p.n_kf, kLbgMaxKeyframes), p.n_points, p.n_planes,
                                p.n_point_obs + p.n_plane_obs, pw).bytes;
        }
        if (total > c->lba_scratch_bytes) {
            HIP_CHECK(c, hipStreamSynchronize(s));
            if (c->d_lba_scratch) (void)hipFree(c->d_lba_scratch);
            c->d_lba_scratch = nullptr;
            c->lba_scratch_bytes = 0;
            HIP_CHECK(c, hipMalloc(&c->d_lba_scratch, total));
            c->lba_scratch_bytes = total;
        }
        if (n > c->lba_off_cap) {
            HIP_CHECK(c, hipStreamSynchronize(s));
            if (c->d_lba_off) (void)hipFree(c->d_lba_off);
            c->d_lba_off = nullptr;
            HIP_CHECK(c, hipMalloc(&c->d_lba_off, (size_t)n * sizeof(long long)));
            c->lba_off_cap = n;
        }
        if (lbg_ctl_ints(n) > c->lba_ctl_cap) {
            HIP_CHECK(c, hipStreamSynchronize(s));
            if (c->d_lba_ctl) (void)hipFree(c->d_lba_ctl);
            c->d_lba_ctl = nullptr;
            HIP_CHECK(c, hipMalloc(&c->d_lba_ctl, lbg_ctl_ints(n) * sizeof(int)));
            c->lba_ctl_cap = lbg_ctl_ints(n);
        }
        // workgroups per problem: the context's setting, else as many as fill the chip's CUs (one each), at most 8
        int team = c->lba_team;
        if (team <= 0) team = std::max(1, std::min(8, c->num_cus / n));
        HIP_CHECK(c, hipMemcpyAsync(c->d_lba_off, off.data(), (size_t)n * sizeof(long long), hipMemcpyHostToDevice, s));
        LbgBatch B{n, d_problems, c->d_lba_off, c->d_lba_scratch, d_kfs, d_points, d_point_obs, d_planes, d_plane_obs,
                   d_kf_out, d_pt_out, d_pl_out, d_point_obs_outlier, d_plane_obs_outlier, d_results, d_stop_flags,
                   c->lba_stop_after, team, c->solve_fail_mask, c->d_lba_ctl, pw, lba_rows_max_team()};
        HIP_CHECK(c, lba_run_g2o(B, C, s, c->timer));
        HIP_CHECK(c, hipEventRecord(c->lba_done, s));
        if (stop_src) {  // host-buffer entry: mirror the caller's bool into the device-visible flag while it runs
            hipEvent_t ev;
            HIP_CHECK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            HIP_CHECK(c, hipEventRecord(ev, s));
            for (;;) {
                if (*stop_src) *stop_mirror = 1;
                const hipError_t q = hipEventQuery(ev);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) {
                    (void)hipEventDestroy(ev);
                    HIP_CHECK(c, q);
                }
                std::this_thread::sleep_for(std::chrono::microseconds(50));
            }
            HIP_CHECK(c, hipEventDestroy(ev));
        }
        return SPSLAM_OK;
    }
    // work tables: edge chunks, landmark chunks, keyframe tasks, pose-pair (+ bs) tasks per problem
    std::vector<int2> ec, lc, kt, pt, qt, sg, pm;
    int max_kf = 1;
    for (int i = 0; i < n; i++) max_kf = std::max(max_kf, problems[i].n_kf);
    const int seg_own = lba_seg_own(std::min(max_kf, kLbaMaxKeyframes));
    size_t total = 0;
    for (int i = 0; i < n; i++) {
        const spslam_lba_problem& p = problems[i];
        if (p.n_kf < 0 || p.n_points < 0 || p.n_planes < 0 || p.n_point_obs < 0 || p.n_plane_obs < 0)
            return fail(c, SPSLAM_ERR_ARG, "negative count in LBA problem%s", "");
        if ((p.n_points && (!d_points || !d_point_obs || !d_pt_out || !d_point_obs_outlier)) ||
            (p.n_planes && (!d_planes || !d_plane_obs || !d_pl_out || !d_plane_obs_outlier)))
            return fail(c, SPSLAM_ERR_ARG, "missing LBA buffers%s", "");
        const int E = p.n_point_obs + p.n_plane_obs, L = p.n_points + p.n_planes;
        off[i] = (long long)total;
        total += lba_layout(p.n_kf, p.n_points, p.n_planes, E).bytes;
        if (p.n_kf > kLbaMaxKeyframes) continue;  // rejected on the device (status -2)
        for (int e = 0; e < E; e += kLbaChunk) ec.push_back(int2{i, e});
        for (int l = 0; l < L; l += kLbaChunk) lc.push_back(int2{i, l});
        for (int k = 0; k < p.n_kf; k++) kt.push_back(int2{i, k});
        const int npmax = p.n_kf;  // bound on the free poses; surplus tasks exit on the device
        // pose-pair and right-hand-side Schur tasks (the latter encoded -(p + 1)) only where the reduced system
        // may exceed the matrix-core path (6 np > 16 x kLbaMfmaTiles rows), which forms both
        if (6 * npmax > 16 * kLbaMfmaTiles) {
            for (int q = 0; q < npmax * (npmax + 1) / 2; q++) pt.push_back(int2{i, q});
            for (int q = 0; q < npmax; q++) pt.push_back(int2{i, -(q + 1)});
        }
        for (int q = 0; q < p.n_plane_obs; q += kLbaPlaneEdgesPerTask) qt.push_back(int2{i, p.n_point_obs + q});
        for (int e = 0; e < p.n_point_obs; e += seg_own) sg.push_back(int2{i, e});
        for (int q = 0; q < p.n_planes; q += kLbaChunk / 64) pm.push_back(int2{i, p.n_points + q});
    }
    if (total > c->lba_scratch_bytes) {
        HIP_CHECK(c, hipStreamSynchronize(s));
        if (c->d_lba_scratch) (void)hipFree(c->d_lba_scratch);
        c->d_lba_scratch = nullptr;
        c->lba_scratch_bytes = 0;
        HIP_CHECK(c, hipMalloc(&c->d_lba_scratch, total));
        c->lba_scratch_bytes = total;
    }
    if (n > c->lba_off_cap) {
        HIP_CHECK(c, hipStreamSynchronize(s));
        if (c->d_lba_off) (void)hipFree(c->d_lba_off);
        c->d_lba_off = nullptr;
        HIP_CHECK(c, hipMalloc(&c->d_lba_off, (size_t)n * sizeof(long long)));
        c->lba_off_cap = n;
    }
    std::vector<int2> work;
    work.reserve(ec.size() + lc.size() + kt.size() + pt.size() + qt.size() + sg.size() + pm.size() + 1);
    work.insert(work.end(), ec.begin(), ec.end());
    work.insert(work.end(), lc.begin(), lc.end());
    work.insert(work.end(), kt.begin(), kt.end());
    work.insert(work.end(), pt.begin(), pt.end());
    work.insert(work.end(), qt.begin(), qt.end());
    work.insert(work.end(), sg.begin(), sg.end());
    work.insert(work.end(), pm.begin(), pm.end());
    work.push_back(int2{0, 0});  // active counter
    if (work.size() > c->lba_work_cap) {
        HIP_CHECK(c, hipStreamSynchronize(s));
        if (c->d_lba_work) (void)hipFree(c->d_lba_work);
        c->d_lba_work = nullptr;
        c->lba_work_cap = 0;
        HIP_CHECK(c, hipMalloc(&c->d_lba_work, work.size() * sizeof(int2)));
        c->lba_work_cap = work.size();
    }
    HIP_CHECK(c, hipMemcpyAsync(c->d_lba_off, off.data(), (size_t)n * sizeof(long long), hipMemcpyHostToDevice, s));
    HIP_CHECK(c, hipMemcpyAsync(c->d_lba_work, work.data(), work.size() * sizeof(int2), hipMemcpyHostToDevice, s));
    const int2* w0 = c->d_lba_work;
    LbaWork W{w0, (int)ec.size(), w0 + ec.size(), (int)lc.size(), w0 + ec.size() + lc.size(), (int)kt.size(),
              w0 + ec.size() + lc.size() + kt.size(), (int)pt.size(),
              w0 + ec.size() + lc.size() + kt.size() + pt.size(), (int)qt.size(),
              w0 + ec.size() + lc.size() + kt.size() + pt.size() + qt.size(), (int)sg.size(),
              w0 + ec.size() + lc.size() + kt.size() + pt.size() + qt.size() + sg.size(), (int)pm.size(), seg_own};
    LbaBatch B{n, d_problems, c->d_lba_off, c->d_lba_scratch, d_kfs, d_points, d_point_obs, d_planes, d_plane_obs,
               d_kf_out, d_pt_out, d_pl_out, d_point_obs_outlier, d_plane_obs_outlier, d_results,
               (int*)(c->d_lba_work + work.size() - 1), d_stop_flags, c->lba_stop_after};
    // optimize(5) + optimize(10), at most 10 trials per iteration, plus the two structure steps
    HIP_CHECK(c, lba_run(B, W, C, 15 * 10 + 4, s, c->timer, nullptr, stop_src, stop_mirror));
    HIP_CHECK(c, hipEventRecord(c->lba_done, s));
    return SPSLAM_OK;
}
}  // namespace

int spslam_lba_set_team(spslam_ctx* c, int workgroups) {
    if (!c || workgroups < 0 || workgroups > kLbgTeamMax) return SPSLAM_ERR_ARG;
    c->lba_team = workgroups;
    return SPSLAM_OK;
}

int spslam_lba_set_order(spslam_ctx* c, int order) {
    if (!c || (order != SPSLAM_LBA_G2O_ORDER && order != SPSLAM_LBA_FAST_ORDER)) return SPSLAM_ERR_ARG;
    c->lba_order = order;
    return SPSLAM_OK;
}

int spslam_lba_debug_stop_after(spslam_ctx* c, int trials) {
    if (!c || trials < -1) return SPSLAM_ERR_ARG;
    c->lba_stop_after = trials;
    return SPSLAM_OK;
}

int spslam_lba_optimize_batch_device(spslam_ctx* c, int n, const spslam_lba_problem* problems,
                                     const spslam_lba_problem* d_problems, const spslam_lba_keyframe* d_kfs,
                                     const spslam_lba_point* d_points, const spslam_lba_point_obs* d_point_obs,
                                     const spslam_lba_plane* d_planes, const spslam_lba_plane_obs* d_plane_obs,
                                     const spslam_plane_config* cfg, float* d_kf_out, float* d_pt_out,
                                     float* d_pl_out, uint8_t* d_point_obs_outlier, uint8_t* d_plane_obs_outlier,
                                     spslam_lba_result* d_results, const int32_t* d_stop_flags, void* hip_stream) {
    return lba_batch(c, n, problems, d_problems, d_kfs, d_points, d_point_obs, d_planes, d_plane_obs, cfg, d_kf_out,
                     d_pt_out, d_pl_out, d_point_obs_outlier, d_plane_obs_outlier, d_results, d_stop_flags,
                     hip_stream, nullptr, nullptr);
}

int spslam_lba_optimize(spslam_ctx* c, const spslam_lba_problem* problem, const spslam_lba_keyframe* kfs,
                        const spslam_lba_point* points, const spslam_lba_point_obs* point_obs,
                        const spslam_lba_plane* planes, const spslam_lba_plane_obs* plane_obs,
                        const spslam_plane_config* cfg, float* kf_out, float* pt_out, float* pl_out,
                        uint8_t* point_obs_outlier, uint8_t* plane_obs_outlier, spslam_lba_result* result,
                        const volatile uint8_t* stop_flag) {
    if (!c || !problem || !cfg || !result) return SPSLAM_ERR_ARG;
    spslam_lba_problem P = *problem;
    P.kf_offset = P.point_offset = P.plane_offset = 0;
    const size_t nk = P.n_kf, np = P.n_points, nq = P.n_planes, npo = P.n_point_obs, nqo = P.n_plane_obs;
    if ((nk && (!kfs || !kf_out)) || (np && (!points || !pt_out)) || (nq && (!planes || !pl_out)) ||
        (npo && (!point_obs || !point_obs_outlier)) || (nqo && (!plane_obs || !plane_obs_outlier)))
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_lba_optimize");
    HIP_CHECK(c, hipSetDevice(c->device));
    size_t sz[] = {sizeof P,
                   nk * sizeof(spslam_lba_keyframe), np * sizeof(spslam_lba_point), npo * sizeof(spslam_lba_point_obs),
                   nq * sizeof(spslam_lba_plane), nqo * sizeof(spslam_lba_plane_obs), nk * 64, np * 12, nq * 16,
                   npo, nqo, sizeof(spslam_lba_result)};
    size_t bytes = 0, o[12];
    for (int i = 0; i < 12; i++) { o[i] = bytes; bytes += (sz[i] + 255) / 256 * 256; }
    if (bytes > c->lba_stage_bytes) {
        if (c->d_lba_stage) (void)hipFree(c->d_lba_stage);
        c->d_lba_stage = nullptr;
        c->lba_stage_bytes = 0;
        HIP_CHECK(c, hipMalloc(&c->d_lba_stage, bytes));
        c->lba_stage_bytes = bytes;
    }
    uint8_t* q = c->d_lba_stage;
    const void* src[] = {&P, kfs, points, point_obs, planes, plane_obs};
    for (int i = 0; i < 6; i++)
        if (sz[i]) HIP_CHECK(c, hipMemcpyAsync(q + o[i], src[i], sz[i], hipMemcpyHostToDevice, c->stream));
    if (stop_flag && !c->h_lba_stop) {
        HIP_CHECK(c, hipHostMalloc((void**)&c->h_lba_stop, sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
        HIP_CHECK(c, hipHostGetDevicePointer((void**)&c->d_lba_stop, c->h_lba_stop, 0));
    }
    if (stop_flag) *(volatile int32_t*)c->h_lba_stop = *stop_flag ? 1 : 0;
    int rc = lba_batch(
        c, 1, &P, (const spslam_lba_problem*)(q + o[0]), (const spslam_lba_keyframe*)(q + o[1]),
        (const spslam_lba_point*)(q + o[2]), (const spslam_lba_point_obs*)(q + o[3]),
        (const spslam_lba_plane*)(q + o[4]), (const spslam_lba_plane_obs*)(q + o[5]), cfg, (float*)(q + o[6]),
        (float*)(q + o[7]), (float*)(q + o[8]), q + o[9], q + o[10], (spslam_lba_result*)(q + o[11]),
        stop_flag ? c->d_lba_stop : nullptr, c->stream, stop_flag, stop_flag ? c->h_lba_stop : nullptr);
    if (rc) return rc;
    void* dst[] = {kf_out, pt_out, pl_out, point_obs_outlier, plane_obs_outlier, result};
    for (int i = 0; i < 6; i++)
        if (sz[6 + i]) HIP_CHECK(c, hipMemcpyAsync(dst[i], q + o[6 + i], sz[6 + i], hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return result->status == 0 ? SPSLAM_OK : fail(c, SPSLAM_ERR_ARG, "LBA problem rejected (status %s)", "< 0");
}

int spslam_planes_associate_batch_device(spslam_ctx* c, int n_frames, const spslam_assoc_frame* d_frames,
                                         const void* d_planes_a, int stride_a, const int* d_count_a, int cap_a,
                                         const void* d_planes_b, int stride_b, const int* d_count_b, int cap_b,
                                         const spslam_map_plane* d_map, const float* d_boundary_xyz, int max_map,
                                         const spslam_assoc_params* params, int32_t* d_match, int32_t* d_parallel,
                                         int32_t* d_vertical, int* d_new_plane, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (n_frames < 1 || !d_frames || !params || !d_match || !d_parallel || !d_vertical || max_map < 0 ||
        (cap_a > 0 && (!d_planes_a || !d_count_a || stride_a < 16)) || cap_a < 0 || cap_b < 0 ||
        (cap_b > 0 && (!d_planes_b || !d_count_b || stride_b < 16)) || (max_map > 0 && (!d_map || !d_boundary_xyz)))
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_planes_associate_batch_device");
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the default stream (header)
    const size_t need = std::max<size_t>((size_t)n_frames * (cap_a + cap_b) * max_map * sizeof(float), 256);
    if (need > c->assoc_dist_bytes) {
        HIP_CHECK(c, hipStreamSynchronize(s));
        if (c->d_assoc_dist) (void)hipFree(c->d_assoc_dist);
        c->d_assoc_dist = nullptr;
        c->assoc_dist_bytes = 0;
        HIP_CHECK(c, hipMalloc(&c->d_assoc_dist, need));
        c->assoc_dist_bytes = need;
    }
    AssocSources S{(const uint8_t*)d_planes_a, cap_b > 0 ? (const uint8_t*)d_planes_b : nullptr, stride_a,
                   stride_b, d_count_a, cap_b > 0 ? d_count_b : nullptr, cap_a, cap_b};
    HIP_CHECK(c, assoc_launch(n_frames, d_frames, S, d_map, d_boundary_xyz, max_map, *params, c->d_assoc_dist,
                              d_match, d_parallel, d_vertical, d_new_plane, s, c->timer));
    return SPSLAM_OK;
}

int spslam_planes_associate(spslam_ctx* c, const spslam_assoc_frame* frame, const float* coefs, int n_planes,
                            const spslam_map_plane* map_planes, int n_map, const float* boundary_xyz,
                            int n_boundary, const spslam_assoc_params* params, int32_t* match, int32_t* parallel,
                            int32_t* vertical, int* new_plane) {
    if (!c || !frame || !params || n_planes < 0 || n_map < 0 || n_boundary < 0 ||
        (n_planes && (!coefs || !match || !parallel || !vertical)) || (n_map && !map_planes) ||
        (n_boundary && !boundary_xyz))
        return SPSLAM_ERR_ARG;
    for (int j = 0; j < n_map; j++)
        if (map_planes[j].n_boundary < 0 || map_planes[j].boundary_offset < 0 ||
            (long long)map_planes[j].boundary_offset + map_planes[j].n_boundary > n_boundary)
            return fail(c, SPSLAM_ERR_ARG, "map plane boundary range outside the boundary array%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    spslam_assoc_frame F = *frame;
    F.map_offset = 0;
    F.n_map = n_map;
    const int cap = std::max(n_planes, 1);
    size_t sz[] = {sizeof F, (size_t)cap * 16, sizeof(int), (size_t)std::max(n_map, 1) * sizeof(spslam_map_plane),
                   (size_t)std::max(n_boundary, 1) * 12, (size_t)cap * 4 * 3, sizeof(int)};
    size_t o[7], bytes = 0;
    for (int i = 0; i < 7; i++) { o[i] = bytes; bytes += (sz[i] + 255) / 256 * 256; }
    uint8_t* q = nullptr;
    HIP_CHECK(c, hipMallocAsync((void**)&q, bytes, c->stream));
    const void* src[] = {&F, coefs, &n_planes, map_planes, boundary_xyz};
    const size_t len[] = {sizeof F, (size_t)n_planes * 16, sizeof(int), (size_t)n_map * sizeof(spslam_map_plane),
                          (size_t)n_boundary * 12};
    for (int i = 0; i < 5; i++)
        if (len[i]) HIP_CHECK(c, hipMemcpyAsync(q + o[i], src[i], len[i], hipMemcpyHostToDevice, c->stream));
    auto* d_out = (int32_t*)(q + o[5]);
    if (F.carry && n_planes) {  // the frame's current associations are the starting state
        HIP_CHECK(c, hipMemcpyAsync(d_out, match, (size_t)n_planes * 4, hipMemcpyHostToDevice, c->stream));
        HIP_CHECK(c, hipMemcpyAsync(d_out + cap, parallel, (size_t)n_planes * 4, hipMemcpyHostToDevice, c->stream));
        HIP_CHECK(c, hipMemcpyAsync(d_out + 2 * cap, vertical, (size_t)n_planes * 4, hipMemcpyHostToDevice, c->stream));
    }
    int rc = spslam_planes_associate_batch_device(
        c, 1, (const spslam_assoc_frame*)(q + o[0]), q + o[1], 16, (const int*)(q + o[2]), cap, nullptr, 0, nullptr,
        0, (const spslam_map_plane*)(q + o[3]), (const float*)(q + o[4]), n_map, params, d_out, d_out + cap,
        d_out + 2 * cap, (int*)(q + o[6]), c->stream);
    if (rc) { (void)hipFreeAsync(q, c->stream); return rc; }
    int np = 0;
    if (n_planes) {
        HIP_CHECK(c, hipMemcpyAsync(match, d_out, (size_t)n_planes * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(c, hipMemcpyAsync(parallel, d_out + cap, (size_t)n_planes * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(c, hipMemcpyAsync(vertical, d_out + 2 * cap, (size_t)n_planes * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_CHECK(c, hipMemcpyAsync(&np, q + o[6], sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipFreeAsync(q, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (new_plane) *new_plane = np;
    return SPSLAM_OK;
}

int spslam_search_by_projection_batch_device(spslam_ctx* c, int n_frames, const spslam_proj_frame* d_frames,
                                             const spslam_proj_point* d_points, int max_points,
                                             const spslam_keypoint* d_keys_un, const uint8_t* d_desc,
                                             const float* d_uright, const int32_t* d_grid_off,
                                             const int32_t* d_grid_idx, const int* d_counts, int cap,
                                             const spslam_match_params* params, int32_t* d_match, int* d_nmatches,
                                             void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (!c->frame_ready) return fail(c, SPSLAM_ERR_NOT_READY, "spslam_frame_configure not called%s", "");
    if (n_frames < 1 || !d_frames || max_points < 0 || (max_points > 0 && !d_points) || !d_keys_un || !d_desc ||
        !d_uright || !d_grid_off || !d_grid_idx || !d_counts || cap < 1 || cap > (1 << 20) || !params ||
        !d_match || !d_nmatches)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_search_by_projection_batch_device");
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the default stream (header)
    const size_t n = (size_t)n_frames * std::max(max_points, 1);
    const size_t need = n * sizeof(MatchWindow) + 256 + n * sizeof(int2);
    if (need > c->match_scratch_bytes) {
        HIP_CHECK(c, hipStreamSynchronize(s));
        if (c->d_match_scratch) (void)hipFree(c->d_match_scratch);
        c->d_match_scratch = nullptr;
        c->match_scratch_bytes = 0;
        HIP_CHECK(c, hipMalloc(&c->d_match_scratch, need));
        c->match_scratch_bytes = need;
    }
    auto* win = (MatchWindow*)c->d_match_scratch;
    auto* pushes = (int2*)(c->d_match_scratch + ((n * sizeof(MatchWindow) + 255) & ~(size_t)255));
    MatchGeom g{};
    g.fx = c->fg.fx; g.fy = c->fg.fy; g.cx = c->fg.cx; g.cy = c->fg.cy; g.bf = c->fg.bf;
    g.min_x = c->fg.min_x; g.max_x = c->fg.max_x; g.min_y = c->fg.min_y; g.max_y = c->fg.max_y;
    g.ginv_x = c->fg.ginv_x; g.ginv_y = c->fg.ginv_y;
    for (int l = 0; l < 8; l++) g.scale[l] = l < c->p.nlevels ? c->scale[l] : 0.f;
    MatchCurrent cur{d_keys_un, d_desc, d_uright, d_grid_off, d_grid_idx, d_counts, cap};
    HIP_CHECK(c, match_launch(n_frames, d_frames, d_points, max_points, cur, g, *params, win, pushes, d_match,
                              d_nmatches, s, c->timer));
    return SPSLAM_OK;
}

int spslam_search_by_projection(spslam_ctx* c, const spslam_proj_frame* frame, const spslam_proj_point* points,
                                const spslam_keypoint* keys_un, const uint8_t* desc, const float* uright, int n_kp,
                                const int32_t* grid_off, const int32_t* grid_idx, const spslam_match_params* params,
                                int32_t* match, int* nmatches) {
    if (!c || !frame || !params || !grid_off || !nmatches || n_kp < 0 || frame->n_points < 0 ||
        (frame->n_points && !points) || (n_kp && (!keys_un || !desc || !uright || !grid_idx || !match)))
        return SPSLAM_ERR_ARG;
    constexpr int kCells = SPSLAM_GRID_COLS * SPSLAM_GRID_ROWS;
    if (grid_off[0] != 0 || grid_off[kCells] > n_kp)
        return fail(c, SPSLAM_ERR_ARG, "grid CSR does not fit the keypoints%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    spslam_proj_frame F = *frame;
    F.point_offset = 0;
    const int np = F.n_points, cap = std::max(n_kp, 1);
    size_t sz[] = {sizeof F, (size_t)std::max(np, 1) * sizeof(spslam_proj_point), (size_t)cap * sizeof(spslam_keypoint),
                   (size_t)cap * 32, (size_t)cap * 4, (kCells + 1) * 4, (size_t)cap * 4, sizeof(int), (size_t)cap * 4,
                   sizeof(int)};
    size_t o[10], bytes = 0;
    for (int i = 0; i < 10; i++) { o[i] = bytes; bytes += (sz[i] + 255) / 256 * 256; }
    uint8_t* q = nullptr;
    HIP_CHECK(c, hipMallocAsync((void**)&q, bytes, c->stream));
    const void* src[] = {&F, points, keys_un, desc, uright, grid_off, grid_idx, &n_kp};
    const size_t len[] = {sizeof F, (size_t)np * sizeof(spslam_proj_point), (size_t)n_kp * sizeof(spslam_keypoint),
                          (size_t)n_kp * 32, (size_t)n_kp * 4, (kCells + 1) * 4, (size_t)grid_off[kCells] * 4,
                          sizeof(int)};
    for (int i = 0; i < 8; i++)
        if (len[i]) HIP_CHECK(c, hipMemcpyAsync(q + o[i], src[i], len[i], hipMemcpyHostToDevice, c->stream));
    int rc = spslam_search_by_projection_batch_device(
        c, 1, (const spslam_proj_frame*)(q + o[0]), (const spslam_proj_point*)(q + o[1]), np,
        (const spslam_keypoint*)(q + o[2]), q + o[3], (const float*)(q + o[4]), (const int32_t*)(q + o[5]),
        (const int32_t*)(q + o[6]), (const int*)(q + o[7]), cap, params, (int32_t*)(q + o[8]), (int*)(q + o[9]),
        c->stream);
    if (rc) { (void)hipFreeAsync(q, c->stream); return rc; }
    if (n_kp) HIP_CHECK(c, hipMemcpyAsync(match, q + o[8], (size_t)n_kp * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(nmatches, q + o[9], sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipFreeAsync(q, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return SPSLAM_OK;
}

int spslam_grab_rgbd_batch_device(spslam_ctx* c, int n_frames, const uint8_t* d_color, size_t color_frame_stride,
                                  int color_stride, const void* d_depth, size_t depth_frame_stride, int depth_stride,
                                  int w, int h, const spslam_grab_params* params, uint8_t* d_gray, float* d_depth_out,
                                  void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (n_frames < 1 || !d_color || !d_depth || !params || !d_gray || !d_depth_out || w < 1 || h < 1 ||
        (params->channels != 1 && params->channels != 3 && params->channels != 4) ||
        color_stride < w * params->channels || depth_stride < w ||
        (n_frames > 1 && (color_frame_stride < (size_t)color_stride * h || depth_frame_stride < (size_t)depth_stride * h)))
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_grab_rgbd_batch_device");
    HIP_CHECK(c, hipSetDevice(c->device));
    GrabArgs a{d_color, color_frame_stride, color_stride, d_depth, depth_frame_stride, depth_stride, w, h, *params,
               d_gray, d_depth_out, nullptr, 0, 1, 0, 0, 0.f, 0.f, 0.f, 0.f};
    // a CV_32F depth with |factor - 1| <= 1e-5 is used as is (Tracking.cc:228)
    if (!params->depth_u16 && std::fabs(params->depth_scale - 1.0f) <= 1e-5f) a.p.depth_scale = 1.0f;
    // the organized cloud of the plane stage in the same pass (spslam_grab_fuse_cloud)
    const bool cloud = c->grab_cloud && c->planes_ready && w == c->pg.w && h == c->pg.h && n_frames <= c->p.max_batch;
    if (cloud) {
        const PlaneGeom& g = c->pg;
        a.cloud = c->pb.cloud; a.cloud_fs = c->pb.cloud_fs;
        a.ds = g.ds; a.cW = g.W; a.cN = g.N;
        a.fx = g.fx; a.fy = g.fy; a.cx = g.cx; a.cy = g.cy;
    }
    HIP_CHECK(c, grab_launch(n_frames, a, (hipStream_t)hip_stream, c->timer));
    if (cloud) c->cloud_tag[c->cloud_set] = {d_depth_out, n_frames};
    return SPSLAM_OK;
}

int spslam_grab_fuse_cloud(spslam_ctx* c, int enable) {
    if (!c) return SPSLAM_ERR_ARG;
    c->grab_cloud = enable != 0;
    if (!enable) c->cloud_tag[0] = c->cloud_tag[1] = {};
    return SPSLAM_OK;
}

int spslam_grab_rgbd(spslam_ctx* c, const uint8_t* color, int color_stride, const void* depth, int depth_stride,
                     int w, int h, const spslam_grab_params* params, uint8_t* gray, float* depth_out) {
    if (!c || !color || !depth || !params || !gray || !depth_out || w < 1 || h < 1 ||
        (params->channels != 1 && params->channels != 3 && params->channels != 4) ||
        color_stride < w * params->channels || depth_stride < w)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_grab_rgbd");
    HIP_CHECK(c, hipSetDevice(c->device));
    const size_t de = params->depth_u16 ? 2 : 4;
    const size_t cb = (size_t)color_stride * h, db = (size_t)depth_stride * h * de, gb = (size_t)w * h;
    const size_t o1 = (cb + 255) / 256 * 256, o2 = o1 + (db + 255) / 256 * 256, o3 = o2 + (gb + 255) / 256 * 256;
    uint8_t* q = nullptr;
    HIP_CHECK(c, hipMallocAsync((void**)&q, o3 + gb * 4, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(q, color, cb, hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(q + o1, depth, db, hipMemcpyHostToDevice, c->stream));
    int rc = spslam_grab_rgbd_batch_device(c, 1, q, cb, color_stride, q + o1, (size_t)depth_stride * h, depth_stride,
                                           w, h, params, q + o2, (float*)(q + o3), c->stream);
    if (rc) { (void)hipFreeAsync(q, c->stream); return rc; }
    HIP_CHECK(c, hipMemcpyAsync(gray, q + o2, gb, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(depth_out, q + o3, gb * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipFreeAsync(q, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return SPSLAM_OK;
}

int spslam_track_graph_batch_device(spslam_ctx* c, int n_frames, int stage, const spslam_track_batch* batch,
                                    void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (n_frames < 1 || !batch || stage < SPSLAM_TRACK_MOTION_MODEL || stage > SPSLAM_TRACK_LAST_FRAME)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_track_graph_batch_device");
    const spslam_track_batch& b = *batch;
    const bool common = b.kp_counts && b.cap >= 1 && b.cap <= (1 << 20) && b.proj_frames && b.proj_match &&
                        b.proj_points && b.edge_of_kp;
    bool ok = common;
    if (stage == SPSLAM_TRACK_MOTION_PRIOR) {
        ok = b.proj_frames && b.velocity;
    } else if (stage == SPSLAM_TRACK_LAST_FRAME) {
        ok = common && b.keys_un && b.local_frames && b.local_points && b.local_match && b.results &&
             b.point_outlier && b.point_outlier_local && b.next_frames && b.next_points && b.velocity;
    } else if (stage == SPSLAM_TRACK_DISCARD) {
        ok = ok && b.taken && b.local_frames && b.results && b.point_outlier;
        if (b.next_match)  // the plane-outlier discard needs the first association and its edge flags
            ok = ok && b.next_parallel && b.next_vertical && b.plane_outlier && b.assoc_match && b.assoc_parallel &&
                 b.assoc_vertical && b.cap_a >= 0 && b.cap_b >= 0 && (b.cap_a == 0 || b.count_a) &&
                 (b.cap_b == 0 || b.count_b);
    } else {
        ok = ok && b.keys_un && b.uright && b.problems && b.points && b.cap_a >= 0 && b.cap_b >= 0 &&
             (b.cap_a == 0 || (b.planes_a && b.count_a && b.stride_a >= 16)) &&
             (b.cap_b == 0 || (b.planes_b && b.count_b && b.stride_b >= 16)) &&
             (b.cap_a + b.cap_b == 0 || (b.planes && b.map && b.assoc_match && b.assoc_parallel && b.assoc_vertical));
        if (stage == SPSLAM_TRACK_LOCAL_MAP)
            ok = ok && b.local_frames && b.local_points && b.local_match && b.results && b.point_outlier;
    }
    static const char* names[5] = {"MOTION_MODEL", "DISCARD", "LOCAL_MAP", "MOTION_PRIOR", "LAST_FRAME"};
    if (!ok) return fail(c, SPSLAM_ERR_ARG, "missing buffer for stage %s of spslam_track_graph_batch_device",
                         names[stage]);
    HIP_CHECK(c, hipSetDevice(c->device));
    TrackArgs a{};
    a.b = b;
    if (b.cap_b == 0) a.b.count_b = nullptr;
    for (int l = 0; l < kMaxLevels; l++)
        a.inv_sigma2[l] = c->inv_sigma2[std::min<int>(l, (int)c->inv_sigma2.size() - 1)];
    HIP_CHECK(c, track_launch(n_frames, stage, a, (hipStream_t)hip_stream, c->timer));
    return SPSLAM_OK;
}

int spslam_track_refkf_batch_device(spslam_ctx* c, int n_frames, int stage, const spslam_track_batch* mm,
                                    const spslam_refkf_batch* rk, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (n_frames < 1 || !mm || !rk || (stage != SPSLAM_REFKF_PREPARE && stage != SPSLAM_REFKF_SELECT))
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_track_refkf_batch_device");
    const spslam_track_batch& b = *mm;
    const spslam_refkf_batch& r = *rk;
    bool ok = b.kp_counts && b.cap >= 1 && b.cap <= (1 << 20) && b.proj_frames && b.proj_points && b.proj_match &&
              b.edge_of_kp && b.point_outlier && r.nmatches && r.fallback;
    if (stage == SPSLAM_REFKF_PREPARE)
        ok = ok && b.problems && b.planes && b.plane_outlier && r.refkf_counts;
    else
        ok = ok && r.bow_nmatches && r.bow_match && r.refkf_rows && r.refkf_index && r.rows_stride >= 1 &&
             r.refkf_sets && r.assoc_frames && r.apply && r.refkf_match && r.refkf_frames && r.refkf_assoc &&
             (!b.seen || b.local_frames);
    if (!ok)
        return fail(c, SPSLAM_ERR_ARG, "missing buffer for spslam_track_refkf_batch_device stage %s",
                    stage == SPSLAM_REFKF_PREPARE ? "PREPARE" : "SELECT");
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, refkf_launch(n_frames, stage, b, r, (hipStream_t)hip_stream));
    return SPSLAM_OK;
}

int spslam_track_refkf_vote_batch_device(spslam_ctx* c, int n_frames, const spslam_track_batch* mm,
                                         const spslam_refkf_vote* vote, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (n_frames < 1 || !mm || !vote)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_track_refkf_vote_batch_device");
    const spslam_track_batch& b = *mm;
    const spslam_refkf_vote& v = *vote;
    if (v.n_kf < 1 || v.n_kf > 1024 || v.ids_per_kf < 1 || v.new_kf >= v.n_kf)
        return fail(c, SPSLAM_ERR_ARG, "spslam_track_refkf_vote_batch_device: n_kf outside 1 .. 1024, ids_per_kf < 1 "
                    "or new_kf >= n_kf%s", "");
    const bool ok = b.kp_counts && b.cap >= 1 && b.cap <= (1 << 20) && b.proj_frames && b.proj_points &&
                    b.proj_match && b.edge_of_kp && b.point_outlier && v.kf_base && v.kf_sets && v.refkf_index &&
                    v.refkf_sets;
    if (!ok) return fail(c, SPSLAM_ERR_ARG, "missing buffer for spslam_track_refkf_vote_batch_device%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, refkf_vote_launch(n_frames, b, v, (hipStream_t)hip_stream));
    return SPSLAM_OK;
}

int spslam_masked_frame_copy_device(spslam_ctx* c, int n_frames, const uint8_t* flags, int n_regions,
                                    const spslam_frame_region* regions, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (n_frames < 1 || !flags || n_regions < 0 || n_regions > kMaxFrameRegions || (n_regions && !regions))
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_masked_frame_copy_device");
    FrameRegions G{};
    G.n = n_regions;
    for (int k = 0; k < n_regions; k++) {
        const spslam_frame_region& r = regions[k];
        if (!r.dst || !r.src || r.frame_bytes < 0 || r.frame_bytes % 4 || r.dst_stride % 4 || r.src_stride % 4 ||
            ((uintptr_t)r.dst | (uintptr_t)r.src) % 4 || r.frame_bytes > r.dst_stride || r.frame_bytes > r.src_stride)
            return fail(c, SPSLAM_ERR_ARG, "bad region of %s", "spslam_masked_frame_copy_device");
        G.r[k] = r;
    }
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, masked_frame_copy_launch(n_frames, flags, G, (hipStream_t)hip_stream));
    return SPSLAM_OK;
}

int spslam_search_local_points_batch_device(spslam_ctx* c, int n_frames, const spslam_local_frame* d_frames,
                                            const spslam_local_point* d_points, int max_points,
                                            const spslam_keypoint* d_keys_un, const uint8_t* d_desc,
                                            const float* d_uright, const int32_t* d_grid_off,
                                            const int32_t* d_grid_idx, const int* d_counts, int cap,
                                            const uint8_t* d_taken, const spslam_local_params* params,
                                            int32_t* d_match, int* d_nmatches, uint8_t* d_in_view,
                                            const int32_t* d_seen, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (!c->frame_ready) return fail(c, SPSLAM_ERR_NOT_READY, "spslam_frame_configure not called%s", "");
    if (n_frames < 1 || !d_frames || max_points < 0 || (max_points > 0 && !d_points) || !d_keys_un || !d_desc ||
        !d_uright || !d_grid_off || !d_grid_idx || !d_counts || cap < 1 || cap > (1 << 20) || !params ||
        !d_match || !d_nmatches)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_search_local_points_batch_device");
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the default stream (header)
    const size_t need = (size_t)n_frames * std::max(max_points, 1) * sizeof(LocalWindow) + 256;
    if (need > c->match_scratch_bytes) {
        HIP_CHECK(c, hipStreamSynchronize(s));
        if (c->d_match_scratch) (void)hipFree(c->d_match_scratch);
        c->d_match_scratch = nullptr;
        c->match_scratch_bytes = 0;
        HIP_CHECK(c, hipMalloc(&c->d_match_scratch, need));
        c->match_scratch_bytes = need;
    }
    MatchGeom g{};
    g.fx = c->fg.fx; g.fy = c->fg.fy; g.cx = c->fg.cx; g.cy = c->fg.cy; g.bf = c->fg.bf;
    g.min_x = c->fg.min_x; g.max_x = c->fg.max_x; g.min_y = c->fg.min_y; g.max_y = c->fg.max_y;
    g.ginv_x = c->fg.ginv_x; g.ginv_y = c->fg.ginv_y;
    for (int l = 0; l < 8; l++) g.scale[l] = l < c->p.nlevels ? c->scale[l] : 0.f;
    LocalConsts P{params->th, params->nn_ratio, params->view_cos_limit,
                  std::log(c->p.scale_factor),  // Frame::mfLogScaleFactor = log(mfScaleFactor), float
                  c->p.nlevels, d_seen};
    MatchCurrent cur{d_keys_un, d_desc, d_uright, d_grid_off, d_grid_idx, d_counts, cap};
    HIP_CHECK(c, local_match_launch(n_frames, d_frames, d_points, max_points, cur, g, P, d_taken,
                                    (LocalWindow*)c->d_match_scratch, d_match, d_nmatches, d_in_view, s, c->timer));
    return SPSLAM_OK;
}

int spslam_search_local_points(spslam_ctx* c, const spslam_local_frame* frame, const spslam_local_point* points,
                               const spslam_keypoint* keys_un, const uint8_t* desc, const float* uright, int n_kp,
                               const int32_t* grid_off, const int32_t* grid_idx, const uint8_t* taken,
                               const spslam_local_params* params, int32_t* match, int* nmatches, uint8_t* in_view) {
    if (!c || !frame || !params || !grid_off || !nmatches || n_kp < 0 || frame->n_points < 0 ||
        (frame->n_points && !points) || (n_kp && (!keys_un || !desc || !uright || !grid_idx || !match)))
        return SPSLAM_ERR_ARG;
    constexpr int kCells = SPSLAM_GRID_COLS * SPSLAM_GRID_ROWS;
    if (grid_off[0] != 0 || grid_off[kCells] > n_kp)
        return fail(c, SPSLAM_ERR_ARG, "grid CSR does not fit the keypoints%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    spslam_local_frame F = *frame;
    F.point_offset = 0;
    const int np = F.n_points, cap = std::max(n_kp, 1);
    size_t sz[] = {sizeof F, (size_t)std::max(np, 1) * sizeof(spslam_local_point), (size_t)cap * sizeof(spslam_keypoint),
                   (size_t)cap * 32, (size_t)cap * 4, (kCells + 1) * 4, (size_t)cap * 4, sizeof(int), (size_t)cap,
                   (size_t)cap * 4, sizeof(int), (size_t)std::max(np, 1)};
    size_t o[12], bytes = 0;
    for (int i = 0; i < 12; i++) { o[i] = bytes; bytes += (sz[i] + 255) / 256 * 256; }
    uint8_t* q = nullptr;
    HIP_CHECK(c, hipMallocAsync((void**)&q, bytes, c->stream));
    const void* src[] = {&F, points, keys_un, desc, uright, grid_off, grid_idx, &n_kp, taken};
    const size_t len[] = {sizeof F, (size_t)np * sizeof(spslam_local_point), (size_t)n_kp * sizeof(spslam_keypoint),
                          (size_t)n_kp * 32, (size_t)n_kp * 4, (kCells + 1) * 4, (size_t)grid_off[kCells] * 4,
                          sizeof(int), taken ? (size_t)n_kp : 0};
    for (int i = 0; i < 9; i++)
        if (len[i]) HIP_CHECK(c, hipMemcpyAsync(q + o[i], src[i], len[i], hipMemcpyHostToDevice, c->stream));
    int rc = spslam_search_local_points_batch_device(
        c, 1, (const spslam_local_frame*)(q + o[0]), (const spslam_local_point*)(q + o[1]), np,
        (const spslam_keypoint*)(q + o[2]), q + o[3], (const float*)(q + o[4]), (const int32_t*)(q + o[5]),
        (const int32_t*)(q + o[6]), (const int*)(q + o[7]), cap, taken ? q + o[8] : nullptr, params,
        (int32_t*)(q + o[9]), (int*)(q + o[10]), q + o[11], nullptr, c->stream);
    if (rc) { (void)hipFreeAsync(q, c->stream); return rc; }
    if (n_kp) HIP_CHECK(c, hipMemcpyAsync(match, q + o[9], (size_t)n_kp * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(nmatches, q + o[10], sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (in_view && np) HIP_CHECK(c, hipMemcpyAsync(in_view, q + o[11], (size_t)np, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipFreeAsync(q, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return SPSLAM_OK;
}

// ---------------------------------------------------------------- bag of words
// TemplatedVocabulary::loadFromTextFile (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424), host side,
// then one HBM blob: descriptors, children CSR, weights, word ids.
int spslam_bow_load_vocabulary(spslam_ctx* c, const char* text, size_t len, int* k_out, int* L_out, int* n_nodes_out,
                               int* n_words_out) {
    if (!c || (!text && len)) return SPSLAM_ERR_ARG;
    std::istringstream f(std::string(text ? text : "", len));
    std::string line;
    std::getline(f, line);
    std::stringstream ss;
    ss << line;
    int k = 0, L = 0, n1 = 0, n2 = 0;
    ss >> k >> L >> n1 >> n2;
    if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3)
        return fail(c, SPSLAM_ERR_ARG, "vocabulary header is not DBoW2 text%s", "");
    std::vector<int> parent(1, 0);
    std::vector<std::vector<int>> children(1);
    std::vector<uint8_t> desc(32, 0);
    std::vector<double> weight(1, 0.0);
    std::vector<uint32_t> word(1, 0);
    uint32_t n_words = 0;
    while (!f.eof()) {  // the reference's loop: an empty last line still makes a node
        std::string sn;
        std::getline(f, sn);
        std::stringstream sl;
        sl << sn;
        const int nid = (int)parent.size();
        int pid = 0, leaf = 0;
        sl >> pid;
        if (pid < 0 || pid >= nid) return fail(c, SPSLAM_ERR_ARG, "vocabulary node with a bad parent%s", "");
        sl >> leaf;
        std::stringstream sd;
        for (int i = 0; i < 32; i++) {
            std::string e;
            sl >> e;
            sd << e << " ";
        }
        uint8_t d[32] = {0};  // FORB::fromString leaves unparsed bytes unset (uninitialised there, zero here)
        for (int i = 0; i < 32; i++) {
            int v;
            sd >> v;
            if (!sd.fail()) d[i] = (uint8_t)v;
        }
        double w = 0.0;
        sl >> w;
        parent.push_back(pid);
        children.emplace_back();
        children[pid].push_back(nid);
        desc.insert(desc.end(), d, d + 32);
        weight.push_back(w);
        word.push_back(leaf > 0 ? n_words++ : 0u);
    }
    const int n = (int)parent.size();
    std::vector<int> cbeg(n), ccnt(n), cids;
    cids.reserve(n);
    for (int i = 0; i < n; i++) {
        cbeg[i] = (int)cids.size();
        ccnt[i] = (int)children[i].size();
        cids.insert(cids.end(), children[i].begin(), children[i].end());
    }
    if (cids.empty()) cids.push_back(0);
    const size_t sz[] = {(size_t)n * 32, (size_t)n * 4, (size_t)n * 4, cids.size() * 4, (size_t)n * 8, (size_t)n * 4};
    size_t off[6], bytes = 0;
    for (int i = 0; i < 6; i++) { off[i] = bytes; bytes += (sz[i] + 255) / 256 * 256; }
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (c->d_vocab) (void)hipFree(c->d_vocab);
    c->d_vocab = nullptr;
    c->vocab = VocabDev{};
    HIP_CHECK(c, hipMalloc(&c->d_vocab, bytes));
    const void* src[] = {desc.data(), cbeg.data(), ccnt.data(), cids.data(), weight.data(), word.data()};
    for (int i = 0; i < 6; i++) HIP_CHECK(c, hipMemcpy(c->d_vocab + off[i], src[i], sz[i], hipMemcpyHostToDevice));
    VocabDev& V = c->vocab;
    V.n_nodes = n; V.k = k; V.L = L; V.scoring = n1; V.weighting = n2;
    V.desc = (const uint4*)(c->d_vocab + off[0]);
    V.child_begin = (const int*)(c->d_vocab + off[1]);
    V.child_count = (const int*)(c->d_vocab + off[2]);
    V.child_ids = (const int*)(c->d_vocab + off[3]);
    V.weight = (const double*)(c->d_vocab + off[4]);
    V.word_id = (const uint32_t*)(c->d_vocab + off[5]);
    if (k_out) *k_out = k;
    if (L_out) *L_out = L;
    if (n_nodes_out) *n_nodes_out = n;
    if (n_words_out) *n_words_out = (int)n_words;
    return SPSLAM_OK;
}

int spslam_bow_transform_batch_device(spslam_ctx* c, int n_frames, const uint8_t* d_desc, const int* d_counts,
                                      int cap, int levelsup, uint32_t* d_bow_words, double* d_bow_values,
                                      int* d_n_bow, uint32_t* d_fv_nodes, int32_t* d_fv_start,
                                      int32_t* d_fv_features, int* d_n_fv, void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    if (!c->d_vocab) return fail(c, SPSLAM_ERR_NOT_READY, "no vocabulary loaded (spslam_bow_load_vocabulary)%s", "");
    if (n_frames < 1 || !d_desc || !d_counts || cap < 1 || cap > 8192 || !d_bow_words || !d_bow_values || !d_n_bow ||
        !d_fv_nodes || !d_fv_start || !d_fv_features || !d_n_fv)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_bow_transform_batch_device");
    HIP_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)hip_stream;
    if (c->vocab.n_nodes < 2) {  // empty vocabulary: transform clears both vectors
        HIP_CHECK(c, hipMemsetAsync(d_n_bow, 0, (size_t)n_frames * sizeof(int), s));
        HIP_CHECK(c, hipMemsetAsync(d_n_fv, 0, (size_t)n_frames * sizeof(int), s));
        return SPSLAM_OK;
    }
    const size_t n = (size_t)n_frames * cap;
    const size_t need = n * 16 + 512;
    if (need > c->bow_scratch_bytes) {
        HIP_CHECK(c, hipStreamSynchronize(s));
        if (c->d_bow_scratch) (void)hipFree(c->d_bow_scratch);
        c->d_bow_scratch = nullptr;
        c->bow_scratch_bytes = 0;
        HIP_CHECK(c, hipMalloc(&c->d_bow_scratch, need));
        c->bow_scratch_bytes = need;
    }
    auto* s_weight = (double*)c->d_bow_scratch;
    auto* s_word = (uint32_t*)(c->d_bow_scratch + ((n * 8 + 255) & ~(size_t)255));
    auto* s_node = s_word + ((n + 63) & ~(size_t)63);
    BowOut out{d_bow_words, d_bow_values, d_n_bow, d_fv_nodes, d_fv_start, d_fv_features, d_n_fv};
    HIP_CHECK(c, bow_transform_launch(c->vocab, n_frames, d_desc, d_counts, cap, levelsup, s_word, s_weight, s_node,
                                      out, s, c->timer));
    return SPSLAM_OK;
}

// grow the BoW drop-in staging buffer
static int bow_stage(spslam_ctx* c, size_t bytes) {
    if (bytes <= c->bow_stage_bytes) return SPSLAM_OK;
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (c->d_bow_stage) (void)hipFree(c->d_bow_stage);
    c->d_bow_stage = nullptr;
    c->bow_stage_bytes = 0;
    HIP_CHECK(c, hipMalloc(&c->d_bow_stage, bytes));
    c->bow_stage_bytes = bytes;
    return SPSLAM_OK;
}

int spslam_bow_transform(spslam_ctx* c, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words,
                         double* bow_values, int* n_bow, uint32_t* fv_nodes, int32_t* fv_start,
                         int32_t* fv_features, int* n_fv) {
    if (!c || n < 0 || (n && !desc) || !n_bow || !n_fv || n > 8192 || !fv_start ||
        (n && (!bow_words || !bow_values || !fv_nodes || !fv_features)))
        return SPSLAM_ERR_ARG;
    if (!c->d_vocab) return fail(c, SPSLAM_ERR_NOT_READY, "no vocabulary loaded (spslam_bow_load_vocabulary)%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    const int cap = std::max(n, 1);
    const size_t sz[] = {(size_t)cap * 32, 4, (size_t)cap * 4, (size_t)cap * 8, 4, (size_t)cap * 4,
                         (size_t)(cap + 1) * 4, (size_t)cap * 4, 4};
    size_t o[9], bytes = 0;
    for (int i = 0; i < 9; i++) { o[i] = bytes; bytes += (sz[i] + 255) / 256 * 256; }
    if (int rc = bow_stage(c, bytes)) return rc;
    uint8_t* q = c->d_bow_stage;
    if (n) HIP_CHECK(c, hipMemcpyAsync(q + o[0], desc, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(q + o[1], &n, 4, hipMemcpyHostToDevice, c->stream));
    int rc = spslam_bow_transform_batch_device(c, 1, q + o[0], (const int*)(q + o[1]), cap, levelsup,
                                               (uint32_t*)(q + o[2]), (double*)(q + o[3]), (int*)(q + o[4]),
                                               (uint32_t*)(q + o[5]), (int32_t*)(q + o[6]), (int32_t*)(q + o[7]),
                                               (int*)(q + o[8]), c->stream);
    if (rc) return rc;
    HIP_CHECK(c, hipMemcpyAsync(n_bow, q + o[4], 4, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(n_fv, q + o[8], 4, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (*n_bow) {
        HIP_CHECK(c, hipMemcpy(bow_words, q + o[2], (size_t)*n_bow * 4, hipMemcpyDeviceToHost));
        HIP_CHECK(c, hipMemcpy(bow_values, q + o[3], (size_t)*n_bow * 8, hipMemcpyDeviceToHost));
    }
    if (*n_fv) {
        HIP_CHECK(c, hipMemcpy(fv_nodes, q + o[5], (size_t)*n_fv * 4, hipMemcpyDeviceToHost));
        HIP_CHECK(c, hipMemcpy(fv_start, q + o[6], (size_t)(*n_fv + 1) * 4, hipMemcpyDeviceToHost));
        int m = 0;
        std::memcpy(&m, fv_start + *n_fv, 4);
        if (m) HIP_CHECK(c, hipMemcpy(fv_features, q + o[7], (size_t)m * 4, hipMemcpyDeviceToHost));
    } else {
        fv_start[0] = 0;
    }
    return SPSLAM_OK;
}

int spslam_search_by_bow_batch_device(spslam_ctx* c, int n_pairs, const int32_t* d_pairs,
                                      const spslam_bow_side* kf, const spslam_bow_side* fr,
                                      const spslam_bow_params* params, int32_t* d_match, int* d_nmatches,
                                      void* hip_stream) {
    if (!c) return SPSLAM_ERR_ARG;
    auto side_ok = [](const spslam_bow_side* b, bool keyframe) {
        return b && b->desc && b->keys && b->counts && b->fv_nodes && b->fv_start && b->fv_features && b->n_fv &&
               b->cap >= 1 && b->cap <= 8192 && (!keyframe || b->has_point);
    };
    if (n_pairs < 1 || !d_pairs || !side_ok(kf, true) || !side_ok(fr, false) || !params || !d_match || !d_nmatches)
        return fail(c, SPSLAM_ERR_ARG, "bad argument%s", " to spslam_search_by_bow_batch_device");
    HIP_CHECK(c, hipSetDevice(c->device));
    BowSide K{kf->desc, kf->keys, kf->has_point, kf->counts, kf->fv_nodes, kf->fv_start, kf->fv_features, kf->n_fv,
              kf->cap};
    BowSide F{fr->desc, fr->keys, nullptr, fr->counts, fr->fv_nodes, fr->fv_start, fr->fv_features, fr->n_fv, fr->cap};
    HIP_CHECK(c, bow_search_launch(n_pairs, (const int2*)d_pairs, K, F, params->nn_ratio, params->check_orientation,
                                   d_match, d_nmatches, (hipStream_t)hip_stream, c->timer));
    return SPSLAM_OK;
}

int spslam_search_by_bow(spslam_ctx* c, const uint8_t* kf_desc, const spslam_keypoint* kf_keys,
                         const uint8_t* kf_has_point, int kf_n, const uint32_t* kf_fv_nodes,
                         const int32_t* kf_fv_start, const int32_t* kf_fv_features, int kf_n_fv,
                         const uint8_t* f_desc, const spslam_keypoint* f_keys, int f_n, const uint32_t* f_fv_nodes,
                         const int32_t* f_fv_start, const int32_t* f_fv_features, int f_n_fv,
                         const spslam_bow_params* params, int32_t* match, int* nmatches) {
    if (!c || !params || !nmatches || kf_n < 0 || f_n < 0 || kf_n > 8192 || f_n > 8192 || kf_n_fv < 0 ||
        f_n_fv < 0 || kf_n_fv > std::max(kf_n, 1) || f_n_fv > std::max(f_n, 1) || !kf_fv_start || !f_fv_start ||
        (kf_n && (!kf_desc || !kf_keys || !kf_has_point)) || (f_n && (!f_desc || !f_keys || !match)) ||
        (kf_n_fv && (!kf_fv_nodes || !kf_fv_features)) || (f_n_fv && (!f_fv_nodes || !f_fv_features)))
        return SPSLAM_ERR_ARG;
    const int kc = std::max(kf_n, 1), fc = std::max(f_n, 1);
    const int km = kf_fv_start[kf_n_fv], fm = f_fv_start[f_n_fv];
    if (km < 0 || km > kf_n || fm < 0 || fm > f_n)
        return fail(c, SPSLAM_ERR_ARG, "FeatureVector does not fit the features%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    // keyframe slot 0 and frame slot 0 of a one-pair batch
    const size_t sz[] = {(size_t)kc * 32, (size_t)kc * sizeof(spslam_keypoint), (size_t)kc, 4, (size_t)kc * 4,
                         (size_t)(kc + 1) * 4, (size_t)kc * 4, 4,
                         (size_t)fc * 32, (size_t)fc * sizeof(spslam_keypoint), 4, (size_t)fc * 4,
                         (size_t)(fc + 1) * 4, (size_t)fc * 4, 4, 8, (size_t)fc * 4, 4};
    size_t o[18], bytes = 0;
    for (int i = 0; i < 18; i++) { o[i] = bytes; bytes += (sz[i] + 255) / 256 * 256; }
    if (int rc = bow_stage(c, bytes)) return rc;
    uint8_t* q = c->d_bow_stage;
    const int32_t pair[2] = {0, 0};
    const void* src[] = {kf_desc, kf_keys, kf_has_point, &kf_n, kf_fv_nodes, kf_fv_start, kf_fv_features, &kf_n_fv,
                         f_desc, f_keys, &f_n, f_fv_nodes, f_fv_start, f_fv_features, &f_n_fv, pair};
    const size_t len[] = {(size_t)kf_n * 32, (size_t)kf_n * sizeof(spslam_keypoint), (size_t)kf_n, 4,
                          (size_t)kf_n_fv * 4, (size_t)(kf_n_fv + 1) * 4, (size_t)km * 4, 4,
                          (size_t)f_n * 32, (size_t)f_n * sizeof(spslam_keypoint), 4, (size_t)f_n_fv * 4,
                          (size_t)(f_n_fv + 1) * 4, (size_t)fm * 4, 4, 8};
    for (int i = 0; i < 16; i++)
        if (len[i]) HIP_CHECK(c, hipMemcpyAsync(q + o[i], src[i], len[i], hipMemcpyHostToDevice, c->stream));
    spslam_bow_side K{q + o[0], (const spslam_keypoint*)(q + o[1]), q + o[2], (const int*)(q + o[3]),
                      (const uint32_t*)(q + o[4]), (const int32_t*)(q + o[5]), (const int32_t*)(q + o[6]),
                      (const int*)(q + o[7]), kc, 0};
    spslam_bow_side F{q + o[8], (const spslam_keypoint*)(q + o[9]), nullptr, (const int*)(q + o[10]),
                      (const uint32_t*)(q + o[11]), (const int32_t*)(q + o[12]), (const int32_t*)(q + o[13]),
                      (const int*)(q + o[14]), fc, 0};
    int rc = spslam_search_by_bow_batch_device(c, 1, (const int32_t*)(q + o[15]), &K, &F, params,
                                               (int32_t*)(q + o[16]), (int*)(q + o[17]), c->stream);
    if (rc) return rc;
    if (f_n) HIP_CHECK(c, hipMemcpyAsync(match, q + o[16], (size_t)f_n * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(nmatches, q + o[17], 4, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return SPSLAM_OK;
}

int spslam_set_timing(spslam_ctx* c, int enable) {
    if (!c) return SPSLAM_ERR_ARG;
    (void)hipSetDevice(c->device);
    if (enable && !c->timer) c->timer = new EventTimer();
    if (!enable && c->timer) { delete c->timer; c->timer = nullptr; }
    if (c->timer) c->timer->reset();
    return SPSLAM_OK;
}

int spslam_kernel_times(spslam_ctx* c, double* total_ms, long long* launches, int max_kinds) {
    if (!c) return SPSLAM_ERR_ARG;
    const int n = std::min(max_kinds, (int)kNumKernelKinds);
    if (c->timer) c->timer->collect();
    for (int k = 0; k < n; k++) {
        if (total_ms) total_ms[k] = c->timer ? c->timer->total_ms[k] : 0.0;
        if (launches) launches[k] = c->timer ? c->timer->count[k] : 0;
    }
    return n;
}

const char* spslam_kernel_name(int kind) { return kernel_kind_name(kind); }

int spslam_orb_debug_stage(spslam_ctx* c, int frame, int level, int stage, void* out, int cap, int* n) {
    if (!c || !out || level < 0 || level >= c->p.nlevels) return SPSLAM_ERR_ARG;
    if (!c->last_frames || frame < 0 || frame >= c->last_frames)
        return fail(c, SPSLAM_ERR_NOT_READY, "no such frame in the last call%s", "");
    HIP_CHECK(c, hipSetDevice(c->device));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    HIP_CHECK(c, hipDeviceSynchronize());
    const LevelGeom& L = c->geom.lv[level];
    if (stage == 0 || stage == 1) {
        const uint8_t* src;
        size_t pitch;
        if (stage == 0) {
            src = (level == 0 ? c->last_gray : L.img) +
                  (size_t)frame * (level == 0 ? c->last_frame_stride : (size_t)L.frame_stride);
            pitch = level == 0 ? c->last_stride : L.stride;
        } else {
            src = L.blur + (size_t)frame * L.blur_frame_stride;
            pitch = L.bpitch;
        }
        HIP_CHECK(c, hipMemcpy2D(out, L.w, src, pitch, L.w, L.h, hipMemcpyDeviceToHost));
        if (n) *n = L.w * L.h;
        return SPSLAM_OK;
    }
    spslam_keypoint* o = (spslam_keypoint*)out;
    if (stage == 2) {
        const int ncells = L.nRows * L.nCols;
        std::vector<uint16_t> cnt(ncells);
        std::vector<uint32_t> cand((size_t)ncells * kCellCap);
        const size_t cell0 = (size_t)frame * c->geom.cells_per_frame + L.cell_base;
        HIP_CHECK(c, hipMemcpy(cnt.data(), c->b.cand_cnt + cell0, ncells * sizeof(uint16_t), hipMemcpyDeviceToHost));
        HIP_CHECK(c, hipMemcpy(cand.data(), c->b.cand + cell0 * kCellCap, cand.size() * 4, hipMemcpyDeviceToHost));
        int k = 0;
        for (int ci = 0; ci < ncells; ci++)
            for (int j = 0; j < cnt[ci]; j++, k++) {
                if (k >= cap) continue;
                const uint32_t v = cand[(size_t)ci * kCellCap + j];
                o[k] = spslam_keypoint{(float)(v & 0xFFF), (float)((v >> 12) & 0xFFF), 7.f, -1.f, (float)(v >> 24), 0, -1};
            }
        *n = k;
        return k > cap ? SPSLAM_ERR_CAPACITY : SPSLAM_OK;
    }
    if (stage == 3) {
        int cnt = 0;
        HIP_CHECK(c, hipMemcpy(&cnt, c->b.lvl_cnt + frame * kMaxLevels + level, sizeof(int), hipMemcpyDeviceToHost));
        std::vector<LevelKp> v(cnt);
        if (cnt)
            HIP_CHECK(c, hipMemcpy(v.data(), c->b.lvl_kp + (size_t)frame * c->geom.lvl_kp_per_frame + L.kp_base,
                                   cnt * sizeof(LevelKp), hipMemcpyDeviceToHost));
        for (int i = 0; i < cnt && i < cap; i++)
            o[i] = spslam_keypoint{(float)v[i].x, (float)v[i].y, (float)L.patch_size, -1.f, (float)v[i].response,
                                   level, -1};
        *n = cnt;
        return cnt > cap ? SPSLAM_ERR_CAPACITY : SPSLAM_OK;
    }
    return fail(c, SPSLAM_ERR_ARG, "unknown stage%s", "");
}

}  // extern "C"
