// The batched tracking step as one C-ABI call (include/spslam_gpu.h "whole step"): GrabImageRGBD -> ORB
// extraction || plane extraction + supposed planes -> the tracking tail (Frame keypoint steps,
// SearchByProjection, AssociatePlanesByBoundary, the PoseOptimization graphs, PoseOptimization,
// SearchLocalPoints, the second association and PoseOptimization) -- the reference's Tracking::GrabImageRGBD ->
// Frame constructor -> TrackWithMotionModel -> TrackLocalMap (src/Tracking.cc:208-244, 951-1068) for a batch of
// frames, on HIP streams and events this object owns.  Pipelined: batch k+1's extraction (grab + ORB on one
// stream, planes on another) runs beside batch k's tail, the extraction outputs double-buffered (set k % 2),
// set j rewritten only after the tail that read it has finished.  Every stage is the library's own batched
// entry point; this file is orchestration only, a client of the public ABI.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <new>

#include "../../include/spslam_gpu.h"

struct spslam_step {
    spslam_ctx* ctx = nullptr;
    spslam_step_config cfg{};
    spslam_step_set set[2]{};
    spslam_step_tail tail{};
    int planes_cap = 0, supp_cap = 0, inlier_cap = 0, contour_cap = 0, line_cap = 0, patch_points = 0;
    hipStream_t s_tail = nullptr, s_orb = nullptr, s_planes = nullptr;
    hipEvent_t ev_orb[2]{}, ev_planes[2]{}, ev_tail[2]{}, ev_grab[2]{}, ev_fork = nullptr, ev_join = nullptr;
    bool primed = false;
    long long k = 0;
    void* owned[64]{};  // buffers this object allocated (NULL members of the caller's sets / tail)
    int n_owned = 0;
};

namespace {

template <class T>
int own(spslam_step* st, T*& p, size_t bytes) {
    if (p) return SPSLAM_OK;
    if (st->n_owned >= 64) return SPSLAM_ERR_ARG;
    void* q = nullptr;
    if (hipMalloc(&q, bytes ? bytes : 16) != hipSuccess) return SPSLAM_ERR_HIP;
    if (hipMemset(q, 0, bytes ? bytes : 16) != hipSuccess) return SPSLAM_ERR_HIP;
    st->owned[st->n_owned++] = q;
    p = static_cast<T*>(q);
    return SPSLAM_OK;
}

#define TRY(x)                         \
    do {                               \
        const int rc_ = (x);           \
        if (rc_ != SPSLAM_OK) return rc_; \
    } while (0)

int alloc_missing(spslam_step* st) {
    const size_t B = (size_t)st->cfg.n_frames, px = (size_t)st->cfg.width * st->cfg.height, cap = st->cfg.kp_cap;
    for (auto& s : st->set) {
        TRY(own(st, s.gray, B * px));
        TRY(own(st, s.depth, B * px * 4));
        TRY(own(st, s.kps, B * cap * sizeof(spslam_keypoint)));
        TRY(own(st, s.desc, B * cap * 32));
        TRY(own(st, s.counts, B * 4));
        TRY(own(st, s.planes, B * st->planes_cap * sizeof(spslam_plane)));
        TRY(own(st, s.plane_counts, B * 4));
        TRY(own(st, s.inliers, B * st->inlier_cap * 4));
        TRY(own(st, s.contours, B * st->contour_cap * 4));
        TRY(own(st, s.supposed, B * st->supp_cap * sizeof(spslam_supposed_plane)));
        TRY(own(st, s.supposed_counts, B * 4));
        TRY(own(st, s.lines, B * st->line_cap * 4));
        TRY(own(st, s.patch, B * st->supp_cap * st->patch_points * 12));
    }
    spslam_step_tail& t = st->tail;
    const size_t P = (size_t)st->planes_cap + st->supp_cap, pe = 3 * P;
    TRY(own(st, t.keys_un, B * cap * sizeof(spslam_keypoint)));
    TRY(own(st, t.mv_depth, B * cap * 4));
    TRY(own(st, t.uright, B * cap * 4));
    TRY(own(st, t.grid_off, B * (64 * 48 + 1) * 4));
    TRY(own(st, t.grid_idx, B * cap * 4));
    TRY(own(st, t.match, B * cap * 4));
    TRY(own(st, t.nmatches, B * 4));
    TRY(own(st, t.taken, B * cap));
    TRY(own(st, t.local_match, B * cap * 4));
    TRY(own(st, t.local_nmatches, B * 4));
    TRY(own(st, t.edge_of_kp, B * cap * 4));
    for (int g = 0; g < 2; g++) {
        for (int a = 0; a < 3; a++) TRY(own(st, t.assoc[g][a], B * P * 4));
        TRY(own(st, t.new_plane[g], B * 4));
        TRY(own(st, t.problems[g], B * sizeof(spslam_pose_problem)));
        TRY(own(st, t.points[g], B * cap * sizeof(spslam_point_obs)));
        TRY(own(st, t.planes[g], B * pe * sizeof(spslam_plane_obs)));
        TRY(own(st, t.point_outlier[g], B * cap));
        TRY(own(st, t.plane_outlier[g], B * pe));
        TRY(own(st, t.results[g], B * sizeof(spslam_pose_result)));
    }
    return SPSLAM_OK;
}

// spslam_track_batch of graph g (0 = motion model, 1 = local map) on extraction set j
spslam_track_batch track_batch(const spslam_step* st, int j, int g, const spslam_step_tracking& in) {
    const spslam_step_set& s = st->set[j];
    const spslam_step_tail& t = st->tail;
    spslam_track_batch b{};
    b.keys_un = t.keys_un;
    b.uright = t.uright;
    b.kp_counts = s.counts;
    b.cap = st->cfg.kp_cap;
    b.proj_frames = in.proj_frames;
    b.proj_points = in.proj_points;
    b.proj_match = t.match;
    b.local_frames = in.local_frames;
    b.local_points = in.local_points;
    b.local_match = t.local_match;
    b.taken = t.taken;
    b.planes_a = s.planes;
    b.planes_b = s.supposed;
    b.count_a = s.plane_counts;
    b.count_b = s.supposed_counts;
    b.stride_a = (int)sizeof(spslam_plane);
    b.stride_b = (int)sizeof(spslam_supposed_plane);
    b.cap_a = st->planes_cap;
    b.cap_b = st->supp_cap;
    b.map = in.map;
    b.assoc_match = t.assoc[g][0];
    b.assoc_parallel = t.assoc[g][1];
    b.assoc_vertical = t.assoc[g][2];
    b.assoc_frames_next = in.assoc_frames2;
    b.plane_outlier = t.plane_outlier[0];
    b.next_match = t.assoc[1][0];
    b.next_parallel = t.assoc[1][1];
    b.next_vertical = t.assoc[1][2];
    b.problems = t.problems[g];
    b.points = t.points[g];
    b.planes = t.planes[g];
    b.edge_of_kp = t.edge_of_kp;
    b.results = t.results[0];
    b.point_outlier = t.point_outlier[0];
    b.fx = st->cfg.fx;
    b.fy = st->cfg.fy;
    b.cx = st->cfg.cx;
    b.cy = st->cfg.cy;
    b.bf = st->cfg.bf;
    return b;
}

int grab(spslam_step* st, int j, const spslam_step_frames& fr, hipStream_t s) {
    const spslam_step_config& c = st->cfg;
    return spslam_grab_rgbd_batch_device(st->ctx, c.n_frames, fr.color, fr.color_frame_stride, fr.color_stride,
                                         fr.depth, fr.depth_frame_stride, fr.depth_stride, c.width, c.height,
                                         &c.grab, st->set[j].gray, st->set[j].depth, s);
}
int orb(spslam_step* st, int j, hipStream_t s) {
    const spslam_step_config& c = st->cfg;
    const spslam_step_set& x = st->set[j];
    return spslam_orb_extract_batch_device(st->ctx, x.gray, c.n_frames, (size_t)c.width * c.height, c.width, x.kps,
                                           x.desc, x.counts, c.kp_cap, s);
}
int planes(spslam_step* st, int j, hipStream_t s) {
    const spslam_step_config& c = st->cfg;
    const spslam_step_set& x = st->set[j];
    const size_t fs = (size_t)c.width * c.height;
    TRY(spslam_planes_extract_batch_device(st->ctx, x.depth, c.n_frames, fs, c.width, x.planes, x.plane_counts,
                                           x.inliers, x.contours, s));
    return spslam_planes_generate_from_boundaries_batch_device(st->ctx, x.depth, c.n_frames, fs, c.width, x.planes,
                                                               x.plane_counts, x.contours, x.supposed,
                                                               x.supposed_counts, x.lines, x.patch, s);
}

// frame steps, SearchByProjection, then TrackWithMotionModel / TrackLocalMap from the matches on (pipeline.py
// HotPath._tail / pose)
int tail(spslam_step* st, int j, const spslam_step_tracking& in, hipStream_t s) {
    const spslam_step_config& c = st->cfg;
    const spslam_step_set& x = st->set[j];
    spslam_step_tail& t = st->tail;
    const int B = c.n_frames, cap = c.kp_cap;
    TRY(spslam_frame_rgbd_batch_device(st->ctx, x.kps, x.counts, cap, x.depth, B, (size_t)c.width * c.height,
                                       c.width, t.keys_un, t.mv_depth, t.uright, t.grid_off, t.grid_idx,
                                       x.plane_counts, x.supposed_counts, s));
    TRY(spslam_search_by_projection_batch_device(st->ctx, B, in.proj_frames, in.proj_points, in.max_proj_points,
                                                 t.keys_un, x.desc, t.uright, t.grid_off, t.grid_idx, x.counts, cap,
                                                 &c.match, t.match, t.nmatches, s));
    auto associate = [&](int g, const spslam_assoc_frame* fr) {
        return spslam_planes_associate_batch_device(st->ctx, B, fr, x.planes, (int)sizeof(spslam_plane),
                                                    x.plane_counts, st->planes_cap, x.supposed,
                                                    (int)sizeof(spslam_supposed_plane), x.supposed_counts,
                                                    st->supp_cap, in.map, in.boundary_xyz, in.max_map, &c.assoc,
                                                    t.assoc[g][0], t.assoc[g][1], t.assoc[g][2], t.new_plane[g], s);
    };
    auto pose = [&](int g) {
        return spslam_pose_optimize_batch_device(st->ctx, B, t.problems[g], t.points[g], t.planes[g], &c.pose,
                                                 nullptr, t.results[g], t.point_outlier[g], t.plane_outlier[g], s);
    };
    TRY(associate(0, in.assoc_frames1));
    spslam_track_batch b0 = track_batch(st, j, 0, in);
    TRY(spslam_track_graph_batch_device(st->ctx, B, SPSLAM_TRACK_MOTION_MODEL, &b0, s));
    TRY(pose(0));
    TRY(spslam_track_graph_batch_device(st->ctx, B, SPSLAM_TRACK_DISCARD, &b0, s));
    TRY(spslam_search_local_points_batch_device(st->ctx, B, in.local_frames, in.local_points, in.max_local_points,
                                                t.keys_un, x.desc, t.uright, t.grid_off, t.grid_idx, x.counts, cap,
                                                t.taken, &c.local, t.local_match, t.local_nmatches, nullptr,
                                                nullptr, s));
    TRY(associate(1, in.assoc_frames2));
    spslam_track_batch b1 = track_batch(st, j, 1, in);
    TRY(spslam_track_graph_batch_device(st->ctx, B, SPSLAM_TRACK_LOCAL_MAP, &b1, s));
    return pose(1);
}

// batch into extraction set j on the extraction streams (pipeline.py HotPath._extract)
int extract(spslam_step* st, int j, const spslam_step_frames& fr) {
    if (hipStreamWaitEvent(st->s_orb, st->ev_tail[j], 0) != hipSuccess) return SPSLAM_ERR_HIP;
    TRY(spslam_planes_select_cloud_set(st->ctx, j));  // (before the grab: a fused grab writes the set's cloud)
    TRY(grab(st, j, fr, st->s_orb));
    if (hipEventRecord(st->ev_grab[j], st->s_orb) != hipSuccess) return SPSLAM_ERR_HIP;
    if (hipStreamWaitEvent(st->s_planes, st->ev_grab[j], 0) != hipSuccess) return SPSLAM_ERR_HIP;
    TRY(planes(st, j, st->s_planes));
    if (hipEventRecord(st->ev_planes[j], st->s_planes) != hipSuccess) return SPSLAM_ERR_HIP;
    TRY(orb(st, j, st->s_orb));
    if (hipEventRecord(st->ev_orb[j], st->s_orb) != hipSuccess) return SPSLAM_ERR_HIP;
    return SPSLAM_OK;
}

}  // namespace

extern "C" {

int spslam_step_create(spslam_ctx* ctx, const spslam_step_config* cfg, const spslam_step_set* sets,
                       const spslam_step_tail* tail, spslam_step** out) {
    if (!ctx || !cfg || !out || cfg->n_frames <= 0 || cfg->width <= 0 || cfg->height <= 0 || cfg->kp_cap <= 0)
        return SPSLAM_ERR_ARG;
    *out = nullptr;
    spslam_step* st = new (std::nothrow) spslam_step;
    if (!st) return SPSLAM_ERR_ARG;
    st->ctx = ctx;
    st->cfg = *cfg;
    if (sets) {
        st->set[0] = sets[0];
        st->set[1] = sets[1];
    }
    if (tail) st->tail = *tail;
    int rc = spslam_planes_capacity(ctx, &st->planes_cap, &st->inlier_cap, &st->contour_cap);
    if (rc == SPSLAM_OK) rc = spslam_supposed_capacity(ctx, &st->supp_cap, &st->line_cap, &st->patch_points);
    if (rc == SPSLAM_OK) rc = alloc_missing(st);
    int lo = 0, hi = 0;
    if (rc == SPSLAM_OK && hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) rc = SPSLAM_ERR_HIP;
    // the tracking tail is a chain of latency-bound one-workgroup-per-frame kernels: high priority in the
    // pipelined step, so its workgroups dispatch ahead of the next batch's extraction
    auto mk = [&](hipStream_t* s, bool high) {
        if (rc == SPSLAM_OK && hipStreamCreateWithPriority(s, hipStreamNonBlocking, high ? hi : lo) != hipSuccess)
            rc = SPSLAM_ERR_HIP;
    };
    mk(&st->s_tail, cfg->pipelined && cfg->tail_priority);
    mk(&st->s_orb, cfg->orb_priority);
    mk(&st->s_planes, cfg->planes_priority);
    hipEvent_t* evs[] = {&st->ev_orb[0], &st->ev_orb[1], &st->ev_planes[0], &st->ev_planes[1], &st->ev_tail[0],
                         &st->ev_tail[1], &st->ev_grab[0], &st->ev_grab[1], &st->ev_fork, &st->ev_join};
    for (hipEvent_t* e : evs)
        if (rc == SPSLAM_OK && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) rc = SPSLAM_ERR_HIP;
    if (rc != SPSLAM_OK) {
        spslam_step_destroy(st);
        return rc;
    }
    *out = st;
    return SPSLAM_OK;
}

int spslam_step_buffers(const spslam_step* st, spslam_step_set* sets, spslam_step_tail* tail) {
    if (!st) return SPSLAM_ERR_ARG;
    if (sets) {
        sets[0] = st->set[0];
        sets[1] = st->set[1];
    }
    if (tail) *tail = st->tail;
    return SPSLAM_OK;
}

int spslam_step_run(spslam_step* st, const spslam_step_frames* next, const spslam_step_tracking* tracking) {
    if (!st || !next || !tracking) return SPSLAM_ERR_ARG;
    if (!st->cfg.pipelined) {
        // serial: grab, then planes (second stream) beside ORB, joined before the tail
        TRY(grab(st, 0, *next, st->s_tail));
        if (hipEventRecord(st->ev_fork, st->s_tail) != hipSuccess) return SPSLAM_ERR_HIP;
        if (hipStreamWaitEvent(st->s_planes, st->ev_fork, 0) != hipSuccess) return SPSLAM_ERR_HIP;
        TRY(planes(st, 0, st->s_planes));
        TRY(orb(st, 0, st->s_tail));
        if (hipEventRecord(st->ev_join, st->s_planes) != hipSuccess) return SPSLAM_ERR_HIP;
        if (hipStreamWaitEvent(st->s_tail, st->ev_join, 0) != hipSuccess) return SPSLAM_ERR_HIP;
        TRY(tail(st, 0, *tracking, st->s_tail));
        st->k++;
        return SPSLAM_OK;
    }
    if (!st->primed) return SPSLAM_ERR_NOT_READY;  // spslam_step_prime first
    const int j = (int)(st->k % 2);
    TRY(extract(st, 1 - j, *next));  // batch k+1
    if (hipStreamWaitEvent(st->s_tail, st->ev_orb[j], 0) != hipSuccess) return SPSLAM_ERR_HIP;
    if (hipStreamWaitEvent(st->s_tail, st->ev_planes[j], 0) != hipSuccess) return SPSLAM_ERR_HIP;
    TRY(tail(st, j, *tracking, st->s_tail));  // batch k
    if (hipEventRecord(st->ev_tail[j], st->s_tail) != hipSuccess) return SPSLAM_ERR_HIP;
    st->k++;
    return SPSLAM_OK;
}

int spslam_step_prime(spslam_step* st, const spslam_step_frames* first) {
    if (!st || !first) return SPSLAM_ERR_ARG;
    if (!st->cfg.pipelined) return SPSLAM_OK;
    TRY(extract(st, 0, *first));
    st->primed = true;
    return SPSLAM_OK;
}

int spslam_step_sync(spslam_step* st) {
    if (!st) return SPSLAM_ERR_ARG;
    for (hipStream_t s : {st->s_orb, st->s_planes, st->s_tail})
        if (s && hipStreamSynchronize(s) != hipSuccess) return SPSLAM_ERR_HIP;
    return SPSLAM_OK;
}

void* spslam_step_stream(const spslam_step* st) { return st ? (void*)st->s_tail : nullptr; }

void spslam_step_destroy(spslam_step* st) {
    if (!st) return;
    spslam_step_sync(st);
    for (hipEvent_t e : {st->ev_orb[0], st->ev_orb[1], st->ev_planes[0], st->ev_planes[1], st->ev_tail[0],
                         st->ev_tail[1], st->ev_grab[0], st->ev_grab[1], st->ev_fork, st->ev_join})
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t s : {st->s_orb, st->s_planes, st->s_tail})
        if (s) (void)hipStreamDestroy(s);
    for (int i = 0; i < st->n_owned; i++) (void)hipFree(st->owned[i]);
    delete st;
}

}  // extern "C"
