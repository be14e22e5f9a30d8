// gfx950 kernel for the Tracking-side graph bookkeeping between matching and
// PoseOptimization (include/spslam_gpu.h, spslam_track_graph_batch_device):
//   TrackWithMotionModel  src/Tracking.cc:951-1000 (graph, outlier discard)
//   TrackLocalMap         src/Tracking.cc:1055-1068
//   PoseOptimization's edge loops  src/Optimizer.cc:561-640 (points), 681-860
//                                  (plane, parallel, vertical edges)
//
// One 256-thread workgroup per frame.  The reference walks mvpMapPoints in
// keypoint order and push_back's one edge per set entry; here every 256-key
// chunk is a ballot/popcount block scan, so edge e of the device graph is the
// e-th set entry exactly as in the reference's vpEdgesMono/Stereo insertion
// order.  The work is index bookkeeping over <= cap keys (HBM/latency bound,
// a few microseconds per batch); no arithmetic touches the values it moves.
#include <hip/hip_runtime.h>

#include "wave_priority.h"

#include "track_launch.h"

namespace spslam {

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ const float* plane_coef(const spslam_track_batch& B, int f, int j, int na) {
    if (j < na) return (const float*)((const uint8_t*)B.planes_a + ((size_t)f * B.cap_a + j) * B.stride_a);
    return (const float*)((const uint8_t*)B.planes_b + ((size_t)f * B.cap_b + (j - na)) * B.stride_b);
}

__global__ __launch_bounds__(kThreads) void track_graph_kernel(TrackArgs A, int stage) {
    tail_wave_priority();
    const spslam_track_batch& B = A.b;
    const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    __shared__ int wsum[kThreads / 64];
    const int n = min(B.kp_counts[f], B.cap);
    const size_t ko = (size_t)f * B.cap;
    const spslam_proj_frame& PF = B.proj_frames[f];

    if (stage == SPSLAM_TRACK_DISCARD) {
        // src/Tracking.cc:986-1000, then ORBmatcher.cc:95-97's "already has a map point with observations"
        for (int i = t; i < n; i += kThreads) {
            const int e = B.edge_of_kp[ko + i];
            bool tk = false;
            if (e >= 0 && !B.point_outlier[ko + e])
                tk = B.proj_points[PF.point_offset + B.proj_match[ko + i]].n_obs > 0;
            B.taken[ko + i] = (uint8_t)tk;
        }
        if (t < 16) {
            const float v = B.results[f].Tcw[t];
            B.local_frames[f].Tcw[t] = v;
            if (B.assoc_frames_next) B.assoc_frames_next[f].Tcw[t] = v;
        }
        // src/Tracking.cc:1004-1028: associations whose edge is an outlier are dropped; the rest are the
        // second association's starting state.  Edge e of a kind is found by the same ballot scan that
        // laid the plane edges out (match, then parallel, then vertical, frame-plane order).
        if (B.next_match && wave == 0) {
            const int na = min(B.count_a[f], B.cap_a);
            const int nb = B.count_b ? min(B.count_b[f], B.cap_b) : 0;
            const int M = na + nb, PC = B.cap_a + B.cap_b;
            const size_t ao = (size_t)f * PC, po = (size_t)f * 3 * PC;
            const int32_t* src[3] = {B.assoc_match, B.assoc_parallel, B.assoc_vertical};
            int32_t* dst[3] = {B.next_match, B.next_parallel, B.next_vertical};
            int np = 0;
            for (int kind = 0; kind < 3; kind++) {
                for (int j0 = 0; j0 < M; j0 += 64) {
                    const int j = j0 + lane;
                    const int mp = j < M ? src[kind][ao + j] : -1;
                    const unsigned long long m = __ballot(mp >= 0);
                    if (j < M) {
                        const int e = np + __popcll(m & ((1ull << lane) - 1ull));
                        dst[kind][ao + j] = (mp >= 0 && !B.plane_outlier[po + e]) ? mp : -1;
                    }
                    np += __popcll(m);
                }
            }
        }
        return;
    }

    // ---- point edges (src/Optimizer.cc:561-640), keypoint order
    const bool local = stage == SPSLAM_TRACK_LOCAL_MAP;
    const int lpo = local ? B.local_frames[f].point_offset : 0;
    int base = 0;
    for (int i0 = 0; i0 < n; i0 += kThreads) {
        const int i = i0 + t;
        const float* xw = nullptr;
        if (i < n) {
            if (!local) {
                const int m = B.proj_match[ko + i];
                if (m >= 0) xw = B.proj_points[PF.point_offset + m].xw;
            } else {
                const int lm = B.local_match[ko + i];
                if (lm >= 0) {
                    xw = B.local_points[lpo + lm].xw;
                } else {
                    const int e = B.edge_of_kp[ko + i];
                    if (e >= 0 && !B.point_outlier[ko + e]) xw = B.proj_points[PF.point_offset + B.proj_match[ko + i]].xw;
                }
            }
        }
        const bool has = xw != nullptr;
        const unsigned long long m = __ballot(has);
        if (lane == 0) wsum[wave] = __popcll(m);
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kThreads / 64; w++) {
            before += w < wave ? wsum[w] : 0;
            total += wsum[w];
        }
        const int e = base + before + __popcll(m & ((1ull << lane) - 1ull));
        if (has) {
            const spslam_keypoint& k = B.keys_un[ko + i];
            spslam_point_obs o;
            o.u = k.x;
            o.v = k.y;
            o.ur = B.uright[ko + i];
            o.inv_sigma2 = A.inv_sigma2[min(max(k.octave, 0), kMaxLevels - 1)];
            o.xw[0] = xw[0];
            o.xw[1] = xw[1];
            o.xw[2] = xw[2];
            o.kp_index = i;
            B.points[ko + e] = o;
        }
        if (!local && i < n) B.edge_of_kp[ko + i] = has ? e : -1;
        base += total;
        __syncthreads();  // wsum reuse
    }

    // ---- plane edges (src/Optimizer.cc:681-860): planes, then parallel, then vertical, frame-plane order
    const int na = min(B.count_a[f], B.cap_a);
    const int nb = B.count_b ? min(B.count_b[f], B.cap_b) : 0;
    const int M = na + nb, PC = B.cap_a + B.cap_b;
    const size_t ao = (size_t)f * PC, po = (size_t)f * 3 * PC;
    int np = 0;
    if (wave == 0) {
        const int32_t* src[3] = {B.assoc_match, B.assoc_parallel, B.assoc_vertical};
        for (int kind = 0; kind < 3; kind++) {
            for (int j0 = 0; j0 < M; j0 += 64) {
                const int j = j0 + lane;
                const int mp = j < M ? src[kind][ao + j] : -1;
                const unsigned long long m = __ballot(mp >= 0);
                if (mp >= 0) {
                    const int e = np + __popcll(m & ((1ull << lane) - 1ull));
                    const float* c = plane_coef(B, f, j, na);
                    const spslam_map_plane& W = B.map[mp];
                    spslam_plane_obs o;
                    for (int q = 0; q < 4; q++) { o.meas[q] = c[q]; o.world[q] = W.world[q]; }
                    o.kind = kind;
                    o.plane_index = j;
                    o.map_plane_id = W.id;
                    o.pad = 0;
                    B.planes[po + e] = o;
                }
                np += __popcll(m);
            }
        }
    }
    if (t == 0) {
        spslam_pose_problem P;
        const float* T = local ? B.results[f].Tcw : PF.Tcw;
        for (int q = 0; q < 16; q++) P.Tcw[q] = T[q];
        P.fx = B.fx; P.fy = B.fy; P.cx = B.cx; P.cy = B.cy; P.bf = B.bf;
        P.n_points = base;
        P.n_planes = np;
        P.point_offset = (int32_t)ko;
        P.plane_offset = (int32_t)po;
        P.pad = 0;
        B.problems[f] = P;
    }
}

}  // namespace

hipError_t track_launch(int n_frames, int stage, const TrackArgs& a, hipStream_t s, KernelTimer* timer) {
    if (timer) timer->begin(kKindTrack, s);
    hipLaunchKernelGGL(track_graph_kernel, dim3(n_frames), dim3(kThreads), 0, s, a, stage);
    if (timer) timer->end(kKindTrack, s);
    return hipGetLastError();
}

}  // namespace spslam
