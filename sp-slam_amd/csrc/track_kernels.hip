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

// cv::Mat float product C = A * B of 4x4 row-major matrices (double accumulation, rounded once)
__device__ __forceinline__ void mat4_mul(const float* A, const float* Bm, float* C) {
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 4; k++) s = __dadd_rn(s, __dmul_rn((double)A[4 * i + k], (double)Bm[4 * k + j]));
            C[4 * i + j] = (float)s;
        }
}

// Frame::GetRotationInverse / GetCameraCenter as a 4x4 (Tracking.cc:446-448): [Rcw^T | -Rcw^T tcw]
__device__ __forceinline__ void inverse_pose(const float* T, float* W) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
#pragma unroll
        for (int j = 0; j < 3; j++) W[4 * i + j] = T[4 * j + i];
        double s = 0.0;  // mOw = -mRcw.t() * mtcw (Frame::UpdatePoseMatrices)
#pragma unroll
        for (int k = 0; k < 3; k++) s = __dadd_rn(s, __dmul_rn(-(double)T[4 * k + i], (double)T[4 * k + 3]));
        W[4 * i + 3] = (float)s;
    }
    W[12] = W[13] = W[14] = 0.f;
    W[15] = 1.f;
}

// a keypoint's map point after TrackLocalMap: the local-map match, else the motion-model match that survived
// the discard.  Returns the index into the local (l >= 0) or last-frame (l < 0, m) point arrays, or false.
__device__ __forceinline__ bool map_point_of(const spslam_track_batch& B, size_t ko, int i, int lpo, int* l,
                                             int* m) {
    const int lm = B.local_match[ko + i];
    if (lm >= 0) {
        *l = lpo + lm;
        return true;
    }
    const int e = B.edge_of_kp[ko + i];
    if (e >= 0 && !B.point_outlier[ko + e]) {
        *l = -1;
        *m = B.proj_match[ko + i];
        return true;
    }
    return false;
}

__global__ __launch_bounds__(kThreads) void track_graph_kernel(TrackArgs A, int stage) {
    tail_wave_priority();
    const spslam_track_batch& B = A.b;
    const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    __shared__ int wsum[kThreads / 64];
    const int n = min(B.kp_counts[f], B.cap);
    const size_t ko = (size_t)f * B.cap;
    const spslam_proj_frame& PF = B.proj_frames[f];

    if (stage == SPSLAM_TRACK_MOTION_PRIOR) {
        // TrackWithMotionModel: mCurrentFrame.SetPose(mVelocity * mLastFrame.mTcw) (Tracking.cc:958)
        if (t == 0) {
            float Tl[16], V[16], P[16];
            for (int q = 0; q < 16; q++) { Tl[q] = PF.Tlw[q]; V[q] = B.velocity[16 * f + q]; }
            mat4_mul(V, Tl, P);
            for (int q = 0; q < 16; q++) {
                const_cast<spslam_proj_frame*>(B.proj_frames)[f].Tcw[q] = P[q];  // the stage writes the prediction
                if (B.assoc_frames_first) B.assoc_frames_first[f].Tcw[q] = P[q];
            }
        }
        return;
    }

    if (stage == SPSLAM_TRACK_LAST_FRAME) {
        // Track(): mVelocity = mCurrentFrame.mTcw * LastTwc (:443-450), VO-match clean-up (:456-466) and
        // outlier drop (:484-488); mLastFrame = Frame(mCurrentFrame) (:505)
        const int lpo = B.local_frames[f].point_offset;
        int base = 0, nb = 0;  // local-map graph edge index / surviving points so far
        for (int i0 = 0; i0 < n; i0 += kThreads) {
            const int i = i0 + t;
            int l = -1, m = -1;
            const bool has = i < n && map_point_of(B, ko, i, lpo, &l, &m);
            const unsigned long long mh = __ballot(has);
            if (lane == 0) wsum[wave] = __popcll(mh);
            __syncthreads();
            int before = 0, total = 0;
#pragma unroll
            for (int w = 0; w < kThreads / 64; w++) {
                before += w < wave ? wsum[w] : 0;
                total += wsum[w];
            }
            __syncthreads();
            const int e2 = base + before + __popcll(mh & ((1ull << lane) - 1ull));
            int n_obs = 0;
            if (has) n_obs = l >= 0 ? B.local_points[l].n_obs : B.proj_points[PF.point_offset + m].n_obs;
            const bool keep = has && !B.point_outlier_local[ko + e2] && n_obs >= 1;
            const unsigned long long mk = __ballot(keep);
            if (lane == 0) wsum[wave] = __popcll(mk);
            __syncthreads();
            int kb = 0, kt = 0;
#pragma unroll
            for (int w = 0; w < kThreads / 64; w++) {
                kb += w < wave ? wsum[w] : 0;
                kt += wsum[w];
            }
            if (keep) {
                const int j = nb + kb + __popcll(mk & ((1ull << lane) - 1ull));
                spslam_proj_point o;
                const spslam_keypoint& k = B.keys_un[ko + i];
                const float* xw;
                const uint8_t* d;
                if (l >= 0) {
                    const spslam_local_point& L = B.local_points[l];
                    xw = L.xw; d = L.desc; o.id = L.id;
                } else {
                    const spslam_proj_point& Pp = B.proj_points[PF.point_offset + m];
                    xw = Pp.xw; d = Pp.desc; o.id = Pp.id;
                }
                o.xw[0] = xw[0]; o.xw[1] = xw[1]; o.xw[2] = xw[2];
                o.angle = k.angle;
                o.octave = k.octave;
                o.n_obs = n_obs;
                o.last_index = i;
                for (int q = 0; q < 32; q++) o.desc[q] = d[q];
                B.next_points[ko + j] = o;
            }
            base += total;
            nb += kt;
            __syncthreads();  // wsum reuse
        }
        if (t == 0) {
            const float* Tc = B.results[f].Tcw;
            float W[16], V[16];
            inverse_pose(PF.Tlw, W);
            mat4_mul(Tc, W, V);
            spslam_proj_frame& N = B.next_frames[f];
            for (int q = 0; q < 16; q++) {
                B.velocity[16 * f + q] = V[q];
                N.Tlw[q] = Tc[q];
                N.Tcw[q] = Tc[q];  // replaced by MOTION_PRIOR
            }
            N.point_offset = (int32_t)ko;
            N.n_points = nb;
            N.pad[0] = N.pad[1] = 0;
        }
        return;
    }

    if (stage == SPSLAM_TRACK_DISCARD) {
        // src/Tracking.cc:986-1000, then ORBmatcher.cc:95-97's "already has a map point with observations"
        const spslam_local_frame& LF = B.local_frames[f];
        for (int i = t; i < n; i += kThreads) {
            const int e = B.edge_of_kp[ko + i];
            bool tk = false;
            if (e >= 0 && !B.point_outlier[ko + e])
                tk = B.proj_points[PF.point_offset + B.proj_match[ko + i]].n_obs > 0;
            B.taken[ko + i] = (uint8_t)tk;
            // every motion-model match, inlier or discarded, is mnLastFrameSeen = this frame (:997, :1380-1390)
            if (B.seen && e >= 0) B.seen[LF.seen_offset + B.proj_points[PF.point_offset + B.proj_match[ko + i]].id] = LF.stamp;
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

// TrackWithMotionModel's failure test (src/Tracking.cc:977 and the nmatchesMap count of :986-1053) and the
// switch to TrackReferenceKeyFrame's re-tracking (:796-817); see spslam_gpu.h.  One workgroup per frame.
__global__ __launch_bounds__(kThreads) void refkf_kernel(spslam_track_batch B, spslam_refkf_batch R, int stage) {
    const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    __shared__ int wsum[kThreads / 64];
    const int n = min(B.kp_counts[f], B.cap);
    const size_t ko = (size_t)f * B.cap;
    const spslam_proj_frame& PF = B.proj_frames[f];
    const int nm = R.nmatches[f];
    if (stage == SPSLAM_REFKF_SELECT) {
        const bool fb = R.fallback[f] != 0;
        const bool ap = fb && R.bow_nmatches[f] >= 10;  // TrackReferenceKeyFrame: if(nmatches<10) return false
        // the keyframe's matches as rows of its point set
        const int32_t* rows = R.refkf_rows + (size_t)R.refkf_index[f] * R.rows_stride;
        for (int i = t; i < B.cap; i += kThreads) {
            const int m = ap && i < n ? R.bow_match[ko + i] : -1;
            R.refkf_match[ko + i] = m >= 0 ? rows[m] : -1;
        }
        // mnLastFrameSeen: the motion model's matches that the keyframe's replace lose their stamp; its discarded
        // outliers keep theirs -- unless it stopped at < 10 matches (no discard at all)
        if (ap && B.seen) {
            const spslam_local_frame& LF = B.local_frames[f];
            for (int i = t; i < n; i += kThreads) {
                const int e = B.edge_of_kp[ko + i];
                if (e >= 0 && (nm < 10 || !B.point_outlier[ko + e]))
                    B.seen[LF.seen_offset + B.proj_points[PF.point_offset + B.proj_match[ko + i]].id] = LF.stamp - 1;
            }
        }
        if (t == 0) {
            R.apply[f] = (uint8_t)ap;
            if (R.state) R.state[f] = (int8_t)(ap ? 1 : fb ? 2 : 0);
            spslam_proj_frame& Q = R.refkf_frames[f];
            for (int q = 0; q < 16; q++) Q.Tcw[q] = Q.Tlw[q] = PF.Tlw[q];  // SetPose(mLastFrame.mTcw)
            Q.point_offset = R.refkf_sets[2 * f];
            Q.n_points = ap ? R.refkf_sets[2 * f + 1] : 0;
            Q.pad[0] = Q.pad[1] = 0;
            spslam_assoc_frame A = R.assoc_frames[f];
            for (int q = 0; q < 16; q++) A.Tcw[q] = PF.Tlw[q];
            if (!ap) A.n_map = 0;
            A.carry = nm >= 10 ? 1 : 0;
            R.refkf_assoc[f] = A;
        }
        return;
    }
    // PREPARE -- nmatchesMap: inlier map points with observations, then inlier matched map planes
    int c = 0;
    for (int i = t; i < n; i += kThreads) {
        const int e = B.edge_of_kp[ko + i];
        if (e >= 0 && !B.point_outlier[ko + e] && B.proj_points[PF.point_offset + B.proj_match[ko + i]].n_obs > 0) c++;
    }
    const spslam_pose_problem& P = B.problems[f];
    for (int j = t; j < P.n_planes; j += kThreads)
        if (B.planes[P.plane_offset + j].kind == SPSLAM_PLANE_EDGE && !B.plane_outlier[P.plane_offset + j]) c++;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off);
    if (lane == 0) wsum[wave] = c;
    __syncthreads();
    if (t != 0) return;
    int nmm = 0;
    for (int w = 0; w < kThreads / 64; w++) nmm += wsum[w];
    const bool fb = nm < 10 || nmm < 5;
    R.fallback[f] = (uint8_t)fb;
    R.refkf_counts[f] = fb ? B.kp_counts[f] : 0;
}

// UpdateLocalKeyFrames' pKFmax (src/Tracking.cc:1459-1570) / CreateNewKeyFrame's new keyframe (:1258); see
// spslam_gpu.h spslam_track_refkf_vote_batch_device.  One workgroup per frame: an LDS histogram of the frame's map
// points over their keyframes, then the first maximum in keyframe order.
constexpr int kMaxVoteKf = 1024;

__global__ __launch_bounds__(kThreads) void refkf_vote_kernel(spslam_track_batch B, spslam_refkf_vote V) {
    const int f = blockIdx.x, t = threadIdx.x;
    if (V.new_kf < 0 && V.state && V.state[f] == 2) return;  // LOST: TrackLocalMap does not run
    __shared__ int hist[kMaxVoteKf];
    __shared__ int best_s;
    const int nk = V.n_kf;
    int best = -1;
    if (V.new_kf < 0) {
        for (int j = t; j < nk; j += kThreads) hist[j] = 0;
        __syncthreads();
        const int n = min(B.kp_counts[f], B.cap);
        const size_t ko = (size_t)f * B.cap;
        const spslam_proj_frame& PF = B.proj_frames[f];
        for (int i = t; i < n; i += kThreads) {
            const int e = B.edge_of_kp[ko + i];
            if (e < 0 || B.point_outlier[ko + e]) continue;
            const int j = B.proj_points[PF.point_offset + B.proj_match[ko + i]].id / V.ids_per_kf;
            if (j >= 0 && j < nk) atomicAdd(&hist[j], 1);
        }
        __syncthreads();
        if (t == 0) {
            int mx = 0;
            for (int j = 0; j < nk; j++)
                if (hist[j] > mx) { mx = hist[j]; best = j; }  // if(it->second>max): the first maximum
            best_s = best;
        }
        __syncthreads();
        best = best_s;
    } else {
        best = V.new_kf;
    }
    if (t != 0) return;
    const int q = best >= 0 ? V.kf_base[f] + best : V.refkf_index[f];  // no map point: pKFmax stays NULL
    V.refkf_index[f] = q;
    V.refkf_sets[2 * f] = V.kf_sets[2 * q];
    V.refkf_sets[2 * f + 1] = V.kf_sets[2 * q + 1];
    if (V.refkf_pairs) {
        V.refkf_pairs[2 * f] = q;
        V.refkf_pairs[2 * f + 1] = f;
    }
}

// dst[f] = src[f] of every region for the flagged frames, 4 bytes per lane
__global__ __launch_bounds__(256) void masked_frame_copy_kernel(const uint8_t* __restrict__ flags, FrameRegions G) {
    const int f = blockIdx.x;
    if (!flags[f]) return;
    for (int k = 0; k < G.n; k++) {
        const spslam_frame_region& r = G.r[k];
        uint32_t* d = (uint32_t*)((uint8_t*)r.dst + f * r.dst_stride);
        const uint32_t* sp = (const uint32_t*)((const uint8_t*)r.src + f * r.src_stride);
        const int64_t nw = r.frame_bytes / 4;
        for (int64_t i = threadIdx.x; i < nw; i += blockDim.x) d[i] = sp[i];
    }
}

}  // namespace

hipError_t refkf_vote_launch(int n_frames, const spslam_track_batch& mm, const spslam_refkf_vote& v, hipStream_t s) {
    hipLaunchKernelGGL(refkf_vote_kernel, dim3(n_frames), dim3(kThreads), 0, s, mm, v);
    return hipGetLastError();
}

hipError_t refkf_launch(int n_frames, int stage, const spslam_track_batch& mm, const spslam_refkf_batch& rk,
                        hipStream_t s) {
    hipLaunchKernelGGL(refkf_kernel, dim3(n_frames), dim3(kThreads), 0, s, mm, rk, stage);
    return hipGetLastError();
}

hipError_t masked_frame_copy_launch(int n_frames, const uint8_t* flags, const FrameRegions& regions, hipStream_t s) {
    hipLaunchKernelGGL(masked_frame_copy_kernel, dim3(n_frames), dim3(256), 0, s, flags, regions);
    return hipGetLastError();
}

hipError_t track_launch(int n_frames, int stage, const TrackArgs& a, hipStream_t s, KernelTimer* timer) {
    if (timer) timer->begin(kKindTrack, s);
    hipLaunchKernelGGL(track_graph_kernel, dim3(n_frames), dim3(kThreads), 0, s, a, stage);
    if (timer) timer->end(kKindTrack, s);
    return hipGetLastError();
}

}  // namespace spslam
