// ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) on gfx950
// (src/ORBmatcher.cc:1328-1470, Frame::GetFeaturesInArea src/Frame.cc:427-480,
// DescriptorDistance :1647-1662, ComputeThreeMaxima :1601-1642) for a batch of
// frame pairs, with TrackWithMotionModel's second search at 2*th when fewer
// than retry_below matches (src/Tracking.cc:968-975).  Semantics:
// oracle/match_oracle.cpp.
//
//   match_window_kernel  grid (frame, 16 last-frame points), 16 lanes per point:
//                        projection and search window (redundantly per lane),
//                        the window's grid cells spread over the lanes, every
//                        candidate's Hamming distance (v_bcnt over the XOR of 8
//                        dwords); keeps the kProjKeys (6) best as (distance << 20 | CSR
//                        position), which orders ties like the reference's
//                        cell-by-cell scan, merged over the lanes (keys are
//                        unique, so the merge is the serial scan's result);
//   match_assign_kernel  grid (frame), one wave: the reference's loop is
//                        sequential only through `mvpMapPoints[i2] taken`, so
//                        the wave walks the points in order, accepts each
//                        point's precomputed best unless an earlier point took
//                        that keypoint, and only then re-scans the window
//                        cooperatively (64 lanes, min over keys) excluding the
//                        taken keypoints (LDS bitmap); then the rotation
//                        histogram check.
// Float expressions follow the reference build's contraction pattern; the
// cv::Mat products are accumulated in double and rounded once (oracle header).
#include <hip/hip_runtime.h>

#include "wave_priority.h"

#include "match_launch.h"

namespace spslam {
namespace match {

constexpr int kThreads = 256, kCols = SPSLAM_GRID_COLS, kRows = SPSLAM_GRID_ROWS, kHisto = 30, kThHigh = 100;
constexpr uint32_t kNone = 0xffffffffu;
// lanes per last-frame point in match_window_kernel: the serial chain of dependent loads (cell bounds,
// grid index, keypoint, descriptor) per candidate is what the in-step time of the window search is made of
// when the extraction streams load the memory system, so the window's cells are split over the lanes
constexpr int kGrp = 16, kPtsPerBlock = kThreads / kGrp;
// local-map windows are a few cells (radius 2.5-4 px x scale): 4 lanes per local point
constexpr int kLGrp = 4, kLPtsPerBlock = kThreads / kLGrp;

// insert a key into the ascending K smallest (keys unique; kNone = +inf)
template <int K>
__device__ __forceinline__ void insk(uint32_t (&b)[K], uint32_t x) {
#pragma unroll
    for (int q = 0; q < K; q++) {
        const uint32_t lo = min(b[q], x);
        x = max(b[q], x);
        b[q] = lo;
    }
}

__device__ __forceinline__ void mat3_mul(const float* T, const float* x, const float* c, bool transpose, double sign,
                                         float* y) {
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++)
            s = __dadd_rn(s, __dmul_rn((double)(transpose ? T[4 * k + r] : T[4 * r + k]), (double)x[k]));
        s = __dmul_rn(s, sign);
        if (c) s = __dadd_rn(s, (double)c[r]);
        y[r] = (float)s;
    }
}

__device__ __forceinline__ int hamming(const uint4& a0, const uint4& a1, const uint8_t* b) {
    const uint4 b0 = *(const uint4*)b, b1 = *(const uint4*)(b + 16);
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// bForward / bBackward of one frame pair (src/ORBmatcher.cc:1336-1349)
__device__ __forceinline__ void direction(const spslam_proj_frame& F, const MatchGeom& g, bool mono, bool* fwd,
                                          bool* bwd) {
    const float tcw[3] = {F.Tcw[3], F.Tcw[7], F.Tcw[11]};
    const float tlw[3] = {F.Tlw[3], F.Tlw[7], F.Tlw[11]};
    float twc[3], tlc[3];
    mat3_mul(F.Tcw, tcw, nullptr, true, -1.0, twc);
    mat3_mul(F.Tlw, twc, tlw, false, 1.0, tlc);
    const float mb = __fdiv_rn(g.bf, g.fx);
    *fwd = tlc[2] > mb && !mono;
    *bwd = -tlc[2] > mb && !mono;
}

// Candidate test of GetFeaturesInArea + the stereo check; returns the key or kNone.
template <class Win>
__device__ __forceinline__ uint32_t candidate_key(const Win& w, const MatchCurrent& C, const float* uright,
                                                  const uint8_t* desc, const spslam_keypoint* kun, int j, int k,
                                                  const uint4& d0, const uint4& d1, const MatchGeom& g) {
    const spslam_keypoint kp = kun[k];
    const bool check = (w.min_level > 0) || (w.max_level >= 0);
    if (check) {
        if (kp.octave < w.min_level) return kNone;
        if (w.max_level >= 0 && kp.octave > w.max_level) return kNone;
    }
    const float dx = __fsub_rn(kp.x, w.u), dy = __fsub_rn(kp.y, w.v);
    if (!(fabsf(dx) < w.r && fabsf(dy) < w.r)) return kNone;
    const float urk = uright[k];
    if (urk > 0) {
        const float ur = __fmaf_rn(-g.bf, w.invzc, w.u);
        const float er = fabsf(__fsub_rn(ur, urk));
        if (er > w.r) return kNone;
    }
    return ((uint32_t)hamming(d0, d1, desc + 32 * (size_t)k) << 20) | (uint32_t)j;
}

template <int K>
__global__ __launch_bounds__(kThreads) void match_window_kernel(const spslam_proj_frame* __restrict__ frames,
                                                                const spslam_proj_point* __restrict__ points,
                                                                int max_points, MatchCurrent C, MatchGeom g, float th,
                                                                int mono, int retry_below, int pass,
                                                                const int* __restrict__ nmatches,
                                                                MatchWindowK<K>* __restrict__ win) {
    tail_wave_priority();
    const int f = blockIdx.x, sub = threadIdx.x & (kGrp - 1);
    const int i = blockIdx.y * kPtsPerBlock + (int)(threadIdx.x / kGrp);
    const spslam_proj_frame& F = frames[f];
    if (pass == 1 && !(retry_below > 0 && nmatches[f] < retry_below)) return;
    if (i >= F.n_points || i >= max_points) return;  // uniform over the point's lanes, as every return below
    MatchWindowK<K> w{};
#pragma unroll
    for (int q = 0; q < K; q++) {
        w.best[q] = kNone;
        w.kp[q] = -1;
    }
    w.valid = 0;
    w.x0 = 1;
    w.x1 = 0;
    const spslam_proj_point p = points[F.point_offset + i];
    bool fwd, bwd;
    direction(F, g, mono != 0, &fwd, &bwd);
    const float tcw[3] = {F.Tcw[3], F.Tcw[7], F.Tcw[11]};
    float x3Dc[3];
    mat3_mul(F.Tcw, p.xw, tcw, false, 1.0, x3Dc);
    const float invzc = (float)__ddiv_rn(1.0, (double)x3Dc[2]);
    MatchWindowK<K>* W = win + (size_t)f * max_points + i;
    if (invzc < 0) { if (sub == 0) *W = w; return; }
    const float u = __fmaf_rn(__fmul_rn(g.fx, x3Dc[0]), invzc, g.cx);
    const float v = __fmaf_rn(__fmul_rn(g.fy, x3Dc[1]), invzc, g.cy);
    if (u < g.min_x || u > g.max_x || v < g.min_y || v > g.max_y) { if (sub == 0) *W = w; return; }
    const int oct = p.octave;
    const float th_eff = pass == 1 ? __fmul_rn(2.0f, th) : th;
    const float r = __fmul_rn(th_eff, g.scale[oct]);
    w.u = u; w.v = v; w.r = r; w.invzc = invzc;
    if (fwd) { w.min_level = oct; w.max_level = -1; }
    else if (bwd) { w.min_level = 0; w.max_level = oct; }
    else { w.min_level = oct - 1; w.max_level = oct + 1; }
    w.valid = 1;
    // GetFeaturesInArea cell range
    const int x0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(u, g.min_x), r), g.ginv_x)));
    const int x1 = min(kCols - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(u, g.min_x), r), g.ginv_x)));
    const int y0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(v, g.min_y), r), g.ginv_y)));
    const int y1 = min(kRows - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(v, g.min_y), r), g.ginv_y)));
    if (x0 >= kCols || x1 < 0 || y0 >= kRows || y1 < 0) { if (sub == 0) *W = w; return; }
    w.x0 = (int16_t)x0; w.x1 = (int16_t)x1; w.y0 = (int16_t)y0; w.y1 = (int16_t)y1;
    const int32_t* GO = C.grid_off + (size_t)f * (kCols * kRows + 1);
    const int32_t* GI = C.grid_idx + (size_t)f * C.cap;
    const spslam_keypoint* kun = C.kun + (size_t)f * C.cap;
    const uint8_t* desc = C.desc + (size_t)f * C.cap * 32;
    const float* uright = C.uright + (size_t)f * C.cap;
    const uint4 d0 = *(const uint4*)p.desc, d1 = *(const uint4*)(p.desc + 16);
    uint32_t bk[K];
#pragma unroll
    for (int q = 0; q < K; q++) bk[q] = kNone;
    // the window's cells (column-major, as the reference scans them) dealt round-robin to the point's lanes;
    // x1 < x0 or y1 < y0 (an empty range) gives no cells
    const int nrows = y1 - y0 + 1, ncells = x1 >= x0 && nrows > 0 ? (x1 - x0 + 1) * nrows : 0;
    for (int cell = sub; cell < ncells; cell += kGrp) {
        const int cx = cell / nrows, c = (x0 + cx) * kRows + y0 + (cell - cx * nrows);
        const int j0 = GO[c], j1 = GO[c + 1];
        for (int j = j0; j < j1; j++) insk(bk, candidate_key(w, C, uright, desc, kun, j, GI[j], d0, d1, g));
    }
#pragma unroll
    for (int o = kGrp / 2; o >= 1; o >>= 1) {
        uint32_t pk[K];
#pragma unroll
        for (int q = 0; q < K; q++) pk[q] = (uint32_t)__shfl_xor((int)bk[q], o);
#pragma unroll
        for (int q = 0; q < K; q++) insk(bk, pk[q]);
    }
    // lanes 0 .. K-1 resolve best[sub]'s keypoint and angle (read by the in-order walk)
    static_assert(K <= kGrp, "a lane per key");
    uint32_t mine = kNone;
#pragma unroll
    for (int q = 0; q < K; q++)
        if (sub == q) mine = bk[q];
    if (sub < K && mine != kNone) {
        const int k = GI[mine & 0xfffff];
        W->kp[sub] = k;
        W->kang[sub] = kun[k].angle;
    }
    if (sub == 0) {
        // kp / kang: written by lanes 0 .. K-1
        W->u = w.u; W->v = w.v; W->r = w.r; W->invzc = w.invzc;
        W->x0 = w.x0; W->x1 = w.x1; W->y0 = w.y0; W->y1 = w.y1;
        W->min_level = w.min_level; W->max_level = w.max_level; W->valid = w.valid; W->pad = 0;
#pragma unroll
        for (int q = 0; q < K; q++) W->best[q] = bk[q];
    }
    if (sub < K && mine == kNone) W->kp[sub] = -1;
}

// ComputeThreeMaxima
__device__ void three_maxima(const int* h, int* i1, int* i2, int* i3) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < kHisto; i++) {
        const int s = h[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < __fmul_rn(0.1f, (float)max1)) { ind2 = -1; ind3 = -1; }
    else if (max3 < __fmul_rn(0.1f, (float)max1)) ind3 = -1;
    *i1 = ind1; *i2 = ind2; *i3 = ind3;
}

template <int K>
__global__ __launch_bounds__(64) void match_assign_kernel(const spslam_proj_frame* __restrict__ frames,
                                                          const spslam_proj_point* __restrict__ points, int max_points,
                                                          MatchCurrent C, MatchGeom g, int check_ori, int retry_below,
                                                          int pass, const MatchWindowK<K>* __restrict__ win,
                                                          int2* __restrict__ pushes, int32_t* __restrict__ match,
                                                          int* __restrict__ nmatches) {
    tail_wave_priority();
    extern __shared__ uint32_t taken[];  // [ceil(cap / 32)], then claim[cap]
    __shared__ int hist[kHisto];
    __shared__ int ind[3];
    const int f = blockIdx.x, lane = threadIdx.x;
    const spslam_proj_frame& F = frames[f];
    if (pass == 1 && !(retry_below > 0 && nmatches[f] < retry_below)) return;
    const int n_kp = min(C.counts[f], C.cap), np = min(F.n_points, max_points);
    int32_t* M = match + (size_t)f * C.cap;
    const int words = (C.cap + 31) / 32;
    // claim[k]: per pass, first the earliest blocking acceptance of keypoint k, then the last committed one
    // (~0u / 0: none) -- one LDS atomic per lane instead of a 64-step shuffle scan per pass
    uint32_t* claim = taken + words;
    for (int k = lane; k < n_kp; k += 64) claim[k] = ~0u;
    for (int k = lane; k < n_kp; k += 64) M[k] = -1;  // fill(mvpMapPoints, NULL)
    for (int k = lane; k < words; k += 64) taken[k] = 0;
    if (lane < kHisto) hist[lane] = 0;
    __syncthreads();
    const MatchWindowK<K>* Wf = win + (size_t)f * max_points;
    const int32_t* GO = C.grid_off + (size_t)f * (kCols * kRows + 1);
    const int32_t* GI = C.grid_idx + (size_t)f * C.cap;
    const spslam_keypoint* kun = C.kun + (size_t)f * C.cap;
    const uint8_t* desc = C.desc + (size_t)f * C.cap * 32;
    const float* uright = C.uright + (size_t)f * C.cap;
    const spslam_proj_point* P = points + F.point_offset;
    int2* PU = pushes + (size_t)f * max_points;
    const float factor = __fdiv_rn(1.0f, (float)kHisto);
    int n_push = 0;
#ifdef SPSLAM_LA_DIAG  // diagnostic build: passes, serial stops and window re-scans per frame (device printf)
    int d_pass = 0, d_stop = 0, d_rescan = 0;
    const long long d_t0 = wall_clock64();
#endif
    // every lane fetches its point's precomputed state, one round of loads per 64 points, issued one chunk
    // ahead (in flight during the previous chunk's walk) ...
    MatchWindowK<K> wn{};
    int nobs_n = 0;
    float pang_n = 0.f;
    if (lane < np) { wn = Wf[lane]; nobs_n = P[lane].n_obs; pang_n = P[lane].angle; }
    for (int c0 = 0; c0 < np; c0 += 64) {
        const int i = c0 + lane;
        int valid = 0, blocking = 0;
        uint32_t best[K];
        int b[K];
        float kang[K];
#pragma unroll
        for (int q = 0; q < K; q++) {
            best[q] = kNone;
            b[q] = -1;
            kang[q] = 0.f;
        }
        float pangle = 0.f;
        const MatchWindowK<K> w = wn;
        const int nobs = nobs_n;
        const float pang = pang_n;
        if (i + 64 < np) { wn = Wf[i + 64]; nobs_n = P[i + 64].n_obs; pang_n = P[i + 64].angle; }
        if (i < np) {
            valid = w.valid;
#pragma unroll
            for (int q = 0; q < K; q++) {
                best[q] = w.best[q];
                if (valid && best[q] != kNone) {
                    b[q] = w.kp[q];  // resolved by the window kernel
                    kang[q] = w.kang[q];
                }
            }
            blocking = nobs > 0;
            pangle = pang;
        }
        // ... then the reference's loop over the 64 points, in passes: every point still to do takes the first of
        // its smallest keys whose keypoint is free; the points before the first one that cannot be decided
        // that way -- all K keys taken (a window re-scan), or its keypoint taken by an earlier point of the pass
        // that blocks it (a map point with observations) -- are committed together, in order; that point is
        // then walked alone (the reference's step with the updated taken set) and the next pass starts after it.
        const int m = min(64, np - c0);
        int start = 0;
        while (start < m) {
#ifdef SPSLAM_LA_DIAG
            d_pass++;
#endif
            uint32_t keyl = kNone;
            int bl = -1;
            float kangl = 0.f;
            bool rescanl = false;
            const bool act = lane >= start && lane < m && valid;
            if (act) {
#pragma unroll
                for (int q = 0; q < K; q++) {
                    if (keyl != kNone || rescanl || best[q] == kNone) continue;
                    if (!((taken[b[q] >> 5] >> (b[q] & 31)) & 1)) { keyl = best[q]; bl = b[q]; kangl = kang[q]; }
                    else if (q == K - 1) rescanl = true;
                }
            }
            const bool acc = act && !rescanl && keyl != kNone && (int)(keyl >> 20) <= kThHigh;
            const bool accb = acc && blocking;
            // conflicts with earlier blocking acceptances (the earliest blocking lane per keypoint)
            auto wsync = [] {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            };
            if (accb) atomicMin(&claim[bl], (uint32_t)lane);
            wsync();
            const bool conflict = acc && claim[bl] < (uint32_t)lane;
            wsync();
            if (acc) claim[bl] = 0u;  // reused below as "last committed lane + 1" (0: none)
            wsync();
            const bool stop = act && (rescanl || (acc && conflict));
            const unsigned long long sm = __ballot(stop);
            const int first = sm ? __ffsll((long long)sm) - 1 : m;
            const bool commit = acc && lane < first;
            const unsigned long long cm = __ballot(commit);
            // the last committed assignment of a keypoint wins, as in the reference's order
            if (commit) atomicMax(&claim[bl], (uint32_t)lane + 1u);
            wsync();
            const bool last = commit && claim[bl] == (uint32_t)lane + 1u;
            wsync();
            if (acc) claim[bl] = ~0u;
            int bin = 0;
            if (commit) {
                if (last) M[bl] = c0 + lane;
                if (blocking) atomicOr(&taken[bl >> 5], 1u << (bl & 31));
                if (check_ori) {
                    float rot = __fsub_rn(pangle, kangl);
                    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
                    bin = (int)roundf(__fmul_rn(rot, factor));
                    if (bin == kHisto) bin = 0;
                    atomicAdd(&hist[bin], 1);
                }
                PU[n_push + __popcll(cm & ((1ull << lane) - 1ull))] = make_int2(bl, bin);
            }
            n_push += __popcll(cm);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (first >= m) break;
#ifdef SPSLAM_LA_DIAG
            d_stop++;
#endif
            // the point that stopped the pass, alone (the reference's step for it)
            const int L = first;
            uint32_t bestL = kNone;
            int bL = -1;
            float kangL = 0.f;
            bool rescan = false;
#pragma unroll
            for (int q = 0; q < K; q++) {
                const uint32_t kq = (uint32_t)__shfl((int)best[q], L);
                const int bq = __shfl(b[q], L);
                const float aq = __shfl(kang[q], L);
                if (bestL != kNone || rescan || kq == kNone) continue;  // sorted: kNone ends the list
                if (!((taken[bq >> 5] >> (bq & 31)) & 1)) { bestL = kq; bL = bq; kangL = aq; }
                else if (q == K - 1) rescan = true;
            }
            if (rescan) {
#ifdef SPSLAM_LA_DIAG
                d_rescan++;
#endif
                // an earlier point holds this keypoint: search the window again without the taken ones
                const MatchWindowK<K> w = Wf[c0 + L];
                const spslam_proj_point& p = P[c0 + L];
                const uint4 d0 = *(const uint4*)p.desc, d1 = *(const uint4*)(p.desc + 16);
                uint32_t mn = kNone;
                for (int ix = w.x0; ix <= w.x1; ix++)
                    for (int iy = w.y0; iy <= w.y1; iy++) {
                        const int c = ix * kRows + iy;
                        for (int j = GO[c] + lane; j < GO[c + 1]; j += 64) {
                            const int k = GI[j];
                            if ((taken[k >> 5] >> (k & 31)) & 1) continue;
                            mn = min(mn, candidate_key(w, C, uright, desc, kun, j, k, d0, d1, g));
                        }
                    }
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
                bestL = mn;
                if (bestL != kNone) {
                    bL = GI[bestL & 0xfffff];
                    kangL = kun[bL].angle;
                }
            }
            start = L + 1;
            if (bestL == kNone || (int)(bestL >> 20) > kThHigh) continue;
            const int blockL = __shfl(blocking, L);
            const float pangL = __shfl(pangle, L);
            if (lane == 0) {
                M[bL] = c0 + L;
                if (blockL) taken[bL >> 5] |= 1u << (bL & 31);
                int binL = 0;
                if (check_ori) {
                    float rot = __fsub_rn(pangL, kangL);
                    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
                    binL = (int)roundf(__fmul_rn(rot, factor));
                    if (binL == kHisto) binL = 0;
                    hist[binL]++;
                }
                PU[n_push] = make_int2(bL, binL);
            }
            n_push++;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();
    int n = n_push;
    if (check_ori) {
        if (lane == 0) three_maxima(hist, &ind[0], &ind[1], &ind[2]);
        __syncthreads();
        const int i1 = ind[0], i2 = ind[1], i3 = ind[2];
        int removed = 0;
        for (int q = lane; q < n_push; q += 64) {
            const int2 e = PU[q];
            if (e.y != i1 && e.y != i2 && e.y != i3) {
                M[e.x] = -1;
                removed++;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) removed += __shfl_xor(removed, o);
        n -= removed;
    }
    if (lane == 0) nmatches[f] = n;
#ifdef SPSLAM_LA_DIAG
    if (lane == 0)
        printf("MA pass %d np %d nkp %d passes %d stops %d rescans %d matches %d us %.1f\n", pass, np, n_kp, d_pass,
               d_stop, d_rescan, n, (double)(wall_clock64() - d_t0) * 0.01);
#endif
}

// ---------------------------------------------------------------------------
// Tracking::SearchLocalPoints: isInFrustum + PredictScale per local point,
// then ORBmatcher::SearchByProjection(F, vpMapPoints, th) (src/ORBmatcher.cc:
// 45-130).  Same two-kernel shape: the window kernel keeps the kLocalKeys (6)
// smallest keys over the window (initially taken keypoints excluded); the
// in-order walk needs the best AND the second best among the keypoints still
// free (the ratio test), which the keys give unless in-loop assignments took
// all but one of them -- then the wave re-scans for both.
template <int K>
__global__ __launch_bounds__(kThreads) void local_window_kernel(const spslam_local_frame* __restrict__ frames,
                                                                const spslam_local_point* __restrict__ points,
                                                                int max_points, MatchCurrent C, MatchGeom g,
                                                                LocalConsts P, const uint8_t* __restrict__ taken_in,
                                                                LocalWindowK<K>* __restrict__ win,
                                                                uint8_t* __restrict__ in_view) {
    tail_wave_priority();
    const int f = blockIdx.x, sub = threadIdx.x & (kLGrp - 1);
    const int i = blockIdx.y * kLPtsPerBlock + (int)(threadIdx.x / kLGrp);
    const spslam_local_frame& F = frames[f];
    if (i >= F.n_points || i >= max_points) return;  // uniform over the point's lanes, as every return below
    LocalWindowK<K> w{};
#pragma unroll
    for (int q = 0; q < K; q++) {
        w.best[q] = kNone;
        w.kp[q] = -1;
        w.oct[q] = -1;
    }
    w.x0 = 1;
    w.x1 = 0;
    LocalWindowK<K>* W = win + (size_t)f * max_points + i;
    const spslam_local_point& p = points[F.point_offset + i];
    // points the frame already tracks (mnLastFrameSeen == the frame) are skipped before isInFrustum
    // (Tracking.cc:1396-1401); their mbTrackInView stays false
    if (P.seen && P.seen[F.seen_offset + p.id] == F.stamp) {
        if (sub == 0) {
            if (in_view) in_view[F.point_offset + i] = 0;
            *W = w;
        }
        return;
    }
    bool in = false;
    // Frame::isInFrustum(pMP, 0.5)
    const float tcw[3] = {F.Tcw[3], F.Tcw[7], F.Tcw[11]};
    float Pc[3], Ow[3];
    mat3_mul(F.Tcw, p.xw, tcw, false, 1.0, Pc);
    float u = 0.f, v = 0.f, invz = 0.f, viewCos = 0.f;
    int level = 0;
    do {
        if (Pc[2] < 0.0f) break;
        invz = __fdiv_rn(1.0f, Pc[2]);
        u = __fmaf_rn(__fmul_rn(g.fx, Pc[0]), invz, g.cx);
        v = __fmaf_rn(__fmul_rn(g.fy, Pc[1]), invz, g.cy);
        if (u < g.min_x || u > g.max_x || v < g.min_y || v > g.max_y) break;
        const float maxD = __fmul_rn(1.2f, p.max_dist), minD = __fmul_rn(0.8f, p.min_dist);
        mat3_mul(F.Tcw, tcw, nullptr, true, -1.0, Ow);
        const float PO[3] = {__fsub_rn(p.xw[0], Ow[0]), __fsub_rn(p.xw[1], Ow[1]), __fsub_rn(p.xw[2], Ow[2])};
        float sq = __fmul_rn(PO[0], PO[0]);
        sq = __fadd_rn(sq, __fmul_rn(PO[1], PO[1]));
        sq = __fadd_rn(sq, __fmul_rn(PO[2], PO[2]));
        const float dist = (float)__dsqrt_rn((double)sq);  // cv::norm
        if (dist < minD || dist > maxD) break;
        double dot = __dmul_rn((double)PO[0], (double)p.normal[0]);
        dot = __dadd_rn(dot, __dmul_rn((double)PO[1], (double)p.normal[1]));
        dot = __dadd_rn(dot, __dmul_rn((double)PO[2], (double)p.normal[2]));
        viewCos = (float)__ddiv_rn(dot, (double)dist);
        if (viewCos < P.view_cos_limit) break;
        // PredictScale: ceil(log(ratio) / mfLogScaleFactor); the correctly rounded logf gives the same
        // level as glibc's for every float ratio (tests/test_libm_restated.py)
        const float ratio = __fdiv_rn(p.max_dist, dist);
        int n = (int)ceilf(__fdiv_rn((float)log((double)ratio), P.log_scale_factor));
        level = n < 0 ? 0 : (n >= P.n_levels ? P.n_levels - 1 : n);
        in = true;
    } while (false);
    if (in_view && sub == 0) in_view[F.point_offset + i] = in;
    if (!in) { if (sub == 0) *W = w; return; }
    float r = viewCos > 0.998f ? 2.5f : 4.0f;  // RadiusByViewingCos
    if (P.th != 1.0f) r = __fmul_rn(r, P.th);
    const float rs = __fmul_rn(r, g.scale[level]);
    w.u = u; w.v = v; w.rs = rs; w.ur = __fmaf_rn(-g.bf, invz, u);
    w.level = (int8_t)level;
    w.in_view = 1;
    const int x0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(u, g.min_x), rs), g.ginv_x)));
    const int x1 = min(kCols - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(u, g.min_x), rs), g.ginv_x)));
    const int y0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(v, g.min_y), rs), g.ginv_y)));
    const int y1 = min(kRows - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(v, g.min_y), rs), g.ginv_y)));
    if (x0 >= kCols || x1 < 0 || y0 >= kRows || y1 < 0) { if (sub == 0) *W = w; return; }
    w.x0 = (int16_t)x0; w.x1 = (int16_t)x1; w.y0 = (int16_t)y0; w.y1 = (int16_t)y1;
    // the frame-to-frame candidate test with its window: same expressions (ur = fma(-mbf, invz, u))
    MatchWindow mw{};
    mw.u = u; mw.v = v; mw.r = rs; mw.invzc = invz;
    mw.min_level = (int8_t)(level - 1);
    mw.max_level = (int8_t)level;
    const int32_t* GO = C.grid_off + (size_t)f * (kCols * kRows + 1);
    const int32_t* GI = C.grid_idx + (size_t)f * C.cap;
    const spslam_keypoint* kun = C.kun + (size_t)f * C.cap;
    const uint8_t* desc = C.desc + (size_t)f * C.cap * 32;
    const float* uright = C.uright + (size_t)f * C.cap;
    const uint8_t* tk = taken_in ? taken_in + (size_t)f * C.cap : nullptr;
    const uint4 d0 = *(const uint4*)p.desc, d1 = *(const uint4*)(p.desc + 16);
    uint32_t bk[K];
#pragma unroll
    for (int q = 0; q < K; q++) bk[q] = kNone;
    // the window's cells dealt round-robin to the point's lanes, the lanes' smallest keys merged (unique keys)
    const int nrows = y1 - y0 + 1, ncells = x1 >= x0 && nrows > 0 ? (x1 - x0 + 1) * nrows : 0;
    for (int cell = sub; cell < ncells; cell += kLGrp) {
        const int cx = cell / nrows, c = (x0 + cx) * kRows + y0 + (cell - cx * nrows);
        const int j0 = GO[c], j1 = GO[c + 1];
        for (int j = j0; j < j1; j++) {
            const int k = GI[j];
            if (tk && tk[k]) continue;
            insk(bk, candidate_key(mw, C, uright, desc, kun, j, k, d0, d1, g));
        }
    }
#pragma unroll
    for (int o = kLGrp / 2; o >= 1; o >>= 1) {
        uint32_t pk[K];
#pragma unroll
        for (int q = 0; q < K; q++) pk[q] = (uint32_t)__shfl_xor((int)bk[q], o);
#pragma unroll
        for (int q = 0; q < K; q++) insk(bk, pk[q]);
    }
    // the keypoint and octave of each key (read by the in-order walk), resolved here
#pragma unroll
    for (int q = 0; q < K; q++) {
        w.best[q] = bk[q];
        if (bk[q] != kNone) {
            w.kp[q] = GI[bk[q] & 0xfffff];
            w.oct[q] = (int8_t)kun[w.kp[q]].octave;
        }
    }
    if (sub == 0) *W = w;
}

template <int K>
__global__ __launch_bounds__(64) void local_assign_kernel(const spslam_local_frame* __restrict__ frames,
                                                          const spslam_local_point* __restrict__ points,
                                                          int max_points, MatchCurrent C, MatchGeom g, LocalConsts P,
                                                          const uint8_t* __restrict__ taken_in,
                                                          const LocalWindowK<K>* __restrict__ win,
                                                          int32_t* __restrict__ match, int* __restrict__ nmatches) {
    tail_wave_priority();
    extern __shared__ uint32_t taken[];  // [ceil(cap / 32)], then claim[cap]
    const int f = blockIdx.x, lane = threadIdx.x;
    const spslam_local_frame& F = frames[f];
    const int n_kp = min(C.counts[f], C.cap), np = min(F.n_points, max_points);
    int32_t* M = match + (size_t)f * C.cap;
    const int words = (C.cap + 31) / 32;
    // claim[k]: the first lane of the current pass whose acceptance takes keypoint k (~0u: none); replaces a
    // 64-step shuffle scan per pass with one LDS atomic and two reads
    uint32_t* claim = taken + words;
    for (int k = lane; k < n_kp; k += 64) claim[k] = ~0u;
    const uint8_t* tk = taken_in ? taken_in + (size_t)f * C.cap : nullptr;
    for (int k = lane; k < n_kp; k += 64) M[k] = -1;
    // the taken bits: 8 coalesced byte loads in flight per lane, two words per ballot (a lane building its own
    // word byte by byte waited out 32 dependent loads per word)
    const int wset = tk ? 2 * ((n_kp + 63) / 64) : 0;  // words written from the flags (the rest are zero)
    for (int wd = wset + lane; wd < words; wd += 64) taken[wd] = 0u;
    for (int base = 0; base < n_kp && tk; base += 64 * 8) {
        uint8_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int k = base + 64 * u + lane;
            v[u] = tk[min(k, n_kp - 1)] & (uint8_t)(k < n_kp);  // unconditional load: no wait at a branch join
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const unsigned long long m = __ballot(v[u] != 0);
            const int wd = (base >> 5) + 2 * u;
            if (lane < 2 && wd + lane < min(words, wset)) taken[wd + lane] = (uint32_t)(m >> (32 * lane));
        }
    }
    __syncthreads();
    const LocalWindowK<K>* Wf = win + (size_t)f * max_points;
    const int32_t* GO = C.grid_off + (size_t)f * (kCols * kRows + 1);
    const int32_t* GI = C.grid_idx + (size_t)f * C.cap;
    const spslam_keypoint* kun = C.kun + (size_t)f * C.cap;
    const uint8_t* desc = C.desc + (size_t)f * C.cap * 32;
    const float* uright = C.uright + (size_t)f * C.cap;
    const spslam_local_point* Pp = points + F.point_offset;
    int nm = 0;
#ifdef SPSLAM_LA_DIAG  // diagnostic build: passes, serial stops and window re-scans per frame (device printf)
    int d_pass = 0, d_stop = 0, d_rescan = 0;
    const long long d_t0 = wall_clock64();
#endif
    LocalWindowK<K> wn{};  // the next chunk's window states, loaded one chunk ahead
    if (lane < np) wn = Wf[lane];
    for (int c0 = 0; c0 < np; c0 += 64) {
        const int i = c0 + lane;
        int valid = 0;
        uint32_t best[K];
        int b[K], oc[K];
#pragma unroll
        for (int q = 0; q < K; q++) {
            best[q] = kNone;
            b[q] = -1;
            oc[q] = -1;
        }
        const LocalWindowK<K> w = wn;
        if (i + 64 < np) wn = Wf[i + 64];
        if (i < np) {
            valid = w.in_view;
#pragma unroll
            for (int q = 0; q < K; q++) {
                best[q] = w.best[q];
                if (valid && best[q] != kNone) {
                    b[q] = w.kp[q];  // resolved by the window kernel
                    oc[q] = w.oct[q];
                }
            }
        }
        // the reference's loop in passes (as in match_assign_kernel): every point still to do evaluates its best
        // and second best free keys from its smallest keys; the points before the first one that cannot be decided
        // that way -- a re-scan, or one of its two keypoints taken by an earlier acceptance of the pass -- are
        // committed together; that point is walked alone and the next pass starts after it.
        const int m = min(64, np - c0);
        auto ratio_ok = [&](uint32_t k1, uint32_t k2, int o1, int o2) {
            const int bestDist = (int)(k1 >> 20), bestDist2 = k2 != kNone ? (int)(k2 >> 20) : 256;
            const int bestLevel2 = k2 != kNone ? o2 : -1;
            if (bestDist > kThHigh) return false;
            return !(o1 == bestLevel2 && (float)bestDist > __fmul_rn(P.nn_ratio, (float)bestDist2));
        };
        int start = 0;
        while (start < m) {
#ifdef SPSLAM_LA_DIAG
            d_pass++;
#endif
            const bool act = lane >= start && lane < m && valid;
            uint32_t k1 = kNone, k2 = kNone;
            int b1 = -1, b2 = -1, o1 = -1, o2 = -1, nk = 0;
            if (act) {
#pragma unroll
                for (int q = 0; q < K; q++) {
                    if (best[q] == kNone) continue;
                    nk++;
                    if ((taken[b[q] >> 5] >> (b[q] & 31)) & 1) continue;
                    if (k1 == kNone) { k1 = best[q]; b1 = b[q]; o1 = oc[q]; }
                    else if (k2 == kNone) { k2 = best[q]; b2 = b[q]; o2 = oc[q]; }
                }
            }
            const bool rescanl = act && nk == K && k2 == kNone;
            const bool acc = act && !rescanl && k1 != kNone && ratio_ok(k1, k2, o1, o2);
            // conflict: an earlier accepting lane of this pass takes my best or second-best keypoint
            if (acc) atomicMin(&claim[b1], (uint32_t)lane);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const bool conflict = act && k1 != kNone &&
                                  (claim[b1] < (uint32_t)lane || (b2 >= 0 && claim[b2] < (uint32_t)lane));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (acc) claim[b1] = ~0u;
            const bool stop = act && (rescanl || (k1 != kNone && conflict));
            const unsigned long long sm = __ballot(stop);
            const int first = sm ? __ffsll((long long)sm) - 1 : m;
            const bool commit = acc && lane < first;
            if (commit) {
                M[b1] = c0 + lane;
                atomicOr(&taken[b1 >> 5], 1u << (b1 & 31));
            }
            nm += __popcll(__ballot(commit));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (first >= m) break;
            const int L = first;
            start = L + 1;
#ifdef SPSLAM_LA_DIAG
            d_stop++;
#endif
            k1 = kNone; k2 = kNone; b1 = -1; o1 = -1; o2 = -1; nk = 0;
#pragma unroll
            for (int q = 0; q < K; q++) {
                const uint32_t kq = (uint32_t)__shfl((int)best[q], L);
                const int bq = __shfl(b[q], L), oq = __shfl(oc[q], L);
                if (kq == kNone) continue;
                nk++;
                if ((taken[bq >> 5] >> (bq & 31)) & 1) continue;
                if (k1 == kNone) { k1 = kq; b1 = bq; o1 = oq; }
                else if (k2 == kNone) { k2 = kq; o2 = oq; }
            }
            if (nk == K && k2 == kNone) {
                // in-loop assignments took all but one of the keys: best and second best over the window again
#ifdef SPSLAM_LA_DIAG
                d_rescan++;
#endif
                const LocalWindowK<K> w = Wf[c0 + L];
                MatchWindow mw{};
                mw.u = w.u; mw.v = w.v; mw.r = w.rs;
                mw.invzc = 0.f;
                mw.min_level = (int8_t)(w.level - 1);
                mw.max_level = w.level;
                const spslam_local_point& p = Pp[c0 + L];
                const uint4 d0 = *(const uint4*)p.desc, d1 = *(const uint4*)(p.desc + 16);
                uint32_t m1 = kNone, m2 = kNone;
                for (int ix = w.x0; ix <= w.x1; ix++)
                    for (int iy = w.y0; iy <= w.y1; iy++) {
                        const int c = ix * kRows + iy;
                        for (int j = GO[c] + lane; j < GO[c + 1]; j += 64) {
                            const int k = GI[j];
                            if ((taken[k >> 5] >> (k & 31)) & 1) continue;
                            // candidate_key's stereo test recomputes ur from invzc; use the stored mTrackProjXR
                            const spslam_keypoint kp = kun[k];
                            if (kp.octave < mw.min_level || kp.octave > mw.max_level) continue;
                            if (!(fabsf(__fsub_rn(kp.x, w.u)) < w.rs && fabsf(__fsub_rn(kp.y, w.v)) < w.rs)) continue;
                            const float urk = uright[k];
                            if (urk > 0 && fabsf(__fsub_rn(w.ur, urk)) > w.rs) continue;
                            const uint32_t key = ((uint32_t)hamming(d0, d1, desc + 32 * (size_t)k) << 20) | (uint32_t)j;
                            if (key < m1) { m2 = m1; m1 = key; }
                            else if (key < m2) m2 = key;
                        }
                    }
                // wave top-2: the smallest key, then the smallest key above it
                uint32_t t1 = m1;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) t1 = min(t1, (uint32_t)__shfl_xor((int)t1, o));
                uint32_t t2 = m1 == t1 ? m2 : m1;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) t2 = min(t2, (uint32_t)__shfl_xor((int)t2, o));
                k1 = t1;
                k2 = t2;
                b1 = k1 != kNone ? GI[k1 & 0xfffff] : -1;
                o1 = b1 >= 0 ? kun[b1].octave : -1;
                o2 = k2 != kNone ? kun[GI[k2 & 0xfffff]].octave : -1;
            }
            if (k1 == kNone || !ratio_ok(k1, k2, o1, o2)) continue;
            if (lane == 0) {
                M[b1] = c0 + L;
                taken[b1 >> 5] |= 1u << (b1 & 31);
            }
            nm++;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    if (lane == 0) nmatches[f] = nm;
#ifdef SPSLAM_LA_DIAG
    if (lane == 0)
        printf("LA np %d nkp %d passes %d stops %d rescans %d matches %d us %.1f\n", np, n_kp, d_pass, d_stop,
               d_rescan, nm, (double)(wall_clock64() - d_t0) * 0.01);
#endif
}

}  // namespace match

hipError_t local_match_launch(int n_frames, const spslam_local_frame* frames, const spslam_local_point* points,
                              int max_points, const MatchCurrent& cur, const MatchGeom& g, const LocalConsts& P,
                              const uint8_t* taken_in, LocalWindow* win, int32_t* match, int* nmatches,
                              uint8_t* in_view, hipStream_t s, KernelTimer* timer) {
    // taken bits + the claim table in dynamic LDS (opted in up to 160 KB: caps up to ~39K keypoints)
    const size_t lds = (size_t)((cur.cap + 31) / 32) * 4 + (size_t)cur.cap * 4;
    if (n_frames < 1 || max_points < 0 || cur.cap < 1 || lds > 160 * 1024) return hipErrorInvalidValue;
    static const hipError_t lds_attr = [] {
        const hipError_t a = hipFuncSetAttribute((const void*)match::local_assign_kernel<kLocalKeys>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return a != hipSuccess ? a : hipFuncSetAttribute((const void*)match::local_assign_kernel<kFewKeys>,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }();
    if (lds_attr != hipSuccess) return lds_attr;
    if (timer) timer->begin(kKindLocalMatch, s);
    auto run = [&](auto* w) {
        constexpr int K = sizeof(w->best) / sizeof(w->best[0]);
        if (max_points > 0)
            hipLaunchKernelGGL(match::local_window_kernel<K>,
                               dim3(n_frames, (max_points + match::kLPtsPerBlock - 1) / match::kLPtsPerBlock),
                               dim3(match::kThreads), 0, s, frames, points, max_points, cur, g, P, taken_in, w, in_view);
        hipLaunchKernelGGL(match::local_assign_kernel<K>, dim3(n_frames), dim3(64), lds, s,
                           frames, points, max_points, cur, g, P, taken_in, w, match, nmatches);
    };
    if (n_frames <= kSmallBatchKeys) run(win);
    else run(reinterpret_cast<LocalWindowK<kFewKeys>*>(win));
    if (timer) timer->end(kKindLocalMatch, s);
    return hipGetLastError();
}

hipError_t match_launch(int n_frames, const spslam_proj_frame* frames, const spslam_proj_point* points,
                        int max_points, const MatchCurrent& cur, const MatchGeom& g, const spslam_match_params& P,
                        MatchWindow* win, int2* pushes, int32_t* match, int* nmatches, hipStream_t s,
                        KernelTimer* timer) {
    // taken bits + the claim table in dynamic LDS (opted in up to 150 KB: caps up to ~36K keypoints)
    const size_t lds = (size_t)((cur.cap + 31) / 32) * 4 + (size_t)cur.cap * 4;
    if (n_frames < 1 || max_points < 0 || cur.cap < 1 || lds > 150 * 1024) return hipErrorInvalidValue;
    static const hipError_t lds_attr = [] {
        const hipError_t a = hipFuncSetAttribute((const void*)match::match_assign_kernel<kProjKeys>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        return a != hipSuccess ? a : hipFuncSetAttribute((const void*)match::match_assign_kernel<kFewKeys>,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    }();
    if (lds_attr != hipSuccess) return lds_attr;
    if (timer) timer->begin(kKindMatch, s);
    const int passes = P.retry_below > 0 ? 2 : 1;
    auto run = [&](auto* w) {
        constexpr int K = sizeof(w->best) / sizeof(w->best[0]);
        for (int pass = 0; pass < passes; pass++) {
            if (max_points > 0)
                hipLaunchKernelGGL(match::match_window_kernel<K>,
                                   dim3(n_frames, (max_points + match::kPtsPerBlock - 1) / match::kPtsPerBlock),
                                   dim3(match::kThreads), 0, s, frames, points, max_points, cur, g, P.th, P.mono,
                                   P.retry_below, pass, nmatches, w);
            hipLaunchKernelGGL(match::match_assign_kernel<K>, dim3(n_frames), dim3(64), lds, s, frames, points,
                               max_points, cur, g, P.check_orientation, P.retry_below, pass, w, pushes, match, nmatches);
        }
    };
    if (n_frames <= kSmallBatchKeys) run(win);
    else run(reinterpret_cast<MatchWindowK<kFewKeys>*>(win));
    if (timer) timer->end(kKindMatch, s);
    return hipGetLastError();
}

}  // namespace spslam
