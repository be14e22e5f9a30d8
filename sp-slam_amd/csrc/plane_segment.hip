// gfx950 segmentation stage of Frame::ComputePlanesFromOrganizedPointCloud
// (src/Frame.cc:876-934): pcl::OrganizedMultiPlaneSegmentation::segmentAndRefine
// (PCL 1.8, PlaneCoefficientComparator + PlaneRefinementComparator), the
// boundary extraction, Frame's sign flip and PlaneNotSeen.
//
// One 1024-thread workgroup per frame.  Phases (each a block-wide barrier
// apart); the per-frame maps live in LDS when they fit (C2: 214x160), in
// global scratch otherwise (C5):
//   A  row runs: one wave per cloud row; ballots give the comparator's
//      horizontal/vertical edge bits (LDS bitmaps) and each pixel's run head
//   B  union-find over run heads, one vertical link per run overlap
//      (min-index linking with atomicMin => root = first raster pixel)
//   C  path flattening;  D  labels = rank of the root (PCL's label order),
//      component sizes by wave-aggregated atomics;  E  components > MinSize
//   G  per component, one wave: raster-order member list and PCL's float
//      mean/covariance accumulation (terms staged through LDS, nine lanes
//      each own one accumulator, so the sums are the reference's sequence)
//   H  eigen33 / viewpoint / curvature filter (models)
//   K  refinement: the reference's two raster passes are row recurrences;
//      one wave evaluates each row with a scan over composed per-pixel
//      transfer functions (constant label, or pass-through-if-accepted
//      bitmask over models), so a row costs O(log 64) instead of O(W)
//      dependent steps; grow events are emitted in the reference's order
//   L  Frame.cc:912-934 sign flip + PlaneNotSeen;  M  inlier lists
//   N  findLabeledRegionBoundary: Moore tracing from per-pixel 8-neighbour
//      masks, one wave per plane (count pass, offsets, write pass)
// Reference semantics are restated in oracle/plane_oracle.cpp:268-470.
#include "libm_restated.h"
#include <hip/hip_runtime.h>

#include "plane_launch.h"
#include "plane_not_seen.h"

// The early wave exits below (surplus waves end while the rest of the workgroup still meets __syncthreads)
// rely on gfx9's s_barrier waiting only for the waves that have not ended.  Other targets keep every wave to
// the end of the kernel.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__) && !defined(SPSLAM_SEG_NO_EARLY_EXIT)
#define SPSLAM_SEG_NO_EARLY_EXIT 1
#endif

namespace spslam {
namespace planes {

#ifndef SPSLAM_SEG_THREADS
#define SPSLAM_SEG_THREADS 1024
#endif
constexpr int kSegThreads = SPSLAM_SEG_THREADS;
// Fast refinement paths: the waves beyond max(models, SPSLAM_SEG_MIN_LIVE) end after refinement pass
// SPSLAM_SEG_EXIT_PASS's descriptors (measurement knobs; see plane_segment_kernel phase K)
#ifndef SPSLAM_SEG_EXIT_PASS
#define SPSLAM_SEG_EXIT_PASS 0
#endif
#ifndef SPSLAM_SEG_MIN_LIVE
#define SPSLAM_SEG_MIN_LIVE 8
#endif
constexpr int kSegWaves = kSegThreads / 64;
constexpr int kMaxBig = 255;          // components > MinSize per frame (u8 tags)
constexpr int kMaxRowWords = 8;       // W <= 512
#ifndef SPSLAM_SEG_COV_AHEAD
#define SPSLAM_SEG_COV_AHEAD 4
#endif
constexpr int kPD = SPSLAM_SEG_COV_AHEAD;  // phase G: member coordinate chunks in flight per wave
constexpr int kLdsBytes = 160 * 1024;

struct SegShared {
    int wsum[kSegWaves];
    int misc[8];
    int nbig;
    int big_label[kMaxBig];
    int big_size[kMaxBig];
    int big_off[kMaxBig];
    float big_par[kMaxBig][4];
    float big_cen[kMaxBig][4];
    float big_curv[kMaxBig];
    uint8_t big_state[kMaxBig + 1];
    int nmodel;
    int model_big[kMaxPlanesPerFrame];
    float model_coef[kMaxPlanesPerFrame][4];
    int model_grown[kMaxPlanesPerFrame];
    int nkept;
    int kept[kMaxPlanesPerFrame];
    int con_len[kMaxPlanesPerFrame];
    int con_start[kMaxPlanesPerFrame];
    alignas(16) float stage[kSegWaves][9][64];   // covariance terms of one 64-pixel chunk, per wave
};

// The whole frame lives in one workgroup (one CU): workgroup scope is enough
// for every global-memory hand-off, and avoids the L2 writeback/invalidate an
// agent-scope fence costs on gfx950.
__device__ __forceinline__ int ld_wg(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int uf_find(const int* P, int x) {
    int p = ld_wg(&P[x]);
    while (p != x) { x = p; p = ld_wg(&P[x]); }
    return x;
}
// Lock-free union with min-index linking: P[x] <= x always, a root is the
// smallest index of its tree.
__device__ void uf_union(int* P, int a, int b) {
    a = uf_find(P, a);
    b = uf_find(P, b);
    while (a != b) {
        if (a < b) { const int t = a; a = b; b = t; }
        const int old = __hip_atomic_fetch_min(&P[a], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old == a) return;
        a = uf_find(P, old);
        b = uf_find(P, b);
    }
}

// The LDS instance's parents: 16-bit pixel indices (N < 0xFFFF), kNone16 = invalid point; the same 2N bytes later
// hold the tag / model map and the contour masks.  gfx950's LDS has no 16-bit min, so the link is a 32-bit
// compare-and-swap on the word holding the entry.
constexpr uint32_t kNone16 = 0xFFFFu;
__device__ __forceinline__ int ld16(const uint16_t* P, int x) {
    return __hip_atomic_load(&P[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int uf_find16(const uint16_t* P, int x) {
    int p = ld16(P, x);
    while (p != x) { x = p; p = ld16(P, x); }
    return x;
}
// P[a] = min(P[a], b); returns the previous P[a]
__device__ __forceinline__ int fetch_min16(uint16_t* P, int a, int b) {
    uint32_t* w = (uint32_t*)P + (a >> 1);
    const int sh = (a & 1) << 4;
    uint32_t old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (true) {
        const int cur = (int)((old >> sh) & 0xFFFFu);
        if (cur <= b) return cur;
        const uint32_t nw = (old & ~(0xFFFFu << sh)) | ((uint32_t)b << sh);
        if (__hip_atomic_compare_exchange_strong(w, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP))
            return cur;
    }
}
__device__ void uf_union16(uint16_t* P, int a, int b) {
    a = uf_find16(P, a);
    b = uf_find16(P, b);
    while (a != b) {
        if (a < b) { const int t = a; a = b; b = t; }
        const int old = fetch_min16(P, a, b);
        if (old == a) return;
        a = uf_find16(P, old);
        b = uf_find16(P, b);
    }
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return (1ull << lane) - 1ull;
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void block_sync() {
    __syncthreads();   // workgroup-scope release/acquire (global and LDS)
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
    const int lo = __shfl_up((int)(uint32_t)v, d), hi = __shfl_up((int)(uint32_t)(v >> 32), d);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
// Exclusive wave prefix sum of v; *total = wave sum.
__device__ __forceinline__ int wave_excl(int v, int* total) {
    const int lane = threadIdx.x & 63;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    *total = __shfl(x, 63);
    return x - v;
}

// pcl::computeRoots / eigen33 (float), see oracle/plane_oracle.cpp.
__device__ void roots2(float b, float c, float* r) {
    r[0] = 0.f;
    float d = (float)(b * b - 4.0 * c);
    if (d < 0.0) d = 0.0;
    const float sd = sqrtf(d);
    r[2] = 0.5f * (b + sd);
    r[1] = 0.5f * (b - sd);
}
__device__ void eigen33_min(const float (&m0)[3][3], float* eval, float* evec) {
    float scale = 0.f;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) scale = fmaxf(scale, fabsf(m0[i][j]));
    if (scale <= 1.17549435e-38f) scale = 1.f;
    float m[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) m[i][j] = m0[i][j] / scale;
    float r[3];
    const float c0 = m[0][0] * m[1][1] * m[2][2] + 2.f * m[0][1] * m[0][2] * m[1][2] - m[0][0] * m[1][2] * m[1][2] -
                     m[1][1] * m[0][2] * m[0][2] - m[2][2] * m[0][1] * m[0][1];
    const float c1 = m[0][0] * m[1][1] - m[0][1] * m[0][1] + m[0][0] * m[2][2] - m[0][2] * m[0][2] +
                     m[1][1] * m[2][2] - m[1][2] * m[1][2];
    const float c2 = m[0][0] + m[1][1] + m[2][2];
    if (fabsf(c0) < 1.1920929e-07f) {
        roots2(c2, c1, r);
    } else {
        const float s_inv3 = (float)(1.0 / 3.0), s_sqrt3 = sqrtf(3.0f);
        const float c2_over_3 = c2 * s_inv3;
        float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
        if (a_over_3 > 0.f) a_over_3 = 0.f;
        const float half_b = 0.5f * (c0 + c2_over_3 * (2.f * c2_over_3 * c2_over_3 - c1));
        float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
        if (q > 0.f) q = 0.f;
        const float rho = sqrtf(-a_over_3);
        const float theta = libm::atan2f_(sqrtf(-q), half_b) * s_inv3;  // glibc-exact (libm_restated.h)
        float st, ct;
        libm::sincosf_(theta, &st, &ct);
        r[0] = c2_over_3 + 2.f * rho * ct;
        r[1] = c2_over_3 - rho * (ct + s_sqrt3 * st);
        r[2] = c2_over_3 - rho * (ct - s_sqrt3 * st);
        float t;
        if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
        if (r[1] >= r[2]) {
            t = r[1]; r[1] = r[2]; r[2] = t;
            if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
        }
        if (r[0] <= 0) roots2(c2, c1, r);
    }
    *eval = r[0] * scale;
    for (int i = 0; i < 3; i++) m[i][i] -= r[0];
    float v[3][3];
    const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    float len[3];
    for (int k = 0; k < 3; k++) {
        const float* a = m[pr[k][0]];
        const float* b = m[pr[k][1]];
        v[k][0] = a[1] * b[2] - a[2] * b[1];
        v[k][1] = a[2] * b[0] - a[0] * b[2];
        v[k][2] = a[0] * b[1] - a[1] * b[0];
        len[k] = v[k][0] * v[k][0] + v[k][1] * v[k][1] + v[k][2] * v[k][2];
    }
    int k = 2;
    if (len[0] >= len[1] && len[0] >= len[2]) k = 0;
    else if (len[1] >= len[0] && len[1] >= len[2]) k = 1;
    const float sl = sqrtf(len[k]);
    for (int j = 0; j < 3; j++) evec[j] = v[k][j] / sl;
}

// Eigen SSE predux order for a Vector4f dot.
__device__ __forceinline__ float dot4(const float* a, const float* b) {
    const float p0 = a[0] * b[0], p1 = a[1] * b[1], p2 = a[2] * b[2], p3 = a[3] * b[3];
    return (p0 + p2) + (p1 + p3);
}

// ---------------------------------------------------------------------------
// Refinement.  A pixel's state is 0 or model+1.  Per row, each pixel maps the
// state arriving along the row chain (from the previous pixel of the pass
// order) to its final state: a constant (already labelled, or grown from the
// previous row, which the reference does first), or "keep the incoming model
// if this point is within 0.02 m of it".  Such maps compose associatively.
struct Fn {
    uint64_t m;  // pass-through models (bit v-1 for state v), when c < 0
    int c;       // constant output, or -1
};
__device__ __forceinline__ int fn_apply(const Fn& f, int L) {
    if (f.c >= 0) return f.c;
    return (L > 0 && ((f.m >> (L - 1)) & 1ull)) ? L : 0;
}
__device__ __forceinline__ Fn fn_then(const Fn& first, const Fn& second) {
    if (second.c >= 0) return second;
    if (first.c >= 0) return Fn{0ull, fn_apply(second, first.c)};
    return Fn{first.m & second.m, -1};
}

// PlaneRefinementComparator::compare (absolute 0.02 m): float expression,
// compared after promotion as the reference does.
__device__ __forceinline__ bool ptp_ok(const float* m, float x, float y, float z) {
    const float e = m[0] * x + m[1] * y + m[2] * z + m[3];
    return fabsf(e) < 0.02f;
}

template <int K, class T>
__device__ __forceinline__ T sel(const T (&a)[K], int k) {
    T v = 0;
#pragma unroll
    for (int j = 0; j < K; j++)
        if (j == k) v = a[j];
    return v;
}

// One refinement pass by one wave (reference: OrganizedMultiPlaneSegmentation
// ::refine, the forward loop r = 0..H-2 / c = 0..W-2 growing right then
// down, and the backward loop r = H-1..1 / c = W-1..0 growing left (row-wrap
// at c = 0) then up).  Lane l owns pass positions p = l*K + k; column
// c = p (forward) or W-1-p (backward).  Grow events are appended to ev[] in
// the reference's order: events of a source row are emitted once both of
// their target rows are final.  Returns the number of events appended.
template <int K>
__device__ __forceinline__ int refine_pass(SegShared& S, uint8_t* state, const uint64_t* cbits, const float* X, const float* Y,
                           const float* Z, int W, int H, bool bw, int* ev, int ev_base) {
    const int RW = (W + 63) >> 6;
    const int lane = threadIdx.x & 63;
    const int nmodel = S.nmodel;
    const int lastLane = (W - 1) / K, lastK = (W - 1) - lastLane * K;
    // per-position flags are K-bit masks (bit k = position lane*K+k)
    int prevS[K];
    int pvm = 0, pcm = 0;  // previous row: valid points, grown along the chain
#pragma unroll
    for (int k = 0; k < K; k++) prevS[k] = 0;
    int carry = 0, ng = 0;
    // prefetch of the next row (its state is not touched by the current step)
    float qx[K], qy[K], qz[K];
    int qs[K];
    // unconditional clamped loads, masked at use (see refine_rows)
#define SPSLAM_REFINE_FETCH(STEP)                                                  \
    {                                                                              \
        const int st_ = min((STEP), H - 1);                                        \
        const int r_ = bw ? H - 1 - st_ : st_;                                     \
        _Pragma("unroll") for (int k = 0; k < K; k++) {                            \
            const int p = min(lane * K + k, W - 1);                                \
            const int i = r_ * W + (bw ? W - 1 - p : p);                           \
            qs[k] = state[i];                                                      \
            qx[k] = X[i]; qy[k] = Y[i]; qz[k] = Z[i];                              \
        }                                                                          \
    }
    SPSLAM_REFINE_FETCH(0)
    for (int step = 0; step < H; step++) {
        const int r = bw ? H - 1 - step : step;
        int s0[K], fin[K];
        float px[K], py[K], pz[K];
        int vm = 0;
#pragma unroll
        for (int k = 0; k < K; k++) {
            const bool in = lane * K + k < W;
            s0[k] = in ? qs[k] : 0; px[k] = in ? qx[k] : 0.f; py[k] = in ? qy[k] : 0.f; pz[k] = in ? qz[k] : 0.f;
            if (in && isfinite(px[k])) vm |= 1 << k;
        }
        SPSLAM_REFINE_FETCH(step + 1)
        // neighbours across lanes: previous row at position p+1, current row at p-1 / position 0
        const int nbS = __shfl_down(prevS[0], 1);
        const int nb = __shfl_down(pvm | (pcm << 8), 1);
        const int nbV = nb & 1, nbC = (nb >> 8) & 1;
        const int pvV = (__shfl_up(vm, 1) >> (K - 1)) & 1;
        const int cur0V = __shfl(vm, 0) & 1;
        const int wrapV = (__shfl(pvm, lastLane) >> lastK) & 1;
        // rows without a growable point (unlabelled, valid, within 0.02 m of some
        // model) keep their states: skip the composition
        int any = 0;
        for (int w = 0; w < RW; w++) any |= cbits[r * RW + w] != 0ull;
        int gm = 0, cm = 0;  // grown from the previous row / along the row chain
        if (!any) {
#pragma unroll
            for (int k = 0; k < K; k++) fin[k] = s0[k];
        } else {
        int cand = 0;
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int p = lane * K + k;
            if (p < W) {
                const int c = bw ? W - 1 - p : p;
                cand |= (int)((cbits[r * RW + (c >> 6)] >> (c & 63)) & 1ull) << k;
            }
        }
        Fn g[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int p = lane * K + k;
            const int c = bw ? W - 1 - p : p;
            const int vk = (vm >> k) & 1, pvk = (pvm >> k) & 1;
            const int pv1 = k < K - 1 ? (pvm >> (k + 1)) & 1 : nbV;   // previous row, position p+1
            const int vm1 = k > 0 ? (vm >> (k - 1)) & 1 : pvV;        // current row, position p-1
            // vertical source: the previous row's pixel in this column
            bool act;
            if (!bw) act = step >= 1 && c <= W - 2 && pvk && pv1 && vk;
            else act = step >= 1 && pvk && (c >= 1 ? pv1 : cur0V) && vk;
            if (p >= W) {
                g[k] = Fn{0ull, 0};
            } else if (s0[k]) {
                g[k] = Fn{0ull, s0[k]};
            } else if (!((cand >> k) & 1)) {
                g[k] = Fn{0ull, 0};
            } else if (act && prevS[k] && ptp_ok(S.model_coef[prevS[k] - 1], px[k], py[k], pz[k])) {
                g[k] = Fn{0ull, prevS[k]};
                gm |= 1 << k;
            } else {
                bool link;
                if (!bw) link = p >= 1 && r <= H - 2 && vm1 && vk;
                else if (p >= 1) link = r >= 1 && vm1 && vk;
                else link = step >= 1 && wrapV && vk;
                if (link) {
                    uint64_t m = 0;
                    for (int v = 0; v < nmodel; v++)
                        if (ptp_ok(S.model_coef[v], px[k], py[k], pz[k])) m |= 1ull << v;
                    g[k] = Fn{m, -1};
                } else {
                    g[k] = Fn{0ull, 0};
                }
            }
        }
        // compose along the row: lane-local, then a wave inclusive scan
        Fn F = g[0];
#pragma unroll
        for (int k = 1; k < K; k++) F = fn_then(F, g[k]);
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const Fn o{shfl_up64(F.m, off), __shfl_up(F.c, off)};
            if (lane >= off) F = fn_then(o, F);
        }
        Fn ex{shfl_up64(F.m, 1), __shfl_up(F.c, 1)};
        if (lane == 0) ex = Fn{~0ull, -1};
        int L = fn_apply(ex, bw ? carry : 0);
#pragma unroll
        for (int k = 0; k < K; k++) {
            fin[k] = fn_apply(g[k], L);
            if (g[k].c < 0 && fin[k] != 0) cm |= 1 << k;
            L = fin[k];
            const int p = lane * K + k;
            if (p < W && s0[k] == 0 && fin[k] != 0) state[r * W + (bw ? W - 1 - p : p)] = (uint8_t)fin[k];
        }
        }
        carry = __shfl(sel<K>(fin, lastK), lastLane);
        // emit the events of the previous row's sources, in pass order
        if (step >= 1) {
            const int chain0 = __shfl(cm, 0) & 1, fin0 = __shfl(fin[0], 0);
            int n = 0;
#pragma unroll
            for (int k = 0; k < K; k++) {
                const int p = lane * K + k;
                int fa = 0;
                if (p <= W - 2) fa = k < K - 1 ? (pcm >> (k + 1)) & 1 : nbC;
                else if (p == W - 1 && bw) fa = chain0;
                n += fa + ((gm >> k) & 1);
            }
            int tot;
            int o = ev_base + ng + wave_excl(n, &tot);
#pragma unroll
            for (int k = 0; k < K; k++) {
                const int p = lane * K + k;
                const int c = bw ? W - 1 - p : p;
                // A: along the source row (forward: right, backward: left / row wrap)
                int fa = 0, ta = 0, ma = 0;
                if (p <= W - 2) {
                    fa = k < K - 1 ? (pcm >> (k + 1)) & 1 : nbC;
                    ma = k < K - 1 ? prevS[k + 1] : nbS;
                    ta = bw ? (r + 1) * W + c - 1 : (r - 1) * W + c + 1;
                } else if (p == W - 1 && bw) {
                    fa = chain0; ma = fin0; ta = r * W + W - 1;
                }
                if (fa) ev[o++] = ta | ((ma - 1) << 24);
                // B: into this row (forward: down, backward: up)
                if ((gm >> k) & 1) ev[o++] = (r * W + c) | ((fin[k] - 1) << 24);
            }
            ng += tot;
        }
#pragma unroll
        for (int k = 0; k < K; k++) prevS[k] = fin[k];
        pvm = vm;
        pcm = cm;
    }
    return ng;
#undef SPSLAM_REFINE_FETCH
}

// Fast paths (nmodel <= kFastModels = 14, or <= kWideModels = 30).  Before
// each pass every point gets a descriptor, computed in parallel: one bit per
// model whose plane is within 0.02 m of the point (only for valid, still
// unlabelled points), an "act" bit (its vertical source may grow it) and a
// "link" bit (its chain source may grow it) -- source and source-neighbour
// validity, row limits of the reference loops.  Narrow: 16 bits (models 0-13,
// act 14, link 15) in two byte planes; wide: one 32-bit word (models 0-29, act
// 30, link 31).  The pass itself then only composes per-pixel transfer
// functions (a constant flag; the constant state, or the complement of the
// pass-through set, so 0 is the identity), scanned with DPP.  Which grow event
// produced each new label is re-derived afterwards from the final states, in
// parallel, in the reference's event order.
constexpr int kFastModels = 14;
constexpr int kWideModels = 30;
template <bool kWide>
struct Desc;
template <>
struct Desc<false> {
    static constexpr uint32_t kAcc = 0x3FFFu, kAct = 0x4000u, kLink = 0x8000u;
    static constexpr uint32_t kConst = 0x10000u, kVal = 0xFFFFu;  // transfer functions
    uint8_t* lo;
    uint8_t* hi;
    __device__ __forceinline__ uint32_t get(int i) const { return lo[i] | ((uint32_t)hi[i] << 8); }
    __device__ __forceinline__ void put(int i, uint32_t d) const {
        lo[i] = (uint8_t)d;
        hi[i] = (uint8_t)(d >> 8);
    }
};
template <>
struct Desc<true> {
    static constexpr uint32_t kAcc = 0x3FFFFFFFu, kAct = 0x40000000u, kLink = 0x80000000u;
    static constexpr uint32_t kConst = 0x80000000u, kVal = 0x3FFFFFFFu;
    uint32_t* w;
    __device__ __forceinline__ uint32_t get(int i) const { return w[i]; }
    __device__ __forceinline__ void put(int i, uint32_t d) const { w[i] = d; }
};

template <class D>
__device__ __forceinline__ uint32_t fn_pass(uint32_t f, uint32_t L) {  // f: complemented pass-through set
    return (L > 0 && !((f >> ((L - 1) & 31)) & 1u)) ? L : 0u;
}
template <class D>
__device__ __forceinline__ uint32_t fn_then(uint32_t first, uint32_t second) {
    const uint32_t through = D::kConst | fn_pass<D>(second, first & D::kVal);
    const uint32_t both = first | second;
    const uint32_t r = (first & D::kConst) ? through : both;
    return (second & D::kConst) ? second : r;
}
template <class D>
__device__ __forceinline__ uint32_t fn_apply(uint32_t f, uint32_t L) {
    return (f & D::kConst) ? (f & D::kVal) : fn_pass<D>(f, L);
}
// Inclusive wave scan of fn_then (lane order), DPP row shifts + row broadcasts (0 = identity fills).
template <class D>
__device__ __forceinline__ uint32_t fn_scan(uint32_t x) {
#define SPSLAM_DPP(V, CTRL, ROWS, BC) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(V), CTRL, ROWS, 0xF, BC))
    x = fn_then<D>(SPSLAM_DPP(x, 0x111, 0xF, true), x);   // row_shr:1
    x = fn_then<D>(SPSLAM_DPP(x, 0x112, 0xF, true), x);   // row_shr:2
    x = fn_then<D>(SPSLAM_DPP(x, 0x114, 0xF, true), x);   // row_shr:4
    x = fn_then<D>(SPSLAM_DPP(x, 0x118, 0xF, true), x);   // row_shr:8
    x = fn_then<D>(SPSLAM_DPP(x, 0x142, 0xA, false), x);  // row_bcast:15
    x = fn_then<D>(SPSLAM_DPP(x, 0x143, 0xC, false), x);  // row_bcast:31
#undef SPSLAM_DPP
    return x;
}

// Descriptor of point i for one pass (see above).  Point validity (isfinite(x)) comes from the valid-point
// bitmap ok[H][RW]; the backward pass reuses the forward pass's accept set `prev` (a point unlabelled now was
// unlabelled then), so only the forward pass reads coordinates.
template <class D>
__device__ __forceinline__ uint32_t refine_desc(const uint8_t* state, const float* X, const float* Y, const float* Z,
                                                const uint64_t* ok, int RW, const float (*coef)[4], int nmodel,
                                                int W, int H, int i, bool bw, uint32_t prev) {
    if (state[i]) return 0;
    const int r = i / W, c = i - r * W;
    auto valid = [&](int rr, int cc) { return (bool)((ok[rr * RW + (cc >> 6)] >> (cc & 63)) & 1ull); };
    uint32_t acc = 0;
    if (!bw) {
        if (!valid(r, c)) return 0;
        const float x = X[i], y = Y[i], z = Z[i];
        for (int v = 0; v < nmodel; v++)
            if (ptp_ok(coef[v], x, y, z)) acc |= 1u << v;
    } else {
        acc = prev & D::kAcc;
    }
    if (!acc) return 0;
    bool act, link;
    if (!bw) {  // sources (r-1, c) [needs (r-1, c+1)] and (r, c-1)
        act = r >= 1 && c <= W - 2 && valid(r - 1, c) && valid(r - 1, c + 1);
        link = c >= 1 && r <= H - 2 && valid(r, c - 1);
    } else {    // sources (r+1, c) [needs flat index before it] and flat i+1 (row wrap at c = W-1)
        act = r <= H - 2 && valid(r + 1, c) && (c >= 1 ? valid(r + 1, c - 1) : valid(r, W - 1));
        link = (c <= W - 2 ? r >= 1 && valid(r, c + 1) : r <= H - 2 && valid(r + 1, 0));
    }
    return acc | (act ? D::kAct : 0u) | (link ? D::kLink : 0u);
}

template <int K, class D>
__device__ __forceinline__ void refine_rows(uint8_t* state, const D desc, const uint64_t* cbits, int W, int H,
                                            bool bw) {
    constexpr bool kWide = D::kAcc > 0xFFFFu;
    const int lane = threadIdx.x & 63;
    const int RW = (W + 63) >> 6;
    const int lastLane = (W - 1) / K, lastK = (W - 1) - lastLane * K;
    uint32_t prevS[K];
#pragma unroll
    for (int k = 0; k < K; k++) prevS[k] = 0;
    uint32_t carry = 0;
    // Next row's values, loaded unconditionally (positions past the row and the row after the last read a
    // clamped in-range pixel and are masked at use) and kept raw until then, so the only wait for them is
    // the one before their use one row later.
    uint32_t qs[K], q0[K], q1[K];
    uint64_t qc = 0;
#define SPSLAM_FAST_FETCH(STEP)                                                    \
    {                                                                              \
        const int st_ = min((STEP), H - 1);                                        \
        const int r_ = bw ? H - 1 - st_ : st_;                                     \
        _Pragma("unroll") for (int k = 0; k < K; k++) {                            \
            const int p = min(lane * K + k, W - 1);                                \
            const int i = r_ * W + (bw ? W - 1 - p : p);                           \
            qs[k] = state[i];                                                      \
            if constexpr (kWide) {                                                 \
                q0[k] = desc.w[i];                                                 \
            } else {                                                               \
                q0[k] = desc.lo[i];                                                \
                q1[k] = desc.hi[i];                                                \
            }                                                                      \
        }                                                                          \
        qc = cbits[r_ * RW + min(lane, RW - 1)];                                   \
    }
    SPSLAM_FAST_FETCH(0)
    for (int step = 0; step < H; step++) {
        const int r = bw ? H - 1 - step : step;
        uint32_t s0[K], d[K], fin[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const bool in = lane * K + k < W;
            s0[k] = in ? qs[k] : 0u;
            if constexpr (kWide) d[k] = in ? q0[k] : 0u;
            else d[k] = in ? (q0[k] | (q1[k] << 8)) : 0u;
        }
        // rows without a growable point keep their states (lanes < RW hold the row's candidate words)
        const bool any = __ballot(lane < RW && qc != 0ull) != 0ull;
        SPSLAM_FAST_FETCH(step + 1)
        if (!any) {
#pragma unroll
            for (int k = 0; k < K; k++) fin[k] = s0[k];
        } else {
            uint32_t g[K];
#pragma unroll
            for (int k = 0; k < K; k++) {
                const uint32_t acc = d[k] & D::kAcc, U = prevS[k];
                const bool grant = (d[k] & D::kAct) && U && ((acc >> ((U - 1) & 31)) & 1u);
                uint32_t e = (d[k] & D::kLink) ? (~acc & D::kVal) : D::kConst;
                e = grant ? (D::kConst | U) : e;
                e = acc ? e : D::kConst;
                g[k] = s0[k] ? (D::kConst | s0[k]) : e;
            }
            uint32_t F = g[0];
#pragma unroll
            for (int k = 1; k < K; k++) F = fn_then<D>(F, g[k]);
            F = fn_scan<D>(F);
            // the lane below's inclusive scan by DPP (wave_shr:1; lane 0 gets 0, the identity): a ds_bpermute here
            // would make its wait also wait for the next row's LDS prefetch issued above
            const uint32_t ex = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)F, 0x138, 0xF, 0xF, false);
            uint32_t L = fn_apply<D>(ex, bw ? carry : 0u);
#pragma unroll
            for (int k = 0; k < K; k++) {
                fin[k] = fn_apply<D>(g[k], L);
                L = fin[k];
                const int p = lane * K + k;
                if (p < W && s0[k] == 0 && fin[k] != 0) state[r * W + (bw ? W - 1 - p : p)] = (uint8_t)fin[k];
            }
        }
        if (bw) carry = (uint32_t)__builtin_amdgcn_readlane((int)sel<K>(fin, lastK), lastLane);
#pragma unroll
        for (int k = 0; k < K; k++) prevS[k] = fin[k];
    }
#undef SPSLAM_FAST_FETCH
}

// Grow events of one finished fast pass, appended at ev[] in the reference's
// order (sources in pass order; per source: along the row, then across rows).
// Returns the number of events (uniform).
template <class D>
__device__ __forceinline__ int refine_events(SegShared& S, const uint8_t* state, const D desc, int W, int H, int N,
                                             bool bw, int* ev, int nw) {  // nw: the workgroup's live waves
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int M = (H - 1) * W;
    // how target j grew in this pass: 0 not, 1 along its row (chain), 2 from the other row
    auto how = [&](int j, int vsrc) -> int {
        const uint32_t dj = desc.get(j);
        if (!(dj & D::kAcc) || !state[j]) return 0;
        if (dj & D::kAct) {
            const int U = state[vsrc];
            if (U && ((dj >> (U - 1)) & 1u)) return 2;
        }
        return 1;
    };
    auto events = [&](int q, int* tA, int* tB) {
        const int s = bw ? N - 1 - q : q;
        *tA = bw ? s - 1 : s + 1;
        *tB = bw ? s - W : s + W;
        const int a = how(*tA, bw ? *tA + W : *tA - W) == 1;
        const int b = how(*tB, s) == 2;
        return a | (b << 1);
    };
    const int span = (M + nw * 64 - 1) / (nw * 64) * 64;
    const int q0 = wave * span, q1 = min(M, q0 + span);
    int cnt = 0;
    for (int base = q0; base < q1; base += 64) {
        const int q = base + lane;
        int tA, tB, e = 0;
        if (q < q1) e = events(q, &tA, &tB);
        cnt += __popcll(__ballot(e & 1)) + __popcll(__ballot(e & 2));
    }
    if (lane == 0) S.wsum[wave] = cnt;
    __syncthreads();
    int off = 0, total = 0;
    for (int j = 0; j < nw; j++) {
        if (j < wave) off += S.wsum[j];
        total += S.wsum[j];
    }
    const uint64_t lt = lanemask_lt();
    for (int base = q0; base < q1; base += 64) {
        const int q = base + lane;
        int tA = 0, tB = 0, e = 0;
        if (q < q1) e = events(q, &tA, &tB);
        const uint64_t ma = __ballot(e & 1), mb = __ballot(e & 2);
        int pos = off + __popcll(ma & lt) + __popcll(mb & lt);
        if (e & 1) ev[pos++] = tA | ((state[tA] - 1) << 24);
        if (e & 2) ev[pos] = tB | ((state[tB] - 1) << 24);
        off += __popcll(ma) + __popcll(mb);
    }
    __syncthreads();
    return total;
}

// 8-neighbour offsets of findLabeledRegionBoundary, packed 2 bits each (+1).
constexpr uint32_t kDX = (0u << 0) | (0u << 2) | (1u << 4) | (2u << 6) | (2u << 8) | (2u << 10) | (1u << 12) | (0u << 14);
constexpr uint32_t kDY = (1u << 0) | (0u << 2) | (0u << 4) | (0u << 6) | (1u << 8) | (2u << 10) | (2u << 12) | (2u << 14);
__device__ __forceinline__ int ddx(int d) { return (int)((kDX >> (2 * d)) & 3u) - 1; }
__device__ __forceinline__ int ddy(int d) { return (int)((kDY >> (2 * d)) & 3u) - 1; }

__device__ __forceinline__ int nb_bits(const uint8_t* state, int W, int H, int x, int y, int lab, bool same) {
    int m = 0;
    for (int d = 0; d < 8; d++) {
        const int u = x + ddx(d), v = y + ddy(d);
        if (u >= 0 && u < W && v >= 0 && v < H && ((state[v * W + u] == lab) == same)) m |= 1 << d;
    }
    return m;
}

// Moore tracing from `start` (reference: findLabeledRegionBoundary); writes
// at most cap indices, returns the full length.
// Inlined so the LDS instance walks with ds_read (a called function sees generic pointers: flat loads).
__device__ __forceinline__ int trace_contour(const uint8_t* state, const uint8_t* nmask, int W, int H, int N, int start, int lab,
                             int32_t* out, int cap) {
    int cx = start % W, cy = start / W;
    const int ne = nb_bits(state, W, H, cx, cy, lab, false);
    if (!ne) return 0;
    int dir = __builtin_ctz(ne);
    int n = 0, cur = start;
    if (n < cap) out[n] = start;
    n++;
    do {
        const int m = state[cur] == lab ? nmask[cur] : nb_bits(state, W, H, cx, cy, lab, true);
        const int sh = (dir + 1) & 7;
        const int rot = ((m >> sh) | (m << (8 - sh))) & 0xFF;
        const int nIdx = rot ? (sh + __builtin_ctz(rot)) & 7 : dir;
        dir = (nIdx + 4) & 7;
        cx += ddx(nIdx);
        cy += ddy(nIdx);
        cur = cy * W + cx;
        if (n < cap) out[n] = cur;
        n++;
    } while (cur != start && n < 8 * N);
    return n;
}

template <bool kLdsMaps, int K>
#ifdef SPSLAM_SEG_NUM_VGPR
__attribute__((amdgpu_waves_per_eu(SPSLAM_SEG_NUM_VGPR)))
#endif
__global__ __launch_bounds__(kSegThreads) void plane_segment_kernel(
    PlaneGeom g, PlaneBuffers b, spslam_plane* __restrict__ planes_out, int* __restrict__ plane_counts, int planes_cap,
    int32_t* __restrict__ inliers_out, int32_t* __restrict__ contours_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    __shared__ SegShared S;
    const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int W = g.W, H = g.H, N = g.N, RW = (W + 63) >> 6;
    uint64_t* hbits = (uint64_t*)dyn;      // comparator edge to the left neighbour, [H][RW]
    uint64_t* vbits = hbits + H * RW;      // comparator edge to the upper neighbour
    uint64_t* okbits = vbits + H * RW;     // valid points
    uint8_t* state = kLdsMaps ? (uint8_t*)(okbits + H * RW) : b.maps + f * b.maps_fs;  // [N] tag / model+1
    uint8_t* nmask = state + N;                                                         // [N] contour masks
    uint16_t* P16 = (uint16_t*)state;      // LDS instance: parents, then labels (phases A-F)
    const float* X = b.cloud + f * b.cloud_fs;
    const float* Y = X + N;
    const float* Z = X + 2 * N;
    const float* Nx = b.normal + f * b.normal_fs;
    const float* Ny = Nx + N;
    const float* Nz = Nx + 2 * N;
    const float* PD = b.pd + f * b.pd_fs;
    int* P = (int*)(b.labels + f * b.labels_fs);   // global instance: parents, then labels (-1 = invalid point)
    int* rankA = b.work + f * b.work_fs;           // [N] global instance: label of each root pixel
    int* sizes = rankA + N;                        // [N] per label (big ones: -(index+1))
    int* members = sizes + 2 * N;                  // [N] member lists of big components (LDS instance: 16-bit)
    auto mem_at = [&](int k) -> int {
        if constexpr (kLdsMaps) return ((const uint16_t*)members)[k];
        else return members[k];
    };
    auto mem_put = [&](int k, int i) {
        if constexpr (kLdsMaps) ((uint16_t*)members)[k] = (uint16_t)i;
        else members[k] = i;
    };
    int* ev = b.grown + f * b.grown_fs;            // [N] grow events: target | model << 24
    spslam_plane* planes = planes_out + (size_t)f * planes_cap;
    int32_t* inl = inliers_out + (size_t)f * g.inlier_cap;
    int32_t* con = contours_out + (size_t)f * g.contour_cap;
    long long* ts = b.ts + f * 16;
#define STAMP(k) do { if (t == 0) ts[k] = (long long)__builtin_amdgcn_s_memrealtime(); } while (0)
    STAMP(15);
    if (t < kMaxPlanesPerFrame) S.model_grown[t] = 0;

    // PlaneCoefficientComparator::compare (i1 = current, i2 = neighbour).  Its z = x * 0 + y * 0 + z * 1: a
    // cloud point's x, y and z are finite or NaN together (plane_cloud_kernel), so z * z is Z * Z bit for bit
    // (a zero's sign aside, which the square drops) and x, y are not read.
    auto cmp = [&](int i1, int i2) {
        const float z = Z[i1];
        float threshold = g.dist_th;
        threshold *= z * z;
        const float nd = Nx[i1] * Nx[i2] + Ny[i1] * Ny[i2] + Nz[i1] * Nz[i2];
        return (fabsf(PD[i1] - PD[i2]) < threshold) && (nd > g.ang_cos);
    };
    auto bit = [&](const uint64_t* m, int r, int c) { return (int)((m[r * RW + (c >> 6)] >> (c & 63)) & 1ull); };

    // ---- A: edge bits and run heads, one wave per row
    for (int r = wave; r < H; r += kSegWaves) {
        int carry = 0;
        for (int k = 0; k < RW; k++) {
            const int c = (k << 6) + lane;
            const bool in = c < W;
            const int i = r * W + c;
            bool h = false, v = false, valid = false;
            if (in) {
                valid = isfinite(Z[i]);  // (isfinite(x), see cmp)
                h = c >= 1 && cmp(i, i - 1);
                v = r >= 1 && cmp(i, i - W);
            }
            const uint64_t hb = __ballot(h), vb = __ballot(v), ob = __ballot(valid);
            if (lane == 0) { hbits[r * RW + k] = hb; vbits[r * RW + k] = vb; okbits[r * RW + k] = ob; }
            const uint64_t sb = __ballot(in && !h);
            const uint64_t upto = lane == 63 ? sb : (sb & ((2ull << lane) - 1ull));
            const int head = upto ? r * W + (k << 6) + 63 - __clzll(upto) : carry;
            if (in) {
                if constexpr (kLdsMaps) P16[i] = (uint16_t)(valid ? head : (int)kNone16);
                else P[i] = valid ? head : -1;
            }
            carry = __shfl(head, 63);
        }
    }
    block_sync();
    STAMP(0);
    // ---- B: one union per vertical run overlap
    for (int i = W + t; i < N; i += kSegThreads) {
        const int r = i / W, c = i - r * W;
        if (!bit(vbits, r, c)) continue;
        if (c >= 1 && bit(hbits, r, c) && bit(hbits, r - 1, c) && bit(vbits, r, c - 1)) continue;
        if constexpr (kLdsMaps) uf_union16(P16, ld16(P16, i), ld16(P16, i - W));
        else uf_union(P, ld_wg(&P[i]), ld_wg(&P[i - W]));
    }
    block_sync();
    STAMP(1);
    // ---- C: flatten
    for (int i = t; i < N; i += kSegThreads) {
        if constexpr (kLdsMaps) {
            const int p = P16[i];
            if (p != (int)kNone16) P16[i] = (uint16_t)uf_find16(P16, p);
        } else {
            const int p = P[i];
            if (p >= 0) P[i] = uf_find(P, p);
        }
    }
    block_sync();
    STAMP(2);
    // ---- D: labels = rank of the root; sizes.  The LDS instance relabels in place: a root's entry becomes its
    //         label (its lanes remember which pixels were roots), then every other pixel reads its root's entry.
    const int span = (N + kSegWaves * 64 - 1) / (kSegWaves * 64) * 64;
    // component sizes: one atomic per run of equal labels among a wave's 64 pixels.  The LDS instance counts in
    // 16-bit halves of the (still unused) covariance staging area when the labels fit (a count <= N < 2^16 never
    // carries into the next half); after phase E the same halves hold each label's tag.
    uint32_t* sz16 = (uint32_t*)&S.stage[0][0][0];
    constexpr int kSz16 = (int)(sizeof(S.stage) / sizeof(uint16_t));
    bool lsz = false;
    auto size_of = [&](int L) -> int {
        if (lsz) return (int)((sz16[L >> 1] >> ((L & 1) << 4)) & 0xFFFFu);
        return sizes[L];
    };
    auto count_run = [&](int L) {
        const int prevL = __shfl_up(L, 1);
        const bool chg = lane == 0 || prevL != L;
        const uint64_t cb = __ballot(chg);
        if (chg && L >= 0) {
            const uint64_t rest = lane == 63 ? 0ull : (cb >> (lane + 1));
            const int len = rest ? __builtin_ctzll(rest) + 1 : 64 - lane;
            if (lsz) atomicAdd(&sz16[L >> 1], (uint32_t)len << ((L & 1) << 4));
            else atomicAdd(&sizes[L], len);
        }
    };
    auto is_root = [&](int i) {
        if constexpr (kLdsMaps) return (int)P16[i] == i;
        else return P[i] == i;
    };
    {
        const int w0 = wave * span, w1 = min(N, w0 + span);
        int cnt = 0;
        for (int base = w0; base < w1; base += 64) {
            const int i = base + lane;
            cnt += __popcll(__ballot(i < w1 && is_root(i)));
        }
        if (lane == 0) S.wsum[wave] = cnt;
        __syncthreads();
        int wb = 0, ncomp = 0;
        for (int j = 0; j < kSegWaves; j++) {
            if (j < wave) wb += S.wsum[j];
            ncomp += S.wsum[j];
        }
        uint64_t rmask = 0;  // (LDS instance) chunk k of this lane's pixels: bit k = root
        for (int base = w0, k = 0; base < w1; base += 64, k++) {
            const int i = base + lane;
            const bool root = i < w1 && is_root(i);
            const uint64_t m = __ballot(root);
            if (root) {
                const int L = wb + __popcll(m & lanemask_lt());
                if constexpr (kLdsMaps) {
                    P16[i] = (uint16_t)L;
                    rmask |= 1ull << k;
                } else {
                    rankA[i] = L;
                }
            }
            wb += __popcll(m);
        }
        lsz = kLdsMaps && ncomp <= kSz16;
        if (lsz) {
            for (int k = t; k < (ncomp + 1) >> 1; k += kSegThreads) sz16[k] = 0;
        } else {
            for (int k = t; k < ncomp; k += kSegThreads) sizes[k] = 0;
        }
        if (t == 0) S.misc[1] = ncomp;
        block_sync();
        for (int base = w0, k = 0; base < w1; base += 64, k++) {
            const int i = base + lane;
            int L = -1;
            if (i < w1) {
                if constexpr (kLdsMaps) {
                    const int p = P16[i];
                    if (p != (int)kNone16) {
                        const bool root = (rmask >> k) & 1ull;
                        L = root ? p : (int)P16[p];
                        if (!root) P16[i] = (uint16_t)L;
                    }
                    if (b.keep_labels) P[i] = L;
                } else {
                    const int p = P[i];
                    if (p >= 0) L = rankA[p];
                    P[i] = L;
                }
            }
            count_run(L);
        }
    }
    block_sync();
    STAMP(3);
    // ---- E: components larger than MinSize, in label order
    const int ncomp = S.misc[1];
    {
        const int lspan = (ncomp + kSegWaves * 64 - 1) / (kSegWaves * 64) * 64;
        const int w0 = wave * lspan, w1 = min(ncomp, w0 + lspan);
        int cnt = 0;
        for (int base = w0; base < w1; base += 64) {
            const int L = base + lane;
            cnt += __popcll(__ballot(L < w1 && (unsigned)size_of(L) > (unsigned)g.min_size));
        }
        __syncthreads();
        if (lane == 0) S.wsum[wave] = cnt;
        __syncthreads();
        int wb = 0, nbig = 0;
        for (int j = 0; j < kSegWaves; j++) {
            if (j < wave) wb += S.wsum[j];
            nbig += S.wsum[j];
        }
        for (int base = w0; base < w1; base += 64) {
            const int L = base + lane;
            const bool big = L < w1 && (unsigned)size_of(L) > (unsigned)g.min_size;
            const uint64_t m = __ballot(big);
            const int j = wb + __popcll(m & lanemask_lt());
            if (big && j < kMaxBig) {
                S.big_label[j] = L;
                S.big_size[j] = size_of(L);
            }
            wb += __popcll(m);
        }
        __syncthreads();
        if (t == 0) {
            S.nbig = min(nbig, kMaxBig);
            int off = 0;
            for (int j = 0; j < S.nbig; j++) { S.big_off[j] = off; off += S.big_size[j]; }
        }
        __syncthreads();
        if (lsz) {  // the halves become tags: 0, or j + 1 for big component j
            for (int k = t; k < (ncomp + 1) >> 1; k += kSegThreads) sz16[k] = 0;
            __syncthreads();
            for (int j = t; j < S.nbig; j += kSegThreads) ((uint16_t*)sz16)[S.big_label[j]] = (uint16_t)(j + 1);
        } else {
            for (int j = t; j < S.nbig; j += kSegThreads) sizes[S.big_label[j]] = -(j + 1);
        }
    }
    block_sync();
    const int nbig = S.nbig;
    // ---- F: per-pixel component tag
    auto tag_of = [&](int L) {
        if (L < 0) return 0;
        if (lsz) return (int)((const uint16_t*)sz16)[L];
        const int z = sizes[L];
        return z < 0 ? -z : 0;
    };
    if constexpr (kLdsMaps) {
        // the byte map overwrites the 16-bit labels: block j's tags (bytes [b0, b0 + 4T) = labels [b0 / 2, ...))
        // are stored once every label of the block is read; they cover labels of earlier blocks only
        constexpr int kU = 4;
        for (int b0 = 0; b0 < N; b0 += kU * kSegThreads) {
            int tg[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int i = b0 + u * kSegThreads + t;
                const int L = i < N ? (int)P16[i] : (int)kNone16;
                tg[u] = tag_of(L == (int)kNone16 ? -1 : L);
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int i = b0 + u * kSegThreads + t;
                if (i < N) state[i] = (uint8_t)tg[u];
            }
        }
    } else {
        for (int i = t; i < N; i += kSegThreads) state[i] = (uint8_t)tag_of(P[i]);
    }
    block_sync();
    STAMP(5);
    // ---- G: member lists of the big components in raster order (each wave counts its stripe's members per
    //         component, a prefix over the stripes places them), then per component, one wave: PCL's float
    //         mean/covariance accumulation over its member list (terms staged through LDS, nine lanes each own
    //         one accumulator, so the sums are the reference's sequence; a chunk's zero padding adds nothing)
    {
        uint32_t(*cnt)[256] = (uint32_t(*)[256]) & S.stage[0][0][0];
        static_assert(sizeof(S.stage) >= sizeof(uint32_t) * kSegWaves * 256, "member counters");
        for (int k = t; k < kSegWaves * 256; k += kSegThreads) (&cnt[0][0])[k] = 0;
        __syncthreads();
        const int w0 = wave * span, w1 = min(N, w0 + span);
        // one round per distinct tag of a 64-pixel chunk
        auto stripe = [&](bool place) {
            for (int base = w0; base < w1; base += 64) {
                const int i = base + lane;
                const int tg = i < w1 ? (int)state[i] : 0;
                uint64_t rem = __ballot(tg != 0);
                while (rem) {
                    const int tq = __shfl(tg, __builtin_ctzll(rem));
                    const uint64_t m = __ballot(tg == tq);
                    if (place && tg == tq) mem_put((int)cnt[wave][tq] + __popcll(m & lanemask_lt()), i);
                    if (lane == 0) cnt[wave][tq] += __popcll(m);
                    rem &= ~m;
                }
            }
        };
        stripe(false);
        __syncthreads();
        for (int j = t; j < nbig; j += kSegThreads) {
            int o = S.big_off[j];
            for (int w = 0; w < kSegWaves; w++) {
                const int c = (int)cnt[w][j + 1];
                cnt[w][j + 1] = o;
                o += c;
            }
        }
        __syncthreads();
        stripe(true);
        __syncthreads();
    }
    for (int j = wave; j < nbig; j += kSegWaves) {
        const int n = S.big_size[j], o = S.big_off[j];
        float* st = &S.stage[wave][0][0];
        float acc = 0.f;
        auto chunk = [&](int c0, float px, float py, float pz) __attribute__((always_inline)) {
            const int cnt = min(64, n - c0), pad = (cnt + 3) & ~3;
            if (lane < cnt) {
                st[0 * 64 + lane] = px * px; st[1 * 64 + lane] = px * py; st[2 * 64 + lane] = px * pz;
                st[3 * 64 + lane] = py * py; st[4 * 64 + lane] = py * pz; st[5 * 64 + lane] = pz * pz;
                st[6 * 64 + lane] = px; st[7 * 64 + lane] = py; st[8 * 64 + lane] = pz;
            } else if (lane < pad) {
                for (int q = 0; q < 9; q++) st[q * 64 + lane] = 0.f;
            }
            wave_sync();
            if (lane < 9) {
                // the chunk's terms in two batches of 8 loads issued together (one LDS round trip per batch, not
                // per 4 values), added in order; entries past the padding are loaded but not added
                const float4* row = (const float4*)(st + lane * 64);
                const int nq = pad >> 2;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    float4 v[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) v[q] = row[8 * h + q];
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        if (8 * h + q < nq) {
                            acc += v[q].x;
                            acc += v[q].y;
                            acc += v[q].z;
                            acc += v[q].w;
                        }
                    }
                }
            }
            wave_sync();
        };
        if constexpr (K <= 4) {
            // coordinates kPD chunks ahead (a chunk's adds take ~0.3 us, a cloud load's round trip several times that:
            // with one chunk ahead the walk waited on every chunk's loads), member indices (LDS) one chunk further
            auto idx_at = [&](int c0) { return c0 + lane < n ? mem_at(o + c0 + lane) : -1; };
            float cx[kPD], cy[kPD], cz[kPD];
#pragma unroll
            for (int d = 0; d < kPD; d++) {
                const int id = idx_at(64 * d);
                cx[d] = 0.f; cy[d] = 0.f; cz[d] = 0.f;
                if (id >= 0) { cx[d] = X[id]; cy[d] = Y[id]; cz[d] = Z[id]; }
            }
            int inext = idx_at(64 * kPD);
            for (int c00 = 0; c00 < n; c00 += 64 * kPD)
#pragma unroll
            for (int d = 0; d < kPD; d++) {
                const int c0 = c00 + 64 * d;
                if (c0 >= n) break;  // (uniform)
                const float px = cx[d], py = cy[d], pz = cz[d];
                cx[d] = 0.f; cy[d] = 0.f; cz[d] = 0.f;
                if (inext >= 0) { cx[d] = X[inext]; cy[d] = Y[inext]; cz[d] = Z[inext]; }
                inext = idx_at(c0 + 64 * (kPD + 1));
                chunk(c0, px, py, pz);
            }
        } else {
            // member indices two chunks ahead, coordinates one chunk ahead (the 512-wide instance: more lookahead
            // spills there)
            auto idx_at = [&](int c0) { return c0 + lane < n ? mem_at(o + c0 + lane) : -1; };
            int icur = idx_at(0), inext = idx_at(64);
            float px = 0.f, py = 0.f, pz = 0.f;
            if (icur >= 0) { px = X[icur]; py = Y[icur]; pz = Z[icur]; }
            for (int c0 = 0; c0 < n; c0 += 64) {
                const int i2 = idx_at(c0 + 128);
                float nx = 0.f, ny = 0.f, nz = 0.f;
                if (inext >= 0) { nx = X[inext]; ny = Y[inext]; nz = Z[inext]; }
                chunk(c0, px, py, pz);
                px = nx; py = ny; pz = nz;
                inext = i2;
            }
        }
        if (lane < 9) acc /= (float)n;
        float a[9];
        for (int k = 0; k < 9; k++) a[k] = __shfl(acc, k);
        if (lane == 0) {
            float cov[3][3];
            cov[0][0] = a[0] - a[6] * a[6];
            cov[0][1] = a[1] - a[6] * a[7];
            cov[0][2] = a[2] - a[6] * a[8];
            cov[1][1] = a[3] - a[7] * a[7];
            cov[1][2] = a[4] - a[7] * a[8];
            cov[2][2] = a[5] - a[8] * a[8];
            cov[1][0] = cov[0][1]; cov[2][0] = cov[0][2]; cov[2][1] = cov[1][2];
            float ev0, evec[3];
            eigen33_min(cov, &ev0, evec);
            const float eig_sum = cov[0][0] + cov[1][1] + cov[2][2];
            S.big_curv[j] = eig_sum != 0 ? fabsf(ev0 / eig_sum) : 0.f;
            S.big_par[j][0] = evec[0]; S.big_par[j][1] = evec[1]; S.big_par[j][2] = evec[2]; S.big_par[j][3] = 0.f;
            S.big_cen[j][0] = a[6]; S.big_cen[j][1] = a[7]; S.big_cen[j][2] = a[8]; S.big_cen[j][3] = 1.f;
        }
    }
    block_sync();
    STAMP(6);
    // ---- H: plane sign via the (accumulating) viewpoint vector, curvature filter
    if (t == 0) {
        float vp[4] = {0, 0, 0, 0};
        int nm = 0;
        S.big_state[0] = 0;
        for (int j = 0; j < nbig; j++) {
            float pp[4] = {S.big_par[j][0], S.big_par[j][1], S.big_par[j][2], 0.f};
            pp[3] = -1 * dot4(pp, S.big_cen[j]);
            for (int k = 0; k < 4; k++) vp[k] -= S.big_cen[j][k];
            if (dot4(vp, pp) < 0) {
                for (int k = 0; k < 4; k++) pp[k] *= -1;
                pp[3] = 0;
                pp[3] = -1 * dot4(pp, S.big_cen[j]);
            }
            S.big_state[j + 1] = 0;
            if (S.big_curv[j] < 0.001f && nm < kMaxPlanesPerFrame) {
                S.model_big[nm] = j;
                for (int k = 0; k < 4; k++) S.model_coef[nm][k] = pp[k];
                S.big_state[j + 1] = (uint8_t)(nm + 1);
                nm++;
            }
        }
        S.nmodel = nm;
    }
    __syncthreads();
    const int nmodel = S.nmodel;
    if (t == 0) ts[13] = nmodel;
    for (int i = t; i < N; i += kSegThreads) {
        const int s = state[i];
        if (s) state[i] = S.big_state[s];
    }
    block_sync();
    STAMP(7);
    // ---- K: refinement (two passes), one wave per pass
    uint64_t* cbits = hbits;  // rows with growable points (hbits no longer needed)
    // Live waves from the first pass's serial row walk on: on the fast paths max(models, 8) waves stay (the
    // rest end once the first pass's descriptors are written -- their VGPRs go back to the other streams'
    // waves for the rest of the kernel; s_barrier waits on surviving waves only).  Measured on the pipelined
    // C2 step against ending at pass 1 or before pass 0, and against 1 / 6 / 12 live waves
    // (profiles/r02/ab_seg_live_waves).
#if !defined(SPSLAM_SEG_NO_EARLY_EXIT) && !defined(SPSLAM_SEG_EXIT_AT_N_ONLY)  // (measurement variants)
    const int nlive = (nmodel > 0 && nmodel <= kWideModels) ? min(max(nmodel, SPSLAM_SEG_MIN_LIVE), kSegWaves) : kSegWaves;
#else
    const int nlive = kSegWaves;
#endif
    const int tlive = nlive * 64;
    // two passes over the fast-path descriptors (D: narrow or wide format); false: this wave has ended its part
    auto fast_refine = [&](const auto desc) -> bool {
        using D = decltype(desc);
        int ng = 0;
        if (SPSLAM_SEG_EXIT_PASS < 0 && wave >= nlive) return false;  // phase H ended with a barrier
        for (int pass = 0; pass < 2; pass++) {
            const bool bw = pass == 1;
            for (int r = wave; r < H; r += pass > SPSLAM_SEG_EXIT_PASS ? nlive : kSegWaves)
                for (int k = 0; k < RW; k++) {
                    const int c = (k << 6) + lane, i = r * W + c;
                    uint32_t dsc = 0;
                    if (c < W) {
                        dsc = refine_desc<D>(state, X, Y, Z, okbits, RW, S.model_coef, nmodel, W, H, i, bw,
                                             bw ? desc.get(i) : 0u);
                        desc.put(i, dsc);
                    }
                    const uint64_t m = __ballot(dsc != 0);
                    if (lane == 0) cbits[r * RW + k] = m;
                }
            __syncthreads();
            if (pass == 0) STAMP(10);
            if (pass == SPSLAM_SEG_EXIT_PASS && wave >= nlive) return false;  // no barrier before the caller's return
            if (wave == 0) refine_rows<K>(state, desc, cbits, W, H, bw);
            __syncthreads();
            if (pass == 0) STAMP(11);
            ng += refine_events(S, state, desc, W, H, N, bw, ev + ng, pass >= SPSLAM_SEG_EXIT_PASS ? nlive : kSegWaves);
        }
        if (t == 0) { S.misc[0] = ng; ts[12] = ng; }
        return true;
    };
    bool live = true;
#ifdef SPSLAM_MEASURE_SKIP_REFINE  // measurement variant only (marginal step cost): no refinement
    if (nmodel > 0 && nmodel <= kFastModels) {
        if (t == 0) S.misc[0] = 0;
    } else if (false) {
#else
    if (nmodel > 0 && nmodel <= kFastModels) {
#endif
        // narrow descriptors: low bytes in the contour-mask map (the masks come later), high bytes in the
        // covariance staging area (phase G is over) in the LDS instance (the host picks it only when
        // N <= sizeof(S.stage)), else in the rank scratch (dead since phase D); fixed per instance so every
        // access is a ds_* or global_* one, never flat
        live = fast_refine(Desc<false>{nmask, kLdsMaps ? (uint8_t*)&S.stage[0][0][0] : (uint8_t*)rankA});
    } else if (nmodel > 0 && nmodel <= kWideModels) {
        // wide descriptors: one word per point in the rank scratch
        live = fast_refine(Desc<true>{(uint32_t*)rankA});
#ifndef SPSLAM_SEG_NO_GENERAL  // measurement variant only: frames with more than kFastModels models are not refined
    } else if (nmodel > 0) {
        // general path: accept masks over up to 64 models evaluated in the pass
        for (int r = wave; r < H; r += kSegWaves)
            for (int k = 0; k < RW; k++) {
                const int c = (k << 6) + lane, i = r * W + c;
                bool cand = false;
                if (c < W && state[i] == 0) {
                    const float x = X[i], y = Y[i], z = Z[i];
                    if (isfinite(x))
                        for (int v = 0; v < nmodel && !cand; v++) cand = ptp_ok(S.model_coef[v], x, y, z);
                }
                const uint64_t m = __ballot(cand);
                if (lane == 0) cbits[r * RW + k] = m;
            }
        __syncthreads();
        if (wave == 0) {
            int ng = refine_pass<K>(S, state, cbits, X, Y, Z, W, H, false, ev, 0);
            ng += refine_pass<K>(S, state, cbits, X, Y, Z, W, H, true, ev, ng);
            if (lane == 0) S.misc[0] = ng;
        }
#endif
    } else if (t == 0) {
        S.misc[0] = 0;
    }
    if (!live) return;
    block_sync();
    for (int e = t; e < S.misc[0]; e += tlive) atomicAdd(&S.model_grown[ev[e] >> 24], 1);
    __syncthreads();
    STAMP(8);
    // ---- L: Frame.cc:912-934: d >= 0, PlaneNotSeen; inlier offsets
    if (t == 0) {
        int nk = 0;
        for (int m = 0; m < nmodel; m++) {
            float cf[4] = {S.model_coef[m][0], S.model_coef[m][1], S.model_coef[m][2], S.model_coef[m][3]};
            if (cf[3] < 0)
                for (int k = 0; k < 4; k++) cf[k] = -cf[k];
            bool seen = false;
            for (int q = 0; q < nk && !seen; q++) {
                seen = plane_seen_by(planes[q].coef, cf);
            }
            if (seen || nk >= planes_cap) continue;
            for (int k = 0; k < 4; k++) planes[nk].coef[k] = cf[k];
            S.kept[nk++] = m;
        }
        S.nkept = nk;
        int off = 0;
        for (int q = 0; q < nk; q++) {
            const int m = S.kept[q];
            const int n = min(S.big_size[S.model_big[m]] + S.model_grown[m], g.inlier_cap - off);
            planes[q].inlier_offset = off;
            planes[q].n_inliers = n;
            off += n;
        }
        plane_counts[f] = nk;
    }
    __syncthreads();
    const int nk = S.nkept, ng = S.misc[0];
    // ---- M: inlier lists (component members in raster order, then grown points in grow order);
    //         8-neighbour same-state masks for the contour walk
    for (int i = t; i < N; i += tlive) {
        const int s = state[i];
        nmask[i] = s ? (uint8_t)nb_bits(state, W, H, i % W, i / W, s, true) : 0;
    }
    for (int q = wave; q < nk; q += nlive) {
        const int m = S.kept[q], j = S.model_big[m], n = S.big_size[j], o = S.big_off[j];
        const int dst = planes[q].inlier_offset, lim = planes[q].n_inliers;
        for (int k = lane; k < min(n, lim); k += 64) inl[dst + k] = mem_at(o + k);
        // contour start = the model's last inlier (segmentAndRefine's max_inlier_idx):
        // its last grow event, else its last component member
        int last = -1;
        for (int e1 = ng; e1 > 0; e1 -= 64) {
            const int e = e1 - 64 + lane;
            const uint64_t mk = __ballot(e >= 0 && (ev[e] >> 24) == m);
            if (mk) {
                last = ev[e1 - 64 + (63 - __clzll(mk))] & 0xFFFFFF;
                break;
            }
        }
        if (lane == 0) S.con_start[q] = last >= 0 ? last : mem_at(o + n - 1);
        int w = n;
        for (int e0 = 0; e0 < ng; e0 += 64) {
            const int e = e0 + lane;
            const int x = e < ng ? ev[e] : -1;
            const bool hit = x >= 0 && (x >> 24) == m;
            const uint64_t mk = __ballot(hit);
            const int pos = w + __popcll(mk & lanemask_lt());
            if (hit && pos < lim) inl[dst + pos] = x & 0xFFFFFF;
            w += __popcll(mk);
        }
    }
    block_sync();
    STAMP(4);
    // ---- N: contours (findLabeledRegionBoundary from the model's last inlier, on refined labels)
    // Waves without a contour end here: a wave's VGPRs are released when it ends (LDS only with the
    // workgroup), and s_barrier waits on the surviving waves only, so the remaining barriers stay correct.
    // The walks take ~0.35 ms per frame; meanwhile other streams' waves can use those registers.
#ifndef SPSLAM_SEG_NO_EARLY_EXIT
    if (wave >= max(nk, 1)) return;
#endif
    // Each boundary is walked once, recorded while it is measured into a provisional slot of 2 x n_inliers
    // points (the label scratch sizes..rootOf, 2N ints, dead since phase F; the slots sum to <= 2N); once the
    // lengths fix the final offsets, each live wave moves its plane's walk into place.  A walk longer than its
    // slot (a pathological boundary revisiting its pixels) is walked again, straight into its final place.
    int32_t* ctmp = sizes;
    for (int q = wave; q < nk; q += kSegWaves)
        if (lane == 0) {
            const int m = S.kept[q];
            S.con_len[q] = trace_contour(state, nmask, W, H, N, S.con_start[q], m + 1,
                                         ctmp + 2 * planes[q].inlier_offset, 2 * planes[q].n_inliers);
        }
    __syncthreads();
    if (t == 0) {
        int coff = 0;
        for (int q = 0; q < nk; q++) {
            planes[q].contour_offset = coff;
            planes[q].n_contour = min(S.con_len[q], g.contour_cap - coff);
            coff += planes[q].n_contour;
        }
    }
    block_sync();
    for (int q = wave; q < nk; q += kSegWaves) {
        const int n = planes[q].n_contour, off = planes[q].contour_offset;
        if (S.con_len[q] <= 2 * planes[q].n_inliers) {
            const int32_t* src = ctmp + 2 * planes[q].inlier_offset;
            for (int k = lane; k < n; k += 64) con[off + k] = src[k];
        } else if (lane == 0) {
            trace_contour(state, nmask, W, H, N, S.con_start[q], S.kept[q] + 1, con + off, n);
        }
    }
    STAMP(9);
#undef STAMP
}

}  // namespace planes

size_t plane_segment_lds_bytes(const PlaneGeom& g, bool* in_lds) {
    const size_t RW = (g.W + 63) / 64;
    const size_t bits = 3 * g.H * RW * sizeof(uint64_t);
    const size_t maps = ((size_t)2 * g.N + 15) / 16 * 16;
    // the LDS instance also keeps the refinement descriptors' high bytes in SegShared::stage, its parents are
    // 16-bit (kNone16 reserved) and its relabelling marks roots in one 64-bit mask per lane
    const bool fits = sizeof(planes::SegShared) + bits + maps <= (size_t)planes::kLdsBytes &&
                      (size_t)g.N <= sizeof(planes::SegShared::stage) && g.N < (int)planes::kNone16 &&
                      g.N <= 64 * planes::kSegThreads;
    if (in_lds) *in_lds = fits;
    return bits + (fits ? maps : 0);
}

hipError_t plane_segment_launch(const PlaneGeom& g, const PlaneBuffers& b, int n, spslam_plane* planes,
                                int* plane_counts, int planes_cap, int32_t* inliers, int32_t* contours,
                                hipStream_t s) {
    if (g.W > 64 * planes::kMaxRowWords || g.N >= (1 << 24)) return hipErrorInvalidValue;
    bool in_lds = false;
    const size_t dyn = plane_segment_lds_bytes(g, &in_lds);
    if (sizeof(planes::SegShared) + dyn > (size_t)planes::kLdsBytes) return hipErrorInvalidValue;
    auto launch = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, dim3(n), dim3(planes::kSegThreads), dyn, s, g, b, planes, plane_counts, planes_cap,
                           inliers, contours);
    };
    auto lds_attr = [](const void* k) {
        return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(planes::kLdsBytes - sizeof(planes::SegShared)));
    };
    static const hipError_t a4 = lds_attr((const void*)planes::plane_segment_kernel<true, 4>);
    static const hipError_t a8 = lds_attr((const void*)planes::plane_segment_kernel<true, 8>);
    (void)a4;
    (void)a8;
    // lane positions per refinement row: 4 for W <= 256, 8 for W <= 512
    if (in_lds) {
        if (g.W <= 256) launch(planes::plane_segment_kernel<true, 4>);
        else launch(planes::plane_segment_kernel<true, 8>);
    } else {
        if (g.W <= 256) launch(planes::plane_segment_kernel<false, 4>);
        else launch(planes::plane_segment_kernel<false, 8>);
    }
    return hipGetLastError();
}

}  // namespace spslam
