// Map::AssociatePlanesByBoundary on gfx950 (src/Map.cc:196-359): frame planes
// against the map planes of the frame's map, for a batch of frames.
// Semantics: oracle/assoc_oracle.cpp.
//
//   assoc_dist_kernel    grid (frame, map plane): the map plane's boundary cloud
//                        is streamed once per 8 frame planes; every thread keeps
//                        8 running minima of |pM . (p, 1)| (float, exact min, so
//                        the order of the reduction does not matter), then wave
//                        and workgroup minima -> dist[frame][plane][map plane]
//                        (-1 where the angle test fails and the reference never
//                        computes the distance);
//   assoc_decide_kernel  grid (frame): one thread per frame plane walks the map
//                        planes in id order with the reference's running
//                        thresholds; mbNewPlane by a workgroup OR.
// Float dot products use the reference build's FMA contraction pattern (GCC
// -O3 -march=native): fma(a2, b2, fma(a0, b0, a1*b1)) (+ a3).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "wave_priority.h"

#include "assoc_launch.h"

namespace spslam {
namespace assoc {

constexpr int kThreads = 256, kWaves = kThreads / 64, kGroup = 8;

__device__ __forceinline__ float dot3(const float* a, const float* b) {
    return __fmaf_rn(a[2], b[2], __fmaf_rn(a[0], b[0], __fmul_rn(a[1], b[1])));
}

// Frame::ComputePlaneWorldCoeff: transpose(Tcw) * coef, cv::Mat float gemm (double accumulation)
__device__ __forceinline__ void world_coeff(const float* T, const float* c, float* pM) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) s = __dadd_rn(s, __dmul_rn((double)T[4 * k + j], (double)c[k]));
        pM[j] = (float)s;
    }
}

__device__ __forceinline__ const float* coef_of(const AssocSources& S, int f, int i, int na) {
    return i < na ? (const float*)(S.a + ((size_t)f * S.cap_a + i) * S.stride_a)
                  : (const float*)(S.b + ((size_t)f * S.cap_b + (i - na)) * S.stride_b);
}

__device__ __forceinline__ void plane_counts(const AssocSources& S, int f, int* na, int* nb) {
    *na = min(S.count_a[f], S.cap_a);
    *nb = S.count_b ? min(S.count_b[f], S.cap_b) : 0;
}

__global__ __launch_bounds__(kThreads) void assoc_dist_kernel(const spslam_assoc_frame* __restrict__ frames,
                                                              AssocSources S, const spslam_map_plane* __restrict__ map,
                                                              const float* __restrict__ boundary, int max_map,
                                                              float angle_th, float* __restrict__ dist) {
    tail_wave_priority();
    __shared__ float pm_s[kGroup][4];
    __shared__ int idx_s[kGroup];
    __shared__ float red[kWaves][kGroup];
    const int f = blockIdx.x, j = blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const spslam_assoc_frame& F = frames[f];
    if (j >= F.n_map) return;
    int na, nb;
    plane_counts(S, f, &na, &nb);
    const int n = na + nb, P = S.cap_a + S.cap_b;
    const spslam_map_plane M = map[F.map_offset + j];
    const float* pts = boundary + 3 * (size_t)M.boundary_offset;
    float* D = dist + (size_t)f * P * max_map;
    for (int i0 = 0; i0 < n; i0 += kGroup) {
        // the frame planes of this group whose normal passes the angle test
        if (t == 0) {
            int g = 0;
            for (int i = i0; i < min(i0 + kGroup, n); i++) {
                float pM[4];
                world_coeff(F.Tcw, coef_of(S, f, i, na), pM);
                const float angle = dot3(pM, M.world);
                if (angle > angle_th || angle < -angle_th) {
                    for (int k = 0; k < 4; k++) pm_s[g][k] = pM[k];
                    idx_s[g++] = i;
                } else {
                    D[(size_t)i * max_map + j] = -1.f;
                }
            }
            for (int k = g; k < kGroup; k++) idx_s[k] = -1;
        }
        __syncthreads();
        float pm[kGroup][4], mn[kGroup];
#pragma unroll
        for (int g = 0; g < kGroup; g++) {
#pragma unroll
            for (int k = 0; k < 4; k++) pm[g][k] = pm_s[g][k];
            mn[g] = 100.f;  // PointDistanceFromPlane: res = 100
        }
        if (idx_s[0] >= 0) {
            for (int p = t; p < M.n_boundary; p += kThreads) {
                const float q[3] = {pts[3 * p], pts[3 * p + 1], pts[3 * p + 2]};
#pragma unroll
                for (int g = 0; g < kGroup; g++) mn[g] = fminf(mn[g], fabsf(__fadd_rn(dot3(pm[g], q), pm[g][3])));
            }
#pragma unroll
            for (int g = 0; g < kGroup; g++) {
                float v = mn[g];
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o));
                if (lane == 0) red[w][g] = v;
            }
        }
        __syncthreads();
        if (t < kGroup && idx_s[t] >= 0) {
            float v = red[0][t];
            for (int k = 1; k < kWaves; k++) v = fminf(v, red[k][t]);
            D[(size_t)idx_s[t] * max_map + j] = v;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(64) void assoc_decide_kernel(const spslam_assoc_frame* __restrict__ frames,
                                                          AssocSources S, const spslam_map_plane* __restrict__ map,
                                                          int max_map, spslam_assoc_params Pm,
                                                          const float* __restrict__ dist, int32_t* __restrict__ match,
                                                          int32_t* __restrict__ parallel,
                                                          int32_t* __restrict__ vertical, int* __restrict__ new_plane) {
    tail_wave_priority();
    const int f = blockIdx.x;
    const spslam_assoc_frame& F = frames[f];
    int na, nb;
    plane_counts(S, f, &na, &nb);
    const int n = na + nb, P = S.cap_a + S.cap_b;
    const float* D = dist + (size_t)f * P * max_map;
    const spslam_map_plane* Mp = map + F.map_offset;
    int unmatched = 0;
    for (int i = threadIdx.x; i < n; i += 64) {
        float pM[4];
        world_coeff(F.Tcw, coef_of(S, f, i, na), pM);
        float ldTh = Pm.dis_th, lverTh = Pm.ver_th, lparTh = Pm.par_th;
        const size_t o = (size_t)f * P + i;
        // the frame's associations are only overwritten when a candidate is found (Map.cc:230-252): a
        // carried call (TrackLocalMap's) starts from what the first call left after the outlier discard
        int32_t m = -1, par = -1, ver = -1;
        if (F.carry) {
            m = match[o];
            par = parallel[o];
            ver = vertical[o];
        }
        for (int j = 0; j < F.n_map; j++) {
            const float angle = dot3(pM, Mp[j].world);
            if (angle > Pm.angle_th || angle < -Pm.angle_th) {
                const float dis = D[(size_t)i * max_map + j];
                if (dis < ldTh) {
                    ldTh = dis;
                    m = F.map_offset + j;
                    continue;
                }
            }
            if (angle < lverTh && angle > -lverTh) {
                lverTh = fabsf(angle);
                ver = F.map_offset + j;
                continue;
            }
            if (angle > lparTh || angle < -lparTh) {
                lparTh = fabsf(angle);
                par = F.map_offset + j;
            }
        }
        match[o] = m;
        parallel[o] = par;
        vertical[o] = ver;
        unmatched |= m < 0;
    }
    const int any = __syncthreads_or(unmatched);
    if (new_plane && threadIdx.x == 0) new_plane[f] = any;
}

// Fused form (the default when the per-frame distance table fits in LDS): one workgroup per frame.  Every
// frame plane's world coefficients are computed once (thread i: plane i), then each wave takes every 4th map
// plane: its lanes stride over that plane's boundary cloud keeping the running minima of |pM . (p, 1)| for
// up to 8 frame planes at a time (those passing the angle test; float minima, exact in any order), and a
// wave reduction writes the distance column.  Two workgroup barriers in all; the decision walk (the
// reference's order over the map planes) then runs from LDS, one thread per frame plane.  One launch of
// n_frames workgroups: inside the pipelined step the tracking chain's launches wait for CU slots behind the
// extraction kernels, so the grid size and the barrier count are the cost.
__global__ __launch_bounds__(kThreads) void assoc_fused_kernel(const spslam_assoc_frame* __restrict__ frames,
                                                               AssocSources S, const spslam_map_plane* __restrict__ map,
                                                               const float* __restrict__ boundary, int max_map,
                                                               spslam_assoc_params Pm, int32_t* __restrict__ match,
                                                               int32_t* __restrict__ parallel,
                                                               int32_t* __restrict__ vertical,
                                                               int* __restrict__ new_plane) {
    tail_wave_priority();
    extern __shared__ float lds[];  // [cap_a + cap_b][max_map] distances, then [cap_a + cap_b][4] world coefs
    const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const spslam_assoc_frame& F = frames[f];
    int na, nb;
    plane_counts(S, f, &na, &nb);
    const int n = na + nb, P = S.cap_a + S.cap_b, nm = F.n_map;
    float* D = lds;
    float* pm_s = lds + (size_t)P * max_map;
#pragma clang loop unroll(disable) interleave(disable) vectorize(disable)
    for (int i = t; i < n; i += kThreads) world_coeff(F.Tcw, coef_of(S, f, i, na), pm_s + 4 * i);
    __syncthreads();
    for (int j = w; j < nm; j += kWaves) {
        const spslam_map_plane M = map[F.map_offset + j];
        const float* pts = boundary + 3 * (size_t)M.boundary_offset;
        for (int i0 = 0; i0 < n; i0 += kGroup) {
            // the frame planes of this group whose normal passes the angle test against map plane j (every
            // lane evaluates the same tests; planes failing it keep the reference's untouched 100)
            float pmr[kGroup][4], mn[kGroup];
            bool pass[kGroup];
#pragma unroll
            for (int q = 0; q < kGroup; q++) {
                const int i = min(i0 + q, n - 1);
#pragma unroll
                for (int k = 0; k < 4; k++)  // wave-uniform: held in scalar registers
                    pmr[q][k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(pm_s[4 * i + k])));
                const float angle = dot3(pmr[q], M.world);
                pass[q] = i0 + q < n && (angle > Pm.angle_th || angle < -Pm.angle_th);
                mn[q] = 100.f;  // PointDistanceFromPlane: res = 100
            }
            for (int p = lane; p < M.n_boundary; p += 64) {
                const float qv[3] = {pts[3 * p], pts[3 * p + 1], pts[3 * p + 2]};
#pragma unroll
                for (int q = 0; q < kGroup; q++)
                    mn[q] = fminf(mn[q], fabsf(__fadd_rn(dot3(pmr[q], qv), pmr[q][3])));
            }
#pragma unroll
            for (int q = 0; q < kGroup; q++) {
                float v = mn[q];
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o));
                if (lane == 0 && i0 + q < n) D[(i0 + q) * max_map + j] = pass[q] ? v : 100.f;
            }
        }
    }
    __syncthreads();
    // the reference's walk over the map planes (Map.cc:207-257), one thread per frame plane
    int unmatched = 0;
    const spslam_map_plane* Mp = map + F.map_offset;
    for (int i = t; i < n; i += kThreads) {
        const float* pM = pm_s + 4 * i;
        float ldTh = Pm.dis_th, lverTh = Pm.ver_th, lparTh = Pm.par_th;
        const size_t o = (size_t)f * P + i;
        int32_t m = -1, par = -1, ver = -1;
        if (F.carry) {
            m = match[o];
            par = parallel[o];
            ver = vertical[o];
        }
        for (int j = 0; j < nm; j++) {
            const float angle = dot3(pM, Mp[j].world);
            if (angle > Pm.angle_th || angle < -Pm.angle_th) {
                const float dis = D[i * max_map + j];
                if (dis < ldTh) {
                    ldTh = dis;
                    m = F.map_offset + j;
                    continue;
                }
            }
            if (angle < lverTh && angle > -lverTh) {
                lverTh = fabsf(angle);
                ver = F.map_offset + j;
                continue;
            }
            if (angle > lparTh || angle < -lparTh) {
                lparTh = fabsf(angle);
                par = F.map_offset + j;
            }
        }
        match[o] = m;
        parallel[o] = par;
        vertical[o] = ver;
        unmatched |= m < 0;
    }
    const int any = __syncthreads_or(unmatched);
    if (new_plane && t == 0) new_plane[f] = any;
}

}  // namespace assoc

hipError_t assoc_launch(int n_frames, const spslam_assoc_frame* frames, const AssocSources& src,
                        const spslam_map_plane* map, const float* boundary, int max_map,
                        const spslam_assoc_params& P, float* dist, int32_t* match, int32_t* parallel,
                        int32_t* vertical, int* new_plane, hipStream_t s, KernelTimer* timer) {
    if (n_frames < 1 || max_map < 0 || src.cap_a < 0 || src.cap_b < 0) return hipErrorInvalidValue;
    if (timer) timer->begin(kKindAssoc, s);
    const size_t lds = (size_t)(src.cap_a + src.cap_b) * (max_map + 4) * sizeof(float);
    if (lds <= 48 * 1024) {
        hipLaunchKernelGGL(assoc::assoc_fused_kernel, dim3(n_frames), dim3(assoc::kThreads), std::max<size_t>(lds, 4),
                           s, frames, src, map, boundary, max_map, P, match, parallel, vertical, new_plane);
        if (timer) timer->end(kKindAssoc, s);
        return hipGetLastError();
    }
    if (max_map > 0)
        hipLaunchKernelGGL(assoc::assoc_dist_kernel, dim3(n_frames, max_map), dim3(assoc::kThreads), 0, s, frames,
                           src, map, boundary, max_map, P.angle_th, dist);
    hipLaunchKernelGGL(assoc::assoc_decide_kernel, dim3(n_frames), dim3(64), 0, s, frames, src, map, max_map, P,
                       dist, match, parallel, vertical, new_plane);
    if (timer) timer->end(kKindAssoc, s);
    return hipGetLastError();
}

}  // namespace spslam
