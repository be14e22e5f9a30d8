// RGB-D Frame per-keypoint steps on gfx950 (src/Frame.cc:146-181): the
// Frame constructor's UndistortKeyPoints (:504-534, cv::undistortPoints),
// ComputeStereoFromRGBD (:743-764) and AssignFeaturesToGrid (:326-341) for a
// batch of frames whose keypoints are already in HBM (ORB stage output).
//
// One 256-thread workgroup per frame: keypoints are processed thread-parallel
// (undistortion in double exactly as OpenCV's 5-iteration loop, depth gather
// at the distorted pixel, grid cell), cell counts are LDS atomics + a block
// scan, and the per-cell index lists are filled by one wave in keypoint order
// (64 keypoints per step, in-wave ranks), so every mGrid[x][y] list is in
// increasing keypoint index like the reference's push_back order.
#include <hip/hip_runtime.h>

#include "wave_priority.h"

#include "frame_launch.h"

namespace spslam {
namespace frame {

constexpr int kThreads = 256;
constexpr int kCells = SPSLAM_GRID_COLS * SPSLAM_GRID_ROWS;

// cv::undistortPoints(src, dst, K, D, noArray(), K) (OpenCV 3.4 cvUndistortPointsInternal).
__device__ void undistort(const FrameGeom& g, float u, float v, float* ou, float* ov) {
    const double fx = g.fx, fy = g.fy, cx = g.cx, cy = g.cy;
    const double ifx = 1. / fx, ify = 1. / fy;
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
    const double xx = fx * x + 0. * y + cx;
    const double yy = 0. * x + fy * y + cy;
    const double ww = 1. / (0. * x + 0. * y + 1.);
    *ou = (float)(xx * ww);
    *ov = (float)(yy * ww);
}

__global__ __launch_bounds__(kThreads) void frame_rgbd_kernel(
    FrameGeom g, const spslam_keypoint* __restrict__ kps, const int* __restrict__ counts, int cap,
    const float* __restrict__ depth, long long depth_fs, int stride, spslam_keypoint* __restrict__ keys_un,
    float* __restrict__ dout, float* __restrict__ urout, int32_t* __restrict__ grid_off,
    int32_t* __restrict__ grid_idx, int* __restrict__ plane_counts, int* __restrict__ supp_counts) {
    tail_wave_priority();
    __shared__ int cnt[kCells];
    __shared__ int wsum[kThreads / 64];
    extern __shared__ int16_t cell_of[];  // [cap]
    const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int n = min(counts[f], cap);
    const spslam_keypoint* K = kps + (size_t)f * cap;
    spslam_keypoint* U = keys_un + (size_t)f * cap;
    const float* D = depth + f * depth_fs;
    if (n == 0 && t == 0) {  // Frame.cc:148-149: no keypoints -> the constructor returns before the planes
        if (plane_counts) plane_counts[f] = 0;
        if (supp_counts) supp_counts[f] = 0;
    }
    for (int c = t; c < kCells; c += kThreads) cnt[c] = 0;
    __syncthreads();
    for (int i = t; i < n; i += kThreads) {
        spslam_keypoint kp = K[i];
        float xu = kp.x, yu = kp.y;
        if (g.undistort) undistort(g, kp.x, kp.y, &xu, &yu);
        // ComputeStereoFromRGBD: imDepth.at<float>(v, u) at the distorted point
        const float d = D[(long long)(int)kp.y * stride + (int)kp.x];
        float dd = -1.f, ur = -1.f;
        if (d > 0) {
            dd = d;
            ur = xu - g.bf / d;
        }
        dout[(size_t)f * cap + i] = dd;
        urout[(size_t)f * cap + i] = ur;
        kp.x = xu;
        kp.y = yu;
        U[i] = kp;
        // PosInGrid
        const int px = (int)roundf((xu - g.min_x) * g.ginv_x);
        const int py = (int)roundf((yu - g.min_y) * g.ginv_y);
        int c = -1;
        if (!(px < 0 || px >= SPSLAM_GRID_COLS || py < 0 || py >= SPSLAM_GRID_ROWS)) {
            c = px * SPSLAM_GRID_ROWS + py;
            atomicAdd(&cnt[c], 1);
        }
        cell_of[i] = (int16_t)c;
    }
    __syncthreads();
    // exclusive scan of the 3072 cell counts (12 per thread)
    constexpr int kPer = kCells / kThreads;
    int loc[kPer], s = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) { loc[k] = cnt[t * kPer + k]; s += loc[k]; }
    int x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int base = x - s;
    for (int w = 0; w < wave; w++) base += wsum[w];
    int32_t* GO = grid_off + (size_t)f * (kCells + 1);
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        cnt[t * kPer + k] = base;  // becomes the fill cursor
        GO[t * kPer + k] = base;
        base += loc[k];
    }
    if (t == kThreads - 1) GO[kCells] = base;
    __syncthreads();
    if (wave == 0) {
        int32_t* GI = grid_idx + (size_t)f * cap;
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            const int c = i < n ? cell_of[i] : -1;
            int rank = 0, tot = 0;
            for (int l = 0; l < 64; l++) {
                const int cl = __shfl(c, l);
                if (cl == c) {
                    tot++;
                    if (l < lane) rank++;
                }
            }
            if (c >= 0) {
                GI[cnt[c] + rank] = i;
            }
            if (c >= 0 && rank == 0) cnt[c] += tot;
        }
    }
}

}  // namespace frame

hipError_t frame_launch(const FrameGeom& g, int n, const spslam_keypoint* kps, const int* counts, int cap,
                        const float* depth, long long depth_fs, int stride, spslam_keypoint* keys_un, float* dout,
                        float* urout, int32_t* grid_off, int32_t* grid_idx, int* plane_counts, int* supp_counts,
                        hipStream_t s, KernelTimer* timer) {
    if (cap < 1 || cap > 32767) return hipErrorInvalidValue;
    if (timer) timer->begin(kKindFrame, s);
    hipLaunchKernelGGL(frame::frame_rgbd_kernel, dim3(n), dim3(frame::kThreads), (size_t)cap * sizeof(int16_t), s, g,
                       kps, counts, cap, depth, depth_fs, stride, keys_un, dout, urout, grid_off, grid_idx,
                       plane_counts, supp_counts);
    if (timer) timer->end(kKindFrame, s);
    return hipGetLastError();
}

}  // namespace spslam
