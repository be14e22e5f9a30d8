// gfx950 kernels for Frame::ComputePlanesFromOrganizedPointCloud
// (src/Frame.cc:854-936) and the PCL 1.8 routines it calls.
//
//   plane_cloud_kernel     organized cloud, stride Cloud.Dis (Frame.cc:857-874)
//   plane_distance_kernel  depth-change map + PCL's two-pass chamfer distance
//                          transform, as two anti-diagonal wavefronts (one
//                          wave lane per cloud row, slope 2): every cell sees
//                          exactly the operands of the reference's raster scan
//   plane_integral_kernel  PCL IntegralImage2D<float,3> of the x/y gradient
//                          images, fp64, same recurrence order, wavefront t=r+c
//   plane_normal_kernel    AVERAGE_3D_GRADIENT normals + flip to viewpoint,
//                          plane_d = p . n (one thread per cloud point)
//   plane_segment_kernel   (plane_segment.hip) connected components, models,
//                          refinement, contours, Frame's post-steps
// Distance map, integral images and normals are bit-identical to the CPU
// restatement; see DESIGN.md for the float/double semantics chosen.
#include <hip/hip_runtime.h>

#include "plane_launch.h"

namespace spslam {
namespace planes {

constexpr int kWaveThreads = 512;  // max cloud rows handled by one wavefront workgroup

__global__ __launch_bounds__(256) void plane_cloud_kernel(PlaneGeom g, const float* __restrict__ depth,
                                                          long long depth_fs, int depth_stride, float* cloud,
                                                          long long cloud_fs) {
    const int f = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    if (i >= g.N) return;
    const int r = i / g.W, c = i - r * g.W;
    const int m = r * g.ds, n = c * g.ds;
    const float z = depth[f * depth_fs + (long long)m * depth_stride + n];
    float* C = cloud + f * cloud_fs;
    C[i] = ((float)n - g.cx) * z / g.fx;
    C[g.N + i] = ((float)m - g.cy) * z / g.fy;
    C[2 * g.N + i] = z;
}

// IntegralImageNormalEstimation::computeFeature depth-change test.
__device__ __forceinline__ bool dc_bad(float za, float zb) {
    const float thr = (0.05f * (fabsf(za) + 1.0f) * 2.0f);
    return fabsf(za - zb) > thr || !isfinite(za) || !isfinite(zb);
}

// Initial distance-map value of cell (r, c): 0 where the depth-change map is 0.
__device__ __forceinline__ float dist_init(const float* Z, int W, int H, int r, int c) {
    const int i = r * W + c;
    bool zero = false;
    if (r < H - 1 && c < W - 1) zero = dc_bad(Z[i], Z[i + 1]) || dc_bad(Z[i], Z[i + W]);
    if (r < H - 1 && c >= 1) zero = zero || dc_bad(Z[i - 1], Z[i]);
    if (r >= 1 && c < W - 1) zero = zero || dc_bad(Z[i - W], Z[i]);
    return zero ? 0.0f : (float)(W + H);
}

__global__ __launch_bounds__(kWaveThreads) void plane_distance_kernel(PlaneGeom g, const float* __restrict__ cloud,
                                                                      long long cloud_fs, float* dist,
                                                                      long long dist_fs) {
    __shared__ float ring[kWaveThreads][4];
    const int f = blockIdx.x, r = threadIdx.x, W = g.W, H = g.H;
    const float* Z = cloud + f * cloud_fs + 2 * g.N;
    float* D = dist + f * dist_fs;
    // pass 1 (top-left to bottom-right), step s handles column c = s - 2r of row r
    float left = 0.f;
    const float row0 = r < H ? dist_init(Z, W, H, r, 0) : 0.f;
    for (int s = 0; s < 2 * (H - 1) + W; s++) {
        const int c = s - 2 * r;
        if (r < H && c >= 0 && c < W) {
            const float center = dist_init(Z, W, H, r, c);
            float v = center;
            if (r > 0 && c > 0) {
                const float upLeft = ring[r - 1][(c - 1) & 3] + 1.4f;
                const float up = ring[r - 1][c & 3] + 1.0f;
                // c == W-1 reads previous_row[W] == this row's element 0 (PCL quirk)
                const float upRight = (c + 1 < W ? ring[r - 1][(c + 1) & 3] : row0) + 1.4f;
                const float lft = left + 1.0f;
                const float mv = fminf(fminf(upLeft, up), fminf(lft, upRight));
                if (mv < center) v = mv;
            }
            ring[r][c & 3] = v;
            left = v;
            D[r * W + c] = v;
        }
        __syncthreads();
    }
    // pass 2 (bottom-right to top-left): step s handles c = W-1 - (s - 2(H-1-r))
    float right = 0.f;
    const float lastcol = r < H ? D[r * W + W - 1] : 0.f;
    for (int s = 0; s < 2 * (H - 1) + W; s++) {
        const int c = W - 1 - (s - 2 * (H - 1 - r));
        if (r < H && c >= 0 && c < W) {
            const float center = D[r * W + c];
            float v = center;
            if (r < H - 1 && c < W - 1) {
                // c == 0 reads next_row[-1] == this row's element W-1 (PCL quirk)
                const float lowerLeft = (c > 0 ? ring[r + 1][(c - 1) & 3] : lastcol) + 1.4f;
                const float lower = ring[r + 1][c & 3] + 1.0f;
                const float lowerRight = ring[r + 1][(c + 1) & 3] + 1.4f;
                const float rgt = right + 1.0f;
                const float mv = fminf(fminf(lowerLeft, lower), fminf(rgt, lowerRight));
                if (mv < center) v = mv;
            }
            ring[r][c & 3] = v;
            right = v;
            D[r * W + c] = v;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kWaveThreads) void plane_integral_kernel(PlaneGeom g, const float* __restrict__ cloud,
                                                                      long long cloud_fs, double* integral,
                                                                      long long integral_fs) {
    __shared__ double ring[kWaveThreads][3][6];
    const int f = blockIdx.x, r = threadIdx.x, W = g.W, H = g.H, N = g.N, IW = W + 1;
    const float* X = cloud + f * cloud_fs;
    const float* Y = X + N;
    const float* Z = X + 2 * N;
    double* I = integral + f * integral_fs;
    for (int c = threadIdx.x; c < IW; c += blockDim.x)
        for (int k = 0; k < 6; k++) I[(size_t)c * 6 + k] = 0.0;  // integral row 0
    if (r < H)
        for (int k = 0; k < 6; k++) I[(size_t)(r + 1) * IW * 6 + k] = 0.0;  // column 0
    double left[6] = {0, 0, 0, 0, 0, 0};
    for (int s = 0; s < W + H - 1; s++) {
        const int c = s - r;
        if (r < H && c >= 0 && c < W) {
            float e[6] = {0, 0, 0, 0, 0, 0};
            if (r >= 1 && r <= H - 2 && c >= 1 && c <= W - 2) {
                const int i = r * W + c;
                e[0] = X[i + 1] - X[i - 1]; e[1] = Y[i + 1] - Y[i - 1]; e[2] = Z[i + 1] - Z[i - 1];
                e[3] = X[i + W] - X[i - W]; e[4] = Y[i + W] - Y[i - W]; e[5] = Z[i + W] - Z[i - W];
            }
            double* out = &I[((size_t)(r + 1) * IW + c + 1) * 6];
#pragma unroll
            for (int k = 0; k < 6; k++) {
                const double up = r > 0 ? ring[r - 1][c % 3][k] : 0.0;
                const double upleft = (r > 0 && c > 0) ? ring[r - 1][(c + 2) % 3][k] : 0.0;
                double v = up + left[k] - upleft;
                v += (double)e[k];
                left[k] = v;
                ring[r][c % 3][k] = v;
                out[k] = v;
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void plane_normal_kernel(PlaneGeom g, const float* __restrict__ cloud,
                                                           long long cloud_fs, const float* __restrict__ dist,
                                                           long long dist_fs, const double* __restrict__ integral,
                                                           long long integral_fs, float* normal, long long normal_fs,
                                                           float* pd, long long pd_fs) {
    const int f = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    if (i >= g.N) return;
    const int W = g.W, H = g.H, N = g.N, IW = W + 1, r = i / W, c = i - r * W;
    const float* X = cloud + f * cloud_fs;
    const float x = X[i], y = X[N + i], z = X[2 * N + i];
    float nx = __builtin_nanf(""), ny = nx, nz = nx;
    const int border = 10;
    if (r >= border && r < H - border && c >= border && c < W - border && isfinite(z)) {
        const float smoothing = fminf(dist[f * dist_fs + i], 10.0f);
        if (smoothing > 2.0f) {
            const int rw = (int)smoothing;
            const int sx = c - rw / 2, sy = r - rw / 2;
            const double* I = integral + f * integral_fs;
            const double* LR = &I[((size_t)(sy + rw) * IW + sx + rw) * 6];
            const double* UL = &I[((size_t)sy * IW + sx) * 6];
            const double* UR = &I[((size_t)sy * IW + sx + rw) * 6];
            const double* LL = &I[((size_t)(sy + rw) * IW + sx) * 6];
            double gx[3], gy[3];
            for (int k = 0; k < 3; k++) {
                gx[k] = LR[k] + UL[k] - UR[k] - LL[k];
                gy[k] = LR[3 + k] + UL[3 + k] - UR[3 + k] - LL[3 + k];
            }
            double nv[3] = {gy[1] * gx[2] - gy[2] * gx[1], gy[2] * gx[0] - gy[0] * gx[2], gy[0] * gx[1] - gy[1] * gx[0]};
            const double len = nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2];
            if (len != 0.0) {
                const double sl = sqrt(len);
                nx = (float)(nv[0] / sl); ny = (float)(nv[1] / sl); nz = (float)(nv[2] / sl);
                const float vx = 0.f - x, vy = 0.f - y, vz = 0.f - z;
                const float cos_theta = (vx * nx + vy * ny + vz * nz);
                if (cos_theta < 0) { nx *= -1; ny *= -1; nz *= -1; }
            }
        }
    }
    float* Nn = normal + f * normal_fs;
    Nn[i] = nx; Nn[N + i] = ny; Nn[2 * N + i] = nz;
    pd[f * pd_fs + i] = x * nx + y * ny + z * nz;
}

}  // namespace planes

using namespace planes;

hipError_t plane_launch(const PlaneGeom& g, const PlaneBuffers& b, int n, const float* depth, long long depth_fs,
                        int depth_stride, spslam_plane* planes, int* plane_counts, int planes_cap, int32_t* inliers,
                        int32_t* contours, hipStream_t s, KernelTimer* timer) {
    if (g.H > kWaveThreads) return hipErrorInvalidValue;
    auto B = [&](int k) { if (timer) timer->begin(k, s); };
    auto E = [&](int k) { if (timer) timer->end(k, s); };
    const dim3 pts((g.N + 255) / 256, n);
    B(kKindPlaneCloud);
    hipLaunchKernelGGL(plane_cloud_kernel, pts, dim3(256), 0, s, g, depth, depth_fs, depth_stride, b.cloud, b.cloud_fs);
    E(kKindPlaneCloud);
    B(kKindPlaneDist);
    hipLaunchKernelGGL(plane_distance_kernel, dim3(n), dim3(kWaveThreads), 0, s, g, b.cloud, b.cloud_fs, b.dist,
                       b.dist_fs);
    E(kKindPlaneDist);
    B(kKindPlaneIntegral);
    hipLaunchKernelGGL(plane_integral_kernel, dim3(n), dim3(kWaveThreads), 0, s, g, b.cloud, b.cloud_fs, b.integral,
                       b.integral_fs);
    E(kKindPlaneIntegral);
    B(kKindPlaneNormal);
    hipLaunchKernelGGL(plane_normal_kernel, pts, dim3(256), 0, s, g, b.cloud, b.cloud_fs, b.dist, b.dist_fs,
                       b.integral, b.integral_fs, b.normal, b.normal_fs, b.pd, b.pd_fs);
    E(kKindPlaneNormal);
    B(kKindPlaneSegment);
    const hipError_t e = plane_segment_launch(g, b, n, planes, plane_counts, planes_cap, inliers, contours, s);
    E(kKindPlaneSegment);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

}  // namespace spslam
