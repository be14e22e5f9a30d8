// gfx950 kernel for Tracking::GrabImageRGBD's image preparation
// (src/Tracking.cc:208-229): colour -> gray (cv::cvtColor 8U, OpenCV's
// fixed-point RGB2Gray: (R*4899 + G*9617 + B*1868 + 2^13) >> 14) and raw depth
// -> f32 metres (cv::Mat::convertTo(CV_32F, mDepthMapFactor): float(d) * factor,
// one rounding).  Pure streaming: 3-5 bytes in and 5 bytes out per pixel, so
// the kernel is HBM bound; each thread moves 8 consecutive pixels of a row
// with 8/16-byte loads and stores (64 px per wave = 1.5 KB of colour, 1 KB of
// depth in, 512 B gray + 2 KB depth out, fully coalesced).
// With a cloud output (CLOUD), the threads of every Cloud.Dis-th row also write the organized cloud's points of
// their 8 pixels (Frame.cc:857-874; the same float expressions as plane_cloud_kernel, so the cloud is bit-identical),
// which saves the plane chain a second pass over the depth lines it samples.
#include <hip/hip_runtime.h>

#include "grab_launch.h"

namespace spslam {

namespace {

constexpr int kThreads = 256;
constexpr int kPx = 8;  // pixels per thread (vector path)
constexpr int kR2Y = 4899, kG2Y = 9617, kB2Y = 1868, kShift = 14;

// c0, c1, c2 = the first three bytes of a pixel; rgb: c0 is red
__device__ __forceinline__ uint32_t gray_of(uint32_t c0, uint32_t c1, uint32_t c2, int rgb) {
    const uint32_t w0 = rgb ? kR2Y : kB2Y, w2 = rgb ? kB2Y : kR2Y;
    return (c0 * w0 + c1 * kG2Y + c2 * w2 + (1u << (kShift - 1))) >> kShift;
}

// Cloud point (m, n) of depth z: cloud[i], cloud[N + i], cloud[2N + i] (plane_cloud_kernel's expressions)
__device__ __forceinline__ void cloud_point(const GrabArgs& a, float* C, int i, int m, int n, float z) {
    C[i] = ((float)n - a.cx) * z / a.fx;
    C[a.cN + i] = ((float)m - a.cy) * z / a.fy;
    C[2 * a.cN + i] = z;
}

template <int CN, bool U16, bool CLOUD>
__global__ __launch_bounds__(kThreads) void grab_vec_kernel(GrabArgs a) {
    const int f = blockIdx.y;
    const int per_row = a.w / kPx;
    const int q = blockIdx.x * kThreads + threadIdx.x;
    if (q >= per_row * a.h) return;
    const int y = q / per_row, x = (q - y * per_row) * kPx;
    const uint8_t* c = a.color + f * a.color_frame_stride + (size_t)y * a.color_stride + (size_t)x * CN;
    uint8_t px[kPx * CN];
    if constexpr (CN == 1) {
        *(uint2*)px = *(const uint2*)c;
    } else if constexpr (CN == 3) {
        const uint2* s = (const uint2*)c;
        uint2* d = (uint2*)px;
        d[0] = s[0]; d[1] = s[1]; d[2] = s[2];
    } else {
        const uint4* s = (const uint4*)c;
        uint4* d = (uint4*)px;
        d[0] = s[0]; d[1] = s[1];
    }
    uint8_t g[kPx];
#pragma unroll
    for (int k = 0; k < kPx; k++)
        g[k] = CN == 1 ? px[k] : (uint8_t)gray_of(px[k * CN], px[k * CN + 1], px[k * CN + 2], a.p.rgb);
    *(uint2*)(a.gray + (size_t)f * a.w * a.h + (size_t)y * a.w + x) = *(const uint2*)g;

    float z[kPx];
    if constexpr (U16) {
        const uint16_t* d = (const uint16_t*)a.depth + f * a.depth_frame_stride + (size_t)y * a.depth_stride + x;
        uint16_t v[kPx];
        *(uint4*)v = *(const uint4*)d;
#pragma unroll
        for (int k = 0; k < kPx; k++) z[k] = __fmul_rn((float)v[k], a.p.depth_scale);
    } else {
        const float* d = (const float*)a.depth + f * a.depth_frame_stride + (size_t)y * a.depth_stride + x;
        *(float4*)z = *(const float4*)d;
        *(float4*)(z + 4) = *(const float4*)(d + 4);
        if (a.p.depth_scale != 1.0f) {
#pragma unroll
            for (int k = 0; k < kPx; k++) z[k] = __fmul_rn(z[k], a.p.depth_scale);
        }
    }
    float* o = a.depth_out + (size_t)f * a.w * a.h + (size_t)y * a.w + x;
    *(float4*)o = *(const float4*)z;
    *(float4*)(o + 4) = *(const float4*)(z + 4);
    if constexpr (CLOUD) {
        const int r = y / a.ds;
        if (r * a.ds != y) return;
        float* C = a.cloud + f * a.cloud_fs;
        const int c0 = (x + a.ds - 1) / a.ds;  // the first sampled column at or after x
        int k0 = c0 * a.ds - x, cc = c0;      // its pixel in this thread's group (the others follow every ds)
#pragma unroll
        for (int k = 0; k < kPx; k++) {
            if (k == k0) {
                cloud_point(a, C, r * a.cW + cc, y, x + k, z[k]);
                k0 += a.ds;
                cc++;
            }
        }
    }
}

// Any width / alignment: one pixel per thread.
__global__ __launch_bounds__(kThreads) void grab_scalar_kernel(GrabArgs a) {
    const int f = blockIdx.y;
    const int q = blockIdx.x * kThreads + threadIdx.x;
    if (q >= a.w * a.h) return;
    const int y = q / a.w, x = q - y * a.w, cn = a.p.channels;
    const uint8_t* c = a.color + f * a.color_frame_stride + (size_t)y * a.color_stride + (size_t)x * cn;
    a.gray[(size_t)f * a.w * a.h + q] = cn == 1 ? c[0] : (uint8_t)gray_of(c[0], c[1], c[2], a.p.rgb);
    float z;
    if (a.p.depth_u16) {
        z = __fmul_rn((float)((const uint16_t*)a.depth)[f * a.depth_frame_stride + (size_t)y * a.depth_stride + x],
                      a.p.depth_scale);
    } else {
        z = ((const float*)a.depth)[f * a.depth_frame_stride + (size_t)y * a.depth_stride + x];
        if (a.p.depth_scale != 1.0f) z = __fmul_rn(z, a.p.depth_scale);
    }
    a.depth_out[(size_t)f * a.w * a.h + q] = z;
    if (a.cloud && y % a.ds == 0 && x % a.ds == 0)
        cloud_point(a, a.cloud + f * a.cloud_fs, (y / a.ds) * a.cW + x / a.ds, y, x, z);
}

bool aligned(const void* p, size_t n) { return ((uintptr_t)p % n) == 0; }

template <int CN, bool U16>
void launch_vec(int n, const GrabArgs& a, hipStream_t s) {
    const int threads = a.w / kPx * a.h;
    const dim3 grid((threads + kThreads - 1) / kThreads, n);
    if (a.cloud) hipLaunchKernelGGL((grab_vec_kernel<CN, U16, true>), grid, dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((grab_vec_kernel<CN, U16, false>), grid, dim3(kThreads), 0, s, a);
}

}  // namespace

hipError_t grab_launch(int n, const GrabArgs& a, hipStream_t s, KernelTimer* timer) {
    const int cn = a.p.channels;
    const size_t de = a.p.depth_u16 ? 2 : 4;
    // vector path: 8-pixel groups with 8/16-byte aligned rows (640x480 / 1280x960 dense frames)
    const size_t cal = cn == 4 ? 16 : 8;
    const bool vec = a.w % kPx == 0 && aligned(a.color, cal) && a.color_stride % cal == 0 &&
                     a.color_frame_stride % cal == 0 && aligned(a.depth, 16) && (a.depth_stride * de) % 16 == 0 &&
                     (a.depth_frame_stride * de) % 16 == 0 && aligned(a.gray, 8) && aligned(a.depth_out, 16);
    if (timer) timer->begin(kKindGrab, s);
    if (vec) {
        if (a.p.depth_u16) {
            if (cn == 1) launch_vec<1, true>(n, a, s);
            else if (cn == 3) launch_vec<3, true>(n, a, s);
            else launch_vec<4, true>(n, a, s);
        } else {
            if (cn == 1) launch_vec<1, false>(n, a, s);
            else if (cn == 3) launch_vec<3, false>(n, a, s);
            else launch_vec<4, false>(n, a, s);
        }
    } else {
        hipLaunchKernelGGL(grab_scalar_kernel, dim3((a.w * a.h + kThreads - 1) / kThreads, n), dim3(kThreads), 0, s,
                           a);
    }
    if (timer) timer->end(kKindGrab, s);
    return hipGetLastError();
}

}  // namespace spslam
