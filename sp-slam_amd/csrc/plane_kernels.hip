// gfx950 kernels for Frame::ComputePlanesFromOrganizedPointCloud
// (src/Frame.cc:854-936) and the PCL 1.8 routines it calls.
//
//   plane_cloud_kernel     organized cloud, stride Cloud.Dis (Frame.cc:857-874)
//   plane_dist_integral_kernel
//                          depth-change map + PCL's two-pass chamfer distance
//                          transform, as two anti-diagonal wavefronts (one
//                          lane per cloud row, slope 2): every cell sees
//                          exactly the operands of the reference's raster scan
//                          (made from the raster cloud through per-row LDS
//                          windows); PCL IntegralImage2D<float,3> of the x/y
//                          gradient images (fp64, same recurrence order) rides
//                          along in the first wavefront
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

// Initial distance-map value of cell (r, c): 0 where the depth-change map is 0.  z(r, c) reads the
// cloud's z.
template <class ZAt>
__device__ __forceinline__ float dist_init(ZAt z, int W, int H, int r, int c) {
    bool zero = false;
    if (r < H - 1 && c < W - 1) zero = dc_bad(z(r, c), z(r, c + 1)) || dc_bad(z(r, c), z(r + 1, c));
    if (r < H - 1 && c >= 1) zero = zero || dc_bad(z(r, c - 1), z(r, c));
    if (r >= 1 && c < W - 1) zero = zero || dc_bad(z(r - 1, c), z(r, c));
    return zero ? 0.0f : (float)(W + H);
}

// Workgroup barrier that orders LDS only: global prefetches of the next wavefront step stay in flight
// across it (nothing another lane reads goes through global memory inside these kernels).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Depth-change distance map (PCL's two-pass chamfer transform) and the six fp64 integral images
// (IntegralImage2D<float,3> of the x / y gradients) in one workgroup per frame.  Both are raster
// recurrences replayed as anti-diagonal wavefronts, one lane per cloud row: the integral image's
// recurrence (up, left, up-left) fits inside the distance pass 1 schedule (slope 2: row r-1 is two
// columns ahead of row r), so both run in the same 2(H-1)+W barrier steps; a 4-column ring per row
// holds what row r+1 still reads.
// Pass 1's operands (each cell's initial distance and its six central differences) are made on chip: per
// chunk of K steps the workgroup stages, for every row, the K + 4 cloud columns that the chunk's cells of
// rows r-1, r, r+1 read (row r-1 runs two columns ahead, row r+1 two behind) in an LDS window, made from the
// depth image's samples (loaded while the previous chunk's steps run) exactly as plane_cloud_kernel makes the
// cloud: nothing is staged through HBM.  Pass 2 visits the cells in exactly the reverse order of pass 1, so in the skewed
// layout both passes read and write one contiguous span per step (the only HBM round trip left: the pass-1
// map, 4 + 4 bytes per cell).  Lanes outside the image compute on unused entries and keep their row state.
// Every cell sees exactly the operands of the reference's raster scans: both outputs stay bit-identical.
template <int MAXR, int K>
__global__ __launch_bounds__(MAXR) void plane_dist_integral_kernel(PlaneGeom g, const float* __restrict__ depth,
                                                                   long long depth_fs, int depth_stride, float* wave,
                                                                   long long wave_fs, float* dist, long long dist_fs,
                                                                   double* integral, long long integral_fs) {
    static_assert(K <= kWaveChunk, "the skewed layout pads kWaveChunk steps of prefetch slack");
    constexpr int WC = K + 4;  // window columns per row: c - 2 .. c + K + 1 around the chunk's first column c
    // slot-major: lane r touches consecutive LDS words
    __shared__ float ring[4][MAXR];
    __shared__ double iring[4][6][MAXR];
    constexpr int WP = WC + 1;  // odd row pitch: the rows' reads of one column spread over the banks
    __shared__ float win[3][MAXR][WP];
    const int f = blockIdx.x, r = threadIdx.x, W = g.W, H = g.H, HP = wave_pitch(H), SK = wave_steps(W, H);
    const float* Z = depth + f * depth_fs;
    // the organized cloud's point (rr, c) from the depth image, as plane_cloud_kernel makes it (same float
    // operations, so the same values)
    auto zof = [&](int rr, int c) { return Z[(long long)(rr * g.ds) * depth_stride + c * g.ds]; };
    float* D = wave + f * wave_fs + r;  // skewed pass-1 distance map (this lane's column)
    // stores of steps where this lane has no cell: one word of the layout's unused leading slack per lane (an
    // address select, not a branch; the line stays in L2 instead of every skewed entry reaching HBM)
    float* Dsink = D;
    float* Dout = dist + f * dist_fs + (long long)r * W;  // raster row r
    const int IW = W + 1;
    double* Iraw = integral + f * integral_fs;
    for (int c = threadIdx.x; c < IW; c += blockDim.x)
        for (int k = 0; k < 6; k++) Iraw[(size_t)c * 6 + k] = 0.0;  // integral row 0
    if (r < H)
        for (int k = 0; k < 6; k++) Iraw[(size_t)(r + 1) * IW * 6 + k] = 0.0;  // column 0
    // raster integral entry (r+1, c+1) of this row; lanes beyond the cloud write into a dummy row
    double* I = Iraw + (size_t)((r < H ? r : H) + 1) * IW * 6 + 6;
    double* Idummy = Iraw + (size_t)(H + 1) * IW * 6;  // sink of the stores of cells outside the cloud
    const bool row_ok = r < H;
    const int rm = r > 0 ? r - 1 : 0, rp = r + 1 < MAXR ? r + 1 : r;  // neighbour rows (reads masked below)
    struct Cell { float center, e[6]; };
    // the windows of the chunk starting at step s0: row rr, columns s0 - 2rr - 2 + i (clamped; the clamped
    // entries feed only cells outside the cloud).  Loaded by the whole workgroup with the window's columns
    // across consecutive lanes (a 64-lane load touches ~6 rows, not 64), straight from the depth image (one
    // plane instead of the cloud's three), held in registers while the previous chunk's steps run, then
    // expanded to x / y / z and stored to LDS.
    const int nthr = blockDim.x;
    float wz[WC];
    auto wcell = [&](int s0, int m, int& rr, int& i, int& ro, int& c) {
        const int q = r + m * nthr;
        rr = q / WC;
        i = q - rr * WC;
        ro = min(rr, H - 1);
        c = min(max(s0 - 2 * rr - 2 + i, 0), W - 1);
    };
    auto wload = [&](int s0) {
#pragma unroll
        for (int m = 0; m < WC; m++) {
            int rr, i, ro, c;
            wcell(s0, m, rr, i, ro, c);
            wz[m] = zof(ro, c);
        }
    };
    auto wstore = [&](int s0) {
#pragma unroll
        for (int m = 0; m < WC; m++) {
            int rr, i, ro, c;
            wcell(s0, m, rr, i, ro, c);
            if (rr < H) {
                const float z = wz[m];
                win[0][rr][i] = ((float)(c * g.ds) - g.cx) * z / g.fx;
                win[1][rr][i] = ((float)(ro * g.ds) - g.cy) * z / g.fy;
                win[2][rr][i] = z;
            }
        }
    };
    // cell (r, c = s0 + j - 2r): the wave_prep operands, from the windows of rows r-1, r, r+1
    auto cell = [&](int s0, int j) {
        const int c = s0 + j - 2 * r;
        auto at = [&](int k, int rr, int cc) { return win[k][rr][cc - s0 + 2 * rr + 2]; };
        Cell o;
        o.center = dist_init([&](int rr, int cc) { return at(2, rr, cc); }, W, H, r, c);
#pragma unroll
        for (int k = 0; k < 6; k++) o.e[k] = 0.f;
        if (r >= 1 && r <= H - 2 && c >= 1 && c <= W - 2) {
#pragma unroll
            for (int k = 0; k < 3; k++) {
                o.e[k] = at(k, r, c + 1) - at(k, r, c - 1);
                o.e[3 + k] = at(k, r + 1, c) - at(k, r - 1, c);
            }
        }
        return o;
    };
    // pass 1 (top-left to bottom-right), step s handles column c = s - 2r of row r
    float left = 0.f;
    double ileft[6] = {0, 0, 0, 0, 0, 0};
    // initial value of (r, 0), which the last column's up-right read sees
    const float row0 = row_ok ? dist_init(zof, W, H, r, 0) : 0.f;
    auto step1 = [&](int s, const Cell& q) {
        const int c = s - 2 * r;
        const bool ok = row_ok && c >= 0 && c < W, inner = r > 0 && c > 0;
        const float upLeft = ring[(c - 1) & 3][rm] + 1.4f;
        const float up = ring[c & 3][rm] + 1.0f;
        // c == W-1 reads previous_row[W] == this row's element 0 (PCL quirk)
        const float upRight = (c + 1 < W ? ring[(c + 1) & 3][rm] : row0) + 1.4f;
        const float lft = left + 1.0f;
        const float mv = fminf(fminf(upLeft, up), fminf(lft, upRight));
        const float v = inner && mv < q.center ? mv : q.center;
        if (ok) {
            ring[c & 3][r] = v;
            left = v;
        }
        *(ok ? D + (s + kWaveChunk) * HP : Dsink) = v;  // entries outside the cloud are never read back
        double iv[6];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const double upI = r > 0 ? iring[c & 3][k][rm] : 0.0;
            const double upleftI = inner ? iring[(c - 1) & 3][k][rm] : 0.0;
            iv[k] = upI + ileft[k] - upleftI;
            iv[k] += (double)q.e[k];
            if (ok) {
                ileft[k] = iv[k];
                iring[c & 3][k][r] = iv[k];
            }
        }
        {  // unconditional store (a branch around it would make the compiler's prefetch waits conservative)
            double2* out = reinterpret_cast<double2*>(ok ? I + c * 6 : Idummy);
            out[0] = make_double2(iv[0], iv[1]);
            out[1] = make_double2(iv[2], iv[3]);
            out[2] = make_double2(iv[4], iv[5]);
        }
    };
    wload(0);
    wstore(0);
    __syncthreads();
    for (int s0 = 0; s0 < SK; s0 += K) {
        Cell cur[K];
#pragma unroll
        for (int j = 0; j < K; j++) cur[j] = cell(s0, j);
        wload(s0 + K);  // in flight during the chunk's steps; the window is dead once every lane has its cells
#pragma unroll
        for (int j = 0; j < K; j++) {
            step1(s0 + j, cur[j]);
            lds_barrier();
        }
        wstore(s0 + K);
        lds_barrier();
    }
    // pass 2 (bottom-right to top-left): iteration j visits the cells pass 1 visited at step SK-1-j
    // (column c = W-1 - (s - 2(H-1-r)) of the reference's order, shifted by the padded steps); each lane
    // reads back only the values it wrote itself
    float right = 0.f;
    const float lastcol = row_ok ? D[(W - 1 + 2 * r + kWaveChunk) * HP] : 0.f;
    auto step2 = [&](int j, float center) {
        const int st = SK - 1 - j, c = st - 2 * r;
        const bool ok = row_ok && c >= 0 && c < W, inner = r < H - 1 && c < W - 1;
        // c == 0 reads next_row[-1] == this row's element W-1 (PCL quirk)
        const float lowerLeft = (c > 0 ? ring[(c - 1) & 3][rp] : lastcol) + 1.4f;
        const float lower = ring[c & 3][rp] + 1.0f;
        const float lowerRight = ring[(c + 1) & 3][rp] + 1.4f;
        const float rgt = right + 1.0f;
        const float mv = fminf(fminf(lowerLeft, lower), fminf(rgt, lowerRight));
        const float v = inner && mv < center ? mv : center;
        if (ok) {
            ring[c & 3][r] = v;
            right = v;
        }
        *(ok ? Dout + c : Dsink) = v;
    };
    auto dval = [&](int j) {
        const int st = SK - 1 - j, c = st - 2 * r;
        return D[((row_ok && c >= 0 && c < W ? st : 0) + kWaveChunk) * HP];
    };
    constexpr int K2 = kWaveChunk;
    float dcur[K2];
#pragma unroll
    for (int j = 0; j < K2; j++) dcur[j] = dval(j);
    for (int j0 = 0; j0 < SK; j0 += K2) {
        float dnxt[K2];
#pragma unroll
        for (int j = 0; j < K2; j++) dnxt[j] = dval(j0 + K2 + j);
#pragma unroll
        for (int j = 0; j < K2; j++) {
            step2(j0 + j, dcur[j]);
            lds_barrier();
        }
#pragma unroll
        for (int j = 0; j < K2; j++) dcur[j] = dnxt[j];
    }
}

__global__ __launch_bounds__(256) void plane_normal_kernel(PlaneGeom g, const float* __restrict__ cloud,
                                                           long long cloud_fs, const float* __restrict__ dist,
                                                           long long dist_fs, const double* __restrict__ integral,
                                                           long long integral_fs, float* normal, long long normal_fs,
                                                           float* pd, long long pd_fs) {
    // XCD-aware order: a frame's blocks on one L2 (the smoothing windows of neighbouring blocks share the
    // integral-image rows)
    const int nb = gridDim.x, id = xcd_remap(blockIdx.y * nb + blockIdx.x, nb * gridDim.y);
    const int f = id / nb, i = (id - f * nb) * 256 + threadIdx.x;
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
    {
        const int rows = wave_pitch(g.H);
        auto* k = g.H <= 192   ? plane_dist_integral_kernel<192, kWaveChunk>
                  : g.H <= 320 ? plane_dist_integral_kernel<320, kWaveChunk>
                               : plane_dist_integral_kernel<kWaveThreads, kWaveChunk / 2>;  // (LDS: 155 KB)
        hipLaunchKernelGGL(k, dim3(n), dim3(rows), 0, s, g, depth, depth_fs, depth_stride, b.wave, b.wave_fs, b.dist,
                           b.dist_fs, b.integral, b.integral_fs);
    }
    E(kKindPlaneDist);
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
