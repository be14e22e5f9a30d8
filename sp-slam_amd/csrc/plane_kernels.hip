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
//   plane_segment_kernel   one 1024-thread workgroup per frame: connected
//                          components (lock-free union-find, roots = first
//                          raster pixel => PCL's label order), per-component
//                          float mean/covariance in PCL's accumulation order,
//                          eigen33, curvature filter, two-pass refinement,
//                          Moore contour tracing, Frame's sign flip and
//                          PlaneNotSeen, output assembly.
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

// ---------------------------------------------------------------------------
// Segmentation.
constexpr int kSegThreads = 1024;

struct SegShared {
    int wsum[kSegThreads / 64];
    int misc[16];
    int nbig;
    int big_label[kMaxPlanesPerFrame * 4];   // big components (size > MinSize), label order
    int big_off[kMaxPlanesPerFrame * 4];
    float big_par[kMaxPlanesPerFrame * 4][4];
    float big_cen[kMaxPlanesPerFrame * 4][4];
    float big_curv[kMaxPlanesPerFrame * 4];
    int nmodel;
    int model_big[kMaxPlanesPerFrame];       // big index of each model
    float model_coef[kMaxPlanesPerFrame][4];
    int model_grown[kMaxPlanesPerFrame];
    int kept[kMaxPlanesPerFrame];
    int nkept;
};
constexpr int kMaxBig = kMaxPlanesPerFrame * 4;

__device__ __forceinline__ int ld_agent(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int uf_find(const int* P, int x) {
    int p = ld_agent(&P[x]);
    while (p != x) { x = p; p = ld_agent(&P[x]); }
    return x;
}
__device__ void uf_unite(int* P, int a, int b) {
    while (true) {
        int ra = uf_find(P, a), rb = uf_find(P, b);
        if (ra == rb) return;
        if (ra > rb) { const int t = ra; ra = rb; rb = t; }
        if (atomicCAS(&P[rb], rb, ra) == rb) return;
    }
}

// Exclusive scan of v over all kSegThreads threads; returns total.
__device__ int seg_scan(int v, int* wsum, int* excl) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int base = 0, total = 0;
    for (int j = 0; j < kSegThreads / 64; j++) {
        if (j < w) base += wsum[j];
        total += wsum[j];
    }
    *excl = base + x - v;
    __syncthreads();
    return total;
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
        const float theta = atan2f(sqrtf(-q), half_b) * s_inv3;
        const float ct = cosf(theta), st = sinf(theta);
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

__global__ __launch_bounds__(kSegThreads) void plane_segment_kernel(
    PlaneGeom g, PlaneBuffers b, spslam_plane* __restrict__ planes_out, int* __restrict__ plane_counts, int planes_cap,
    int32_t* __restrict__ inliers_out, int32_t* __restrict__ contours_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t state[];  // N bytes: model id + 1 per point
    __shared__ SegShared S;
    const int f = blockIdx.x, t = threadIdx.x, W = g.W, H = g.H, N = g.N;
    const float* X = b.cloud + f * b.cloud_fs;
    const float* Y = X + N;
    const float* Z = X + 2 * N;
    const float* Nx = b.normal + f * b.normal_fs;
    const float* Ny = Nx + N;
    const float* Nz = Nx + 2 * N;
    const float* PD = b.pd + f * b.pd_fs;
    int* P = (int*)(b.labels + f * b.labels_fs);   // parent, then labels
    int* root = b.work + f * b.work_fs;             // N
    int* rank = root + N;                           // N
    int* sizes = rank + N;                          // N
    int* members = sizes + N;                       // N
    int* grown = b.grown + f * b.grown_fs;          // N
    int* grown_m = b.grown_model + f * b.grown_fs;  // N
    spslam_plane* planes = planes_out + (size_t)f * planes_cap;
    int32_t* inl = inliers_out + (size_t)f * g.inlier_cap;
    int32_t* con = contours_out + (size_t)f * g.contour_cap;

    // ---- OrganizedConnectedComponentSegmentation with PlaneCoefficientComparator
    for (int i = t; i < N; i += kSegThreads) P[i] = i;
    __syncthreads();
    auto cmp = [&](int i1, int i2) {
        const float z = X[i1] * 0.f + Y[i1] * 0.f + Z[i1] * 1.f;
        float threshold = g.dist_th;
        threshold *= z * z;
        const float nd = Nx[i1] * Nx[i2] + Ny[i1] * Ny[i2] + Nz[i1] * Nz[i2];
        return (fabsf(PD[i1] - PD[i2]) < threshold) && (nd > g.ang_cos);
    };
    for (int i = t; i < N; i += kSegThreads) {
        const int r = i / W, c = i - r * W;
        if (c >= 1 && cmp(i, i - 1)) uf_unite(P, i, i - 1);
        if (r >= 1 && cmp(i, i - W)) uf_unite(P, i, i - W);
    }
    __threadfence();
    __syncthreads();
    for (int i = t; i < N; i += kSegThreads) root[i] = uf_find(P, i);
    __threadfence();
    __syncthreads();
    // label = rank of the component's first raster pixel among all roots
    const int per = (N + kSegThreads - 1) / kSegThreads;
    const int i0 = t * per, i1 = min(N, i0 + per);
    int cnt = 0;
    for (int i = i0; i < i1; i++) cnt += root[i] == i;
    int base;
    const int ncomp = seg_scan(cnt, S.wsum, &base);
    for (int i = i0; i < i1; i++)
        if (root[i] == i) rank[i] = base++;
    __threadfence();
    __syncthreads();
    for (int i = t; i < N; i += kSegThreads) P[i] = rank[root[i]];
    for (int k = t; k < ncomp; k += kSegThreads) sizes[k] = 0;
    __threadfence();
    __syncthreads();
    for (int i = t; i < N; i += kSegThreads) atomicAdd(&sizes[P[i]], 1);
    __threadfence();
    __syncthreads();

    // ---- components larger than MinSize, in label order (segment(), :segment loop)
    {
        const int perc = (ncomp + kSegThreads - 1) / kSegThreads;
        const int k0 = t * perc, k1 = min(ncomp, k0 + perc);
        int nb = 0;
        for (int k = k0; k < k1; k++) nb += (unsigned)sizes[k] > (unsigned)g.min_size;
        int bb;
        const int nbig = seg_scan(nb, S.wsum, &bb);
        for (int k = k0; k < k1; k++)
            if ((unsigned)sizes[k] > (unsigned)g.min_size && bb < kMaxBig) S.big_label[bb++] = k;
        if (t == 0) {
            S.nbig = min(nbig, kMaxBig);
            int off = 0;
            for (int j = 0; j < S.nbig; j++) { S.big_off[j] = off; off += sizes[S.big_label[j]]; }
        }
        __syncthreads();
    }
    const int nbig = S.nbig;
    const int lane = t & 63, wave = t >> 6;
    // member lists (raster order) by per-wave ballot compaction
    for (int j = wave; j < nbig; j += kSegThreads / 64) {
        const int L = S.big_label[j];
        int o = S.big_off[j];
        for (int i0w = 0; i0w < N; i0w += 64) {
            const int i = i0w + lane;
            const bool m = i < N && P[i] == L;
            const unsigned long long mask = __ballot(m);
            if (m) members[o + __popcll(mask & ((1ull << lane) - 1ull))] = i;
            o += __popcll(mask);
        }
    }
    __threadfence();
    __syncthreads();
    // mean + covariance in PCL's float accumulation order: lane k owns term k
    for (int j = wave; j < nbig; j += kSegThreads / 64) {
        const int n = sizes[S.big_label[j]], o = S.big_off[j];
        float acc = 0.f;
        if (lane < 9) {
            for (int q = 0; q < n; q++) {
                const int i = members[o + q];
                const float x = X[i], y = Y[i], z = Z[i];
                float term;
                switch (lane) {
                    case 0: term = x * x; break;
                    case 1: term = x * y; break;
                    case 2: term = x * z; break;
                    case 3: term = y * y; break;
                    case 4: term = y * z; break;
                    case 5: term = z * z; break;
                    case 6: term = x; break;
                    case 7: term = y; break;
                    default: term = z; break;
                }
                acc += term;
            }
            acc /= (float)n;
        }
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
            float ev, evec[3];
            eigen33_min(cov, &ev, evec);
            const float eig_sum = cov[0][0] + cov[1][1] + cov[2][2];
            S.big_curv[j] = eig_sum != 0 ? fabsf(ev / eig_sum) : 0.f;
            S.big_par[j][0] = evec[0]; S.big_par[j][1] = evec[1]; S.big_par[j][2] = evec[2]; S.big_par[j][3] = 0.f;
            S.big_cen[j][0] = a[6]; S.big_cen[j][1] = a[7]; S.big_cen[j][2] = a[8]; S.big_cen[j][3] = 1.f;
        }
    }
    __syncthreads();
    if (t == 0) {
        // plane sign via the (accumulating) viewpoint vector, curvature filter
        float vp[4] = {0, 0, 0, 0};
        int nm = 0;
        for (int j = 0; j < nbig; j++) {
            float pp[4] = {S.big_par[j][0], S.big_par[j][1], S.big_par[j][2], 0.f};
            pp[3] = -1 * dot4(pp, S.big_cen[j]);
            for (int k = 0; k < 4; k++) vp[k] -= S.big_cen[j][k];
            if (dot4(vp, pp) < 0) {
                for (int k = 0; k < 4; k++) pp[k] *= -1;
                pp[3] = 0;
                pp[3] = -1 * dot4(pp, S.big_cen[j]);
            }
            if (S.big_curv[j] < 0.001f && nm < kMaxPlanesPerFrame) {
                S.model_big[nm] = j;
                for (int k = 0; k < 4; k++) S.model_coef[nm][k] = pp[k];
                S.model_grown[nm] = 0;
                nm++;
            }
        }
        S.nmodel = nm;
    }
    __syncthreads();
    const int nmodel = S.nmodel;

    // ---- refinement (PlaneRefinementComparator, 0.02 m): per-point state = model + 1
    for (int i = t; i < N; i += kSegThreads) state[i] = 0;
    __syncthreads();
    for (int m = 0; m < nmodel; m++) {
        const int j = S.model_big[m], n = sizes[S.big_label[j]], o = S.big_off[j];
        for (int q = t; q < n; q += kSegThreads) state[members[o + q]] = (uint8_t)(m + 1);
    }
    __syncthreads();
    if (t == 0) {
        int ng = 0;
        auto grow = [&](int i, int j) {
            const int s = state[i];
            if (!s || state[j]) return;
            const float* m = S.model_coef[s - 1];
            const double ptp = fabsf(m[0] * X[j] + m[1] * Y[j] + m[2] * Z[j] + m[3]);
            if (ptp < 0.02f) {
                state[j] = (uint8_t)s;
                grown[ng] = j;
                grown_m[ng] = s - 1;
                ng++;
            }
        };
        for (int r = 0; r < H - 1; r++)
            for (int c = 0; c < W - 1; c++) {
                const int i = r * W + c;
                if (!state[i]) continue;
                grow(i, i + 1);
                grow(i, i + W);
            }
        for (int r = H - 1; r >= 1; r--)
            for (int c = W - 1; c >= 0; c--) {
                const int i = r * W + c;
                if (!state[i]) continue;
                grow(i, i - 1);  // c == 0: previous row's last element (PCL quirk)
                grow(i, i - W);
            }
        S.misc[0] = ng;
        // ---- Frame.cc:912-934: d >= 0, PlaneNotSeen
        int nk = 0;
        for (int m = 0; m < nmodel; m++) {
            float cf[4] = {S.model_coef[m][0], S.model_coef[m][1], S.model_coef[m][2], S.model_coef[m][3]};
            if (cf[3] < 0)
                for (int k = 0; k < 4; k++) cf[k] = -cf[k];
            bool seen = false;
            for (int q = 0; q < nk && !seen; q++) {
                const spslam_plane& pm = planes[q];
                const float d = pm.coef[3] - cf[3];
                const float angle = pm.coef[0] * cf[0] + pm.coef[1] * cf[1] + pm.coef[2] * cf[2];
                if (d > 0.2f || d < -0.2f) continue;
                if (angle < 0.9397f && angle > -0.9397f) continue;
                seen = true;
            }
            if (seen || nk >= planes_cap) continue;
            for (int k = 0; k < 4; k++) planes[nk].coef[k] = cf[k];
            S.kept[nk++] = m;
        }
        S.nkept = nk;
        // inlier lists: component members (raster order) then grown points (growth order)
        int off = 0;
        for (int q = 0; q < nk; q++) {
            const int m = S.kept[q], j = S.model_big[m], n = sizes[S.big_label[j]];
            planes[q].inlier_offset = off;
            planes[q].n_inliers = n;
            off += n;
            for (int k = 0; k < ng; k++)
                if (grown_m[k] == m) off++;
        }
    }
    __syncthreads();
    const int nk = S.nkept, ng = S.misc[0];
    for (int q = 0; q < nk; q++) {
        const int m = S.kept[q], j = S.model_big[m], n = sizes[S.big_label[j]], o = S.big_off[j];
        const int dst = planes[q].inlier_offset;
        for (int k = t; k < n && dst + k < g.inlier_cap; k += kSegThreads) inl[dst + k] = members[o + k];
    }
    if (t == 0) {
        for (int q = 0; q < nk; q++) {
            const int m = S.kept[q];
            int w = planes[q].inlier_offset + planes[q].n_inliers;
            for (int k = 0; k < ng; k++)
                if (grown_m[k] == m && w < g.inlier_cap) inl[w++] = grown[k];
            planes[q].n_inliers = w - planes[q].inlier_offset;
        }
        // ---- contours: findLabeledRegionBoundary from the first inlier, on refined labels
        const int ddx[8] = {-1, -1, 0, 1, 1, 1, 0, -1}, ddy[8] = {0, -1, -1, -1, 0, 1, 1, 1};
        int coff = 0;
        for (int q = 0; q < nk; q++) {
            const int m = S.kept[q], start = members[S.big_off[S.model_big[m]]];
            const uint8_t lab = (uint8_t)(m + 1);
            planes[q].contour_offset = coff;
            int cx = start % W, cy = start / W, dir = -1;
            for (int d = 0; d < 8; ++d) {
                const int x = cx + ddx[d], y = cy + ddy[d];
                if (x >= 0 && x < W && y >= 0 && y < H && state[y * W + x] != lab) { dir = d; break; }
            }
            int n = 0;
            if (dir != -1) {
                if (coff + n < g.contour_cap) con[coff + n] = start;
                n++;
                int cur = start;
                do {
                    int nIdx = 0;
                    for (int d = 1; d <= 8; ++d) {
                        nIdx = (dir + d) & 7;
                        const int x = cx + ddx[nIdx], y = cy + ddy[nIdx];
                        if (x >= 0 && x < W && y >= 0 && y < H && state[y * W + x] == lab) break;
                    }
                    dir = (nIdx + 4) & 7;
                    cx += ddx[nIdx];
                    cy += ddy[nIdx];
                    cur = cy * W + cx;
                    if (coff + n < g.contour_cap) con[coff + n] = cur;
                    n++;
                } while (cur != start && n < 8 * N);
            }
            planes[q].n_contour = min(n, g.contour_cap - coff);
            coff += planes[q].n_contour;
        }
        plane_counts[f] = nk;
    }
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
    hipLaunchKernelGGL(plane_segment_kernel, dim3(n), dim3(kSegThreads), (size_t)((g.N + 15) / 16 * 16), s, g, b,
                       planes, plane_counts, planes_cap, inliers, contours);
    E(kKindPlaneSegment);
    return hipGetLastError();
}

}  // namespace spslam
