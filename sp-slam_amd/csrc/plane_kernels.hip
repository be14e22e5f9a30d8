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

#include <cstdlib>

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

// ---- the same two recurrences with no workgroup barrier (round 6): one wave per 64 cloud rows, lane = row.
// Pass 1 at wave-local step s has lane l at column c = s - 2 l: a lane's up-row operands (the distance at columns
// c - 1 .. c + 1 and the integral entries at c - 1, c) are what lane l - 1 produced 3, 2 and 1 steps earlier, so
// they arrive by DPP (wave_shr:1) into a 3-deep shift register, one hop per step and no barrier.  The first row of
// wave w > 0 takes the last row of wave w - 1 from a small LDS ring instead (the waves overlap: wave w trails wave
// w - 1 by the 128 steps its 64 rows take; per-chunk progress counters bound the ring).  The cloud operands come
// from the depth image: each lane makes its own row's x / y / z a few columns ahead (plane_cloud_kernel's float
// operations), the rows above and below by DPP from the neighbouring lanes, and a wave's two outer neighbour rows
// are made once into LDS before the passes.  Pass 2 runs the mirrored schedule (lane l + 1's values by wave_shl:1,
// wave w + 1's first row through a ring).  Every cell sees exactly the operands of the reference's raster scans,
// as in plane_dist_integral_kernel, so both outputs stay bit-identical.
constexpr int kXR = 32;  // ring columns of a wave boundary
struct WaveXchg {
    float d1[kXR];       // pass 1: the upper wave's last row (distance)
    double i1[kXR][6];   //         and its integral entries
    float d2[kXR];       // pass 2: the lower wave's first row (distance)
    int prod1, cons1, prod2, cons2;
};
__device__ __forceinline__ float from_above(float v) {  // lane l gets lane l - 1's value (wave_shr:1)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float from_below(float v) {  // lane l gets lane l + 1's value (wave_shl:1)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xF, 0xF, false));
}
__device__ __forceinline__ double from_above_d(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int wave_counter(const int* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void wave_publish(int* p, int v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// bounded wait for a counter (the producers always advance; the bound only guards against a hang)
__device__ __forceinline__ void wave_wait(const int* p, int need) {
    for (int spin = 0; spin < (1 << 18) && wave_counter(p) < need; spin++) __builtin_amdgcn_s_sleep(1);
}

template <int NWV>
__global__ __launch_bounds__(64 * NWV) void plane_wave_kernel(PlaneGeom g, const float* __restrict__ depth,
                                                              long long depth_fs, int depth_stride, float* sink,
                                                              long long sink_fs, float* dist, long long dist_fs,
                                                              double* integral, long long integral_fs) {
    constexpr int K = 6;  // steps per chunk (a multiple of the 3-deep shift registers: no register rotation)
    __shared__ WaveXchg X[NWV > 1 ? NWV - 1 : 1];
    extern __shared__ float outer_rows[];  // per wave: the row above it and the row below it, x | y | z [3][W] each
    const int f = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int W = g.W, H = g.H, r = 64 * w + lane, IW = W + 1;
    const bool row_ok = r < H;
    const int ro = min(r, H - 1);
    const float* Z = depth + f * depth_fs;
    auto zof = [&](int rr, int c) { return Z[(long long)(rr * g.ds) * depth_stride + c * g.ds]; };
    auto xof = [&](int c, float z) { return ((float)(c * g.ds) - g.cx) * z / g.fx; };
    auto yof = [&](int rr, float z) { return ((float)(rr * g.ds) - g.cy) * z / g.fy; };
    float* UP = outer_rows + (size_t)w * 6 * W;  // row 64 w - 1
    float* DN = UP + 3 * W;                      // row 64 w + 64
    {
        const int ru = 64 * w - 1, rd = 64 * w + 64;
        for (int c = lane; c < W; c += 64) {
            if (ru >= 0) {
                const float z = zof(ru, c);
                UP[c] = xof(c, z); UP[W + c] = yof(ru, z); UP[2 * W + c] = z;
            }
            if (rd < H) {
                const float z = zof(rd, c);
                DN[c] = xof(c, z); DN[W + c] = yof(rd, z); DN[2 * W + c] = z;
            }
        }
    }
    if (threadIdx.x < NWV - 1) {
        X[threadIdx.x].prod1 = X[threadIdx.x].cons1 = X[threadIdx.x].prod2 = X[threadIdx.x].cons2 = 0;
    }
    double* Iraw = integral + f * integral_fs;
    for (int c = threadIdx.x; c < IW; c += blockDim.x)
        for (int k = 0; k < 6; k++) Iraw[(size_t)c * 6 + k] = 0.0;  // integral row 0
    if (row_ok)
        for (int k = 0; k < 6; k++) Iraw[(size_t)(r + 1) * IW * 6 + k] = 0.0;  // column 0
    double* I = Iraw + (size_t)(ro + 1) * IW * 6 + 6;  // raster integral entry (r + 1, c + 1) at I + 6 c
    double* Idummy = Iraw + (size_t)(H + 1) * IW * 6;  // sink row of the cells outside the cloud
    float* D = dist + f * dist_fs + (size_t)ro * W;
    float* Dsink = sink + f * sink_fs + threadIdx.x;
    __syncthreads();
    const float row0 = row_ok ? dist_init(zof, W, H, r, 0) : 0.f;
    const bool has_up = w > 0, has_dn = w < NWV - 1;
    // ---------------- pass 1
    // this lane's row in a window of the chunk's columns c0 - 2 .. c0 + K + 1 (c0 = s0 - 2 lane): the own row's
    // horizontal operands and, by DPP, the neighbour rows' values at the cell's column (the row above is two
    // columns ahead: its window index j is column c; the row below two behind: its index j + 4)
    float wx[K + 4], wy[K + 4], wz[K + 4], nz[K];
    auto colz = [&](int c) { return zof(ro, min(max(c, 0), W - 1)); };
    auto fill = [&](int i, int c, float z) {
        const int cc = min(max(c, 0), W - 1);
        wz[i] = z; wx[i] = xof(cc, z); wy[i] = yof(ro, z);
    };
    {
        const int c0 = -2 * lane;
#pragma unroll
        for (int i = 0; i < K + 4; i++) fill(i, c0 - 2 + i, colz(c0 - 2 + i));
#pragma unroll
        for (int i = 0; i < K; i++) nz[i] = colz(c0 + K + 2 + i);
    }
    float nd0 = 0.f, nd1 = 0.f, nd2 = 0.f;  // row above: distance at c + 1, c, c - 1
    double na[6], nb[6], nc[6];             // row above: integral at c + 1, c, c - 1
#pragma unroll
    for (int k = 0; k < 6; k++) na[k] = nb[k] = nc[k] = 0.0;
    float left = 0.f, vprev = 0.f;
    double ileft[6], iprev[6];
#pragma unroll
    for (int k = 0; k < 6; k++) ileft[k] = iprev[k] = 0.0;
    const int S1 = (W + 126 + K - 1) / K * K;
    if (has_up) {  // step -1: the first row's register of the upper row's column 0 (its column c - 1 at step 1)
        wave_wait(&X[w - 1].prod1, 1);
        nd0 = lane == 0 ? X[w - 1].d1[0] : 0.f;
#pragma unroll
        for (int k = 0; k < 6; k++) na[k] = lane == 0 ? X[w - 1].i1[0][k] : 0.0;
    }
    for (int s0 = 0; s0 < S1; s0 += K) {
        const int c0 = s0 - 2 * lane;
        // this chunk: the first row reads the upper wave's last row up to column s0 + K; the last row overwrites
        // ring slots of columns s0 - 126 .. s0 - 121, freed once the lower wave has read up to them
        if (has_up) wave_wait(&X[w - 1].prod1, min(s0 + K + 1, W));
        if (has_dn) wave_wait(&X[w].cons1, min(s0 - 126 + K - kXR, W));
        float nzn[K];
#pragma unroll
        for (int i = 0; i < K; i++) nzn[i] = colz(c0 + 2 * K + 2 + i);  // the next chunk's new columns (in flight)
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int c = c0 + j;
            // the row above: its output of the previous step (column c + 1)
            float vin = from_above(vprev);
            double iin[6];
#pragma unroll
            for (int k = 0; k < 6; k++) iin[k] = from_above_d(iprev[k]);
            if (has_up) {
                const int sl = (c + 1) & (kXR - 1);
                const float rv = X[w - 1].d1[sl];
                vin = lane == 0 ? rv : vin;
#pragma unroll
                for (int k = 0; k < 6; k++) {
                    const double ri = X[w - 1].i1[sl][k];
                    iin[k] = lane == 0 ? ri : iin[k];
                }
            }
            nd2 = nd1; nd1 = nd0; nd0 = vin;
#pragma unroll
            for (int k = 0; k < 6; k++) { nc[k] = nb[k]; nb[k] = na[k]; na[k] = iin[k]; }
            // cloud operands of cell (r, c)
            const int cc = min(max(c, 0), W - 1);
            float ux = from_above(wx[j]), uy = from_above(wy[j]), uz = from_above(wz[j]);
            float dx = from_below(wx[j + 4]), dy = from_below(wy[j + 4]), dz = from_below(wz[j + 4]);
            if (lane == 0 && has_up) { ux = UP[cc]; uy = UP[W + cc]; uz = UP[2 * W + cc]; }
            if (lane == 63 && has_dn) { dx = DN[cc]; dy = DN[W + cc]; dz = DN[2 * W + cc]; }
            bool zero = false;
            const float zc = wz[j + 2];
            if (r < H - 1 && c < W - 1) zero = dc_bad(zc, wz[j + 3]) || dc_bad(zc, dz);
            if (r < H - 1 && c >= 1) zero = zero || dc_bad(wz[j + 1], zc);
            if (r >= 1 && c < W - 1) zero = zero || dc_bad(uz, zc);
            const float center = zero ? 0.0f : (float)(W + H);
            float e[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (r >= 1 && r <= H - 2 && c >= 1 && c <= W - 2) {
                e[0] = wx[j + 3] - wx[j + 1]; e[1] = wy[j + 3] - wy[j + 1]; e[2] = wz[j + 3] - wz[j + 1];
                e[3] = dx - ux; e[4] = dy - uy; e[5] = dz - uz;
            }
            // PCL's pass 1 and IntegralImage2D's recurrence (plane_dist_integral_kernel step1)
            const bool ok = row_ok && c >= 0 && c < W, inner = r > 0 && c > 0;
            const float upLeft = nd2 + 1.4f, up = nd1 + 1.0f;
            const float upRight = (c + 1 < W ? nd0 : row0) + 1.4f;
            const float lft = left + 1.0f;
            const float mv = fminf(fminf(upLeft, up), fminf(lft, upRight));
            const float v = inner && mv < center ? mv : center;
            double iv[6];
#pragma unroll
            for (int k = 0; k < 6; k++) {
                const double upI = r > 0 ? nb[k] : 0.0;
                const double upleftI = inner ? nc[k] : 0.0;
                iv[k] = upI + ileft[k] - upleftI;
                iv[k] += (double)e[k];
            }
            if (ok) {
                left = v;
#pragma unroll
                for (int k = 0; k < 6; k++) ileft[k] = iv[k];
            }
            vprev = v;
#pragma unroll
            for (int k = 0; k < 6; k++) iprev[k] = iv[k];
            *(ok ? D + c : Dsink) = v;  // the pass-1 map: pass 2's centre values, read back by this lane
            {
                double2* out = reinterpret_cast<double2*>(ok ? I + c * 6 : Idummy);
                out[0] = make_double2(iv[0], iv[1]);
                out[1] = make_double2(iv[2], iv[3]);
                out[2] = make_double2(iv[4], iv[5]);
            }
            if (has_dn && lane == 63 && ok) {
                const int sl = c & (kXR - 1);
                X[w].d1[sl] = v;
#pragma unroll
                for (int k = 0; k < 6; k++) X[w].i1[sl][k] = iv[k];
            }
        }
        if (has_dn) wave_publish(&X[w].prod1, max(0, min(s0 + K - 126, W)));
        if (has_up) wave_publish(&X[w - 1].cons1, min(s0 + K + 1, W));
        // the window moves on by K columns
#pragma unroll
        for (int i = 0; i < 4; i++) { wx[i] = wx[K + i]; wy[i] = wy[K + i]; wz[i] = wz[K + i]; }
#pragma unroll
        for (int i = 0; i < K; i++) fill(4 + i, c0 + K + 2 + i, nz[i]);
#pragma unroll
        for (int i = 0; i < K; i++) nz[i] = nzn[i];
    }
    const float lastcol = left;  // this row's pass-1 value at column W - 1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the pass-1 map is read back below (same lane)
    // ---------------- pass 2 (bottom-right to top-left): lane l at step s has column c = W - 1 - s + 2 (lb - l)
    const int lb = min(63, H - 1 - 64 * w);
    const int S2 = (W + 2 * lb + K - 1) / K * K;
    auto dval = [&](int c) { return D[min(max(c, 0), W - 1)]; };
    float dcur[K];
#pragma unroll
    for (int j = 0; j < K; j++) dcur[j] = dval(W - 1 - j + 2 * (lb - lane));
    float right = 0.f, vp2 = 0.f;
    float ld0 = 0.f, ld1 = 0.f, ld2 = 0.f;  // row below: distance at c - 1, c, c + 1
    const bool up_ring = w > 0;             // this wave's first row feeds the upper wave's last row
    if (has_dn) {  // step -1: the last row's register of the lower row's column W - 1 (its column c + 1 at step 1)
        wave_wait(&X[w].prod2, 1);
        ld0 = lane == 63 ? X[w].d2[(W - 1) & (kXR - 1)] : 0.f;
    }
    for (int s0 = 0; s0 < S2; s0 += K) {
        const int cA = W - 1 - s0 + 2 * (lb - lane);  // this lane's column at the chunk's first step
        // the last row reads the lower wave's first row down to column W - 2 - (s0 + K - 1) + ...; the first row
        // overwrites ring slots freed once the upper wave has read them
        if (has_dn) wave_wait(&X[w].prod2, min(s0 + K + 1, W));
        if (up_ring) wave_wait(&X[w - 1].cons2, min(s0 + K - 2 * lb - kXR, W));
        float dnx[K];
#pragma unroll
        for (int j = 0; j < K; j++) dnx[j] = dval(cA - K - j);
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int c = cA - j;
            float vin = from_below(vp2);
            if (has_dn) {
                const float rv = X[w].d2[(c - 1) & (kXR - 1)];
                vin = lane == 63 ? rv : vin;
            }
            ld2 = ld1; ld1 = ld0; ld0 = vin;
            const bool ok = row_ok && c >= 0 && c < W, inner = r < H - 1 && c < W - 1;
            const float lowerLeft = (c > 0 ? ld0 : lastcol) + 1.4f;
            const float lower = ld1 + 1.0f;
            const float lowerRight = ld2 + 1.4f;
            const float rgt = right + 1.0f;
            const float mv = fminf(fminf(lowerLeft, lower), fminf(rgt, lowerRight));
            const float center = dcur[j];
            const float v = inner && mv < center ? mv : center;
            if (ok) right = v;
            vp2 = v;
            *(ok ? D + c : Dsink) = v;
            if (up_ring && lane == 0 && ok) X[w - 1].d2[c & (kXR - 1)] = v;
        }
        if (up_ring) wave_publish(&X[w - 1].prod2, max(0, min(s0 + K - 2 * lb, W)));
        if (has_dn) wave_publish(&X[w].cons2, min(s0 + K + 1, W));
#pragma unroll
        for (int j = 0; j < K; j++) dcur[j] = dnx[j];
    }
}

// ---- the same wavefronts split by output (round 6): three workgroups per frame, each on its own CU, each running
// plane_wave_kernel's schedule for one third of its work -- ROLE 0 the distance map (both passes; it needs only the
// depth: no x / y, no divisions), ROLE 1 the integral images of the horizontal differences (channels 0..2, the own
// row's x / y / z at c - 1, c + 1), ROLE 2 those of the vertical differences (channels 3..5, the rows above and below
// by DPP).  A single wave per 64 rows is bound by its instruction issue (~170 instructions per cell step in
// plane_wave_kernel); split three ways the longest role issues ~70, and the roles run side by side.  Same operands,
// same operations per output: bit-identical to plane_wave_kernel.
template <int NWV, int ROLE>
__device__ __forceinline__ void plane_wave_role(const PlaneGeom& g, const float* __restrict__ depth, long long depth_fs,
                                                int depth_stride, float* sink, long long sink_fs, float* dist,
                                                long long dist_fs, double* integral, long long integral_fs,
                                                WaveXchg* X, float* outer_rows) {
    constexpr int K = 6;
    constexpr bool kDist = ROLE == 0, kXY = ROLE != 0;
    constexpr int k0 = ROLE == 2 ? 3 : 0;  // the role's first integral channel
    const int f = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int W = g.W, H = g.H, r = 64 * w + lane, IW = W + 1;
    const bool row_ok = r < H;
    const int ro = min(r, H - 1);
    const float* Z = depth + f * depth_fs;
    auto zof = [&](int rr, int c) { return Z[(long long)(rr * g.ds) * depth_stride + c * g.ds]; };
    auto xof = [&](int c, float z) { return ((float)(c * g.ds) - g.cx) * z / g.fx; };
    auto yof = [&](int rr, float z) { return ((float)(rr * g.ds) - g.cy) * z / g.fy; };
    float* UP = outer_rows + (size_t)w * 6 * W;  // row 64 w - 1: x | y | z (ROLE 0: z only)
    float* DN = UP + 3 * W;                      // row 64 w + 64
    {
        const int ru = 64 * w - 1, rd = 64 * w + 64;
        for (int c = lane; c < W; c += 64) {
            if (ru >= 0) {
                const float z = zof(ru, c);
                if constexpr (kXY) { UP[c] = xof(c, z); UP[W + c] = yof(ru, z); }
                UP[2 * W + c] = z;
            }
            if (rd < H) {
                const float z = zof(rd, c);
                if constexpr (kXY) { DN[c] = xof(c, z); DN[W + c] = yof(rd, z); }
                DN[2 * W + c] = z;
            }
        }
    }
    if (threadIdx.x < NWV - 1) {
        X[threadIdx.x].prod1 = X[threadIdx.x].cons1 = X[threadIdx.x].prod2 = X[threadIdx.x].cons2 = 0;
    }
    double* Iraw = integral + f * integral_fs;
    if constexpr (!kDist) {
        for (int c = threadIdx.x; c < IW; c += blockDim.x)
            for (int k = 0; k < 3; k++) Iraw[(size_t)c * 6 + k0 + k] = 0.0;  // integral row 0
        if (row_ok)
            for (int k = 0; k < 3; k++) Iraw[(size_t)(r + 1) * IW * 6 + k0 + k] = 0.0;  // column 0
    }
    double* I = Iraw + (size_t)(ro + 1) * IW * 6 + 6 + k0;  // raster integral entry (r + 1, c + 1), the role's channels
    double* Idummy = Iraw + (size_t)(H + 1) * IW * 6 + k0;   // sink row of the cells outside the cloud
    float* D = dist + f * dist_fs + (size_t)ro * W;
    float* Dsink = sink + f * sink_fs + threadIdx.x;
    __syncthreads();
    const bool has_up = w > 0, has_dn = w < NWV - 1;
    // ---------------- pass 1 (plane_wave_kernel's schedule; each role keeps the state of its own outputs)
    float wx[K + 4], wy[K + 4], wz[K + 4], nz[K];
    auto colz = [&](int c) { return zof(ro, min(max(c, 0), W - 1)); };
    auto fill = [&](int i, int c, float z) {
        wz[i] = z;
        if constexpr (kXY) {
            const int cc = min(max(c, 0), W - 1);
            wx[i] = xof(cc, z); wy[i] = yof(ro, z);
        }
    };
    {
        const int c0 = -2 * lane;
#pragma unroll
        for (int i = 0; i < K + 4; i++) fill(i, c0 - 2 + i, colz(c0 - 2 + i));
#pragma unroll
        for (int i = 0; i < K; i++) nz[i] = colz(c0 + K + 2 + i);
    }
    const float row0 = kDist && row_ok ? dist_init(zof, W, H, r, 0) : 0.f;
    float nd0 = 0.f, nd1 = 0.f, nd2 = 0.f;  // ROLE 0, the row above: distance at c + 1, c, c - 1
    double na[3], nb[3], nc[3];             // ROLES 1, 2, the row above: integral at c + 1, c, c - 1
#pragma unroll
    for (int k = 0; k < 3; k++) na[k] = nb[k] = nc[k] = 0.0;
    float left = 0.f, vprev = 0.f;
    double ileft[3], iprev[3];
#pragma unroll
    for (int k = 0; k < 3; k++) ileft[k] = iprev[k] = 0.0;
    const int S1 = (W + 126 + K - 1) / K * K;
    if (has_up) {  // step -1: the first row's register of the upper row's column 0
        wave_wait(&X[w - 1].prod1, 1);
        if constexpr (kDist) {
            nd0 = lane == 0 ? X[w - 1].d1[0] : 0.f;
        } else {
#pragma unroll
            for (int k = 0; k < 3; k++) na[k] = lane == 0 ? X[w - 1].i1[0][k] : 0.0;
        }
    }
    for (int s0 = 0; s0 < S1; s0 += K) {
        const int c0 = s0 - 2 * lane;
        if (has_up) wave_wait(&X[w - 1].prod1, min(s0 + K + 1, W));
        if (has_dn) wave_wait(&X[w].cons1, min(s0 - 126 + K - kXR, W));
        float nzn[K];
#pragma unroll
        for (int i = 0; i < K; i++) nzn[i] = colz(c0 + 2 * K + 2 + i);
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int c = c0 + j;
            const int sl = (c + 1) & (kXR - 1);
            const bool ok = row_ok && c >= 0 && c < W, inner = r > 0 && c > 0;
            const int cc = min(max(c, 0), W - 1);
            if constexpr (kDist) {
                float vin = from_above(vprev);
                if (has_up) {
                    const float rv = X[w - 1].d1[sl];
                    vin = lane == 0 ? rv : vin;
                }
                nd2 = nd1; nd1 = nd0; nd0 = vin;
                float uz = from_above(wz[j]), dz = from_below(wz[j + 4]);
                if (lane == 0 && has_up) uz = UP[2 * W + cc];
                if (lane == 63 && has_dn) dz = DN[2 * W + cc];
                bool zero = false;
                const float zc = wz[j + 2];
                if (r < H - 1 && c < W - 1) zero = dc_bad(zc, wz[j + 3]) || dc_bad(zc, dz);
                if (r < H - 1 && c >= 1) zero = zero || dc_bad(wz[j + 1], zc);
                if (r >= 1 && c < W - 1) zero = zero || dc_bad(uz, zc);
                const float center = zero ? 0.0f : (float)(W + H);
                const float upLeft = nd2 + 1.4f, up = nd1 + 1.0f;
                const float upRight = (c + 1 < W ? nd0 : row0) + 1.4f;
                const float lft = left + 1.0f;
                const float mv = fminf(fminf(upLeft, up), fminf(lft, upRight));
                const float v = inner && mv < center ? mv : center;
                if (ok) left = v;
                vprev = v;
                *(ok ? D + c : Dsink) = v;
                if (has_dn && lane == 63 && ok) X[w].d1[c & (kXR - 1)] = v;
            } else {
                double iin[3];
#pragma unroll
                for (int k = 0; k < 3; k++) iin[k] = from_above_d(iprev[k]);
                if (has_up) {
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const double ri = X[w - 1].i1[sl][k];
                        iin[k] = lane == 0 ? ri : iin[k];
                    }
                }
#pragma unroll
                for (int k = 0; k < 3; k++) { nc[k] = nb[k]; nb[k] = na[k]; na[k] = iin[k]; }
                float e[3] = {0.f, 0.f, 0.f};
                if constexpr (ROLE == 1) {
                    if (r >= 1 && r <= H - 2 && c >= 1 && c <= W - 2) {
                        e[0] = wx[j + 3] - wx[j + 1]; e[1] = wy[j + 3] - wy[j + 1]; e[2] = wz[j + 3] - wz[j + 1];
                    }
                } else {
                    float ux = from_above(wx[j]), uy = from_above(wy[j]), uz = from_above(wz[j]);
                    float dx = from_below(wx[j + 4]), dy = from_below(wy[j + 4]), dz = from_below(wz[j + 4]);
                    if (lane == 0 && has_up) { ux = UP[cc]; uy = UP[W + cc]; uz = UP[2 * W + cc]; }
                    if (lane == 63 && has_dn) { dx = DN[cc]; dy = DN[W + cc]; dz = DN[2 * W + cc]; }
                    if (r >= 1 && r <= H - 2 && c >= 1 && c <= W - 2) {
                        e[0] = dx - ux; e[1] = dy - uy; e[2] = dz - uz;
                    }
                }
                double iv[3];
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const double upI = r > 0 ? nb[k] : 0.0;
                    const double upleftI = inner ? nc[k] : 0.0;
                    iv[k] = upI + ileft[k] - upleftI;
                    iv[k] += (double)e[k];
                }
                if (ok) {
#pragma unroll
                    for (int k = 0; k < 3; k++) ileft[k] = iv[k];
                }
#pragma unroll
                for (int k = 0; k < 3; k++) iprev[k] = iv[k];
                {
                    double* out = ok ? I + c * 6 : Idummy;
                    if constexpr (ROLE == 1) {
                        *reinterpret_cast<double2*>(out) = make_double2(iv[0], iv[1]);
                        out[2] = iv[2];
                    } else {  // (channel 3 at byte 24 of the 48-byte entry: a double, then a 16-byte pair)
                        out[0] = iv[0];
                        *reinterpret_cast<double2*>(out + 1) = make_double2(iv[1], iv[2]);
                    }
                }
                if (has_dn && lane == 63 && ok) {
                    const int so = c & (kXR - 1);
#pragma unroll
                    for (int k = 0; k < 3; k++) X[w].i1[so][k] = iv[k];
                }
            }
        }
        if (has_dn) wave_publish(&X[w].prod1, max(0, min(s0 + K - 126, W)));
        if (has_up) wave_publish(&X[w - 1].cons1, min(s0 + K + 1, W));
#pragma unroll
        for (int i = 0; i < 4; i++) {
            wz[i] = wz[K + i];
            if constexpr (kXY) { wx[i] = wx[K + i]; wy[i] = wy[K + i]; }
        }
#pragma unroll
        for (int i = 0; i < K; i++) fill(4 + i, c0 + K + 2 + i, nz[i]);
#pragma unroll
        for (int i = 0; i < K; i++) nz[i] = nzn[i];
    }
    if constexpr (!kDist) return;
    // ---------------- pass 2 (ROLE 0): plane_wave_kernel's
    const float lastcol = left;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int lb = min(63, H - 1 - 64 * w);
    const int S2 = (W + 2 * lb + K - 1) / K * K;
    auto dval = [&](int c) { return D[min(max(c, 0), W - 1)]; };
    float dcur[K];
#pragma unroll
    for (int j = 0; j < K; j++) dcur[j] = dval(W - 1 - j + 2 * (lb - lane));
    float right = 0.f, vp2 = 0.f;
    float ld0 = 0.f, ld1 = 0.f, ld2 = 0.f;
    const bool up_ring = w > 0;
    if (has_dn) {
        wave_wait(&X[w].prod2, 1);
        ld0 = lane == 63 ? X[w].d2[(W - 1) & (kXR - 1)] : 0.f;
    }
    for (int s0 = 0; s0 < S2; s0 += K) {
        const int cA = W - 1 - s0 + 2 * (lb - lane);
        if (has_dn) wave_wait(&X[w].prod2, min(s0 + K + 1, W));
        if (up_ring) wave_wait(&X[w - 1].cons2, min(s0 + K - 2 * lb - kXR, W));
        float dnx[K];
#pragma unroll
        for (int j = 0; j < K; j++) dnx[j] = dval(cA - K - j);
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int c = cA - j;
            float vin = from_below(vp2);
            if (has_dn) {
                const float rv = X[w].d2[(c - 1) & (kXR - 1)];
                vin = lane == 63 ? rv : vin;
            }
            ld2 = ld1; ld1 = ld0; ld0 = vin;
            const bool ok = row_ok && c >= 0 && c < W, inner = r < H - 1 && c < W - 1;
            const float lowerLeft = (c > 0 ? ld0 : lastcol) + 1.4f;
            const float lower = ld1 + 1.0f;
            const float lowerRight = ld2 + 1.4f;
            const float rgt = right + 1.0f;
            const float mv = fminf(fminf(lowerLeft, lower), fminf(rgt, lowerRight));
            const float center = dcur[j];
            const float v = inner && mv < center ? mv : center;
            if (ok) right = v;
            vp2 = v;
            *(ok ? D + c : Dsink) = v;
            if (up_ring && lane == 0 && ok) X[w - 1].d2[c & (kXR - 1)] = v;
        }
        if (up_ring) wave_publish(&X[w - 1].prod2, max(0, min(s0 + K - 2 * lb, W)));
        if (has_dn) wave_publish(&X[w].cons2, min(s0 + K + 1, W));
#pragma unroll
        for (int j = 0; j < K; j++) dcur[j] = dnx[j];
    }
}
template <int NWV>
__global__ __launch_bounds__(64 * NWV) void plane_wave_roles_kernel(PlaneGeom g, const float* __restrict__ depth,
                                                                    long long depth_fs, int depth_stride, float* sink,
                                                                    long long sink_fs, float* dist, long long dist_fs,
                                                                    double* integral, long long integral_fs) {
    __shared__ WaveXchg X[NWV > 1 ? NWV - 1 : 1];
    extern __shared__ float outer_rows[];
    // (the sink: one slot per (role, thread), so the roles' stores of cells outside the cloud do not meet)
    float* snk = sink + (size_t)blockIdx.y * 64 * NWV;
    switch (blockIdx.y) {
        case 0: plane_wave_role<NWV, 0>(g, depth, depth_fs, depth_stride, snk, sink_fs, dist, dist_fs, integral,
                                        integral_fs, X, outer_rows); break;
        case 1: plane_wave_role<NWV, 1>(g, depth, depth_fs, depth_stride, snk, sink_fs, dist, dist_fs, integral,
                                        integral_fs, X, outer_rows); break;
        default: plane_wave_role<NWV, 2>(g, depth, depth_fs, depth_stride, snk, sink_fs, dist, dist_fs, integral,
                                         integral_fs, X, outer_rows); break;
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
                        int32_t* contours, hipStream_t s, KernelTimer* timer, bool have_cloud) {
    if (g.H > kWaveThreads) return hipErrorInvalidValue;
    auto B = [&](int k) { if (timer) timer->begin(k, s); };
    auto E = [&](int k) { if (timer) timer->end(k, s); };
    const dim3 pts((g.N + 255) / 256, n);
    if (!have_cloud) {  // (else a fused grab made it: grab_kernels.hip)
        B(kKindPlaneCloud);
        hipLaunchKernelGGL(plane_cloud_kernel, pts, dim3(256), 0, s, g, depth, depth_fs, depth_stride, b.cloud,
                           b.cloud_fs);
        E(kKindPlaneCloud);
    }
    B(kKindPlaneDist);
    static const bool barrier_wave = [] {
        const char* e = getenv("SPSLAM_PLANE_WAVE_BARRIER");
        return e && e[0] == '1';
    }();
    // three workgroups per frame, one per output group (plane_wave_roles_kernel), for small batches: B = 1 serial
    // latency 3.72 -> 3.44 ms p50; one per frame (plane_wave_kernel) for large ones, where the roles' extra
    // workgroups and operand fetches cost the C2 step 3 % (profiles/r06/ab_plane_wave_roles.txt).
    // SPSLAM_PLANE_WAVE=1 / 3 forces one / three.
    static const int wave_groups = [] {
        const char* e = getenv("SPSLAM_PLANE_WAVE");
        return e ? atoi(e) : 0;
    }();
    const bool one_wave_group = wave_groups == 1 || (wave_groups != 3 && n > 16);
    if (!barrier_wave && !one_wave_group) {
        const int nw = (g.H + 63) / 64;
        const size_t lds = (size_t)nw * 6 * g.W * sizeof(float);
        auto* k = nw <= 1 ? plane_wave_roles_kernel<1> : nw <= 2 ? plane_wave_roles_kernel<2>
                : nw <= 3 ? plane_wave_roles_kernel<3> : nw <= 4 ? plane_wave_roles_kernel<4>
                : nw <= 5 ? plane_wave_roles_kernel<5> : nw <= 6 ? plane_wave_roles_kernel<6>
                : nw <= 7 ? plane_wave_roles_kernel<7> : plane_wave_roles_kernel<8>;
        hipLaunchKernelGGL(k, dim3(n, 3), dim3(64 * nw), lds, s, g, depth, depth_fs, depth_stride, b.wave, b.wave_fs,
                           b.dist, b.dist_fs, b.integral, b.integral_fs);
    } else if (!barrier_wave) {
        const int nw = (g.H + 63) / 64;
        const size_t lds = (size_t)nw * 6 * g.W * sizeof(float);
        auto* k = nw <= 1 ? plane_wave_kernel<1> : nw <= 2 ? plane_wave_kernel<2> : nw <= 3 ? plane_wave_kernel<3>
                : nw <= 4 ? plane_wave_kernel<4> : nw <= 5 ? plane_wave_kernel<5> : nw <= 6 ? plane_wave_kernel<6>
                : nw <= 7 ? plane_wave_kernel<7> : plane_wave_kernel<8>;
        hipLaunchKernelGGL(k, dim3(n), dim3(64 * nw), lds, s, g, depth, depth_fs, depth_stride, b.wave, b.wave_fs,
                           b.dist, b.dist_fs, b.integral, b.integral_fs);
    } else {
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
