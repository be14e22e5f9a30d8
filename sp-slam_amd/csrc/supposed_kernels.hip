// Supposed planes from plane boundaries on gfx950:
// Frame::GeneratePlanesFromBoundries (src/Frame.cc:938-998) with its helpers
// IsBorderLine / IsBorderPoint / LineInRange / CaculatePlanes / PlaneNotSeen
// (:1013-1144) and the PCL 1.8.0 SACSegmentation LINE + RANSAC + optimize it
// calls (semantics: oracle/supposed_oracle.cpp).
//
// supp_lines_kernel: one 256-thread workgroup per (frame, boundary).  The
// boundary's points live in LDS (float4, w = organized-cloud index).  Each
// segment() call restarts boost::mt19937(12345), so its draws are a fixed
// sequence, precomputed once per context (kSuppRndTable entries cover the
// worst case).  RANSAC is run speculatively in rounds of kBatch trials:
//   - wave 0 replays the sampler (drawIndexSample's partial Fisher-Yates on
//     the persistent shuffled_indices_, isSampleGood retries); the 64 lanes
//     fetch and reduce 32 draw pairs at a time and the uniform swap chain
//     applies them (the swaps are the same whichever pairs isSampleGood
//     rejects), then the 32 pairs' isSampleGood tests run in parallel and
//     the good ones become trials in order;
//   - all waves count each trial's inliers (wave per trial, lanes over points);
//   - one lane replays computeModel's best/k bookkeeping in trial order and
//     stops exactly where the reference loop stops; trials sampled beyond that
//     point are discarded (the RNG is discarded by the reference too).
// Then selectWithinDistance, optimizeModelCoefficients (sequential float
// centroid / covariance sums, one lane per accumulator, glibc-exact eigen
// solve), the Line.Ratio test, LineInRange, IsBorderLine (thread per line
// point) and the order-preserving removal of the line's points.
//
// supp_assemble_kernel: one wave per frame; boundaries last to first, the
// fitted lines in order: CaculatePlanes + PlaneNotSeen against the growing
// plane list (serial, as in the reference), then the synthetic patches and
// line point lists are written by all lanes.
#include <cfloat>

#include "libm_restated.h"
#include "plane_not_seen.h"
#include "supposed_launch.h"

namespace spslam {
namespace supp {

constexpr int kThreads = 256, kWaves = 4;  // the batched launch (one workgroup per boundary)
constexpr int kMaxWaves = 8;                // small batches: 512 threads (supp_launch)
constexpr int kBatch = 64;       // RANSAC trials per speculative round
constexpr int kLdsPts = 2048;    // boundaries up to this size are held in LDS
constexpr int kMaxTrials = 1001; // RandomSampleConsensus: ++iterations_ > max_iterations_ (1000) -> stop

#ifdef SPSLAM_SUPP_PROF  // diagnostic build: per-boundary phase clocks (100 MHz ticks) in sb.prof
#define SUPP_CLK() ((long long)__builtin_amdgcn_s_memrealtime())
#define SUPP_T(k) do { if (t == 0) { const long long c_ = SUPP_CLK(); pr[k] += c_ - pt; pt = c_; } } while (0)
#else
#define SUPP_T(k) do { } while (0)
#endif

struct Shared {
    int s0[kBatch], s1[kBatch], cnt[kBatch];
    int nb, fail, done, have;
    int iterations, best, best_s0, best_s1;
    double k;
    float line[6];
    float acc[9];
    int red[kMaxWaves];
    int n_inl, flags;
    int s0x[kBatch], s1x[kBatch], nbb[2], failb[2];  // kOverlap: the second sample buffer, both buffers' counts
};

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
template <int NT>
__device__ int block_sum(int v, Shared& S) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) S.red[wave] = v;
    __syncthreads();
    int s = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) s += S.red[w];
    return s;
}

// computeModelCoefficients + tail<3>().normalize() (3-element, unvectorised).
__device__ __forceinline__ void line_from_samples(const float4 a, const float4 b, float* c) {
    c[0] = a.x; c[1] = a.y; c[2] = a.z;
    float d0 = b.x - a.x, d1 = b.y - a.y, d2 = b.z - a.z;
    const float sq = d0 * d0 + d1 * d1 + d2 * d2;
    if (sq > 0.f) {
        const float s = sqrtf(sq);
        d0 /= s; d1 /= s; d2 /= s;
    }
    c[3] = d0; c[4] = d1; c[5] = d2;
}
// Vector4f line_dir.normalize() (SSE lane order, w = 0).
__device__ __forceinline__ void normalize4(float* d) {
    const float sq = (d[0] * d[0] + d[2] * d[2]) + (d[1] * d[1] + 0.f);
    if (sq > 0.f) {
        const float s = sqrtf(sq);
        d[0] /= s; d[1] /= s; d[2] /= s;
    }
}
// ((line_pt - p).cross3(line_dir)).squaredNorm() in Eigen's SSE order.
__device__ __forceinline__ float line_sqd(const float* lp, const float* ld, const float4 p) {
    const float ax = lp[0] - p.x, ay = lp[1] - p.y, az = lp[2] - p.z;
    const float cx = ay * ld[2] - az * ld[1];
    const float cy = az * ld[0] - ax * ld[2];
    const float cz = ax * ld[1] - ay * ld[0];
    return (cx * cx + cz * cz) + (cy * cy + 0.f);
}

// pcl::computeRoots on a scaled matrix (float), glibc-exact transcendental calls.
__device__ void roots2(float b, float c, float* r) {
    r[0] = 0.f;
    float d = (float)(b * b - 4.0 * c);
    if (d < 0.0) d = 0.0;
    const float sd = sqrtf(d);
    r[2] = 0.5f * (b + sd);
    r[1] = 0.5f * (b - sd);
}
__device__ void roots3(const float (&m)[3][3], float* r) {
    const float c0 = m[0][0] * m[1][1] * m[2][2] + 2.f * m[0][1] * m[0][2] * m[1][2] - m[0][0] * m[1][2] * m[1][2] -
                     m[1][1] * m[0][2] * m[0][2] - m[2][2] * m[0][1] * m[0][1];
    const float c1 = m[0][0] * m[1][1] - m[0][1] * m[0][1] + m[0][0] * m[2][2] - m[0][2] * m[0][2] +
                     m[1][1] * m[2][2] - m[1][2] * m[1][2];
    const float c2 = m[0][0] + m[1][1] + m[2][2];
    if (fabsf(c0) < FLT_EPSILON) { roots2(c2, c1, r); return; }
    const float s_inv3 = (float)(1.0 / 3.0), s_sqrt3 = sqrtf(3.0f);
    const float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > 0.f) a_over_3 = 0.f;
    const float half_b = 0.5f * (c0 + c2_over_3 * (2.f * c2_over_3 * c2_over_3 - c1));
    float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
    if (q > 0.f) q = 0.f;
    const float rho = sqrtf(-a_over_3);
    const float theta = libm::atan2f_(sqrtf(-q), half_b) * s_inv3;
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
__device__ float max_abs3(const float (&m)[3][3]) {
    float s = 0.f;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) s = fmaxf(s, fabsf(m[i][j]));
    if (s <= FLT_MIN) s = 1.f;
    return s;
}
// pcl::eigen33(cov, evals) + computeCorrespondingEigenVector(cov, evals[2]).
__device__ void line_direction(const float (&cov)[3][3], float* evec) {
    const float scale = max_abs3(cov);
    float s[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) s[i][j] = cov[i][j] / scale;
    float r[3];
    roots3(s, r);
    const float eval2 = r[2] * scale;
    const float scale2 = max_abs3(cov);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) s[i][j] = cov[i][j] / scale2;
    const float sub = eval2 / scale2;
    for (int i = 0; i < 3; i++) s[i][i] -= sub;
    const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    float v[3][3], len[3];
    for (int k = 0; k < 3; k++) {
        const float* a = s[pr[k][0]];
        const float* b = s[pr[k][1]];
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

struct Cam { float fx, fy, cx, cy, min_x, max_x, min_y, max_y; int w, h, stride; };

// Frame::IsBorderPoint (Frame.cc:1027-1057); window read through the flat
// row-major index of the (continuous) depth image, reads outside the image
// buffer count as invalid (<= 0.05) pixels -- see oracle/supposed_oracle.cpp.
__device__ bool is_border_point(const float4 p, const float* __restrict__ depth, const Cam& K) {
    if (p.z < 0.0f) return false;
    const float invz = 1.0f / p.z;
    const float u = fmaf(K.fx * p.x, invz, K.cx);
    const float v = fmaf(K.fy * p.y, invz, K.cy);
    if (isnan(u) || isnan(v)) return true;
    if (!(fabsf(u) < 1e6f) || !(fabsf(v) < 1e6f)) return false;
    // element offset of window pixel (i, j), or -1 when the reference reads nothing there; 32-bit is exact
    // here (|u|, |v| < 1e6 and w <= 2048 keep j * w + i inside int)
    const int total = K.w * K.h;
    auto offset = [&](int i, int j) -> int {
        if ((unsigned)i < (unsigned)K.w && (unsigned)j < (unsigned)K.h) return j * K.stride + i;
        const int fi = j * K.w + i;
        return (fi >= 0 && fi < total) ? (fi / K.w) * K.stride + fi % K.w : -1;
    };
    int num = 0, nan = 0;
    float res = 0.f;
    // A window row is at most 21 pixels wide (|u| < 1e6: float spacing <= 1/16): its depths are loaded
    // together (unconditional loads from a clamped offset, masked afterwards), then consumed in the
    // reference's order with its early exit; any pixels beyond the batch are read one by one.
    constexpr int kRow = 22;
    const int i0 = (int)(u - 10.f);
    for (int j = (int)(v - 10.f); (float)j < v + 10.f; ++j) {
        float dv[kRow];
#pragma unroll
        for (int k = 0; k < kRow; k++) {
            const int o = offset(i0 + k, j);
            const float x = depth[o < 0 ? 0 : o];
            dv[k] = o < 0 ? 0.f : x;
        }
        int i = i0;
#pragma unroll
        for (int k = 0; k < kRow; k++, ++i) {
            if (!((float)i < u + 10.f)) break;
            const float d = dv[k];
            if ((double)d > 0.05) {
                res += d;
                num++;
            } else if (++nan > 100) {
                return false;
            }
        }
        for (; (float)i < u + 10.f; ++i) {
            const int o = offset(i, j);
            const float d = o < 0 ? 0.f : depth[o];
            if ((double)d > 0.05) {
                res += d;
                num++;
            } else if (++nan > 100) {
                return false;
            }
        }
    }
    if ((double)(p.z - res / (float)num) > 0.1) return false;
    return true;
}

// Frame::LineInRange (Frame.cc:1059-1076).
__device__ bool line_in_range(const float* pc, const Cam& K) {
    if (pc[2] < 0.0f) return false;
    const float invz = 1.0f / pc[2];
    const float u = fmaf(K.fx * pc[0], invz, K.cx);
    const float v = fmaf(K.fy * pc[1], invz, K.cy);
    if (u < K.min_x + 50 || u > K.max_x - 50) return false;
    if (v < K.min_y + 50 || v > K.max_y - 50) return false;
    return true;
}

// selectWithinDistance(coef): flag[i] for the n current points; returns the count.
template <int NT>
__device__ int select_within(const float* coef, const float4* Q, uint8_t* flag, int n, float thr, Shared& S) {
    float lp[3] = {coef[0], coef[1], coef[2]}, ld[3] = {coef[3], coef[4], coef[5]};
    normalize4(ld);
    int c = 0;
    for (int i = threadIdx.x; i < n; i += NT) {
        const bool in = line_sqd(lp, ld, Q[i]) <= thr;
        flag[i] = in;
        c += in;
    }
    return block_sum<NT>(c, S);
}

// 3 waves per SIMD: 168 VGPRs instead of 172, so the LDS (43.9 KB) and not the registers bounds residency at
// 3 workgroups per CU instead of 2 (1.35 -> 0.95 ms per 256 frames alone; profiles/r02/ab_contour_single_walk)
#ifndef SPSLAM_SUPP_OVERLAP
#define SPSLAM_SUPP_OVERLAP 1
#endif
#ifndef SPSLAM_SUPP_OVERLAP_ALL  // measurement knob: the overlap in the 256-thread (batched) instance too
#define SPSLAM_SUPP_OVERLAP_ALL 0
#endif
#ifndef SPSLAM_SUPP_MINB
#define SPSLAM_SUPP_MINB 3
#endif
// NT threads: 256 for batches (SPSLAM_SUPP_MINB workgroups per CU), 512 for a few frames (the inlier counts and the
// point loops over twice the lanes; the sampler chain is wave 0's either way)
template <int NT>
__global__ __launch_bounds__(NT, NT == 256 ? SPSLAM_SUPP_MINB : 1) void supp_lines_kernel(PlaneGeom g, PlaneBuffers pb, SuppParams sp,
                                                              SuppBuffers sb, const float* __restrict__ depth,
                                                              long long depth_fs, int depth_stride,
                                                              const spslam_plane* __restrict__ planes,
                                                              const int* __restrict__ plane_counts,
                                                              const int32_t* __restrict__ contours) {
    __shared__ float4 Qs[kLdsPts];
    __shared__ int shs[kLdsPts];
    __shared__ uint8_t flags_s[kLdsPts];
#ifdef SPSLAM_MEASURE_SKIP_SUPP  // measurement variant only (marginal step cost): no RANSAC work
    if (g.W > 0) return;
#endif
    __shared__ Shared S;
    // 512-thread instance (a few frames): the next RANSAC round is sampled while the other waves count this one's
    // inliers (SPSLAM_SUPP_OVERLAP=0 turns it off)
    constexpr bool kOverlap = SPSLAM_SUPP_OVERLAP && (NT == 512 || SPSLAM_SUPP_OVERLAP_ALL);
    const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int np = min(plane_counts[f], kMaxPlanesPerFrame);
    const spslam_plane* P = planes + (size_t)f * kMaxPlanesPerFrame;
    const int32_t* con = contours + (size_t)f * g.contour_cap;
    const float* X = pb.cloud + f * pb.cloud_fs;
    const float* Y = X + g.N;
    const float* Z = X + 2 * g.N;
    const Cam K{g.fx, g.fy, g.cx, g.cy, sp.min_x, sp.max_x, sp.min_y, sp.max_y, g.w, g.h, depth_stride};
    const float* D = depth + f * depth_fs;
    const float thr = sp.sqr_th_f;
    for (int q = blockIdx.y; q < np; q += gridDim.y) {
        LineCand* C = sb.cand + ((size_t)f * kMaxPlanesPerFrame + q) * kMaxLinesPerBoundary;
        const int bsize = P[q].n_contour, coff = P[q].contour_offset;
        if (bsize < 50) {  // Frame.cc:951-955 (the 0-point case only fills mvBoundaryPoints)
            if (t == 0) sb.n_cand[f * kMaxPlanesPerFrame + q] = 0;
            continue;
        }
        const bool in_lds = bsize <= kLdsPts;
        int32_t* lidx = sb.line_idx + (size_t)f * g.contour_cap + coff;
        // The boundary's points, shuffle state and flags live in LDS (or, for big boundaries, in HBM
        // scratch): the body is instantiated once per case, so the LDS case compiles to ds_* accesses
        // (one pointer selected at run time would make every access a flat one, waited on by both the
        // vector-memory and the LDS counters).
        auto boundary = [&](float4* Q, int* sh, uint8_t* flag) __attribute__((always_inline)) -> int {
#ifdef SPSLAM_SUPP_PROF
        long long pr[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt = SUPP_CLK();
#endif
        for (int i = t; i < bsize; i += NT) {
            const int ci = con[coff + i];
            Q[i] = make_float4(X[ci], Y[ci], Z[ci], __int_as_float(ci));
        }
        __syncthreads();
        SUPP_T(0);
        int n = bsize, used = 0, ncand = 0;
        for (int j = 0; j < kMaxLinesPerBoundary; j++) {
            // ---------------- RandomSampleConsensus::computeModel
            if (t == 0) {
                S.iterations = 0; S.best = -2147483647; S.k = 1.0; S.have = 0; S.done = n < 2;
            }
            if constexpr (kOverlap) {
                if (t < kBatch) S.cnt[t] = 0;
            }
            for (int i = t; i < n; i += NT) sh[i] = i;
            __syncthreads();
            const double one_over_n = 1.0 / (double)n, log_prob = log(1.0 - 0.99);
            int r0 = 0, r1 = 1;   // shuffled_indices_[0], [1] (kept in registers by wave 0)
            uint32_t pos = 0;     // draws applied to the shuffle state
            // Draw pairs already applied, not yet consumed by a trial: pair qh..qn-1 of the last block of 32,
            // lane c holding pair c's sample (bp0, bp1); gmask = its isSampleGood bits.
            int bp0 = 0, bp1 = 0, qh = 0, qn = 0;
            uint64_t gmask = 0;
            uint32_t rnext = wave == 0 ? sb.rnd[lane] : 0u;  // next block's draws, loaded one block ahead
            if constexpr (!kOverlap) {
                while (!S.done) {
                    if (wave == 0) {
                        const int it0 = S.iterations;
                        int nb = 0, chk = 0;  // chk: failed samples of the trial being drawn
                        bool fail = false;
                        while (nb < kBatch && it0 + nb < kMaxTrials) {
                            if (qh == qn) {
                                // apply the next 32 draw pairs to the shuffle state: their swaps do not depend on
                                // whether a pair becomes a trial's sample, so isSampleGood is checked afterwards,
                                // for all 32 pairs at once (the chain keeps one LDS round trip per pair)
                                const uint32_t r = rnext;
                                const uint32_t jv = (lane & 1) ? 1u + r % (uint32_t)(n - 1) : r % (uint32_t)n;
                                pos += 64;
                                rnext = sb.rnd[pos + lane];  // (the table holds one block beyond the worst case)
                                // Branch-free: entries 0 and 1 live in r0 / r1 (their LDS slots are never read), so
                                // a swap that does not touch LDS reads and writes slot 0 (first swap) or 1 (second)
                                // as a sink; per pair two reads, then two writes, and selects.
    #pragma unroll 4
                                for (int c = 0; c < 32; c++) {
                                    const int j0 = __builtin_amdgcn_readlane((int)jv, 2 * c), j1 = __builtin_amdgcn_readlane((int)jv, 2 * c + 1);
                                    const int i0 = j0 > 1 ? j0 : 0, i1 = j1 > 1 ? j1 : 1;
                                    const int x0 = sh[i0], x1 = sh[i1];
                                    const int a0 = r0, b0 = r1;
                                    const int r1m = j0 == 1 ? a0 : b0;  // entry 1 after the first swap
                                    sh[i0] = a0;
                                    sh[i1] = r1m;
                                    r0 = j0 > 1 ? x0 : (j0 == 1 ? b0 : a0);
                                    r1 = j1 > 1 ? (j1 == j0 ? a0 : x1) : r1m;  // j1 == j0: the value the first swap stored
                                    bp0 = lane == c ? r0 : bp0;
                                    bp1 = lane == c ? r1 : bp1;
                                }
                                bool good = false;
                                if (lane < 32) {
                                    const float4 a = Q[bp0], b = Q[bp1];
                                    good = a.x != b.x && a.y != b.y && a.z != b.z;
                                }
                                gmask = __ballot(good);
                                qh = 0;
                                qn = 32;
                            }
                            const uint64_t m = gmask & (~0ull << qh) & 0xFFFFFFFFull;
                            if (m == 0) {  // the rest of the block failed isSampleGood
                                chk += qn - qh;
                                qh = qn;
                                if (chk >= 1000) { fail = true; break; }
                                continue;
                            }
                            const int gi = __ffsll((unsigned long long)m) - 1;
                            if (chk + (gi - qh) >= 1000) { fail = true; break; }  // 1000 failed samples first
                            const int s0v = __builtin_amdgcn_readlane(bp0, gi), s1v = __builtin_amdgcn_readlane(bp1, gi);
                            if (lane == 0) { S.s0[nb] = s0v; S.s1[nb] = s1v; }
                            nb++;
                            chk = 0;
                            qh = gi + 1;
                        }
                        if (lane == 0) { S.nb = nb; S.fail = fail; }
                    }
                    __syncthreads();
                    SUPP_T(1);
                    const int nb = S.nb;
                    {
                        // kBatch / NW trials per wave, NW lanes per trial each counting every NW-th point (the lanes of
                        // a point phase read the same point: an LDS broadcast)
                        constexpr int NW = NT / 64;
                        const int c = wave * (kBatch / NW) + lane / NW, qq = lane % NW;
                        int cnt = 0;
                        if (c < nb) {
                            float L[6];
                            line_from_samples(Q[S.s0[c]], Q[S.s1[c]], L);
                            float ld[3] = {L[3], L[4], L[5]};
                            normalize4(ld);
    #pragma unroll 1
                            for (int i = qq; i < n; i += NW) cnt += line_sqd(L, ld, Q[i]) <= thr;
                        }
    #pragma unroll
                        for (int o = 1; o < NW; o <<= 1) cnt += __shfl_xor(cnt, o);
                        if (qq == 0 && c < nb) S.cnt[c] = cnt;
                    }
                    __syncthreads();
                    SUPP_T(2);
                    if (wave == 0) {
                        // computeModel's bookkeeping over the round's trials, in parallel (lane c = trial c): a
                        // trial improves the model when its count beats the best so far (exclusive prefix max);
                        // k changes only there, so the k each trial's `iterations < k` test sees is the k of the
                        // last improvement before it; the loop stops at the first failed test, or after trial
                        // 1000 - iterations (max_iterations_)
                        const int it0 = S.iterations, best0 = S.best;
                        const double k0 = S.k;
                        const bool act = lane < nb;
                        const int cn = act ? S.cnt[lane] : INT_MIN;
                        int pm = cn, lr;
    #pragma unroll
                        for (int off = 1; off < 64; off <<= 1) {
                            const int y = __shfl_up(pm, off);
                            if (lane >= off) pm = max(pm, y);
                        }
                        int ex = __shfl_up(pm, 1);
                        if (lane == 0) ex = INT_MIN;
                        const bool rec = act && cn > max(ex, best0);
                        double kc = 0.0;
                        if (rec) {
                            const double w = (double)cn * one_over_n;
                            double pno = 1.0 - w * w;
                            pno = fmax(DBL_EPSILON, pno);
                            pno = fmin(1.0 - DBL_EPSILON, pno);
                            kc = log_prob / log(pno);
                        }
                        lr = rec ? lane : -1;
    #pragma unroll
                        for (int off = 1; off < 64; off <<= 1) {
                            const int y = __shfl_up(lr, off);
                            if (lane >= off) lr = max(lr, y);
                        }
                        int lre = __shfl_up(lr, 1);
                        if (lane == 0) lre = -1;
                        const double kb_rec = __shfl(kc, lre < 0 ? 0 : lre);
                        const double kb = lre < 0 ? k0 : kb_rec;
                        const uint64_t m1 = __ballot(act && !((double)(it0 + lane) < kb));
                        const int stop1 = m1 ? __ffsll((unsigned long long)m1) - 1 : 64;
                        const int stop2 = (kMaxTrials - 1) - it0;
                        int proc, it;
                        bool done;
                        if (stop1 < nb && stop1 <= stop2) { proc = stop1; it = it0 + stop1; done = true; }
                        else if (stop2 < nb) { proc = stop2 + 1; it = it0 + stop2 + 1; done = true; }
                        else { proc = nb; it = it0 + nb; done = false; }
                        const uint64_t rm = __ballot(rec) & (proc >= 64 ? ~0ull : ((1ull << proc) - 1ull));
                        double kf = k0;
                        if (rm) {
                            const int L = 63 - __clzll(rm);
                            kf = __shfl(kc, L);
                            if (lane == L) {
                                S.best = cn; S.best_s0 = S.s0[L]; S.best_s1 = S.s1[L]; S.have = 1; S.k = kc;
                            }
                        }
                        if (!done && (S.fail || !((double)it < kf))) done = true;
                        if (lane == 0) {
                            S.iterations = it;
                            S.done = done;
                        }
                    }
                    __syncthreads();
                    SUPP_T(3);
    #ifdef SPSLAM_SUPP_PROF
                    if (t == 0) pr[6]++;
    #endif
                }
            } else {
                // wave 0: one speculative round's samples from trial it0 on, into buffer sb_ (S.s0 / S.s1 or S.s0x /
                // S.s1x; S.nbb[sb_] trials, S.failb[sb_]: 1000 failed samples came first)
                auto sample = [&](int sb_, int it0) __attribute__((always_inline)) {
                    int nb = 0, chk = 0;  // chk: failed samples of the trial being drawn
                    bool fail = false;
                    while (nb < kBatch && it0 + nb < kMaxTrials) {
                        if (qh == qn) {
                            // apply the next 32 draw pairs to the shuffle state: their swaps do not depend on
                            // whether a pair becomes a trial's sample, so isSampleGood is checked afterwards,
                            // for all 32 pairs at once (the chain keeps one LDS round trip per pair)
                            const uint32_t r = rnext;
                            const uint32_t jv = (lane & 1) ? 1u + r % (uint32_t)(n - 1) : r % (uint32_t)n;
                            pos += 64;
                            rnext = sb.rnd[pos + lane];  // (the table holds one block beyond the worst case)
                            // Branch-free: entries 0 and 1 live in r0 / r1 (their LDS slots are never read), so
                            // a swap that does not touch LDS reads and writes slot 0 (first swap) or 1 (second)
                            // as a sink; per pair two reads, then two writes, and selects.
    #pragma unroll 4
                            for (int c = 0; c < 32; c++) {
                                const int j0 = __builtin_amdgcn_readlane((int)jv, 2 * c), j1 = __builtin_amdgcn_readlane((int)jv, 2 * c + 1);
                                const int i0 = j0 > 1 ? j0 : 0, i1 = j1 > 1 ? j1 : 1;
                                const int x0 = sh[i0], x1 = sh[i1];
                                const int a0 = r0, b0 = r1;
                                const int r1m = j0 == 1 ? a0 : b0;  // entry 1 after the first swap
                                sh[i0] = a0;
                                sh[i1] = r1m;
                                r0 = j0 > 1 ? x0 : (j0 == 1 ? b0 : a0);
                                r1 = j1 > 1 ? (j1 == j0 ? a0 : x1) : r1m;  // j1 == j0: the value the first swap stored
                                bp0 = lane == c ? r0 : bp0;
                                bp1 = lane == c ? r1 : bp1;
                            }
                            bool good = false;
                            if (lane < 32) {
                                const float4 a = Q[bp0], b = Q[bp1];
                                good = a.x != b.x && a.y != b.y && a.z != b.z;
                            }
                            gmask = __ballot(good);
                            qh = 0;
                            qn = 32;
                        }
                        const uint64_t m = gmask & (~0ull << qh) & 0xFFFFFFFFull;
                        if (m == 0) {  // the rest of the block failed isSampleGood
                            chk += qn - qh;
                            qh = qn;
                            if (chk >= 1000) { fail = true; break; }
                            continue;
                        }
                        const int gi = __ffsll((unsigned long long)m) - 1;
                        if (chk + (gi - qh) >= 1000) { fail = true; break; }  // 1000 failed samples first
                        const int s0v = __builtin_amdgcn_readlane(bp0, gi), s1v = __builtin_amdgcn_readlane(bp1, gi);
                        if (lane == 0) { (sb_ ? S.s0x : S.s0)[nb] = s0v; (sb_ ? S.s1x : S.s1)[nb] = s1v; }
                        nb++;
                        chk = 0;
                        qh = gi + 1;
                    }
                    if (lane == 0) { S.nbb[sb_] = nb; S.failb[sb_] = fail; }
                };
                // wave 0: computeModel's bookkeeping over the round's trials in buffer sb_, in parallel (lane c = trial
                // c): a trial improves the model when its count beats the best so far (exclusive prefix max); k changes
                // only there, so the k each trial's `iterations < k` test sees is the k of the last improvement before
                // it; the loop stops at the first failed test, or after trial 1000 - iterations (max_iterations_)
                auto decide = [&](int sb_, int nb) __attribute__((always_inline)) {
                    const int it0 = S.iterations, best0 = S.best;
                    const double k0 = S.k;
                    const bool act = lane < nb;
                    const int cn = act ? S.cnt[lane] : INT_MIN;
                    int pm = cn, lr;
    #pragma unroll
                    for (int off = 1; off < 64; off <<= 1) {
                        const int y = __shfl_up(pm, off);
                        if (lane >= off) pm = max(pm, y);
                    }
                    int ex = __shfl_up(pm, 1);
                    if (lane == 0) ex = INT_MIN;
                    const bool rec = act && cn > max(ex, best0);
                    double kc = 0.0;
                    if (rec) {
                        const double w = (double)cn * one_over_n;
                        double pno = 1.0 - w * w;
                        pno = fmax(DBL_EPSILON, pno);
                        pno = fmin(1.0 - DBL_EPSILON, pno);
                        kc = log_prob / log(pno);
                    }
                    lr = rec ? lane : -1;
    #pragma unroll
                    for (int off = 1; off < 64; off <<= 1) {
                        const int y = __shfl_up(lr, off);
                        if (lane >= off) lr = max(lr, y);
                    }
                    int lre = __shfl_up(lr, 1);
                    if (lane == 0) lre = -1;
                    const double kb_rec = __shfl(kc, lre < 0 ? 0 : lre);
                    const double kb = lre < 0 ? k0 : kb_rec;
                    const uint64_t m1 = __ballot(act && !((double)(it0 + lane) < kb));
                    const int stop1 = m1 ? __ffsll((unsigned long long)m1) - 1 : 64;
                    const int stop2 = (kMaxTrials - 1) - it0;
                    int proc, it;
                    bool done;
                    if (stop1 < nb && stop1 <= stop2) { proc = stop1; it = it0 + stop1; done = true; }
                    else if (stop2 < nb) { proc = stop2 + 1; it = it0 + stop2 + 1; done = true; }
                    else { proc = nb; it = it0 + nb; done = false; }
                    const uint64_t rm = __ballot(rec) & (proc >= 64 ? ~0ull : ((1ull << proc) - 1ull));
                    double kf = k0;
                    if (rm) {
                        const int L = 63 - __clzll(rm);
                        kf = __shfl(kc, L);
                        if (lane == L) {
                            S.best = cn; S.best_s0 = (sb_ ? S.s0x : S.s0)[L]; S.best_s1 = (sb_ ? S.s1x : S.s1)[L];
                            S.have = 1; S.k = kc;
                        }
                    }
                    if (!done && (S.failb[sb_] || !((double)it < kf))) done = true;
                    if (lane == 0) {
                        S.iterations = it;
                        S.done = done;
                    }
                };
                // the next round's samples (wave 0) drawn while the other waves count this round's inliers: the
                // draws do not depend on the counts, and a round the bookkeeping does not reach is discarded (the
                // reference discards its RNG too); the next round starts at trial iterations + this round's trials,
                // which is where the bookkeeping continues whenever it does not stop
                if (wave == 0 && !S.done) sample(0, 0);
                __syncthreads();
                SUPP_T(1);
                int cur = 0;
                while (!S.done) {
                    const int nb = S.nbb[cur];
                    if (wave == 0) {
                        if (!S.failb[cur]) sample(cur ^ 1, S.iterations + nb);
                        else if (lane == 0) { S.nbb[cur ^ 1] = 0; S.failb[cur ^ 1] = 1; }
                    } else {
                        // NW - 1 counting waves: NW - 1 lanes per trial, each counting every (NW - 1)-th point; the
                        // partial counts are integers, so their LDS additions give the same total in any order
                        constexpr int LP = NT / 64 - 1;
                        const int u = t - 64, c = u / LP, qq = u - c * LP;
                        if (c < nb) {
                            float L[6];
                            line_from_samples(Q[(cur ? S.s0x : S.s0)[c]], Q[(cur ? S.s1x : S.s1)[c]], L);
                            float ld[3] = {L[3], L[4], L[5]};
                            normalize4(ld);
                            int cnt = 0;
#pragma unroll 1
                            for (int i = qq; i < n; i += LP) cnt += line_sqd(L, ld, Q[i]) <= thr;
                            atomicAdd(&S.cnt[c], cnt);
                        }
                    }
                    __syncthreads();
                    SUPP_T(2);
                    if (wave == 0) {
                        decide(cur, nb);
                        S.cnt[lane] = 0;  // (each lane read its own count above)
                    }
                    __syncthreads();
                    SUPP_T(3);
#ifdef SPSLAM_SUPP_PROF
                    if (t == 0) pr[6]++;
#endif
                    cur ^= 1;
                }
            }
            // ---------------- inliers, optimizeModelCoefficients, refined inliers
            int n_inl = 0;
            if (S.have) {
                float c0[6];
                line_from_samples(Q[S.best_s0], Q[S.best_s1], c0);
                n_inl = select_within<NT>(c0, Q, flag, n, thr, S);
                if (n_inl > 2) {
                    // The two sums below are sequential float chains in point order (one accumulator per lane).
                    // Points outside the line add +0.0f, which leaves a sum that starts at +0.0f unchanged
                    // (it can never be -0.0f), so the loop is branch-free and its LDS loads are issued a
                    // group of 8 ahead of the adds instead of one dependent round trip per point.
                    constexpr int kG = 8;
                    if (wave == 0 && lane < 3) {  // compute3DCentroid (dense): sequential float sums
                        float s = 0.f;
                        int i = 0;
                        for (; i + kG <= n; i += kG) {
                            float v[kG];
#pragma unroll
                            for (int u = 0; u < kG; u++) {
                                const float4 p = Q[i + u];
                                v[u] = flag[i + u] ? (lane == 0 ? p.x : lane == 1 ? p.y : p.z) : 0.f;
                            }
#pragma unroll
                            for (int u = 0; u < kG; u++) s += v[u];
                        }
                        for (; i < n; i++) {
                            const float4 p = Q[i];
                            s += flag[i] ? (lane == 0 ? p.x : lane == 1 ? p.y : p.z) : 0.f;
                        }
                        S.acc[lane] = s / (float)n_inl;
                    }
                    __syncthreads();
                    if (wave == 0 && lane < 6) {  // computeCovarianceMatrix (dense), one accumulator per lane
                        const float cx = S.acc[0], cy = S.acc[1], cz = S.acc[2];
                        auto term = [&](int i) __attribute__((always_inline)) {
                            const float4 p = Q[i];
                            const float x = p.x - cx, y = p.y - cy, z = p.z - cz;
                            const float a = lane == 0 ? y : lane == 1 ? y : lane == 2 ? z : lane == 3 ? x : lane == 4 ? y : z;
                            const float b = lane == 0 ? y : lane == 1 ? z : lane == 2 ? z : x;
                            return flag[i] ? a * b : 0.f;
                        };
                        float s = 0.f;
                        int i = 0;
                        for (; i + kG <= n; i += kG) {
                            float v[kG];
#pragma unroll
                            for (int u = 0; u < kG; u++) v[u] = term(i + u);
#pragma unroll
                            for (int u = 0; u < kG; u++) s += v[u];
                        }
                        for (; i < n; i++) s += term(i);
                        S.acc[3 + lane] = s;
                    }
                    __syncthreads();
                    if (t == 0) {
                        // acc[3..8] = (1,1) (1,2) (2,2) (0,0) (0,1) (0,2)
                        const float cov[3][3] = {{S.acc[6], S.acc[7], S.acc[8]},
                                                 {S.acc[7], S.acc[3], S.acc[4]},
                                                 {S.acc[8], S.acc[4], S.acc[5]}};
                        float ev[3];
                        line_direction(cov, ev);
                        S.line[0] = S.acc[0]; S.line[1] = S.acc[1]; S.line[2] = S.acc[2];
                        S.line[3] = ev[0]; S.line[4] = ev[1]; S.line[5] = ev[2];
                    }
                } else if (t == 0) {
                    for (int k = 0; k < 6; k++) S.line[k] = c0[k];
                }
                __syncthreads();
                float ref[6];
                for (int k = 0; k < 6; k++) ref[k] = S.line[k];
                n_inl = select_within<NT>(ref, Q, flag, n, thr, S);
            } else if (t == 0) {
                for (int k = 0; k < 6; k++) S.line[k] = 0.f;
            }
            __syncthreads();
            SUPP_T(4);
            // ---------------- Frame.cc:961-988
            LineCand& out = C[j];
            if (t == 0) {
                for (int k = 0; k < 6; k++) out.line[k] = S.line[k];
                out.n_inliers = n_inl;
                out.iterations = S.iterations;
                out.idx_off = coff + used;
                int fl = 0;
                if (!((double)n_inl < sp.line_ratio * (double)bsize)) {
                    fl = 1;
                    if (line_in_range(S.line, K)) fl |= 2;
                }
                S.flags = fl;
            }
            ncand = j + 1;
            __syncthreads();
            const int fl = S.flags;
            if (!(fl & 1)) {
                if (t == 0) out.flags = fl;
                break;
            }
            // line points (ExtractIndices, order kept) + removal of them from the set, in place
            int nonborder = 0;
            int wbase = 0, kbase = 0;
            for (int base = 0; base < n; base += NT) {
                const int i = base + t;
                const bool valid = i < n;
                const bool in = valid && flag[i];
                const float4 p = valid ? Q[i] : make_float4(0.f, 0.f, 0.f, 0.f);
                if (in && (fl & 2) && !is_border_point(p, D, K)) nonborder++;
                // exclusive ranks of inliers / kept points within this chunk
                const uint64_t mi = __ballot(in), mk = __ballot(valid && !in);
                const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
                if (lane == 0) { S.s0[wave] = __popcll(mi); S.s1[wave] = __popcll(mk); }
                __syncthreads();
                int oi = wbase, ok = kbase;
                for (int w = 0; w < wave; w++) { oi += S.s0[w]; ok += S.s1[w]; }
                int ti = 0, tk = 0;
                for (int w = 0; w < NT / 64; w++) { ti += S.s0[w]; tk += S.s1[w]; }
                __syncthreads();
                if (in) lidx[used + oi + __popcll(mi & lt)] = __float_as_int(p.w);
                if (valid && !in) Q[ok + __popcll(mk & lt)] = p;
                wbase += ti;
                kbase += tk;
            }
            nonborder = block_sum<NT>(nonborder, S);
            if (t == 0) out.flags = fl | ((fl & 2) && nonborder <= n_inl / 4 ? 4 : 0);
            used += n_inl;
            n = kbase;
            __syncthreads();
            SUPP_T(5);
        }
#ifdef SPSLAM_SUPP_PROF
        if (t == 0) {
            pr[7] = bsize;
            for (int k = 0; k < 8; k++) sb.prof[((size_t)f * kMaxPlanesPerFrame + q) * 8 + k] = pr[k];
        }
#endif
            return ncand;
        };
        const int ncand = in_lds ? boundary(Qs, shs, flags_s)
                                 : boundary(sb.big + (size_t)f * g.contour_cap + coff,
                                            sb.big_sh + (size_t)f * g.contour_cap + coff,
                                            sb.big_flag + (size_t)f * g.contour_cap + coff);
        if (t == 0) sb.n_cand[f * kMaxPlanesPerFrame + q] = ncand;
        __syncthreads();
    }
}

// Frame::CaculatePlanes' plane (Frame.cc:1082-1093) with GCC -O3 -march=native's contractions.
__device__ void supposed_coef(const float* ip, const float* il, float* coef) {
    const float a = fmaf(ip[1], il[5], -(ip[2] * il[4]));
    const float b = fmaf(ip[2], il[3], -(ip[0] * il[5]));
    const float c = fmaf(ip[0], il[4], -(ip[1] * il[3]));
    const float d = fmaf(c, il[2], fmaf(a, il[0], b * il[1]));
    const float v = sqrtf(fmaf(c, c, fmaf(a, a, b * b)));
    coef[0] = a / v; coef[1] = b / v; coef[2] = c / v; coef[3] = -d / v;
    if (coef[3] < 0)
        for (int k = 0; k < 4; k++) coef[k] = -coef[k];
}

__global__ __launch_bounds__(64) void supp_assemble_kernel(SuppParams sp, SuppBuffers sb, int contour_cap,
                                                           const spslam_plane* __restrict__ planes,
                                                           const int* __restrict__ plane_counts,
                                                           spslam_supposed_plane* __restrict__ out,
                                                           int* __restrict__ out_counts,
                                                           int32_t* __restrict__ out_line_idx,
                                                           float* __restrict__ out_patch) {
    __shared__ float pl[kMaxPlanesPerFrame + kMaxSuppPerFrame][4];
    __shared__ int src_cand[kMaxSuppPerFrame];
    __shared__ int n_out;
    const int f = blockIdx.x, lane = threadIdx.x;
    const int np = min(plane_counts[f], kMaxPlanesPerFrame);
    const spslam_plane* P = planes + (size_t)f * kMaxPlanesPerFrame;
    const LineCand* C = sb.cand + (size_t)f * kMaxPlanesPerFrame * kMaxLinesPerBoundary;
    spslam_supposed_plane* O = out + (size_t)f * sp.supp_cap;
    const int cap = min(sp.supp_cap, kMaxSuppPerFrame);
    const int n_patch = sp.n_steps * sp.n_steps;
    if (lane == 0) {
        for (int q = 0; q < np; q++)
            for (int k = 0; k < 4; k++) pl[q][k] = P[q].coef[k];
        int nl = np, ns = 0, loff = 0;
        for (int q = np - 1; q >= 0; --q) {
            const int nc = sb.n_cand[f * kMaxPlanesPerFrame + q];
            for (int j = 0; j < nc; j++) {
                const LineCand& c = C[q * kMaxLinesPerBoundary + j];
                if ((c.flags & 7) != 7) continue;
                float cf[4];
                supposed_coef(pl[q], c.line, cf);
                bool seen = false;
                for (int m = 0; m < nl && !seen; m++)  // PlaneNotSeen (Frame.cc:1116-1130)
                    seen = plane_seen_by(pl[m], cf);
                if (seen) continue;
                if (ns < cap && nl < kMaxPlanesPerFrame + kMaxSuppPerFrame) {
                    for (int k = 0; k < 4; k++) pl[nl][k] = cf[k];
                    nl++;
                    spslam_supposed_plane& o = O[ns];
                    for (int k = 0; k < 4; k++) o.coef[k] = cf[k];
                    for (int k = 0; k < 6; k++) o.line[k] = c.line[k];
                    o.source_plane = q;
                    o.n_line = min(c.n_inliers, sp.line_cap - loff);
                    o.line_offset = loff;
                    o.n_patch = n_patch;
                    o.patch_offset = ns * n_patch;
                    o.pad = 0;
                    loff += o.n_line;
                    src_cand[ns] = q * kMaxLinesPerBoundary + j;
                }
                ns++;
            }
        }
        out_counts[f] = ns;
        n_out = min(ns, cap);
    }
    __syncthreads();
    for (int s = 0; s < n_out; s++) {
        const spslam_supposed_plane& o = O[s];
        const LineCand& c = C[src_cand[s]];
        const int32_t* src = sb.line_idx + (size_t)f * contour_cap + c.idx_off;
        int32_t* dst = out_line_idx + (size_t)f * sp.line_cap + o.line_offset;
        for (int i = lane; i < o.n_line; i += 64) dst[i] = src[i];
        // CaculatePlanes' synthetic patch (Frame.cc:1097-1112), i outer, j inner
        const float* ip = pl[o.source_plane];
        float* pp = out_patch + ((size_t)f * sp.supp_cap + s) * (size_t)n_patch * 3;
        for (int k = lane; k < n_patch; k += 64) {
            const float a = sp.steps[k / sp.n_steps], b = sp.steps[k % sp.n_steps];
            const float x = fmaf(b, ip[0], fmaf(a, o.line[3], o.line[0]));
            const float y = fmaf(b, ip[1], fmaf(a, o.line[4], o.line[1]));
            const float z = (fmaf(o.coef[0], x, o.coef[1] * y) + o.coef[3]) / (-o.coef[2]);
            pp[3 * k] = x;
            pp[3 * k + 1] = y;
            pp[3 * k + 2] = z;
        }
    }
}

}  // namespace supp

hipError_t supp_launch(const PlaneGeom& g, const PlaneBuffers& pb, const SuppParams& sp, const SuppBuffers& sb,
                       int n, const float* depth, long long depth_fs, int depth_stride, const spslam_plane* planes,
                       const int* plane_counts, const int32_t* contours, spslam_supposed_plane* out, int* out_counts,
                       int32_t* out_line_idx, float* out_patch, hipStream_t s, KernelTimer* timer) {
    if (sp.n_steps < 1 || sp.n_steps > kMaxPatchSteps || sp.supp_cap < 1) return hipErrorInvalidValue;
    auto B = [&](int k) { if (timer) timer->begin(k, s); };
    auto E = [&](int k) { if (timer) timer->end(k, s); };
    B(kKindSuppLines);
    if (n <= 16)  // a few frames: each boundary's workgroup on twice the lanes (B = 1 latency)
        hipLaunchKernelGGL(supp::supp_lines_kernel<512>, dim3(n, 16), dim3(512), 0, s, g, pb, sp, sb, depth,
                           depth_fs, depth_stride, planes, plane_counts, contours);
    else
        hipLaunchKernelGGL(supp::supp_lines_kernel<supp::kThreads>, dim3(n, 16), dim3(supp::kThreads), 0, s, g, pb,
                           sp, sb, depth, depth_fs, depth_stride, planes, plane_counts, contours);
    E(kKindSuppLines);
    B(kKindSuppAssemble);
    hipLaunchKernelGGL(supp::supp_assemble_kernel, dim3(n), dim3(64), 0, s, sp, sb, g.contour_cap, planes,
                       plane_counts, out, out_counts, out_line_idx, out_patch);
    E(kKindSuppAssemble);
    return hipGetLastError();
}

// Test hook (spslam_debug_plane_not_seen): Frame::PlaneNotSeen of each candidate against a plane list,
// through the same device predicate the extraction kernels use.
__global__ __launch_bounds__(64) void plane_not_seen_debug_kernel(const float* __restrict__ planes, int n,
                                                                  const float* __restrict__ coefs, int m,
                                                                  int* __restrict__ out) {
    const int k = blockIdx.x * 64 + threadIdx.x;
    if (k >= m) return;
    bool seen = false;
    for (int j = 0; j < n && !seen; j++) seen = plane_seen_by(planes + 4 * j, coefs + 4 * k);
    out[k] = !seen;
}

hipError_t plane_not_seen_debug_launch(const float* planes, int n, const float* coefs, int m, int* out,
                                       hipStream_t s) {
    if (m < 1) return hipSuccess;
    hipLaunchKernelGGL(plane_not_seen_debug_kernel, dim3((m + 63) / 64), dim3(64), 0, s, planes, n, coefs, m, out);
    return hipGetLastError();
}

}  // namespace spslam
