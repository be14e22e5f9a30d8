// gfx950 kernels for SP-SLAM's ORB extractor (reference: src/ORBextractor.cc).
//
// One batched pass over B frames is four kernel kinds:
//   level_kernel          x8  per pyramid level, 64x32 tiles: level image (OpenCV
//                             INTER_LINEAR 8U fixed point from level l-1,
//                             :1107-1132), its 7x7 sigma-2 Gaussian (:1085-1086)
//                             and its FAST-9/16 score map, from one LDS tile
//   fast_cells_kernel     x1  one wave per 30x30 FAST cell of every level: 3x3
//                             NMS at iniThFAST on the score map, retry at
//                             minThFAST if the cell came back empty (:789-829)
//   octree_kernel         x1  one workgroup per (frame, level): DistributeOctTree
//                             (:539-763) as data-parallel passes over the keys
//   desc_kernel           x1  one wave per keypoint: IC_Angle (:77-104) + rotated
//                             BRIEF (:107-147), output assembly (:1075-1104)
//
// Floating point: built with -ffp-contract=off and correctly rounded fp32
// division; the only fused multiply-adds are the explicit ones reproducing the
// reference build's contraction of the BRIEF sample expression.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/spslam_gpu.h"
#include "wave_priority.h"
#include "orb_launch.h"

namespace spslam {

__constant__ int8_t c_pattern[1024] = {
#include "../../include/spslam_brief_pattern.inc"
};
__constant__ int c_umax[16];

__device__ __forceinline__ int cv_round(float v) { return (int)__builtin_rintf(v); }

// ---------------------------------------------------------------------------
// FAST-9/16.  Score = max over the 16 contiguous 9-arcs of min(v - x) and of
// min(x - v), minus 1; equals OpenCV cornerScore<16> for every corner, and
// "corner at threshold t" <=> score >= t.  Since min over an arc of v - x is
// v - max x and max of v - x is v - min x, the score is
//   max(v - min_k max_arc(k) x, max_k min_arc(k) x - v) - 1,
// and both arc extremes come from one packed u16 minimum chain over the
// pairs (255 - x, x) (min of 255 - x = 255 - max x): 16 mads to pack, 64
// packed minima, 16 packed maxima.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u16x2 pmin(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ u16x2 pmax(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ u16x2 psubs(u16x2 a, u16x2 b) { return __builtin_elementwise_sub_sat(a, b); }

__device__ __forceinline__ int fast_score(const uint8_t* p, int P) {
    const int v = p[0];
    const int off[16] = {3 * P,  3 * P + 1,  2 * P + 2,  P + 3,  3,  -P + 3, -2 * P + 2, -3 * P + 1,
                         -3 * P, -3 * P - 1, -2 * P - 2, -P - 3, -3, P - 3,  2 * P - 2,  3 * P - 1};
    u16x2 X[16];
#pragma unroll
    for (int k = 0; k < 16; k++) X[k] = as_u16x2((uint32_t)p[off[k]] * 65535u + 255u);  // (255 - x, x)
    u16x2 m2[16], m4[16];
#pragma unroll
    for (int k = 0; k < 16; k++) m2[k] = pmin(X[k], X[(k + 1) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++) m4[k] = pmin(m2[k], m2[(k + 2) & 15]);
    u16x2 M = as_u16x2(0u);
#pragma unroll
    for (int k = 0; k < 16; k++) M = pmax(M, pmin(pmin(m4[k], m4[(k + 4) & 15]), X[(k + 8) & 15]));
    return max(v + (int)M.x - 255, (int)M.y - v) - 1;
}


// ---------------------------------------------------------------------------
// One pyramid level, one 64x32 output tile per 256-thread workgroup:
//   * the tile plus a 3-pixel halo of level l, resized from level l-1 with
//     OpenCV's INTER_LINEAR 8U fixed point (:1107-1132; per-pixel
//     coefficients from the same double/float expressions OpenCV uses), or
//     read from the input frame at level 0; BORDER_REFLECT_101 outside;
//   * the level image (tile interior) for the next level, IC_Angle and BRIEF;
//   * GaussianBlur 7x7 sigma 2 (:1085-1086), OpenCV's bit-exact 8U fixed point:
//     out = (sum_ij k_i k_j p + 2^15) >> 16 with k = [18,34,48,56,48,34,18];
//   * the FAST score map (0 where no cell window evaluates a pixel).
// The tile is built and read 4 pixels (one dword) at a time: dword global loads realigned with
// v_alignbyte, the resize's byte pairs picked with v_perm and weighted with v_dot2_u32_u16, the
// horizontal blur as two v_dot4_u32_u8 per output, the FAST pre-test on packed u16 pairs.
constexpr int kLH = kLevelTileH + 6, kLW = kLevelTileW + 6;
constexpr int kLG = (kLW + 3) / 4;   // 4-column groups of a tile row (the last holds 2 pad columns)
constexpr int kTinPitch = 4 * kLG;   // 72: dword-aligned rows
constexpr int kLevelThreads = 256;

// BORDER_REFLECT_101 for positions at most one image length outside (tiles
// overhang by < 64 + 3 pixels; levels are >= 64 wide/high).
__device__ __forceinline__ int reflect1(int p, int len) {
    p = p < 0 ? -p : p;
    return p >= len ? 2 * len - 2 - p : p;
}

// OpenCV INTER_LINEAR 8U coefficients for one destination column / row: the
// same double/float expressions as cv::resize.
struct RzCol { int16_t x0, x1, a0, a1; };
__device__ __forceinline__ RzCol resize_coef(double s, int d, int slen, bool horizontal) {
    float fx = (float)((d + 0.5) * s - 0.5);
    int sx = (int)floorf(fx);
    fx -= sx;
    RzCol r;
    if (horizontal) {
        bool tail = false;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= slen) {
            tail = true;
            if (sx >= slen - 1) { fx = 0; sx = slen - 1; }
        }
        const int a0 = (short)cv_round((1.f - fx) * 2048.f), a1 = (short)cv_round(fx * 2048.f);
        r.x0 = (int16_t)sx;
        r.x1 = (int16_t)(tail ? sx : sx + 1);
        r.a0 = (int16_t)(tail ? 2048 : a0);
        r.a1 = (int16_t)(tail ? 0 : a1);
    } else {
        const int b0 = (short)cv_round((1.f - fx) * 2048.f), b1 = (short)cv_round(fx * 2048.f);
        r.x0 = (int16_t)min(max(sx, 0), slen - 1);
        r.x1 = (int16_t)min(max(sx + 1, 0), slen - 1);
        r.a0 = (int16_t)b0;
        r.a1 = (int16_t)b1;
    }
    return r;
}
// The vertical step of the resize for one destination pixel from its two horizontally interpolated rows.
__device__ __forceinline__ uint32_t resize_v(const RzCol& cy, int r0, int r1) {
    return (uint32_t)((((cy.a0 * (r0 >> 4)) >> 16) + ((cy.a1 * (r1 >> 4)) >> 16) + 2) >> 2) & 255u;
}

// A 4-column group of the resized tile whose 8 source bytes per row lie in one window sb..sb+7 (sb = the
// first column's left source): the window is read as 3 aligned dwords from a = sb & ~3, realigned by
// s = sb & 3; sel[j] picks (x0_j, x1_j) of column j into a u16 pair for v_dot2 with coef[j] = (a0, a1).
// a < 0: the group is gathered per pixel (reflected / clamped border columns, unaligned source rows).
struct RzGroup { int a, s; uint32_t sel[4], coef[4]; };

// FAST pre-test for 4 pixels at once (byte j of each word = pixel j; c0 = p[3P], c4 = p[3], c8 = p[-3P],
// c12 = p[-3]): bit j set when some 9-arc may hold pixel j's corner at threshold t, i.e. two consecutive
// compass pixels are both brighter than v + t or both darker than v - t.  Saturated u16 differences
// are non-zero exactly when the comparison holds.
__device__ __forceinline__ uint32_t fast_maybe4(uint32_t V, uint32_t C0, uint32_t C4, uint32_t C8, uint32_t C12,
                                                uint32_t t2) {
    uint32_t res = 0;
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {  // pixels hh (low half) and hh + 2 (high half)
        auto half = [&](uint32_t x) { return as_u16x2((x >> (8 * hh)) & 0x00ff00ffu); };
        const u16x2 v = half(V), t = as_u16x2(t2);
        const u16x2 hi = v + t, lo = psubs(v, t);
        const u16x2 c0 = half(C0), c4 = half(C4), c8 = half(C8), c12 = half(C12);
        const u16x2 b0 = psubs(c0, hi), b4 = psubs(c4, hi), b8 = psubs(c8, hi), b12 = psubs(c12, hi);
        const u16x2 k0 = psubs(lo, c0), k4 = psubs(lo, c4), k8 = psubs(lo, c8), k12 = psubs(lo, c12);
        const u16x2 br = pmax(pmax(pmin(b0, b4), pmin(b4, b8)), pmax(pmin(b8, b12), pmin(b12, b0)));
        const u16x2 dk = pmax(pmax(pmin(k0, k4), pmin(k4, k8)), pmax(pmin(k8, k12), pmin(k12, k0)));
        const uint32_t m = as_u32(pmax(br, dk));
        res |= ((m & 0xffffu) ? 1u : 0u) << hh;
        res |= ((m >> 16) ? 1u : 0u) << (hh + 2);
    }
    return res;
}

// The LDS of one tile (a 256-thread group).
struct LevelLds {
    __attribute__((aligned(16))) uint8_t tin[kLH][kTinPitch];
    __attribute__((aligned(16))) uint16_t th[kLH][kLevelTileW];
    RzCol rx[kTinPitch], ry[kLH];
    RzGroup rg[kLG];
    uint16_t cand[kLevelThreads / 64][kLevelTileH * kLevelTileW / (kLevelThreads / 64)];
    __attribute__((aligned(16))) uint8_t stile[kLevelTileH][kLevelTileW];  // FAST scores of the tile
};

// One 64x32 tile of level l of frame f on the 256 threads t of a group.  Every __syncthreads of the body is
// reached by every thread of the workgroup; `active` false (a group without a tile of its own in the fused
// launch: it repeats a valid tile in its own LDS) suppresses the global stores.
__device__ __forceinline__ void level_tile(const OrbGeom& g, int l, int minTh, int f, int tile, bool active, int t,
                                           LevelLds& sm) {
    const LevelGeom& L = g.lv[l];
    const int lane = t & 63, wave = t >> 6;
    const int x0 = (tile % L.tiles_x) * kLevelTileW, y0 = (tile / L.tiles_x) * kLevelTileH;
    const int w = L.w, h = L.h;
    uint8_t* img = const_cast<uint8_t*>(L.img) + f * L.frame_stride;
    constexpr int kNG = kLH * kLG, kIterG = (kNG + kLevelThreads - 1) / kLevelThreads;
    if (l == 0) {
        // interior tiles: the 72 bytes x0-4 .. x0+67 of each row as aligned dwords, shifted by one byte
        if (x0 >= 4 && x0 + kTinPitch <= w && ((reinterpret_cast<uintptr_t>(img) | (uintptr_t)L.stride) & 3) == 0) {
            uint32_t lo[kIterG], hi[kIterG];
#pragma unroll
            for (int k = 0; k < kIterG; k++) {
                const int q = t + k * kLevelThreads;
                lo[k] = hi[k] = 0;
                if (q < kNG) {
                    const int r = q / kLG, m = q - r * kLG;
                    const uint32_t* row = reinterpret_cast<const uint32_t*>(
                        img + (size_t)reflect1(y0 + r - 3, h) * L.stride + (x0 - 4));
                    lo[k] = row[m];
                    hi[k] = row[m + 1];
                }
            }
#pragma unroll
            for (int k = 0; k < kIterG; k++) {
                const int q = t + k * kLevelThreads;
                if (q < kNG) {
                    const int r = q / kLG, m = q - r * kLG;
                    *reinterpret_cast<uint32_t*>(&sm.tin[r][4 * m]) = __builtin_amdgcn_alignbyte(hi[k], lo[k], 1);
                }
            }
        } else {
            constexpr int kN = kLH * kLW, kIter = (kN + kLevelThreads - 1) / kLevelThreads;
            uint8_t v[kIter];
#pragma unroll
            for (int k = 0; k < kIter; k++) {
                const int q = t + k * kLevelThreads;
                v[k] = 0;
                if (q < kN) {
                    const int r = q / kLW, c = q - r * kLW;
                    const int y = reflect1(y0 + r - 3, h), x = reflect1(min(x0 + c - 3, w + 2), w);
                    v[k] = img[(size_t)y * L.stride + x];
                }
            }
#pragma unroll
            for (int k = 0; k < kIter; k++) {
                const int q = t + k * kLevelThreads;
                if (q < kN) sm.tin[q / kLW][q % kLW] = v[k];
            }
        }
    } else {
        const LevelGeom& S = g.lv[l - 1];
        const uint8_t* src = S.img + f * S.frame_stride;
        if (t < kLG) {
            RzCol cx[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int c = 4 * t + j;
                cx[j] = resize_coef(L.rscale_x, reflect1(min(x0 + c - 3, w + 2), w), S.w, true);
                sm.rx[c] = cx[j];
            }
            const int sb = cx[0].x0, a = sb & ~3;
            bool ok = a + 12 <= S.stride && ((reinterpret_cast<uintptr_t>(src) | (uintptr_t)S.stride) & 3) == 0;
            RzGroup G;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int o0 = cx[j].x0 - sb, o1 = cx[j].x1 - sb;
                ok = ok && o0 >= 0 && o0 <= 7 && o1 >= 0 && o1 <= 7;
                G.sel[j] = (uint32_t)(o0 & 7) | 0x0c00u | ((uint32_t)(o1 & 7) << 16) | 0x0c000000u;
                G.coef[j] = (uint32_t)(uint16_t)cx[j].a0 | ((uint32_t)(uint16_t)cx[j].a1 << 16);
            }
            G.a = ok ? a : -1;
            G.s = sb & 3;
            sm.rg[t] = G;
        } else if (t >= 64 && t < 64 + kLH) {
            sm.ry[t - 64] = resize_coef(L.rscale_y, reflect1(y0 + (t - 64) - 3, h), S.h, false);
        }
        __syncthreads();
        typedef unsigned short u16v2 __attribute__((ext_vector_type(2)));
        auto dot2 = [](uint32_t a, uint32_t b) {
            return (int)__builtin_amdgcn_udot2(__builtin_bit_cast(u16v2, a), __builtin_bit_cast(u16v2, b), 0u, false);
        };
        uint32_t wv[kIterG][6];
#pragma unroll
        for (int k = 0; k < kIterG; k++) {
            const int q = t + k * kLevelThreads;
#pragma unroll
            for (int i = 0; i < 6; i++) wv[k][i] = 0;
            if (q < kNG) {
                const int r = q / kLG, m = q - r * kLG;
                const int a = sm.rg[m].a;
                if (a >= 0) {
                    const RzCol cy = sm.ry[r];
                    const uint32_t* p0 = reinterpret_cast<const uint32_t*>(src + (size_t)cy.x0 * S.stride + a);
                    const uint32_t* p1 = reinterpret_cast<const uint32_t*>(src + (size_t)cy.x1 * S.stride + a);
                    wv[k][0] = p0[0]; wv[k][1] = p0[1]; wv[k][2] = p0[2];
                    wv[k][3] = p1[0]; wv[k][4] = p1[1]; wv[k][5] = p1[2];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kIterG; k++) {
            const int q = t + k * kLevelThreads;
            if (q < kNG) {
                const int r = q / kLG, m = q - r * kLG;
                const RzGroup& G = sm.rg[m];
                const RzCol cy = sm.ry[r];
                uint32_t packed = 0;
                if (G.a >= 0) {
                    const uint32_t s = (uint32_t)G.s;
                    const uint32_t a0 = __builtin_amdgcn_alignbyte(wv[k][1], wv[k][0], s);
                    const uint32_t a1 = __builtin_amdgcn_alignbyte(wv[k][2], wv[k][1], s);
                    const uint32_t b0 = __builtin_amdgcn_alignbyte(wv[k][4], wv[k][3], s);
                    const uint32_t b1 = __builtin_amdgcn_alignbyte(wv[k][5], wv[k][4], s);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int r0 = dot2(__builtin_amdgcn_perm(a1, a0, G.sel[j]), G.coef[j]);
                        const int r1 = dot2(__builtin_amdgcn_perm(b1, b0, G.sel[j]), G.coef[j]);
                        packed |= resize_v(cy, r0, r1) << (8 * j);
                    }
                } else {
                    const uint8_t* r0p = src + (size_t)cy.x0 * S.stride;
                    const uint8_t* r1p = src + (size_t)cy.x1 * S.stride;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int c = 4 * m + j;
                        if (c < kLW) {
                            const RzCol cx = sm.rx[c];
                            const int r0 = r0p[cx.x0] * cx.a0 + r0p[cx.x1] * cx.a1;
                            const int r1 = r1p[cx.x0] * cx.a0 + r1p[cx.x1] * cx.a1;
                            packed |= resize_v(cy, r0, r1) << (8 * j);
                        }
                    }
                }
                *reinterpret_cast<uint32_t*>(&sm.tin[r][4 * m]) = packed;
            }
        }
    }
    __syncthreads();
    const int lr = lane >> 4, lc = (lane & 15) * 4;  // 4 adjacent pixels per lane, 16 lanes per tile row
    if (l > 0) {
        // the level image (tile interior) for the next level, IC_Angle and BRIEF: one dword store per
        // 4 pixels (row pitch L.stride is a multiple of 64; columns past w land in the row padding)
        for (int rb = wave * 4; rb < kLevelTileH; rb += kLevelThreads / 16) {
            const int r = rb + lr;
            if (active && y0 + r < h) {
                const uint32_t* p = reinterpret_cast<const uint32_t*>(&sm.tin[r + 3][lc]);
                *reinterpret_cast<uint32_t*>(img + (size_t)(y0 + r) * L.stride + (x0 + lc)) =
                    __builtin_amdgcn_alignbyte(p[1], p[0], 3);
            }
        }
    }
    // horizontal blur pass over all tile rows, 4 outputs per lane: bytes c..c+11 from three dword LDS reads,
    // output j = dot4(bytes j..j+3, k0..k3) + dot4(bytes j+4..j+7, k4, k5, k6, 0)
    for (int q = t; q < kLH * (kLevelTileW / 4); q += kLevelThreads) {
        const int r = q / (kLevelTileW / 4), c = (q - r * (kLevelTileW / 4)) * 4;
        const uint32_t* w3 = reinterpret_cast<const uint32_t*>(&sm.tin[r][c]);
        const uint32_t a = w3[0], b = w3[1], d = w3[2];
        constexpr uint32_t K0 = 18u | (34u << 8) | (48u << 16) | (56u << 24), K1 = 48u | (34u << 8) | (18u << 16);
        uint32_t o[4];
        o[0] = __builtin_amdgcn_udot4(a, K0, __builtin_amdgcn_udot4(b, K1, 0u, false), false);
#pragma unroll
        for (int j = 1; j < 4; j++)
            o[j] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(b, a, j), K0,
                                          __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d, b, j), K1, 0u, false),
                                          false);
        *reinterpret_cast<uint2*>(&sm.th[r][c]) = make_uint2(o[0] | (o[1] << 16), o[2] | (o[3] << 16));
    }
    __syncthreads();
    uint8_t* blur = L.blur + f * L.blur_frame_stride;
    uint8_t* score = L.score + f * L.blur_frame_stride;
    const int bp = L.bpitch;
    const uint32_t t2 = (uint32_t)minTh | ((uint32_t)minTh << 16);
    // vertical blur pass, 4 pixels per lane (8-byte LDS reads of the row sums, one dword store); FAST
    // pre-test at the lowest threshold, candidates compacted per wave.  A wave owns tile rows
    // {4w..4w+3, 16+4w..16+4w+3}; their scores are assembled in LDS and stored as dwords by the same wave.
    int ncand = 0;
    for (int rb = wave * 4; rb < kLevelTileH; rb += kLevelThreads / 16) {
        const int r = rb + lr, y = y0 + r;
        uint16_t tv[7][4];
#pragma unroll
        for (int i = 0; i < 7; i++) *reinterpret_cast<uint2*>(tv[i]) = *reinterpret_cast<const uint2*>(&sm.th[r + i][lc]);
        uint32_t bw = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int sb = 18 * (tv[0][j] + tv[6][j]) + 34 * (tv[1][j] + tv[5][j]) + 48 * (tv[2][j] + tv[4][j]) +
                           56 * tv[3][j];
            bw |= (uint32_t)min(255, (sb + (1 << 15)) >> 16) << (8 * j);
        }
        if (active && y < h) *reinterpret_cast<uint32_t*>(blur + (size_t)y * bp + (x0 + lc)) = bw;
        *reinterpret_cast<uint32_t*>(&sm.stile[r][lc]) = 0u;
        // the FAST pre-test's 5 pixels for the 4 centres (sm.tin[r+3][lc+3+j]): centre row bytes lc..lc+11
        // and rows r, r+6 bytes lc+3..lc+6, from 7 dword LDS reads, realigned to one word per compass point
        const uint32_t* rc = reinterpret_cast<const uint32_t*>(&sm.tin[r + 3][lc]);
        const uint32_t* ru = reinterpret_cast<const uint32_t*>(&sm.tin[r][lc]);
        const uint32_t* rd = reinterpret_cast<const uint32_t*>(&sm.tin[r + 6][lc]);
        const uint32_t c0w = rc[0], c1w = rc[1], c2w = rc[2];
        const uint32_t V = __builtin_amdgcn_alignbyte(c1w, c0w, 3);
        const uint32_t CR = __builtin_amdgcn_alignbyte(c2w, c1w, 2);
        const uint32_t CU = __builtin_amdgcn_alignbyte(ru[1], ru[0], 3);
        const uint32_t CD = __builtin_amdgcn_alignbyte(rd[1], rd[0], 3);
        const uint32_t mb = (y >= 3 && y < h - 3) ? fast_maybe4(V, CD, CR, CU, c0w, t2) : 0u;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int x = x0 + lc + j;
            const bool maybe = ((mb >> j) & 1u) && x >= 3 && x < w - 3;
            const unsigned long long m = __ballot(maybe);
            if (maybe) sm.cand[wave][ncand + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)(r * kLevelTileW + lc + j);
            ncand += __popcll(m);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int k = lane; k < ncand; k += 64) {
        const int q = sm.cand[wave][k];
        const int r = q / kLevelTileW, c = q - r * kLevelTileW;
        const int sc = max(fast_score(&sm.tin[r + 3][c + 3], kTinPitch), 0);
        sm.stile[r][c] = (uint8_t)(sc >= minTh ? sc : 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int rb = wave * 4; rb < kLevelTileH; rb += kLevelThreads / 16) {
        const int r = rb + lr, y = y0 + r;
        if (active && y < h)
            *reinterpret_cast<uint32_t*>(score + (size_t)y * bp + (x0 + lc)) =
                *reinterpret_cast<const uint32_t*>(&sm.stile[r][lc]);
    }
}

// One launch per large level: one tile per workgroup.  XCD-aware order: the hardware deals consecutive
// workgroups round-robin over the 8 XCDs (one L2 each); remapped, every XCD runs whole frames, so the 3-pixel
// halos a tile shares with its neighbours (and the resize's source rows) are fetched into one L2 once instead
// of by up to 8 L2s (PMC: 3-4x the algorithmic reads without the remap, profiles/r04/pmc_levels_*).
__global__ __launch_bounds__(kLevelThreads) void level_kernel(OrbGeom g, int l, int minTh) {
    orb_wave_priority();
    __shared__ LevelLds sm;
    const int nt = gridDim.x, total = nt * gridDim.y;
    const int id = xcd_remap(blockIdx.y * nt + blockIdx.x, total);
    level_tile(g, l, minTh, id / nt, id - (id / nt) * nt, true, threadIdx.x, sm);
}

// The small levels l0 .. nlevels-1 of one frame in one workgroup (no cross-workgroup hand-off): kLevelGroups
// tiles at a time, one per 256-thread group, level after level; a level's image stores are made visible to
// the workgroup (release / acquire at workgroup scope: the same CU's L1) before the next level reads them.
template <int kLevelGroups>
__global__ __launch_bounds__(kLevelThreads * kLevelGroups) void level_small_kernel(OrbGeom g, int l0, int minTh) {
    orb_wave_priority();
    __shared__ LevelLds sm[kLevelGroups];
    const int grp = threadIdx.x / kLevelThreads, t = threadIdx.x % kLevelThreads, f = blockIdx.x;
    for (int l = l0; l < g.nlevels; l++) {
        const int nt = g.level_tiles[l];
        for (int t0 = 0; t0 < nt; t0 += kLevelGroups) {
            const int tile = t0 + grp;
            level_tile(g, l, minTh, f, min(tile, nt - 1), tile < nt, t, sm[grp]);
            __syncthreads();  // this round's LDS reads are over before the next round's writes
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
}

__device__ __forceinline__ int level_of_cell(const OrbGeom& g, int cid) {
    int l = 0;
    for (int k = 1; k < g.nlevels; k++)
        if (cid >= g.lv[k].cell_base) l = k;
    return l;
}

// FAST cells (:789-829): one wave per 30x30 cell, four cells per workgroup.
// The cell window's evaluated pixels come from the score map; 3x3 non-max
// suppression among corners at iniThFAST, retry at minThFAST if the cell came
// back empty.  Candidates are written in the reference's order (row-major
// inside the cell), packed x | y << 12 | score << 24 with (x, y) relative to
// (minBorderX, minBorderY) as at src/ORBextractor.cc:822-823.
constexpr int kCellScoreMax = kCellWinMax - 6;
// The cell's scores live in LDS with a zero frame (one row above and below, one column left, >= 2 right) and a
// row pitch that is a multiple of 4: lane k evaluates the 4 pixels of group k (row-major groups of 4 columns)
// from two aligned dword reads per row (the 3x3 neighbourhoods of 4 adjacent pixels span 6 columns), so
// neither the bounds tests nor a per-pixel division remain; out-of-cell neighbours read the zero frame (the
// reference's n < thr -> 0).  Candidates keep the reference's row-major order: (group, pixel) order.
constexpr int kScPitchMax = ((kCellScoreMax + 3) & ~3) + 4, kScRowsMax = kCellScoreMax + 2;
__global__ __launch_bounds__(256) void fast_cells_kernel(OrbGeom g, uint32_t* __restrict__ cand,
                                                         uint16_t* __restrict__ cand_cnt, int iniTh, int minTh,
                                                         int cid0, int cid1) {  // this launch's cells [cid0, cid1)
    orb_wave_priority();
    __shared__ __attribute__((aligned(16))) uint8_t scs[4][kScRowsMax * kScPitchMax];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // XCD-aware order (as level_kernel): a frame's cells, whose windows overlap by 6 pixels, on one L2
    const int nb = gridDim.x, id = xcd_remap(blockIdx.y * nb + blockIdx.x, nb * gridDim.y);
    const int f = id / nb, cid = cid0 + (id - f * nb) * 4 + wave;
    if (cid >= cid1) return;
    uint8_t* sc = scs[wave];
    const int l = level_of_cell(g, cid);
    const LevelGeom& L = g.lv[l];
    const int local = cid - L.cell_base;
    const int ci = local / L.nCols, cj = local - ci * L.nCols;
    const size_t cell_slot = (size_t)f * g.cells_per_frame + cid;
    uint32_t* out = cand + cell_slot * kCellCap;
    const int iniY = kMinBorder + ci * L.hCell, iniX = kMinBorder + cj * L.wCell;
    if (iniY >= L.maxBorderY - 3 || iniX >= L.maxBorderX - 6) {
        if (lane == 0) cand_cnt[cell_slot] = 0;
        return;
    }
    const int maxY = min(iniY + L.hCell + 6, L.maxBorderY), maxX = min(iniX + L.wCell + 6, L.maxBorderX);
    const int R = maxY - iniY - 6, C = maxX - iniX - 6;
    const int npx = (R > 0 && C > 0) ? R * C : 0;
    const int G = (C + 3) >> 2, P = 4 * G + 4;  // groups per row, LDS row pitch (score column c at byte c + 1)
    const uint8_t* smap = L.score + f * L.blur_frame_stride + (size_t)(iniY + 3) * L.bpitch + (iniX + 3);
    uint32_t* sc32 = reinterpret_cast<uint32_t*>(sc);
    for (int q = lane; q < ((R + 2) * P) >> 2; q += 64) sc32[q] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float invC = 1.f / (float)max(C, 1);   // p / C exactly for p < 2^12
    for (int p0 = 0; p0 < npx; p0 += 256) {
        uint8_t v[4];
        int at[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int p = p0 + lane + 64 * k;
            v[k] = 0;
            at[k] = -1;
            if (p < npx) {
                const int r = (int)(((float)p + 0.5f) * invC), c = p - r * C;
                v[k] = smap[(size_t)r * L.bpitch + c];
                at[k] = (r + 1) * P + c + 1;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (at[k] >= 0) sc[at[k]] = v[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int ngroups = R * G;
    const float invG = 1.f / (float)max(G, 1);
    const unsigned long long lt = (1ull << lane) - 1ull;
    int base = 0;
    for (int pass = 0; pass < 2; pass++) {
        const int thr = pass == 0 ? iniTh : minTh;
        base = 0;
        for (int g0 = 0; g0 < ngroups; g0 += 64) {
            const int gi = g0 + lane;
            int keep[4] = {0, 0, 0, 0}, sv[4] = {0, 0, 0, 0}, r = 0, c0 = 0;
            if (gi < ngroups) {
                r = (int)(((float)gi + 0.5f) * invG);
                c0 = (gi - r * G) * 4;
                int b[3][6];  // rows r-1, r, r+1; score columns c0-1 .. c0+4
#pragma unroll
                for (int y = 0; y < 3; y++) {
                    const uint32_t* rowp = reinterpret_cast<const uint32_t*>(sc + (r + y) * P + c0);
                    const uint32_t lo = rowp[0], hi = rowp[1];
#pragma unroll
                    for (int k = 0; k < 6; k++) b[y][k] = (int)(((k < 4 ? lo : hi) >> (8 * (k & 3))) & 255u);
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int s = b[1][j + 1];
                    sv[j] = s;
                    bool k = s >= thr && c0 + j < C;
#pragma unroll
                    for (int y = 0; y < 3; y++)
#pragma unroll
                        for (int x = 0; x < 3; x++) {
                            if (y == 1 && x == 1) continue;
                            const int n = b[y][j + x];
                            k = k && (n < thr || s > n);
                        }
                    keep[j] = k;
                }
            }
            unsigned long long m[4];
            int before = 0, total = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                m[j] = __ballot(keep[j]);
                before += __popcll(m[j] & lt);
                total += __popcll(m[j]);
            }
            int pos = base + before;
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (keep[j]) {
                    out[pos++] = (uint32_t)(c0 + j + 3 + cj * L.wCell) | ((uint32_t)(r + 3 + ci * L.hCell) << 12) |
                                 ((uint32_t)sv[j] << 24);
                }
            base += total;
        }
        if (base > 0) break;
    }
    if (lane == 0) cand_cnt[cell_slot] = (uint16_t)base;
}

// ---------------------------------------------------------------------------
// DistributeOctTree (src/ORBextractor.cc:539-763) for one (frame, level) per
// 256-thread workgroup.
//
// The reference walks a std::list, dividing nodes one at a time.  All
// divisions of one main-loop pass are independent, so a pass is done as: one
// sweep over the keys counting each divided node's four children (atomics in
// LDS), block scans that place every child where the reference's push_front
// sequence would put it, and one sweep re-pointing each key at its new node.
// The node table always *is* the list (entry i = i-th list element).  The
// final phase (:673-737) sorts the expandable nodes by (size, creation
// sequence) -- the creation sequence stands in for the reference's pointer
// tie-break, see DESIGN.md -- and finds the division after which the list
// reaches N with one scan instead of one division at a time.
constexpr int kFlagNoMore = 1, kFlagToExp = 2;

// NC = node capacity: the list never exceeds the level's kp_cap (N + 16; the main loop only runs a
// pass when L + 3 * nToExpand <= N, the final phase stops at >= N), so the launcher picks the
// smallest instance that holds every level -- 256 for nFeatures = 1000 (25 KB of LDS, 6 workgroups
// per CU) instead of 1024 (77 KB, 2 per CU).
template <int NC>
struct OctShared {
    short x0[2][NC], y0[2][NC], x1[2][NC], y1[2][NC];
    int cnt[2][NC];
    int seq[2][NC];
    uint8_t flags[2][NC];
    uint8_t div[NC];
    alignas(8) int c4[NC][4];  // child counts, then child positions (-1 = empty); at the end the retained keys
    int sa[NC];      // scan scratch
    int sb[NC];      // scan scratch / remap
    int sc[NC];      // scan scratch / sort
    int cand[NC];
    int cellpre[2048];
    int wsum[4];
    int misc[8];
};

// Exclusive scan of a[0..n) in place (n <= 2048), returns the total.
__device__ int block_scan(int* a, int n, int* wsum) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int v[8], local = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int i = 8 * t + k;
        v[k] = i < n ? a[i] : 0;
        local += v[k];
    }
    int x = local;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int wbase = 0;
    for (int j = 0; j < w; j++) wbase += wsum[j];
    const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    int run = wbase + x - local;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int i = 8 * t + k;
        if (i < n) a[i] = run;
        run += v[k];
    }
    __syncthreads();
    return total;
}

__device__ __forceinline__ int quadrant(int kx, int ky, int x0, int y0, int x1, int y1) {
    const int hx = (int)ceilf((float)(x1 - x0) / 2), hy = (int)ceilf((float)(y1 - y0) / 2);
    const bool left = kx < x0 + hx, top = ky < y0 + hy;
    return left ? (top ? 0 : 2) : (top ? 1 : 3);
}

__device__ __forceinline__ void child_rect(int q, int x0, int y0, int x1, int y1, short& cx0, short& cy0, short& cx1,
                                           short& cy1) {
    const int hx = (int)ceilf((float)(x1 - x0) / 2), hy = (int)ceilf((float)(y1 - y0) / 2);
    cx0 = (short)((q & 1) ? x0 + hx : x0);
    cx1 = (short)((q & 1) ? x1 : x0 + hx);
    cy0 = (short)((q & 2) ? y0 + hy : y0);
    cy1 = (short)((q & 2) ? y1 : y0 + hy);
}

// Where the level's keys live between the passes.  A pass touches every key (its node, and for a divided node
// its quadrant), and there are ~6-10 passes per level, so the keys stay on chip when they fit: RegKeys holds
// KPT keys per thread in registers (key k = threadIdx.x + 256 j, its node index packed 4 per register);
// GlobalKeys is the fallback for levels with more than 256 * KPT candidates (and for the 1024-node instance):
// the keys gathered once into global scratch, their node indices beside them, a node index written only when
// it changes.  Both visit every key once per call, in any order: the passes only count (LDS atomics) and
// re-point keys, and the final retain orders by key index k.
struct GlobalKeys {
    const uint32_t* keys;
    uint16_t* node;
    int C;
    template <class F>
    __device__ __forceinline__ void each(F&& f) {
        for (int k = threadIdx.x; k < C; k += 256) {
            int n = node[k];
            const int n0 = n;
            f(keys[k], k, n);
            if (n != n0) node[k] = (uint16_t)n;
        }
    }
};

template <int KPT>
struct RegKeys {
    uint32_t key[KPT];
    uint32_t nodew[(KPT + 3) / 4];
    int C;
    template <class F>
    __device__ __forceinline__ void each(F&& f) {
        const int t = threadIdx.x;
#pragma unroll
        for (int j = 0; j < KPT; j++) {
            const int k = t + 256 * j;
            if (k >= C) break;
            const int sh = 8 * (j & 3);
            // opaque per visit: otherwise the compiler hoists each key's x / y fields (and unpacked node bytes)
            // out of the pass loop, ~3 registers per key instead of 1.25
            uint32_t kv = key[j];
            asm volatile("" : "+v"(kv));
            int n = (int)((nodew[j >> 2] >> sh) & 0xFFu);
            f(kv, k, n);
            nodew[j >> 2] = (nodew[j >> 2] & ~(0xFFu << sh)) | ((uint32_t)n << sh);
        }
    }
};

// Rebuild the list after dividing the nodes flagged in S.div (proc rank of a
// divided node in S.sb[node] = position in division order, P_c prefix in
// S.sa[node]).  T = number of children pushed.  Returns the new length.
template <int NC, class KS>
__device__ __forceinline__ int rebuild_list(OctShared<NC>& S, int cur, int L, int T, int seqc, KS& ks) {
    const int nb = cur ^ 1;
    // rank of non-divided nodes in list order
    for (int i = threadIdx.x; i < L; i += 256) S.sc[i] = S.div[i] ? 0 : 1;
    __syncthreads();
    const int ND = block_scan(S.sc, L, S.wsum);
    for (int i = threadIdx.x; i < L; i += 256) {
        if (S.div[i]) {
            const int pc = S.sa[i];
            int r = 0;
            for (int q = 0; q < 4; q++) {
                const int n = S.c4[i][q];
                if (n > 0) {
                    const int pos = T - pc - 1 - r;
                    short a, b, c, d;
                    child_rect(q, S.x0[cur][i], S.y0[cur][i], S.x1[cur][i], S.y1[cur][i], a, b, c, d);
                    S.x0[nb][pos] = a; S.y0[nb][pos] = b; S.x1[nb][pos] = c; S.y1[nb][pos] = d;
                    S.cnt[nb][pos] = n;
                    S.seq[nb][pos] = seqc + pc + r;
                    S.flags[nb][pos] = (uint8_t)((n == 1 ? kFlagNoMore : 0) | (n > 1 ? kFlagToExp : 0));
                    S.c4[i][q] = pos;
                    r++;
                } else {
                    S.c4[i][q] = -1;
                }
            }
        } else {
            const int pos = T + S.sc[i];
            S.x0[nb][pos] = S.x0[cur][i]; S.y0[nb][pos] = S.y0[cur][i];
            S.x1[nb][pos] = S.x1[cur][i]; S.y1[nb][pos] = S.y1[cur][i];
            S.cnt[nb][pos] = S.cnt[cur][i];
            S.seq[nb][pos] = S.seq[cur][i];
            S.flags[nb][pos] = (uint8_t)(S.flags[cur][i] & kFlagNoMore);
            S.sb[i] = pos;
        }
    }
    __syncthreads();
    ks.each([&](uint32_t key, int, int& n) {
        if (S.div[n]) {
            const int q = quadrant(key & 0xFFF, (key >> 12) & 0xFFF, S.x0[cur][n], S.y0[cur][n], S.x1[cur][n],
                                   S.y1[cur][n]);
            n = S.c4[n][q];
        } else {
            n = S.sb[n];
        }
    });
    __syncthreads();
    return T + ND;
}

// Count the four children of every node with S.div set.
template <int NC, class KS>
__device__ __forceinline__ void count_children(OctShared<NC>& S, int cur, int L, KS& ks) {
    for (int i = threadIdx.x; i < L; i += 256) S.c4[i][0] = S.c4[i][1] = S.c4[i][2] = S.c4[i][3] = 0;
    __syncthreads();
    ks.each([&](uint32_t key, int, int& n) {
        if (S.div[n]) {
            const int q = quadrant(key & 0xFFF, (key >> 12) & 0xFFF, S.x0[cur][n], S.y0[cur][n], S.x1[cur][n],
                                   S.y1[cur][n]);
            atomicAdd(&S.c4[n][q], 1);
        }
    });
    __syncthreads();
}

// The level's tree from its keys (initial nodes, main-loop passes, final phase, retained keys).
template <int NC, class KS>
__device__ __forceinline__ void octree_body(OctShared<NC>& S, KS& ks, const LevelGeom& Lg, LevelKp* __restrict__ out,
                                            int* __restrict__ out_cnt) {
    const int t = threadIdx.x;
    // --- initial nodes (:542-585)
    const int minX = kMinBorder, maxX = Lg.maxBorderX, minY = kMinBorder, maxY = Lg.maxBorderY;
    const int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    int cur = 0;
    if (t < 4 * nIni) S.sa[t] = 0;
    __syncthreads();
    ks.each([&](uint32_t key, int, int& n) {
        n = (int)((float)(key & 0xFFF) / hX);
        atomicAdd(&S.sa[n], 1);
    });
    __syncthreads();
    if (t == 0) {
        int L = 0;
        for (int i = 0; i < nIni; i++) {
            S.sb[i] = -1;
            if (S.sa[i] == 0) continue;
            S.x0[0][L] = (short)(int)(hX * (float)i); S.y0[0][L] = 0;
            S.x1[0][L] = (short)(int)(hX * (float)(i + 1)); S.y1[0][L] = (short)(maxY - minY);
            S.cnt[0][L] = S.sa[i];
            S.seq[0][L] = i;
            S.flags[0][L] = (uint8_t)(S.sa[i] == 1 ? kFlagNoMore : 0);
            S.sb[i] = L++;
        }
        S.misc[0] = L;
    }
    __syncthreads();
    int L = S.misc[0];
    ks.each([&](uint32_t, int, int& n) { n = S.sb[n]; });
    __syncthreads();
    int seqc = nIni;
    const int N = Lg.nfeat;

    bool finish = (L == 0);
    while (!finish) {
        // ---- main-loop pass (:596-665): divide every node that is not bNoMore
        const int prevSize = L;
        for (int i = t; i < L; i += 256) S.div[i] = (S.flags[cur][i] & kFlagNoMore) ? 0 : 1;
        __syncthreads();
        count_children(S, cur, L, ks);
        for (int i = t; i < L; i += 256) {
            int nc = 0, nm = 0;
            if (S.div[i])
                for (int q = 0; q < 4; q++) { nc += S.c4[i][q] > 0; nm += S.c4[i][q] > 1; }
            S.sa[i] = nc;
            S.sb[i] = nm;
        }
        __syncthreads();
        const int nToExpand = block_scan(S.sb, L, S.wsum);
        const int T = block_scan(S.sa, L, S.wsum);
        L = rebuild_list(S, cur, L, T, seqc, ks);
        seqc += T;
        cur ^= 1;
        if (L >= N || L == prevSize) {
            finish = true;
        } else if (L + nToExpand * 3 > N) {
            // ---- final phase (:673-737)
            while (!finish) {
                const int prev2 = L;
                // candidates = nodes pushed last step with > 1 key
                for (int i = t; i < L; i += 256) S.sc[i] = (S.flags[cur][i] & kFlagToExp) ? 1 : 0;
                __syncthreads();
                const int M = block_scan(S.sc, L, S.wsum);
                for (int i = t; i < L; i += 256)
                    if (S.flags[cur][i] & kFlagToExp) S.cand[S.sc[i]] = i;
                __syncthreads();
                // processing rank: descending (size, seq)
                for (int a = t; a < M; a += 256) {
                    const int ia = S.cand[a], ca = S.cnt[cur][ia], sa = S.seq[cur][ia];
                    int rank = 0;
                    for (int b = 0; b < M; b++) {
                        const int ib = S.cand[b], cb = S.cnt[cur][ib], sb = S.seq[cur][ib];
                        rank += (cb < ca) || (cb == ca && sb < sa);
                    }
                    S.sc[M - 1 - rank] = ia;  // sc[p] = node processed p-th
                }
                for (int i = t; i < L; i += 256) S.div[i] = (S.flags[cur][i] & kFlagToExp) ? 1 : 0;
                __syncthreads();
                count_children(S, cur, L, ks);
                // deltas in processing order
                for (int p = t; p < M; p += 256) {
                    const int i = S.sc[p];
                    int nc = 0;
                    for (int q = 0; q < 4; q++) nc += S.c4[i][q] > 0;
                    S.sa[p] = nc - 1;
                    S.cand[p] = nc;
                }
                if (t == 0) S.misc[1] = M - 1;
                __syncthreads();
                block_scan(S.sa, M, S.wsum);  // exclusive prefix of deltas
                for (int p = t; p < M; p += 256)
                    if (L + S.sa[p] + (S.cand[p] - 1) >= N) atomicMin(&S.misc[1], p);
                __syncthreads();
                const int kstar = S.misc[1];
                // divided = first kstar+1 in processing order; P_c over processing order
                for (int i = t; i < L; i += 256) S.div[i] = 0;
                __syncthreads();
                for (int p = t; p < M; p += 256) {
                    S.sa[p] = p <= kstar ? S.cand[p] : 0;
                    if (p <= kstar) S.div[S.sc[p]] = 1;
                }
                __syncthreads();
                const int T2 = block_scan(S.sa, M, S.wsum);
                // move P_c from processing slot to node slot (sb is free here)
                for (int p = t; p <= kstar; p += 256) S.sb[S.sc[p]] = S.sa[p];
                __syncthreads();
                for (int i = t; i < L; i += 256)
                    if (S.div[i]) S.sa[i] = S.sb[i];
                __syncthreads();
                L = rebuild_list(S, cur, L, T2, seqc, ks);
                seqc += T2;
                cur ^= 1;
                if (L >= N || L == prev2) finish = true;
            }
        }
    }

    // --- retain the best key of each node (:741-760): the first maximum response in key order, i.e. the maximum
    // of (response, -k); the key itself rides in the low word (the child-count table is free here)
    unsigned long long* best = reinterpret_cast<unsigned long long*>(&S.c4[0][0]);
    for (int i = t; i < L; i += 256) best[i] = 0;
    __syncthreads();
    ks.each([&](uint32_t key, int k, int& n) {
        const unsigned long long v = ((unsigned long long)(key >> 24) << 55) |
                                     ((unsigned long long)(0x7FFFFF - k) << 32) | key;
        atomicMax(&best[n], v);
    });
    __syncthreads();
    const int nout = min(L, Lg.kp_cap);
    for (int i = t; i < nout; i += 256) {
        const uint32_t key = (uint32_t)best[i];
        LevelKp kp;
        kp.x = (uint16_t)((key & 0xFFF) + minX);
        kp.y = (uint16_t)(((key >> 12) & 0xFFF) + minY);
        kp.response = (uint16_t)(key >> 24);
        kp.pad = 0;
        out[i] = kp;
    }
    if (t == 0) *out_cnt = nout;
}

// Keys per thread held in registers (the 256-node instance): 40 covers the C2-C4 levels (level 0 of a
// 640x480 frame has ~9K FAST candidates); a level with more keys takes the global path
#ifndef SPSLAM_OCT_KPT
#define SPSLAM_OCT_KPT 40
#endif

template <int NC, int KPT>
__global__ __launch_bounds__(256) void octree_kernel(OrbGeom g, const uint32_t* __restrict__ cand,
                                                     const uint16_t* __restrict__ cand_cnt, uint32_t* __restrict__ keys_all,
                                                     uint16_t* __restrict__ keynode_all, LevelKp* __restrict__ lvl_kp,
                                                     int* __restrict__ lvl_cnt, int l0) {  // levels l0 + blockIdx.x
    orb_wave_priority();
    __shared__ OctShared<NC> S;
    const int l = l0 + blockIdx.x, f = blockIdx.y, t = threadIdx.x;
    const LevelGeom& Lg = g.lv[l];
    const int ncells = Lg.nRows * Lg.nCols;
    const size_t cell0 = (size_t)f * g.cells_per_frame + Lg.cell_base;
    LevelKp* out = lvl_kp + (size_t)f * g.lvl_kp_per_frame + Lg.kp_base;
    int* out_cnt = lvl_cnt + f * kMaxLevels + l;

    // --- candidates in cell order (vToDistributeKeys, :818-826): key k of the level = entry k - cellpre[c] of the
    // cell c holding it
    for (int c = t; c < ncells; c += 256) S.cellpre[c] = cand_cnt[cell0 + c];
    __syncthreads();
    const int C = block_scan(S.cellpre, ncells, S.wsum);
    if constexpr (KPT > 0) {
        static_assert(NC <= 256, "node indices are packed as bytes");
        if (C <= 256 * KPT) {
            RegKeys<KPT> ks;
            ks.C = C;
#pragma unroll
            for (int j = 0; j < KPT; j++) {
                const int k = t + 256 * j;
                ks.key[j] = 0;
                if (k < C) {  // the cell holding key k: the last c with cellpre[c] <= k (empty cells share prefixes)
                    int lo = 0, hi = ncells - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (S.cellpre[mid] <= k) lo = mid; else hi = mid - 1;
                    }
                    ks.key[j] = cand[(cell0 + lo) * kCellCap + (k - S.cellpre[lo])];
                }
            }
#pragma unroll
            for (int j = 0; j < (KPT + 3) / 4; j++) ks.nodew[j] = 0;
            octree_body(S, ks, Lg, out, out_cnt);
            return;
        }
    }
    GlobalKeys ks;
    ks.keys = keys_all + (size_t)f * g.keys_per_frame + Lg.key_base;
    ks.node = keynode_all + (size_t)f * g.keys_per_frame + Lg.key_base;
    ks.C = C;
    uint32_t* keys = keys_all + (size_t)f * g.keys_per_frame + Lg.key_base;
    for (int c = t >> 6; c < ncells; c += 4) {
        const int n = (int)cand_cnt[cell0 + c], o = S.cellpre[c];
        const uint32_t* src = cand + (cell0 + c) * kCellCap;
        for (int j = t & 63; j < n; j += 64) keys[o + j] = src[j];
    }
    __threadfence_block();
    __syncthreads();
    octree_body(S, ks, Lg, out, out_cnt);
}

// ---------------------------------------------------------------------------
// glibc sinf/cosf (|y| < 120) restated; bit-identical to the system libm the
// reference calls at src/ORBextractor.cc:113 over all ORB angles.
struct SinCosT { double sign[4]; double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3; };
__constant__ SinCosT c_sincos[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
__device__ __forceinline__ uint32_t abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }
__device__ __forceinline__ float sincos_poly(double x, double x2, const SinCosT* p, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2, s1 = p->s2 + x2 * p->s3, x7 = x3 * x2, s = x + x3 * p->s1;
        return (float)(s + x7 * s1);
    }
    const double x4 = x2 * x2, c2 = p->c3 + x2 * p->c4, c1 = p->c0 + x2 * p->c1, x6 = x4 * x2, c = c1 + x4 * p->c2;
    return (float)(c + x6 * c2);
}
__device__ void glibc_sincosf(float y, float* sn, float* cs) {
    const double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) { *sn = y; *cs = 1.0f; return; }
        *sn = sincos_poly(x, x * x, &c_sincos[0], 0);
        *cs = sincos_poly(x, x * x, &c_sincos[0], 1);
        return;
    }
    const double r = x * c_sincos[0].hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    const double xr = x - n * c_sincos[0].hpi;
    const double s = c_sincos[0].sign[n & 3];
    const SinCosT* p = (n & 2) ? &c_sincos[1] : &c_sincos[0];
    *sn = sincos_poly(xr * s, xr * xr, p, n);
    *cs = sincos_poly(xr * s, xr * xr, p, n ^ 1);
}

// OpenCV cv::fastAtan2 (degrees).
__device__ float fast_atan2(float y, float x) {
    const float k = (float)(180 / M_PI);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k, p5 = 0.1555786518463281f * k,
                p7 = -0.04432655554792128f * k;
    const float eps = (float)2.220446049250313e-16;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps); c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps); c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// One wave per keypoint slot: orientation on the level image, rotated BRIEF
// on the blurred level, final scaling/placement in reference order.
__global__ __launch_bounds__(256) void desc_kernel(OrbGeom g, const LevelKp* __restrict__ lvl_kp,
                                                   const int* __restrict__ lvl_cnt, spslam_keypoint* __restrict__ out_kp,
                                                   uint8_t* __restrict__ out_desc, int* __restrict__ out_cnt,
                                                   int cap_per_frame) {
    orb_wave_priority();
    // 1-D launch of gx * frames workgroups in XCD-aware order: one frame's keypoints (and its level
    // images / blurred levels, ~1.9 MB at 640x480) stay on one XCD's L2
    const int gx = (g.lvl_kp_per_frame + 3) / 4;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int f = lid / gx, lane = threadIdx.x & 63;
    const int slot = (lid - f * gx) * 4 + (threadIdx.x >> 6);
    if (slot >= g.lvl_kp_per_frame) return;
    int l = 0;
    for (int k = 1; k < g.nlevels; k++)
        if (slot >= g.lv[k].kp_base) l = k;
    const LevelGeom& L = g.lv[l];
    const int i = slot - L.kp_base;
    const int* cnt = lvl_cnt + f * kMaxLevels;
    int off = 0, total = 0;
    for (int k = 0; k < g.nlevels; k++) {
        if (k < l) off += cnt[k];
        total += cnt[k];
    }
    if (slot == 0 && lane == 0) out_cnt[f] = min(total, cap_per_frame);
    if (i >= cnt[l] || off + i >= cap_per_frame) return;
    const LevelKp kp = lvl_kp[(size_t)f * g.lvl_kp_per_frame + slot];
    // IC_Angle (:77-104) on the un-blurred level
    const uint8_t* img = L.img + f * L.frame_stride;
    const int P = L.stride;
    const uint8_t* center = img + (size_t)kp.y * P + kp.x;
    int m10 = 0, m01 = 0;
    if (lane < 31) {
        const int u = lane - 15;
        m10 = u * center[u];
        for (int v = 1; v <= 15; v++) {
            if (abs(u) > c_umax[v]) continue;
            const int vp = center[u + v * P], vm = center[u - v * P];
            m01 += v * (vp - vm);
            m10 += u * (vp + vm);
        }
    }
#pragma unroll
    for (int off2 = 32; off2 >= 1; off2 >>= 1) {
        m10 += __shfl_xor(m10, off2);
        m01 += __shfl_xor(m01, off2);
    }
    const float angle = fast_atan2((float)m01, (float)m10);
    // rotated BRIEF (:107-147) on the blurred level
    const float factorPI = (float)(M_PI / 180.f);
    float sb, ca;
    glibc_sincosf(angle * factorPI, &sb, &ca);
    const uint8_t* bimg = L.blur + f * L.blur_frame_stride;
    const uint8_t* bc = bimg + (size_t)kp.y * L.bpitch + kp.x;
    const size_t o = (size_t)f * cap_per_frame + off + i;
    uint64_t* dd = reinterpret_cast<uint64_t*>(out_desc + o * 32);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int tst = lane + 64 * k;
        int val[2];
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const float x = (float)c_pattern[4 * tst + 2 * e], y = (float)c_pattern[4 * tst + 2 * e + 1];
            const int r = cv_round(__builtin_fmaf(x, sb, y * ca));
            const int c = cv_round(__builtin_fmaf(x, ca, -(y * sb)));
            val[e] = bc[r * L.bpitch + c];
        }
        const unsigned long long m = __ballot(val[0] < val[1]);
        if (lane == 0) dd[k] = m;
    }
    if (lane == 0) {
        spslam_keypoint r;
        float x = (float)kp.x, y = (float)kp.y;
        if (l != 0) { x = x * L.scale; y = y * L.scale; }
        r.x = x; r.y = y;
        r.size = (float)L.patch_size;
        r.angle = angle;
        r.response = (float)kp.response;
        r.octave = l;
        r.class_id = -1;
        out_kp[o] = r;
    }
}

}  // namespace spslam

// ---------------------------------------------------------------------------
// Host-side launchers (called from spslam_capi.cpp).
namespace spslam {

// levels fused into level_small_kernel (SPSLAM_ORB_SMALL_LEVELS=1): the smallest ones whose tiles fit this
// budget per frame (640x480: L4-L7, 114 tiles, 180K px).  Off by default: one launch per level measured 38.8K
// against 37.0K frames/s on the pipelined C2 step (profiles/r04/ab_small_levels.txt) -- the fused kernel's
// 256 workgroups serialise four levels that the per-level launches spread over the whole chip.
constexpr int kSmallLevelTiles = 128;
static bool small_levels_off() {
    static const bool off = [] {
        const char* e = getenv("SPSLAM_ORB_SMALL_LEVELS");
        return !(e && e[0] == '1');
    }();
    return off;
}
// tile groups per level_small_kernel workgroup: 4 (1024 threads, default) or 2 (SPSLAM_ORB_SMALL_GROUPS=2)
static int small_level_groups() {
    static const int n = [] {
        const char* e = getenv("SPSLAM_ORB_SMALL_GROUPS");
        return e && e[0] == '2' ? 2 : 4;
    }();
    return n;
}

hipError_t orb_upload_tables(const int umax[16]) {
    return hipMemcpyToSymbol(HIP_SYMBOL(c_umax), umax, 16 * sizeof(int));
}



// Enqueue the whole ORB pass for n frames on `s`.  g.lv[0].img/stride/
// frame_stride must already point at the caller's gray frames.
const char* kernel_kind_name(int kind) {
    static const char* names[kNumKernelKinds] = {"level_kernel", "fast_cells_kernel", "octree_kernel",
                                                 "desc_kernel", "pose_kernel", "plane_cloud_kernel", "plane_dist_integral_kernel",
                                                 "plane_integral_kernel (fused)", "plane_normal_kernel",
                                                 "plane_segment_kernel", "supp_lines_kernel",
                                                 "supp_assemble_kernel", "frame_rgbd_kernel",
                                                 "lba_batch", "plane_assoc_kernel", "search_projection",
                                                 "search_local_points", "track_graph_kernel", "grab_rgbd_kernel",
                                                 "bow_words_kernel", "bow_vectors_kernel", "bow_search_kernel"};
    return kind >= 0 && kind < kNumKernelKinds ? names[kind] : "?";
}

// the small levels' chain on orb_launch's second stream (SPSLAM_ORB_SPLIT=1): off by default -- 39.5K against
// 40.0K frames/s on the pipelined C2 step (profiles/r04/ab_orb_split.txt): the small levels' launches wait for
// CUs inside the step on either stream, and the second chain only adds contention
static bool orb_split_off() {
    static const bool off = [] {
        const char* e = getenv("SPSLAM_ORB_SPLIT");
        return !(e && e[0] == '1');
    }();
    return off;
}

hipError_t orb_launch(const OrbGeom& g, const OrbBuffers& b, int n, int iniTh, int minTh, spslam_keypoint* kps,
                      uint8_t* desc, int* counts, int cap_per_frame, hipStream_t s, KernelTimer* timer,
                      hipStream_t aux, hipEvent_t ev_fork, hipEvent_t ev_join) {
    auto B = [&](int k) { if (timer) timer->begin(k, s); };
    auto E = [&](int k) { if (timer) timer->end(k, s); };
    // the small levels (at most kSmallLevelTiles tiles per frame together): levels ls .. nlevels - 1
    int ls = g.nlevels, tiles = 0;
    while (ls > 1 && tiles + g.level_tiles[ls - 1] <= kSmallLevelTiles) tiles += g.level_tiles[--ls];
    if (g.nlevels - ls < 2) ls = g.nlevels;
    int maxcap = 0;
    for (int l = 0; l < g.nlevels; l++) maxcap = max(maxcap, g.lv[l].kp_cap);
    auto* octree = maxcap <= 256 ? octree_kernel<256, SPSLAM_OCT_KPT> : octree_kernel<kNodeCap, 0>;
    auto fast = [&](int la, int lb, hipStream_t st) {
        const int c0 = g.lv[la].cell_base, c1 = lb < g.nlevels ? g.lv[lb].cell_base : g.cells_per_frame;
        hipLaunchKernelGGL(fast_cells_kernel, dim3((c1 - c0 + 3) / 4, n), dim3(256), 0, st, g, b.cand, b.cand_cnt,
                           iniTh, minTh, c0, c1);
    };
    auto tree = [&](int la, int lb, hipStream_t st) {
        hipLaunchKernelGGL(octree, dim3(lb - la, n), dim3(256), 0, st, g, b.cand, b.cand_cnt, b.keys, b.keynode,
                           b.lvl_kp, b.lvl_cnt, la);
    };
    auto level = [&](int l, hipStream_t st) {
        hipLaunchKernelGGL(level_kernel, dim3(g.level_tiles[l], n), dim3(kLevelThreads), 0, st, g, l,
                           min(iniTh, minTh));
    };
    if (aux && ev_fork && ev_join && ls < g.nlevels && !orb_split_off() && small_levels_off()) {
        // Two chains from level ls - 1 on: the small levels, their FAST cells and their octrees on `aux`; the large
        // levels' cells and octrees on `s` meanwhile; the descriptors (every level's keypoints) after both.  The
        // small levels' launches are short but wait for CUs inside the pipelined step; off the caller's stream
        // they no longer lengthen its chain.  (Timed: the caller's stream's part.)
        B(kKindLevel);
        for (int l = 0; l < ls; l++) level(l, s);
        E(kKindLevel);
        hipError_t e = hipEventRecord(ev_fork, s);
        if (e == hipSuccess) e = hipStreamWaitEvent(aux, ev_fork, 0);
        if (e != hipSuccess) return e;
        for (int l = ls; l < g.nlevels; l++) level(l, aux);
        fast(ls, g.nlevels, aux);
        tree(ls, g.nlevels, aux);
        e = hipEventRecord(ev_join, aux);
        if (e != hipSuccess) return e;
        B(kKindFast);
        fast(0, ls, s);
        E(kKindFast);
        B(kKindOctree);
        tree(0, ls, s);
        E(kKindOctree);
        e = hipStreamWaitEvent(s, ev_join, 0);
        if (e != hipSuccess) return e;
    } else {
        B(kKindLevel);
        const int l0 = small_levels_off() ? g.nlevels : ls;  // SPSLAM_ORB_SMALL_LEVELS=1: one fused launch
        for (int l = 0; l < l0; l++) level(l, s);
        if (l0 < g.nlevels) {
            if (small_level_groups() == 2)
                hipLaunchKernelGGL(level_small_kernel<2>, dim3(n), dim3(kLevelThreads * 2), 0, s, g, l0, min(iniTh, minTh));
            else
                hipLaunchKernelGGL(level_small_kernel<4>, dim3(n), dim3(kLevelThreads * 4), 0, s, g, l0, min(iniTh, minTh));
        }
        E(kKindLevel);
        B(kKindFast);
        fast(0, g.nlevels, s);
        E(kKindFast);
        B(kKindOctree);
        tree(0, g.nlevels, s);
        E(kKindOctree);
    }
    B(kKindDesc);
    hipLaunchKernelGGL(desc_kernel, dim3((g.lvl_kp_per_frame + 3) / 4 * n), dim3(256), 0, s, g, b.lvl_kp, b.lvl_cnt,
                       kps, desc, counts, cap_per_frame);
    E(kKindDesc);
    return hipGetLastError();
}

}  // namespace spslam
