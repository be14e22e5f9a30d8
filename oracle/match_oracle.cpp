// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// CPU restatement of the matching step between Frame construction and
// PoseOptimization in Tracking::TrackWithMotionModel (src/Tracking.cc:949-980):
//   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
//                                        (src/ORBmatcher.cc:1328-1470)
//   Frame::GetFeaturesInArea             (src/Frame.cc:427-480)
//   ORBmatcher::DescriptorDistance       (src/ORBmatcher.cc:1647-1662)
//   ORBmatcher::ComputeThreeMaxima       (src/ORBmatcher.cc:1601-1642)
// with the caller's retry (`nmatches < 20` -> clear, search again at 2*th,
// src/Tracking.cc:968-975).  The last frame's map points are given as a list
// of the keypoints i with mvpMapPoints[i] && !mvbOutlier[i], in increasing i.
//
// FP: cv::Mat float products (Rcw*x3Dw + tcw, -Rcw^T*tcw, Rlw*twc + tlw) are
// accumulated in double and rounded once (OpenCV's GEMM for float; OpenCV is
// absent here, so this rounding is parity-unpinned).  Float
// expressions follow the reference build's GCC -O3 -march=native contraction
// (u = fma(fx*xc, invzc, cx), ur = fma(-mbf, invzc, u)).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace oracle {
namespace match {

constexpr int kCols = 64, kRows = 48, kHisto = 30, kThHigh = 100;

struct ProjPoint {  // spslam_proj_point
    float xw[3];
    float angle;
    int32_t octave, n_obs, last_index, id;
    uint8_t desc[32];
};
struct ProjFrame {  // spslam_proj_frame
    float Tcw[16];
    float Tlw[16];
    int32_t point_offset, n_points, seen_offset, stamp;
};
struct Keypoint {  // spslam_keypoint
    float x, y, size, angle, response;
    int32_t octave, class_id;
};
struct Geometry {
    float fx, fy, cx, cy, bf;
    float min_x, max_x, min_y, max_y, ginv_x, ginv_y;
    float scale[8];
};
struct Params {
    float th;
    int32_t mono, check_orientation, retry_below;
};

int descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int w = 0; w < 8; w++) {
        uint32_t x, y;
        std::memcpy(&x, a + 4 * w, 4);
        std::memcpy(&y, b + 4 * w, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

// y = A x (+ c) for a 3x3 block of a row-major 4x4 float matrix, double accumulation, one rounding
void mat3_mul(const float* T, const float* x, const float* c, bool transpose, float sign, float* y) {
    for (int r = 0; r < 3; r++) {
        double s = 0.0;
        for (int k = 0; k < 3; k++) s += (double)(transpose ? T[4 * k + r] : T[4 * r + k]) * (double)x[k];
        s *= sign;
        if (c) s += (double)c[r];
        y[r] = (float)s;
    }
}

struct Current {
    const Keypoint* kun;
    const uint8_t* desc;
    const float* uright;
    const int32_t* grid_off;
    const int32_t* grid_idx;
    int n;
};

// Frame::GetFeaturesInArea over the CSR grid (cell (ix, iy) = ix * 48 + iy)
void features_in_area(const Current& F, const Geometry& G, float x, float y, float r, int minLevel, int maxLevel,
                      std::vector<int>& out) {
    out.clear();
    const int nMinCellX = std::max(0, (int)std::floor((x - G.min_x - r) * G.ginv_x));
    if (nMinCellX >= kCols) return;
    const int nMaxCellX = std::min(kCols - 1, (int)std::ceil((x - G.min_x + r) * G.ginv_x));
    if (nMaxCellX < 0) return;
    const int nMinCellY = std::max(0, (int)std::floor((y - G.min_y - r) * G.ginv_y));
    if (nMinCellY >= kRows) return;
    const int nMaxCellY = std::min(kRows - 1, (int)std::ceil((y - G.min_y + r) * G.ginv_y));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const int c = ix * kRows + iy;
            for (int j = F.grid_off[c]; j < F.grid_off[c + 1]; j++) {
                const int k = F.grid_idx[j];
                const Keypoint& kp = F.kun[k];
                if (bCheckLevels) {
                    if (kp.octave < minLevel) continue;
                    if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                }
                const float distx = kp.x - x, disty = kp.y - y;
                if (std::fabs(distx) < r && std::fabs(disty) < r) out.push_back(k);
            }
        }
}

void compute_three_maxima(const int* histo, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < kHisto; i++) {
        const int s = histo[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
}

// One SearchByProjection(CurrentFrame, LastFrame, th, bMono).  match[k]: index into P of the map point
// assigned to current keypoint k (mvpMapPoints), -1 if none; blocking[k]: that map point has observations.
int search_once(const ProjFrame& fr, const ProjPoint* P, const Current& F, const Geometry& G, float th, bool mono,
                bool check_ori, int32_t* match) {
    std::vector<uint8_t> blocking(F.n, 0);
    for (int k = 0; k < F.n; k++) match[k] = -1;
    std::vector<int> rotHist[kHisto];
    const float factor = 1.0f / kHisto;
    float twc[3], tlc[3];
    const float tcw[3] = {fr.Tcw[3], fr.Tcw[7], fr.Tcw[11]};
    const float tlw[3] = {fr.Tlw[3], fr.Tlw[7], fr.Tlw[11]};
    mat3_mul(fr.Tcw, tcw, nullptr, true, -1.0f, twc);  // -Rcw^T tcw
    mat3_mul(fr.Tlw, twc, tlw, false, 1.0f, tlc);       // Rlw twc + tlw
    const float mb = G.bf / G.fx;                       // Frame::mb = mbf / fx
    const bool bForward = tlc[2] > mb && !mono;
    const bool bBackward = -tlc[2] > mb && !mono;
    int nmatches = 0;
    std::vector<int> idx;
    for (int i = 0; i < fr.n_points; i++) {
        const ProjPoint& p = P[i];
        float x3Dc[3];
        mat3_mul(fr.Tcw, p.xw, tcw, false, 1.0f, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        if (invzc < 0) continue;
        const float u = std::fmaf(G.fx * xc, invzc, G.cx);
        const float v = std::fmaf(G.fy * yc, invzc, G.cy);
        if (u < G.min_x || u > G.max_x) continue;
        if (v < G.min_y || v > G.max_y) continue;
        const int nLastOctave = p.octave;
        const float radius = th * G.scale[nLastOctave];
        if (bForward) features_in_area(F, G, u, v, radius, nLastOctave, -1, idx);
        else if (bBackward) features_in_area(F, G, u, v, radius, 0, nLastOctave, idx);
        else features_in_area(F, G, u, v, radius, nLastOctave - 1, nLastOctave + 1, idx);
        if (idx.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int i2 : idx) {
            if (match[i2] >= 0 && blocking[i2]) continue;
            if (F.uright[i2] > 0) {
                const float ur = std::fmaf(-G.bf, invzc, u);
                const float er = std::fabs(ur - F.uright[i2]);
                if (er > radius) continue;
            }
            const int dist = descriptor_distance(p.desc, F.desc + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= kThHigh) {
            match[bestIdx2] = i;
            blocking[bestIdx2] = p.n_obs > 0;
            nmatches++;
            if (check_ori) {
                float rot = p.angle - F.kun[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == kHisto) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    if (check_ori) {
        int h[kHisto];
        for (int b = 0; b < kHisto; b++) h[b] = (int)rotHist[b].size();
        int ind1 = -1, ind2 = -1, ind3 = -1;
        compute_three_maxima(h, ind1, ind2, ind3);
        for (int b = 0; b < kHisto; b++)
            if (b != ind1 && b != ind2 && b != ind3)
                for (int k : rotHist[b]) {
                    match[k] = -1;
                    nmatches--;
                }
    }
    return nmatches;
}

}  // namespace match
}  // namespace oracle

extern "C" {

// geometry: fx fy cx cy bf min_x max_x min_y max_y ginv_x ginv_y scale[8] (19 floats).
// Returns nmatches of the last search (after the retry at 2*th when enabled).
int oracle_search_by_projection(const void* frame, const void* points, const void* keys_un, const uint8_t* desc,
                                const float* uright, int n_kp, const int32_t* grid_off, const int32_t* grid_idx,
                                const float* geometry, const void* params, int32_t* match, int* passes) {
    using namespace oracle::match;
    const ProjFrame& fr = *(const ProjFrame*)frame;
    const ProjPoint* P = (const ProjPoint*)points;
    Geometry G;
    std::memcpy(&G, geometry, sizeof G);
    const Params& prm = *(const Params*)params;
    const Current F{(const Keypoint*)keys_un, desc, uright, grid_off, grid_idx, n_kp};
    int n = search_once(fr, P, F, G, prm.th, prm.mono != 0, prm.check_orientation != 0, match);
    if (passes) *passes = 1;
    if (prm.retry_below > 0 && n < prm.retry_below) {
        n = search_once(fr, P, F, G, 2 * prm.th, prm.mono != 0, prm.check_orientation != 0, match);
        if (passes) *passes = 2;
    }
    return n;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Tracking::SearchLocalPoints (src/Tracking.cc:1375-1425): Frame::isInFrustum
// (src/Frame.cc:369-425, viewing-cosine limit 0.5) with MapPoint::PredictScale
// (src/MapPoint.cc:402-417), then ORBmatcher(0.8).SearchByProjection(F,
// vpMapPoints, th) (src/ORBmatcher.cc:45-130) with RadiusByViewingCos
// (:131-137).  Points the caller already holds (mnLastFrameSeen == current, or
// bad) are left out of the list; `taken` marks keypoints whose mvpMapPoints
// entry is set with Observations() > 0 before the call.
// FP (OpenCV parts parity-unpinned): Rcw*P + tcw and -Rcw^T*tcw as above;
// cv::norm of a float 3-vector = sqrt((double)(float)(x*x + y*y + z*z)) with
// float partial sums; Mat::dot in double with exact products; log / ceil as
// PredictScale writes them (float logf).
namespace oracle {
namespace match {

struct LocalPoint {  // spslam_local_point
    float xw[3], normal[3];
    float min_dist, max_dist;
    int32_t id, n_obs, pad[2];
    uint8_t desc[32];
};
struct LocalFrame {  // spslam_local_frame
    float Tcw[16];
    int32_t point_offset, n_points, seen_offset, stamp;
};
struct LocalParams {  // spslam_local_params
    float th, nn_ratio, view_cos_limit, log_scale_factor;
    int32_t n_levels, pad[3];
};

struct InView {
    bool in;
    float u, ur, v, view_cos;
    int level;
};

InView is_in_frustum(const float* Tcw, const LocalPoint& p, const Geometry& G, const LocalParams& P) {
    InView r{};
    const float tcw[3] = {Tcw[3], Tcw[7], Tcw[11]};
    float Pc[3], Ow[3];
    mat3_mul(Tcw, p.xw, tcw, false, 1.0f, Pc);
    if (Pc[2] < 0.0f) return r;
    const float invz = 1.0f / Pc[2];
    const float u = std::fmaf(G.fx * Pc[0], invz, G.cx);
    const float v = std::fmaf(G.fy * Pc[1], invz, G.cy);
    if (u < G.min_x || u > G.max_x) return r;
    if (v < G.min_y || v > G.max_y) return r;
    const float maxDistance = 1.2f * p.max_dist, minDistance = 0.8f * p.min_dist;
    mat3_mul(Tcw, tcw, nullptr, true, -1.0f, Ow);
    const float PO[3] = {p.xw[0] - Ow[0], p.xw[1] - Ow[1], p.xw[2] - Ow[2]};
    float s = PO[0] * PO[0];
    s = s + PO[1] * PO[1];
    s = s + PO[2] * PO[2];
    const float dist = (float)std::sqrt((double)s);
    if (dist < minDistance || dist > maxDistance) return r;
    double dot = 0.0;
    for (int k = 0; k < 3; k++) dot += (double)PO[k] * (double)p.normal[k];
    const float viewCos = (float)(dot / (double)dist);
    if (viewCos < P.view_cos_limit) return r;
    const float ratio = p.max_dist / dist;
    int nScale = (int)std::ceil(std::log(ratio) / P.log_scale_factor);
    if (nScale < 0) nScale = 0;
    else if (nScale >= P.n_levels) nScale = P.n_levels - 1;
    r.in = true;
    r.u = u;
    r.ur = std::fmaf(-G.bf, invz, u);
    r.v = v;
    r.view_cos = viewCos;
    r.level = nScale;
    return r;
}

int search_local(const LocalFrame& fr, const LocalPoint* P, const Current& F, const Geometry& G,
                 const LocalParams& prm, const uint8_t* taken_in, int32_t* match, uint8_t* in_view) {
    std::vector<uint8_t> taken(F.n, 0);
    for (int k = 0; k < F.n; k++) {
        match[k] = -1;
        taken[k] = taken_in ? taken_in[k] : 0;
    }
    const bool bFactor = prm.th != 1.0f;
    int nmatches = 0;
    std::vector<int> idx;
    for (int i = 0; i < fr.n_points; i++) {
        const InView iv = is_in_frustum(fr.Tcw, P[i], G, prm);
        if (in_view) in_view[i] = iv.in;
        if (!iv.in) continue;
        const int nPredictedLevel = iv.level;
        float r = iv.view_cos > 0.998f ? 2.5f : 4.0f;  // RadiusByViewingCos
        if (bFactor) r *= prm.th;
        const float rs = r * G.scale[nPredictedLevel];
        features_in_area(F, G, iv.u, iv.v, rs, nPredictedLevel - 1, nPredictedLevel, idx);
        if (idx.empty()) continue;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int k : idx) {
            if (taken[k]) continue;
            if (F.uright[k] > 0) {
                const float er = std::fabs(iv.ur - F.uright[k]);
                if (er > rs) continue;
            }
            const int dist = descriptor_distance(P[i].desc, F.desc + 32 * (size_t)k);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = F.kun[k].octave;
                bestIdx = k;
            } else if (dist < bestDist2) {
                bestLevel2 = F.kun[k].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= kThHigh) {
            if (bestLevel == bestLevel2 && bestDist > prm.nn_ratio * bestDist2) continue;
            match[bestIdx] = i;
            taken[bestIdx] = 1;  // a local map point has observations
            nmatches++;
        }
    }
    return nmatches;
}

}  // namespace match
}  // namespace oracle

extern "C" int oracle_search_local_points(const void* frame, const void* points, const void* keys_un,
                                          const uint8_t* desc, const float* uright, int n_kp, const int32_t* grid_off,
                                          const int32_t* grid_idx, const float* geometry, const void* params,
                                          const uint8_t* taken, int32_t* match, uint8_t* in_view) {
    using namespace oracle::match;
    Geometry G;
    std::memcpy(&G, geometry, sizeof G);
    const Current F{(const Keypoint*)keys_un, desc, uright, grid_off, grid_idx, n_kp};
    return search_local(*(const LocalFrame*)frame, (const LocalPoint*)points, F, G, *(const LocalParams*)params,
                        taken, match, in_view);
}
