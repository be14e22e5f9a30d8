// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// CPU restatement of Frame::GeneratePlanesFromBoundries (src/Frame.cc:938-998)
// and its helpers GenerateBoundaryPoints (:1001-1011), IsBorderLine
// (:1013-1025), IsBorderPoint (:1027-1057), LineInRange (:1059-1076),
// CaculatePlanes (:1079-1119) and PlaneNotSeen (:1121-1144), together with
// the PCL 1.8.0 code they call (PCL is not vendored; build.sh:4-8 pins
// pcl-1.8.0):
//   pcl::SACSegmentation<PointXYZRGB>::segment with SACMODEL_LINE, SAC_RANSAC,
//     setOptimizeCoefficients(true), setMaxIterations(1000), default
//     probability 0.99, random_ = false;
//   pcl::SampleConsensusModel (seeded boost::mt19937(12345u) in every
//     constructor, i.e. on every segment() call; rnd() = boost::uniform_int<>
//     (0, INT_MAX) over the 32-bit engine = mt() >> 1, bucket size 2;
//     drawIndexSample's partial Fisher-Yates on the persistent
//     shuffled_indices_; getSamples' 1000 isSampleGood checks);
//   pcl::SampleConsensusModelLine isSampleGood (x, y AND z all differ),
//     computeModelCoefficients, countWithinDistance / selectWithinDistance
//     (Vector4f cross3 + squaredNorm in Eigen's SSE lane order, compared in
//     double), optimizeModelCoefficients (compute3DCentroid +
//     computeCovarianceMatrix on the dense path, pcl::eigen33 values +
//     computeCorrespondingEigenVector of the largest);
//   pcl::RandomSampleConsensus::computeModel (adaptive k, <= 1001 trials);
//   pcl::ExtractIndices (positive / negative, order preserving).
// FP: PCL code uncontracted; expressions of Frame.cc itself with the FMA
// contractions GCC -O3 -march=native emits for them.
// Parity: unpinned against PCL itself (absent).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

namespace oracle {
namespace supposed {

struct P4 { float x, y, z; };

// ---- pcl::computeRoots (common/eigen.hpp), float; same as plane_oracle.cpp
static void roots2(float b, float c, float* r) {
    r[0] = 0.f;
    float d = (float)(b * b - 4.0 * c);
    if (d < 0.0) d = 0.0;
    float sd = std::sqrt(d);
    r[2] = 0.5f * (b + sd);
    r[1] = 0.5f * (b - sd);
}
static void roots3(const float m[3][3], float* r) {
    float c0 = m[0][0] * m[1][1] * m[2][2] + 2.f * m[0][1] * m[0][2] * m[1][2] - m[0][0] * m[1][2] * m[1][2] -
               m[1][1] * m[0][2] * m[0][2] - m[2][2] * m[0][1] * m[0][1];
    float c1 = m[0][0] * m[1][1] - m[0][1] * m[0][1] + m[0][0] * m[2][2] - m[0][2] * m[0][2] + m[1][1] * m[2][2] -
               m[1][2] * m[1][2];
    float c2 = m[0][0] + m[1][1] + m[2][2];
    if (std::fabs(c0) < std::numeric_limits<float>::epsilon()) { roots2(c2, c1, r); return; }
    const float s_inv3 = (float)(1.0 / 3.0);
    const float s_sqrt3 = std::sqrt(3.0f);
    float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > 0.f) a_over_3 = 0.f;
    float half_b = 0.5f * (c0 + c2_over_3 * (2.f * c2_over_3 * c2_over_3 - c1));
    float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
    if (q > 0.f) q = 0.f;
    float rho = std::sqrt(-a_over_3);
    float theta = std::atan2(std::sqrt(-q), half_b) * s_inv3;
    float cos_theta = std::cos(theta), sin_theta = std::sin(theta);
    r[0] = c2_over_3 + 2.f * rho * cos_theta;
    r[1] = c2_over_3 - rho * (cos_theta + s_sqrt3 * sin_theta);
    r[2] = c2_over_3 - rho * (cos_theta - s_sqrt3 * sin_theta);
    if (r[0] >= r[1]) std::swap(r[0], r[1]);
    if (r[1] >= r[2]) {
        std::swap(r[1], r[2]);
        if (r[0] >= r[1]) std::swap(r[0], r[1]);
    }
    if (r[0] <= 0) roots2(c2, c1, r);
}
static float max_abs(const float m[3][3]) {
    float s = 0.f;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) s = std::max(s, std::fabs(m[i][j]));
    if (s <= std::numeric_limits<float>::min()) s = 1.f;
    return s;
}
// pcl::eigen33(mat, evals) then computeCorrespondingEigenVector(mat, evals[2]):
// eigenvector of the largest eigenvalue (sac_model_line.hpp optimizeModelCoefficients).
void line_direction(const float cov[3][3], float* evec) {
    float scale = max_abs(cov), s[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) s[i][j] = cov[i][j] / scale;
    float r[3];
    roots3(s, r);
    const float eval2 = r[2] * scale;            // evals *= scale
    const float scale2 = max_abs(cov);           // recomputed inside computeCorrespondingEigenVector
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) s[i][j] = cov[i][j] / scale2;
    const float sub = eval2 / scale2;
    for (int i = 0; i < 3; i++) s[i][i] -= sub;
    float v[3][3], len[3];
    const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
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
    const float sl = std::sqrt(len[k]);
    for (int j = 0; j < 3; j++) evec[j] = v[k][j] / sl;
}

// Eigen Vector4f::normalize() with w = 0: squaredNorm in SSE predux order
// (x^2 + z^2) + (y^2 + w^2), then lane-wise division by the square root.
static void normalize4(float* d) {
    const float sq = (d[0] * d[0] + d[2] * d[2]) + (d[1] * d[1] + 0.f);
    if (sq > 0.f) {
        const float s = std::sqrt(sq);
        d[0] /= s; d[1] /= s; d[2] /= s;
    }
}
// ((line_pt - p).cross3(line_dir)).squaredNorm(), Vector4f (p.w = 1, line w = 0),
// in Eigen's SSE order; the caller compares it as a double.
float line_sqr_dist(const float* lp, const float* ld, const P4& p) {
    const float ax = lp[0] - p.x, ay = lp[1] - p.y, az = lp[2] - p.z;
    const float cx = ay * ld[2] - az * ld[1];
    const float cy = az * ld[0] - ax * ld[2];
    const float cz = ax * ld[1] - ay * ld[0];
    return (cx * cx + cz * cz) + (cy * cy + 0.f);
}

// std::mt19937 == boost::mt19937; boost::uniform_int<>(0, INT_MAX) -> mt() >> 1.
struct Rnd {
    std::mt19937 mt{12345u};
    uint64_t drawn = 0;
    uint32_t operator()() { drawn++; return (uint32_t)mt() >> 1; }
};

struct Segment {
    bool ok = false;
    float coef[6] = {};
    std::vector<int> inliers;  // positions into the current point set, increasing
    int iterations = 0;
    uint64_t draws = 0;
};

// pcl::SACSegmentation::segment, SACMODEL_LINE + RANSAC + optimize (one call).
Segment segment_line(const std::vector<P4>& pts, double threshold, int max_iterations) {
    Segment S;
    const int n = (int)pts.size();
    if (n < 2) return S;  // getSamples: fewer indices than the sample size -> no model
    Rnd rnd;
    std::vector<int> sh(n);
    for (int i = 0; i < n; i++) sh[i] = i;
    const double sqr_th = threshold * threshold;
    auto count = [&](const float* c) {
        float lp[3] = {c[0], c[1], c[2]}, ld[3] = {c[3], c[4], c[5]};
        normalize4(ld);
        int k = 0;
        for (int i = 0; i < n; i++)
            if ((double)line_sqr_dist(lp, ld, pts[i]) < sqr_th) k++;
        return k;
    };
    auto select = [&](const float* c, std::vector<int>& out) {
        float lp[3] = {c[0], c[1], c[2]}, ld[3] = {c[3], c[4], c[5]};
        normalize4(ld);
        out.clear();
        for (int i = 0; i < n; i++)
            if ((double)line_sqr_dist(lp, ld, pts[i]) < sqr_th) out.push_back(i);
    };
    // RandomSampleConsensus::computeModel
    int iterations = 0, best = -std::numeric_limits<int>::max();
    double k = 1.0;
    const double log_probability = std::log(1.0 - 0.99);
    const double one_over_indices = 1.0 / (double)n;
    bool have = false;
    float best_c[6] = {};
    const unsigned max_skip = (unsigned)max_iterations * 10;
    unsigned skipped = 0;
    while (iterations < k && skipped < max_skip) {
        // getSamples: up to 1000 draws of a good sample
        int s0 = -1, s1 = -1;
        for (int chk = 0; chk < 1000; chk++) {
            for (int i = 0; i < 2; i++) {
                const uint32_t r = rnd();
                std::swap(sh[i], sh[i + (int)(r % (uint32_t)(n - i))]);
            }
            const P4 &a = pts[sh[0]], &b = pts[sh[1]];
            if (a.x != b.x && a.y != b.y && a.z != b.z) { s0 = sh[0]; s1 = sh[1]; break; }
        }
        if (s0 < 0) break;  // "No samples could be selected"
        // computeModelCoefficients
        const P4 &a = pts[s0], &b = pts[s1];
        float c[6] = {a.x, a.y, a.z, b.x - a.x, b.y - a.y, b.z - a.z};
        {   // tail<3>().normalize(): unvectorised squaredNorm of a 3-element segment
            const float sq = c[3] * c[3] + c[4] * c[4] + c[5] * c[5];
            if (sq > 0.f) {
                const float s = std::sqrt(sq);
                c[3] /= s; c[4] /= s; c[5] /= s;
            }
        }
        const int cnt = count(c);
        if (cnt > best) {
            best = cnt;
            std::memcpy(best_c, c, sizeof c);
            have = true;
            const double w = (double)best * one_over_indices;
            double p_no_outliers = 1.0 - w * w;  // pow(w, 2)
            p_no_outliers = std::max(std::numeric_limits<double>::epsilon(), p_no_outliers);
            p_no_outliers = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no_outliers);
            k = log_probability / std::log(p_no_outliers);
        }
        ++iterations;
        if (iterations > max_iterations) break;
    }
    S.iterations = iterations;
    S.draws = rnd.drawn;
    if (!have) return S;
    std::vector<int> inl;
    select(best_c, inl);
    // optimizeModelCoefficients
    float refined[6];
    if (inl.size() <= 2) {
        std::memcpy(refined, best_c, sizeof refined);
    } else {
        float cen[3] = {0.f, 0.f, 0.f};
        for (int i : inl) { cen[0] += pts[i].x; cen[1] += pts[i].y; cen[2] += pts[i].z; }
        const float fn = (float)inl.size();
        for (float& v : cen) v /= fn;
        float cov[3][3] = {};
        for (int i : inl) {
            float px = pts[i].x - cen[0], py = pts[i].y - cen[1], pz = pts[i].z - cen[2];
            cov[1][1] += py * py;
            cov[1][2] += py * pz;
            cov[2][2] += pz * pz;
            const float qx = px * px, qy = py * px, qz = pz * px;  // pt *= pt.x()
            cov[0][0] += qx;
            cov[0][1] += qy;
            cov[0][2] += qz;
        }
        cov[1][0] = cov[0][1]; cov[2][0] = cov[0][2]; cov[2][1] = cov[1][2];
        float ev[3];
        line_direction(cov, ev);
        refined[0] = cen[0]; refined[1] = cen[1]; refined[2] = cen[2];
        refined[3] = ev[0]; refined[4] = ev[1]; refined[5] = ev[2];
    }
    select(refined, S.inliers);
    std::memcpy(S.coef, refined, sizeof refined);
    S.ok = true;
    return S;
}

struct Cam { float fx, fy, cx, cy; int w, h; float min_x, max_x, min_y, max_y; };

// Frame::IsBorderPoint (Frame.cc:1027-1057).  The reference does not bound-
// check the 20x20 window; here it is read through the flat row-major index
// (exactly what the reference reads while that index stays inside the image
// buffer), and a read outside the buffer counts as an invalid (<= 0.05) pixel.
bool is_border_point(const P4& p, const float* depth, int stride, const Cam& K) {
    if (p.z < 0.0f) return false;
    const float invz = 1.0f / p.z;
    const float u = std::fmaf(K.fx * p.x, invz, K.cx);
    const float v = std::fmaf(K.fy * p.y, invz, K.cy);
    const int b = 10;
    // z == 0 (x == 0): u or v is NaN, the window loops run no pixel, res/num is
    // NaN and the final test is false -> border point.  Infinite / huge
    // coordinates are unreachable (x, y are multiples of z); treated as "not border".
    if (std::isnan(u) || std::isnan(v)) return true;
    if (!(std::fabs(u) < 1e6f) || !(std::fabs(v) < 1e6f)) return false;
    int num = 0, nan = 0;
    float res = 0.f;
    const long long total = (long long)stride * K.h;
    for (int j = (int)(v - (float)b); (float)j < v + (float)b; ++j)
        for (int i = (int)(u - (float)b); (float)i < u + (float)b; ++i) {
            const long long fi = (long long)j * stride + i;
            const float d = (fi >= 0 && fi < total) ? depth[fi] : 0.f;
            if ((double)d > 0.05) {
                res += d;
                num++;
            } else {
                nan++;
                if (nan > b * b) return false;
            }
        }
    if ((double)(p.z - res / (float)num) > 0.1) return false;
    return true;
}

// Frame::LineInRange (Frame.cc:1059-1076); mnMinX..mnMaxY from
// Frame::ComputeImageBounds (Frame.cc:536-564: 0, cols, 0, rows without distortion).
bool line_in_range(const float* pc, const Cam& K) {
    if (pc[2] < 0.0f) return false;
    const float invz = 1.0f / pc[2];
    const float u = std::fmaf(K.fx * pc[0], invz, K.cx);
    const float v = std::fmaf(K.fy * pc[1], invz, K.cy);
    if (u < K.min_x + 50 || u > K.max_x - 50) return false;
    if (v < K.min_y + 50 || v > K.max_y - 50) return false;
    return true;
}

// Frame::PlaneNotSeen (Frame.cc:1121-1144); mvNotSeenPlaneCoefficients is
// never written in the reference (SURVEY.md section 8 notes), so only the
// first loop runs.
bool plane_not_seen(const std::vector<std::vector<float>>& planes, const float* c) {
    for (const auto& pm : planes) {
        const float d = pm[3] - c[3];
        const float angle = std::fmaf(pm[2], c[2], std::fmaf(pm[1], c[1], pm[0] * c[0]));  // GCC -O3 -march=native
        if ((double)d > 0.2 || (double)d < -0.2) continue;
        if ((double)angle < 0.9397 && (double)angle > -0.9397) continue;
        return false;
    }
    return true;
}

// Frame::CaculatePlanes' plane (Frame.cc:1082-1093), with GCC's contractions.
void supposed_coef(const float* ip, const float* il, float* coef) {
    const float a = std::fmaf(ip[1], il[5], -(ip[2] * il[4]));
    const float b = std::fmaf(ip[2], il[3], -(ip[0] * il[5]));
    const float c = std::fmaf(ip[0], il[4], -(ip[1] * il[3]));
    const float d = std::fmaf(c, il[2], std::fmaf(a, il[0], b * il[1]));
    const float v = std::sqrt(std::fmaf(c, c, std::fmaf(a, a, b * b)));
    coef[0] = a / v; coef[1] = b / v; coef[2] = c / v; coef[3] = -d / v;
    if (coef[3] < 0)
        for (int k = 0; k < 4; k++) coef[k] = -coef[k];
}

// The 50x50-ish synthetic patch of CaculatePlanes (Frame.cc:1097-1112):
// float loop variables stepped by a double 0.01.
int supposed_patch(const float* ip, const float* il, const float* coef, float* out, int cap) {
    int n = 0;
    for (float i = -0.25f; i < 0.25f;) {
        for (float j = -0.25f; j < 0.25f;) {
            const float x = std::fmaf(j, ip[0], std::fmaf(i, il[3], il[0]));
            const float y = std::fmaf(j, ip[1], std::fmaf(i, il[4], il[1]));
            const float z = (std::fmaf(coef[0], x, coef[1] * y) + coef[3]) / (-coef[2]);
            if (n < cap) { out[3 * n] = x; out[3 * n + 1] = y; out[3 * n + 2] = z; }
            n++;
            j = (float)((double)j + 0.01);
        }
        i = (float)((double)i + 0.01);
    }
    return n;
}

struct Candidate {
    int plane = -1, j = -1;
    int n_inliers = 0, iterations = 0, flags = 0;  // bit0 fitted, bit1 in range, bit2 border line, bit3 added
    float line[6] = {};
    std::vector<int> cloud_idx;  // line points as organized-cloud indices
};

struct Output {
    std::vector<Candidate> cand;
    std::vector<std::vector<float>> coef;  // appended planes
    std::vector<int> cand_of;              // candidate index of each appended plane
};

void generate(const float* depth, int stride, const Cam& K, const P4* cloud, int n_planes, const float* coefs,
              const int* con_off, const int* con_n, const int* contours, double line_ratio, float dis_th,
              Output& O) {
    std::vector<std::vector<float>> planes;
    for (int q = 0; q < n_planes; q++) planes.push_back({coefs[4 * q], coefs[4 * q + 1], coefs[4 * q + 2], coefs[4 * q + 3]});
    O = Output();
    for (int i = n_planes - 1; i >= 0; --i) {
        const int bsize = con_n[i];
        if (bsize < 50) continue;  // (0 -> GenerateBoundaryPoints: output-only, no lines)
        std::vector<int> cur(contours + con_off[i], contours + con_off[i] + bsize);  // cloud indices
        for (int j = 0; j < 4; j++) {
            std::vector<P4> pts(cur.size());
            for (size_t k = 0; k < cur.size(); k++) pts[k] = cloud[cur[k]];
            Segment S = segment_line(pts, (double)dis_th, 1000);
            Candidate C;
            C.plane = i; C.j = j;
            C.iterations = S.iterations;
            C.n_inliers = (int)S.inliers.size();
            std::memcpy(C.line, S.coef, sizeof C.line);
            if ((double)S.inliers.size() < line_ratio * bsize) {
                O.cand.push_back(C);
                break;
            }
            C.flags |= 1;
            std::vector<P4> line_pts;
            for (int k : S.inliers) { C.cloud_idx.push_back(cur[k]); line_pts.push_back(pts[k]); }
            if (line_in_range(S.coef, K)) {
                C.flags |= 2;
                // IsBorderLine (Frame.cc:1013-1025)
                const int s = (int)line_pts.size();
                int res = 0;
                bool border = true;
                for (const P4& p : line_pts) {
                    if (!is_border_point(p, depth, stride, K)) res++;
                    if (res > s / 4) { border = false; break; }
                }
                if (border) {
                    C.flags |= 4;
                    float cf[4];
                    supposed_coef(planes[i].data(), S.coef, cf);
                    if (plane_not_seen(planes, cf)) {
                        C.flags |= 8;
                        planes.push_back({cf[0], cf[1], cf[2], cf[3]});
                        O.coef.push_back(planes.back());
                        O.cand_of.push_back((int)O.cand.size());
                    }
                }
            }
            O.cand.push_back(C);
            // extract.setNegative(true): the remaining points, order kept
            std::vector<int> rest;
            size_t q = 0;
            for (size_t k = 0; k < cur.size(); k++) {
                if (q < S.inliers.size() && S.inliers[q] == (int)k) { q++; continue; }
                rest.push_back(cur[k]);
            }
            cur.swap(rest);
        }
    }
}

}  // namespace supposed
}  // namespace oracle

using namespace oracle::supposed;

extern "C" {

// Frame::PlaneNotSeen of n_coefs candidates against n_planes planes (4 floats each): not_seen[k].
void oracle_plane_not_seen(const float* planes, int n_planes, const float* coefs, int n_coefs, int* not_seen) {
    std::vector<std::vector<float>> P;
    for (int j = 0; j < n_planes; j++) P.emplace_back(planes + 4 * j, planes + 4 * j + 4);
    for (int k = 0; k < n_coefs; k++) not_seen[k] = oracle::supposed::plane_not_seen(P, coefs + 4 * k) ? 1 : 0;
}

void* oracle_supposed_new() { return new Output(); }
void oracle_supposed_free(void* h) { delete (Output*)h; }

// Runs GeneratePlanesFromBoundries on n_planes planes (coefficients +
// contour index lists into the organized cloud `cloud_xyz`; bounds = mnMinX,
// mnMaxX, mnMinY, mnMaxY or NULL for 0, w, 0, h).  Returns the
// number of appended (supposed) planes.
int oracle_supposed_generate(void* h, const float* depth, int w, int hgt, int stride, const float* cloud_xyz,
                             float fx, float fy, float cx, float cy, int n_planes, const float* coefs,
                             const int* con_off, const int* con_n, const int* contours, double line_ratio,
                             float dis_th, const float* bounds) {
    Cam K{fx, fy, cx, cy, w, hgt, 0.f, (float)w, 0.f, (float)hgt};
    if (bounds) { K.min_x = bounds[0]; K.max_x = bounds[1]; K.min_y = bounds[2]; K.max_y = bounds[3]; }
    Output* O = (Output*)h;
    generate(depth, stride, K, (const P4*)cloud_xyz, n_planes, coefs, con_off, con_n, contours, line_ratio, dis_th,
             *O);
    return (int)O->coef.size();
}
int oracle_supposed_n_candidates(void* h) { return (int)((Output*)h)->cand.size(); }
// candidate k: plane, j, n_inliers, iterations, flags, line[6]; returns #line points
int oracle_supposed_candidate(void* h, int k, int* info5, float* line6, int* cloud_idx, int cap) {
    const Candidate& C = ((Output*)h)->cand[k];
    info5[0] = C.plane; info5[1] = C.j; info5[2] = C.n_inliers; info5[3] = C.iterations; info5[4] = C.flags;
    std::memcpy(line6, C.line, sizeof C.line);
    const int n = (int)C.cloud_idx.size();
    if (cloud_idx)
        for (int i = 0; i < n && i < cap; i++) cloud_idx[i] = C.cloud_idx[i];
    return n;
}
// appended plane k: coefficients; returns its candidate index
int oracle_supposed_plane(void* h, int k, float* coef) {
    Output* O = (Output*)h;
    for (int j = 0; j < 4; j++) coef[j] = O->coef[k][j];
    return O->cand_of[k];
}
void oracle_supposed_coef(const float* src_coef, const float* line6, float* coef) {
    supposed_coef(src_coef, line6, coef);
}
int oracle_supposed_patch(const float* src_coef, const float* line6, const float* coef, float* out, int cap) {
    return supposed_patch(src_coef, line6, coef, out, cap);
}
// Standalone RANSAC line segmentation (tests): returns #inliers, writes coef[6], info[2] = iterations, draws.
int oracle_segment_line(const float* xyz, int n, double threshold, float* coef, int* inliers, long long* info) {
    std::vector<P4> pts(n);
    std::memcpy(pts.data(), xyz, (size_t)n * 12);
    Segment S = segment_line(pts, threshold, 1000);
    std::memcpy(coef, S.coef, sizeof S.coef);
    for (size_t i = 0; i < S.inliers.size(); i++) inliers[i] = S.inliers[i];
    info[0] = S.iterations;
    info[1] = (long long)S.draws;
    return S.ok ? (int)S.inliers.size() : -1;
}

}  // extern "C"
