// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h header comment).
//
// Each function cites the reference (or inherited third-party) behaviour it
// restates.  Build flags: -O3 -ffp-contract=off; the only fused multiply-adds
// are the explicit fmaf() calls that reproduce GCC -O3 -march=native
// contraction of the BRIEF sample expression (src/ORBextractor.cc:118-120).
#include "orb_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <utility>

namespace oracle {

static const int8_t kBriefPattern[1024] = {
#include "../include/spslam_brief_pattern.inc"
};

static const int PATCH_SIZE = 31;       // src/ORBextractor.cc:72
static const int HALF_PATCH_SIZE = 15;  // :73
static const int EDGE_THRESHOLD = 19;   // :74

int cv_round(float v) { return (int)std::nearbyint(v); }  // default FE_TONEAREST: half-even
static int cv_round_d(double v) { return (int)std::nearbyint(v); }
static int cv_floor(float v) { int i = (int)v; return i - (i > v); }

// ---------------------------------------------------------------------------
// glibc 2.28+ sinf/cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c,
// sincosf.h, s_sincosf_data.c), restricted to |y| < 120 (all ORB angles are
// in [0, 2*pi]).  Reference call site: (float)cos(angle) / sin(angle) at
// src/ORBextractor.cc:113 resolve to std::cos(float) == cosf.
struct SinCosT { double sign[4]; double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3; };
static const SinCosT kSinCos[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
static inline uint32_t abstop12(float x) { uint32_t u; std::memcpy(&u, &x, 4); return (u >> 20) & 0x7ff; }
static inline float sincos_poly(double x, double x2, const SinCosT* p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2, s1 = p->s2 + x2 * p->s3, x7 = x3 * x2, s = x + x3 * p->s1;
        return (float)(s + x7 * s1);
    }
    double x4 = x2 * x2, c2 = p->c3 + x2 * p->c4, c1 = p->c0 + x2 * p->c1, x6 = x4 * x2, c = c1 + x4 * p->c2;
    return (float)(c + x6 * c2);
}
static inline double reduce_fast(double x, const SinCosT* p, int* np) {
    double r = x * p->hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return x - n * p->hpi;
}
float glibc_sinf(float y) {
    double x = y; const SinCosT* p = &kSinCos[0]; int n;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sincos_poly(x, x * x, p, 0);
    }
    x = reduce_fast(x, p, &n);
    double s = p->sign[n & 3];
    if (n & 2) p = &kSinCos[1];
    return sincos_poly(x * s, x * x, p, n);
}
float glibc_cosf(float y) {
    double x = y; const SinCosT* p = &kSinCos[0]; int n;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sincos_poly(x, x * x, p, 1);
    }
    x = reduce_fast(x, p, &n);
    double s = p->sign[n & 3];
    if (n & 2) p = &kSinCos[1];
    return sincos_poly(x * s, x * x, p, n ^ 1);
}

// OpenCV cv::fastAtan2 (modules/core mathfuncs: atan_f32), degrees.
float fast_atan2(float y, float x) {
    const float k = (float)(180 / M_PI);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k,
                p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float eps = (float)2.220446049250313e-16;  // (float)DBL_EPSILON
    float ax = std::fabs(x), ay = std::fabs(y), a, c, c2;
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

// ---------------------------------------------------------------------------
// OpenCV resize INTER_LINEAR, CV_8U (imgproc/resize.cpp: coefficient setup in
// resize(); HResizeLinear + VResizeLinear<uchar,int,short,FixedPtCast,...>).
void resize_linear_u8(const GrayImage& src, GrayImage& dst, int dw, int dh) {
    const int sw = src.w, sh = src.h;
    dst.w = dw; dst.h = dh; dst.px.assign((size_t)dw * dh, 0);
    const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    std::vector<int> xofs(dw);
    std::vector<short> ialpha(2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        ialpha[2 * dx] = (short)cv_round((1.f - fx) * 2048);
        ialpha[2 * dx + 1] = (short)cv_round(fx * 2048);
    }
    std::vector<int> r0(dw), r1(dw);
    auto hresize = [&](int sy, std::vector<int>& D) {
        const uint8_t* S = &src.px[(size_t)sy * sw];
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (dx < xmax) D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
            else D[dx] = S[sx] * 2048;
        }
    };
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        const int b0 = (short)cv_round((1.f - fy) * 2048), b1 = (short)cv_round(fy * 2048);
        auto clip = [&](int y) { return y < 0 ? 0 : (y >= sh ? sh - 1 : y); };
        hresize(clip(sy), r0);
        hresize(clip(sy + 1), r1);
        uint8_t* D = &dst.px[(size_t)dy * dw];
        for (int x = 0; x < dw; x++)
            D[x] = (uint8_t)((((b0 * (r0[x] >> 4)) >> 16) + ((b1 * (r1[x] >> 4)) >> 16) + 2) >> 2);
    }
}

// ---------------------------------------------------------------------------
// OpenCV GaussianBlur, CV_8U bit-exact fixed-point path (smooth.simd.hpp
// fixedSmoothInvoker; kernel from getGaussianKernelBitExact +
// getGaussianKernelFixedPoint_ED with 8 fraction bits), BORDER_REFLECT_101.
static int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}
void gaussian_blur_7x7_s2(const GrayImage& src, GrayImage& dst) {
    static const int k[7] = {18, 34, 48, 56, 48, 34, 18};
    const int w = src.w, h = src.h;
    std::vector<int> hb((size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int s = 0;
            for (int i = 0; i < 7; i++) s += k[i] * src.at(y, reflect101(x + i - 3, w));
            hb[(size_t)y * w + x] = s;
        }
    dst.w = w; dst.h = h; dst.px.assign((size_t)w * h, 0);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int s = 0;
            for (int i = 0; i < 7; i++) s += k[i] * hb[(size_t)reflect101(y + i - 3, h) * w + x];
            dst.px[(size_t)y * w + x] = (uint8_t)std::min(255, (s + (1 << 15)) >> 16);
        }
}

// ---------------------------------------------------------------------------
// OpenCV FAST_t<16> (features2d/fast.cpp) with cornerScore<16>
// (fast_score.cpp), on the window [y0,y0+h) x [x0,x0+w) of img.
static const int kCircle[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                                   {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// Returns max over the 16 contiguous 9-arcs of min(v - x) and of min(x - v),
// minus 1 (== cornerScore<16> for any pixel that is a corner).
static int fast_raw_score(const GrayImage& img, int y, int x) {
    int v = img.at(y, x), d[16];
    for (int k = 0; k < 16; k++) d[k] = v - img.at(y + kCircle[k][1], x + kCircle[k][0]);
    int best = -1000;
    for (int s = 0; s < 16; s++) {
        int mn = 1000, mx = -1000;
        for (int t = 0; t < 9; t++) { int e = d[(s + t) & 15]; mn = std::min(mn, e); mx = std::max(mx, e); }
        best = std::max(best, std::max(mn, -mx));
    }
    return best - 1;
}

void fast_window(const GrayImage& img, int x0, int y0, int w, int h, int thr, std::vector<KeyPoint>& out) {
    thr = std::min(std::max(thr, 0), 255);
    // score grid: 0 where not a corner (FAST_t memsets each row buffer)
    std::vector<int> sc((size_t)w * h, 0);
    for (int i = 3; i < h - 3; i++)
        for (int j = 3; j < w - 3; j++) {
            // corner iff >= 9 contiguous pixels all > v+thr or all < v-thr
            int s = fast_raw_score(img, y0 + i, x0 + j);
            if (s >= thr) sc[(size_t)i * w + j] = s;
        }
    for (int i = 3; i < h - 3; i++)
        for (int j = 3; j < w - 3; j++) {
            int s = sc[(size_t)i * w + j];
            if (!s) continue;
            bool keep = true;
            for (int dy = -1; dy <= 1 && keep; dy++)
                for (int dx = -1; dx <= 1; dx++)
                    if ((dy || dx) && !(s > sc[(size_t)(i + dy) * w + (j + dx)])) { keep = false; break; }
            if (keep) out.push_back(KeyPoint{(float)j, (float)i, 7.f, -1.f, (float)s, 0, -1});
        }
}

// ---------------------------------------------------------------------------
// ORBextractor::ORBextractor, src/ORBextractor.cc:410-470.
ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
    : nfeatures(_nfeatures), nlevels(_nlevels), iniThFAST(_iniThFAST), minThFAST(_minThFAST),
      scaleFactor(_scaleFactor) {
    mvScaleFactor.resize(nlevels); mvLevelSigma2.resize(nlevels);
    mvScaleFactor[0] = 1.0f; mvLevelSigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
        mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);  // float*double -> float
        mvLevelSigma2[i] = mvScaleFactor[i] * mvScaleFactor[i];
    }
    mvInvScaleFactor.resize(nlevels); mvInvLevelSigma2.resize(nlevels);
    for (int i = 0; i < nlevels; i++) {
        mvInvScaleFactor[i] = 1.0f / mvScaleFactor[i];
        mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
    }
    pyramid.resize(nlevels); blurred.resize(nlevels);
    mnFeaturesPerLevel.resize(nlevels);
    float factor = (float)(1.0f / scaleFactor);
    float nDesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int level = 0; level < nlevels - 1; level++) {
        mnFeaturesPerLevel[level] = cv_round(nDesired);
        sum += mnFeaturesPerLevel[level];
        nDesired *= factor;
    }
    mnFeaturesPerLevel[nlevels - 1] = std::max(nfeatures - sum, 0);

    umax.resize(HALF_PATCH_SIZE + 1);
    int v, v0, vmax = (int)std::floor(HALF_PATCH_SIZE * std::sqrt(2.f) / 2 + 1);
    int vmin = (int)std::ceil(HALF_PATCH_SIZE * std::sqrt(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (v = 0; v <= vmax; ++v) umax[v] = cv_round_d(std::sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
}

// ComputePyramid, src/ORBextractor.cc:1107-1132.  The EDGE_THRESHOLD padding
// (copyMakeBorder) is never read by the RGB-D path: FAST windows start 16 px
// inside, orientation/BRIEF read <= 18 px around keypoints >= 19 px inside,
// and resize reads the un-padded previous level.  So levels are kept un-padded.
void ORBextractor::compute_pyramid(const GrayImage& image) {
    for (int level = 0; level < nlevels; ++level) {
        float scale = mvInvScaleFactor[level];
        int w = cv_round((float)image.w * scale), h = cv_round((float)image.h * scale);
        if (level == 0) pyramid[0] = image;
        else resize_linear_u8(pyramid[level - 1], pyramid[level], w, h);
    }
}

// Per-cell FAST of ComputeKeyPointsOctTree, src/ORBextractor.cc:773-829.
// Output coordinates are relative to (minBorderX, minBorderY) as at :822-823.
void ORBextractor::candidates(int level, std::vector<KeyPoint>& out) {
    const float W = 30;
    const GrayImage& img = pyramid[level];
    const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
    const int maxBorderX = img.w - EDGE_THRESHOLD + 3, maxBorderY = img.h - EDGE_THRESHOLD + 3;
    const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
    for (int i = 0; i < nRows; i++) {
        const float iniY = (float)(minBorderY + i * hCell);
        float maxY = iniY + hCell + 6;
        if (iniY >= maxBorderY - 3) continue;
        if (maxY > maxBorderY) maxY = (float)maxBorderY;
        for (int j = 0; j < nCols; j++) {
            const float iniX = (float)(minBorderX + j * wCell);
            float maxX = iniX + wCell + 6;
            if (iniX >= maxBorderX - 6) continue;
            if (maxX > maxBorderX) maxX = (float)maxBorderX;
            std::vector<KeyPoint> cell;
            fast_window(img, (int)iniX, (int)iniY, (int)maxX - (int)iniX, (int)maxY - (int)iniY, iniThFAST, cell);
            if (cell.empty())
                fast_window(img, (int)iniX, (int)iniY, (int)maxX - (int)iniX, (int)maxY - (int)iniY, minThFAST, cell);
            for (auto& kp : cell) {
                kp.x += j * wCell;
                kp.y += i * hCell;
                out.push_back(kp);
            }
        }
    }
}

// ExtractorNode + DistributeOctTree, src/ORBextractor.cc:481-763.
// The reference sorts (size, ExtractorNode*) pairs (:684), so equal-size ties
// break by heap address, which depends on the allocator.  Here the "address"
// is the node's list-insertion sequence number (later insertion = larger),
// a documented, deterministic pin of that tie-break.
namespace {
struct Node {
    std::vector<KeyPoint> keys;
    int x0, y0, x1, y1;  // UL=(x0,y0) UR=(x1,y0) BL=(x0,y1) BR=(x1,y1)
    std::list<Node>::iterator lit;
    bool noMore = false;
    long seq = 0;
    void divide(Node& n1, Node& n2, Node& n3, Node& n4) const {
        const int halfX = (int)std::ceil((float)(x1 - x0) / 2);
        const int halfY = (int)std::ceil((float)(y1 - y0) / 2);
        n1.x0 = x0; n1.y0 = y0; n1.x1 = x0 + halfX; n1.y1 = y0 + halfY;
        n2.x0 = x0 + halfX; n2.y0 = y0; n2.x1 = x1; n2.y1 = y0 + halfY;
        n3.x0 = x0; n3.y0 = y0 + halfY; n3.x1 = x0 + halfX; n3.y1 = y1;
        n4.x0 = x0 + halfX; n4.y0 = y0 + halfY; n4.x1 = x1; n4.y1 = y1;
        for (const KeyPoint& kp : keys) {
            if (kp.x < n1.x1) { if (kp.y < n1.y1) n1.keys.push_back(kp); else n3.keys.push_back(kp); }
            else if (kp.y < n1.y1) n2.keys.push_back(kp);
            else n4.keys.push_back(kp);
        }
        if (n1.keys.size() == 1) n1.noMore = true;
        if (n2.keys.size() == 1) n2.noMore = true;
        if (n3.keys.size() == 1) n3.noMore = true;
        if (n4.keys.size() == 1) n4.noMore = true;
    }
};
struct Entry { int size; long seq; Node* node; };
bool entry_less(const Entry& a, const Entry& b) { return a.size != b.size ? a.size < b.size : a.seq < b.seq; }
}  // namespace

std::vector<KeyPoint> ORBextractor::distribute_octtree(const std::vector<KeyPoint>& keys, int minX, int maxX,
                                                       int minY, int maxY, int N) {
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    std::list<Node> lNodes;
    long seq = 0;
    std::vector<Node*> ini(nIni);
    for (int i = 0; i < nIni; i++) {
        Node ni;
        ni.x0 = (int)(hX * (float)i); ni.y0 = 0;
        ni.x1 = (int)(hX * (float)(i + 1)); ni.y1 = maxY - minY;
        ni.seq = seq++;
        lNodes.push_back(ni);
        ini[i] = &lNodes.back();
    }
    for (const KeyPoint& kp : keys) ini[(size_t)(kp.x / hX)]->keys.push_back(kp);
    for (auto lit = lNodes.begin(); lit != lNodes.end();) {
        if (lit->keys.size() == 1) { lit->noMore = true; ++lit; }
        else if (lit->keys.empty()) lit = lNodes.erase(lit);
        else ++lit;
    }
    bool finish = false;
    std::vector<Entry> toExpand;
    auto push_child = [&](Node& c, std::vector<Entry>& vec, int* nToExpand) {
        if (c.keys.empty()) return;
        c.seq = seq++;
        lNodes.push_front(c);
        if (c.keys.size() > 1) {
            if (nToExpand) (*nToExpand)++;
            vec.push_back(Entry{(int)c.keys.size(), c.seq, &lNodes.front()});
            lNodes.front().lit = lNodes.begin();
        }
    };
    while (!finish) {
        int prevSize = (int)lNodes.size();
        int nToExpand = 0;
        toExpand.clear();
        for (auto lit = lNodes.begin(); lit != lNodes.end();) {
            if (lit->noMore) { ++lit; continue; }
            Node n1, n2, n3, n4;
            lit->divide(n1, n2, n3, n4);
            push_child(n1, toExpand, &nToExpand);
            push_child(n2, toExpand, &nToExpand);
            push_child(n3, toExpand, &nToExpand);
            push_child(n4, toExpand, &nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            finish = true;
        } else if ((int)lNodes.size() + nToExpand * 3 > N) {
            while (!finish) {
                prevSize = (int)lNodes.size();
                std::vector<Entry> prev = toExpand;
                toExpand.clear();
                std::sort(prev.begin(), prev.end(), entry_less);
                for (int j = (int)prev.size() - 1; j >= 0; j--) {
                    Node n1, n2, n3, n4;
                    prev[j].node->divide(n1, n2, n3, n4);
                    push_child(n1, toExpand, nullptr);
                    push_child(n2, toExpand, nullptr);
                    push_child(n3, toExpand, nullptr);
                    push_child(n4, toExpand, nullptr);
                    lNodes.erase(prev[j].node->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) finish = true;
            }
        }
    }
    std::vector<KeyPoint> result;
    result.reserve(nfeatures);
    for (auto& node : lNodes) {
        const KeyPoint* best = &node.keys[0];
        float maxResponse = best->response;
        for (size_t k = 1; k < node.keys.size(); k++)
            if (node.keys[k].response > maxResponse) { best = &node.keys[k]; maxResponse = best->response; }
        result.push_back(*best);
    }
    return result;
}

// IC_Angle, src/ORBextractor.cc:77-104.
float ic_angle(const GrayImage& img, float px, float py, const std::vector<int>& umax) {
    int m_01 = 0, m_10 = 0;
    const int cy = cv_round(py), cx = cv_round(px);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * img.at(cy, cx + u);
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0, d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int vp = img.at(cy + v, cx + u), vm = img.at(cy - v, cx + u);
            v_sum += vp - vm;
            m_10 += u * (vp + vm);
        }
        m_01 += v * v_sum;
    }
    return fast_atan2((float)m_01, (float)m_10);
}

// ComputeKeyPointsOctTree per level, src/ORBextractor.cc:831-852.
void ORBextractor::keypoints_level(int level, std::vector<KeyPoint>& out) {
    const GrayImage& img = pyramid[level];
    const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
    const int maxBorderX = img.w - EDGE_THRESHOLD + 3, maxBorderY = img.h - EDGE_THRESHOLD + 3;
    std::vector<KeyPoint> cand;
    candidates(level, cand);
    out = distribute_octtree(cand, minBorderX, maxBorderX, minBorderY, maxBorderY, mnFeaturesPerLevel[level]);
    const int scaledPatchSize = (int)(PATCH_SIZE * mvScaleFactor[level]);
    for (auto& kp : out) {
        kp.x += minBorderX; kp.y += minBorderY;
        kp.octave = level;
        kp.size = (float)scaledPatchSize;
    }
    for (auto& kp : out) kp.angle = ic_angle(img, kp.x, kp.y, umax);
}

// computeOrbDescriptor, src/ORBextractor.cc:107-147.  Sample offsets use the
// contraction GCC 11 -O3 -march=native emits for :119-120 on FMA hardware:
// row = fma(x, b, y*a), col = fma(x, a, -(y*b)).
void orb_descriptor(const GrayImage& img, const KeyPoint& kp, uint8_t desc[32]) {
    const float factorPI = (float)(M_PI / 180.f);
    const float angle = kp.angle * factorPI;
    const float a = glibc_cosf(angle), b = glibc_sinf(angle);
    const int cy = cv_round(kp.y), cx = cv_round(kp.x);
    auto sample = [&](int idx) {
        const float x = (float)kBriefPattern[2 * idx], y = (float)kBriefPattern[2 * idx + 1];
        const int r = cv_round(std::fmaf(x, b, y * a));
        const int c = cv_round(std::fmaf(x, a, -(y * b)));
        return (int)img.at(cy + r, cx + c);
    };
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int bit = 0; bit < 8; bit++) {
            int t0 = sample(16 * i + 2 * bit), t1 = sample(16 * i + 2 * bit + 1);
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

// ORBextractor::operator(), src/ORBextractor.cc:1043-1105.
void ORBextractor::extract(const GrayImage& image, std::vector<KeyPoint>& kps, std::vector<uint8_t>& desc) {
    if (image.w == 0 || image.h == 0) return;
    compute_pyramid(image);
    std::vector<std::vector<KeyPoint>> all(nlevels);
    for (int level = 0; level < nlevels; ++level) keypoints_level(level, all[level]);
    kps.clear(); desc.clear();
    for (int level = 0; level < nlevels; ++level) {
        std::vector<KeyPoint>& lk = all[level];
        if (lk.empty()) continue;
        gaussian_blur_7x7_s2(pyramid[level], blurred[level]);
        size_t off = desc.size();
        desc.resize(off + 32 * lk.size());
        for (size_t i = 0; i < lk.size(); i++) orb_descriptor(blurred[level], lk[i], &desc[off + 32 * i]);
        if (level != 0) {
            float scale = mvScaleFactor[level];
            for (auto& kp : lk) { kp.x *= scale; kp.y *= scale; }
        }
        kps.insert(kps.end(), lk.begin(), lk.end());
    }
}

}  // namespace oracle
