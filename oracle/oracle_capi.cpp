// ORACLE -- TEST INFRASTRUCTURE ONLY.  Flat C entry points over the CPU
// restatement so tests/ (ctypes) and bench.py's cpu_baseline leg can drive it.
#include <cstring>
#include <vector>

#include "orb_oracle.h"

using namespace oracle;

namespace {
struct OrbHandle {
    ORBextractor ex;
    OrbHandle(int nf, float sf, int nl, int ini, int mn) : ex(nf, sf, nl, ini, mn) {}
};
GrayImage wrap(const uint8_t* p, int w, int h, int stride) {
    GrayImage g; g.w = w; g.h = h; g.px.resize((size_t)w * h);
    for (int y = 0; y < h; y++) std::memcpy(&g.px[(size_t)y * w], p + (size_t)y * stride, w);
    return g;
}
int copy_kps(const std::vector<KeyPoint>& v, KeyPoint* out, int cap, int* n) {
    *n = (int)v.size();
    if ((int)v.size() > cap) return -1;
    if (!v.empty()) std::memcpy(out, v.data(), v.size() * sizeof(KeyPoint));
    return 0;
}
}  // namespace

extern "C" {

void* oracle_orb_new(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST) {
    return new OrbHandle(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST);
}
void oracle_orb_free(void* h) { delete (OrbHandle*)h; }

int oracle_orb_features_per_level(void* h, int* out) {
    auto& ex = ((OrbHandle*)h)->ex;
    for (int l = 0; l < ex.nlevels; l++) out[l] = ex.mnFeaturesPerLevel[l];
    return ex.nlevels;
}
int oracle_orb_scale_tables(void* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2) {
    auto& ex = ((OrbHandle*)h)->ex;
    for (int l = 0; l < ex.nlevels; l++) {
        scale[l] = ex.mvScaleFactor[l]; inv_scale[l] = ex.mvInvScaleFactor[l];
        sigma2[l] = ex.mvLevelSigma2[l]; inv_sigma2[l] = ex.mvInvLevelSigma2[l];
    }
    return ex.nlevels;
}
int oracle_orb_umax(void* h, int* out) {
    auto& ex = ((OrbHandle*)h)->ex;
    for (size_t i = 0; i < ex.umax.size(); i++) out[i] = ex.umax[i];
    return (int)ex.umax.size();
}

// Full ORBextractor::operator(): keypoints (level order) + N x 32 descriptors.
int oracle_orb_extract(void* h, const uint8_t* gray, int w, int hgt, int stride, KeyPoint* kps, uint8_t* desc,
                       int cap, int* n) {
    auto& ex = ((OrbHandle*)h)->ex;
    std::vector<KeyPoint> v; std::vector<uint8_t> d;
    ex.extract(wrap(gray, w, hgt, stride), v, d);
    int rc = copy_kps(v, kps, cap, n);
    if (rc == 0 && !d.empty()) std::memcpy(desc, d.data(), d.size());
    return rc;
}

// Stage access (valid after oracle_orb_pyramid or oracle_orb_extract).
int oracle_orb_pyramid(void* h, const uint8_t* gray, int w, int hgt, int stride) {
    ((OrbHandle*)h)->ex.compute_pyramid(wrap(gray, w, hgt, stride));
    return 0;
}
int oracle_orb_level_size(void* h, int level, int* w, int* hgt) {
    auto& g = ((OrbHandle*)h)->ex.pyramid[level];
    *w = g.w; *hgt = g.h;
    return 0;
}
int oracle_orb_level_image(void* h, int level, uint8_t* out) {
    auto& g = ((OrbHandle*)h)->ex.pyramid[level];
    std::memcpy(out, g.px.data(), g.px.size());
    return 0;
}
int oracle_orb_level_blurred(void* h, int level, uint8_t* out) {
    auto& ex = ((OrbHandle*)h)->ex;
    GrayImage b;
    gaussian_blur_7x7_s2(ex.pyramid[level], b);
    std::memcpy(out, b.px.data(), b.px.size());
    return 0;
}
int oracle_orb_level_candidates(void* h, int level, KeyPoint* out, int cap, int* n) {
    std::vector<KeyPoint> v;
    ((OrbHandle*)h)->ex.candidates(level, v);
    return copy_kps(v, out, cap, n);
}
int oracle_orb_level_keypoints(void* h, int level, KeyPoint* out, int cap, int* n) {
    std::vector<KeyPoint> v;
    ((OrbHandle*)h)->ex.keypoints_level(level, v);
    return copy_kps(v, out, cap, n);
}

// Known-answer-test hooks for the inherited OpenCV routines.
int oracle_resize_linear(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
    GrayImage s = wrap(src, sw, sh, sw), d;
    resize_linear_u8(s, d, dw, dh);
    std::memcpy(dst, d.px.data(), d.px.size());
    return 0;
}
int oracle_gaussian_blur(const uint8_t* src, int w, int hgt, uint8_t* dst) {
    GrayImage s = wrap(src, w, hgt, w), d;
    gaussian_blur_7x7_s2(s, d);
    std::memcpy(dst, d.px.data(), d.px.size());
    return 0;
}
int oracle_fast(const uint8_t* img, int w, int hgt, int thr, KeyPoint* out, int cap, int* n) {
    GrayImage g = wrap(img, w, hgt, w);
    std::vector<KeyPoint> v;
    fast_window(g, 0, 0, w, hgt, thr, v);
    return copy_kps(v, out, cap, n);
}
float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }
float oracle_sinf(float x) { return glibc_sinf(x); }
float oracle_cosf(float x) { return glibc_cosf(x); }
int oracle_descriptor(const uint8_t* img, int w, int hgt, float x, float y, float angle, uint8_t* desc) {
    GrayImage g = wrap(img, w, hgt, w);
    KeyPoint kp{x, y, 31.f, angle, 0.f, 0, -1};
    orb_descriptor(g, kp, desc);
    return 0;
}

}  // extern "C"
