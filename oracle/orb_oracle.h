// ORACLE -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of SP-SLAM's ORB extractor (reference: src/ORBextractor.cc,
// include/ORBextractor.h), including the OpenCV behaviours it inherits
// (resize INTER_LINEAR fixed point, FAST-9/16 + cornerScore<16> + 3x3 NMS,
// GaussianBlur 7x7 sigma=2 bit-exact fixed point, fastAtan2, cvRound).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this code, and only as the checker / CPU baseline. The product path
// (sp-slam_amd/) never links it.
//
// Parity status: UNPINNED against the reference binary (OpenCV/PCL/Eigen are
// absent from the build container, so the reference cannot be built or run;
// the reference ships no tests or fixtures -- SURVEY.md section 4/8c).
// Pinned instead by independent known-answer tests (tests/test_oracle_orb.py)
// and by restating each inherited third-party routine from its published
// algorithm; every chosen semantic is listed in DESIGN.md "Parity semantics".
#pragma once
#include <cstddef>
#include <cstdint>
#include <list>
#include <vector>

namespace oracle {

// Mirrors cv::KeyPoint's field order/size (28 bytes).
struct KeyPoint {
    float x, y;        // pt
    float size;
    float angle;
    float response;
    int32_t octave;
    int32_t class_id;
};
static_assert(sizeof(KeyPoint) == 28, "KeyPoint layout");

struct GrayImage {
    int w = 0, h = 0;
    std::vector<uint8_t> px;  // row-major, stride == w
    uint8_t at(int y, int x) const { return px[(size_t)y * w + x]; }
};

// --- inherited third-party routines (restated) ---------------------------
// OpenCV resize(INTER_LINEAR) on 8UC1, classic fixed-point path
// (INTER_RESIZE_COEF_BITS = 11, VResizeLinear<uchar,int,short,...> rounding).
void resize_linear_u8(const GrayImage& src, GrayImage& dst, int dw, int dh);
// OpenCV GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on an un-padded 8UC1
// image: bit-exact fixed-point path (kernel [18,34,48,56,48,34,18]/256 per axis).
void gaussian_blur_7x7_s2(const GrayImage& src, GrayImage& dst);
// OpenCV FAST(img_window, kps, thr, nonmax=true), TYPE_9_16 (FAST_t<16>).
void fast_window(const GrayImage& img, int x0, int y0, int w, int h, int thr,
                 std::vector<KeyPoint>& out);
// OpenCV cv::fastAtan2 (degrees, [0,360)).
float fast_atan2(float y, float x);
// glibc sinf / cosf (sysdeps/ieee754/flt-32), restated; equal to the system
// libm on every float in [0, 2*pi] (checked exhaustively).
float glibc_sinf(float y);
float glibc_cosf(float y);
int cv_round(float v);  // round half to even (cvRound on SSE2)

// --- ORBextractor restatement ---------------------------------------------
class ORBextractor {
public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);

    // src/ORBextractor.cc:1043-1105.  Returns keypoints (level order) and
    // descriptors (N x 32).
    void extract(const GrayImage& image, std::vector<KeyPoint>& kps, std::vector<uint8_t>& desc);

    // Stage access for parity tests.
    void compute_pyramid(const GrayImage& image);                         // :1107-1132
    void candidates(int level, std::vector<KeyPoint>& out);               // :789-829 (cell FAST)
    std::vector<KeyPoint> distribute_octtree(const std::vector<KeyPoint>& keys, int minX, int maxX,
                                             int minY, int maxY, int N);   // :539-763
    void keypoints_level(int level, std::vector<KeyPoint>& out);          // :831-852 (+ orientation)

    int nfeatures, nlevels, iniThFAST, minThFAST;
    double scaleFactor;
    std::vector<int> mnFeaturesPerLevel;
    std::vector<int> umax;
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
    std::vector<GrayImage> pyramid;   // un-padded level images
    std::vector<GrayImage> blurred;   // GaussianBlur of each level (filled by extract)
};

float ic_angle(const GrayImage& img, float px, float py, const std::vector<int>& umax);
void orb_descriptor(const GrayImage& blurred, const KeyPoint& kp, uint8_t desc[32]);

}  // namespace oracle
