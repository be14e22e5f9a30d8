// Minimal OpenCV-layout value types for the reference-side shim (tests/shim/reference_shim.cpp).
//
// The reference's call sites hand cv::Mat / cv::KeyPoint to ORBextractor, Frame and Optimizer
// (include/ORBextractor.h:59-61, include/Frame.h, src/Optimizer.cc).  OpenCV is not in this image, so the
// shim compiles against these stand-ins: cv::KeyPoint with OpenCV's member layout {Point2f pt; float size,
// angle, response; int octave, class_id} (28 bytes, the layout spslam_keypoint mirrors) and a cv::Mat that
// owns a dense row-major buffer with OpenCV's rows / cols / step / data / ptr / at accessors.  Only what the
// shim touches is provided.  TEST INFRASTRUCTURE: not part of the product library.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

namespace cv {

struct Point2f {
    float x = 0, y = 0;
};

struct KeyPoint {
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
};
static_assert(sizeof(KeyPoint) == 28, "cv::KeyPoint layout");

enum { CV_8U = 0, CV_16U = 2, CV_32F = 5 };
inline int elem_size(int type) { return type == CV_8U ? 1 : type == CV_16U ? 2 : 4; }

class Mat {
   public:
    int rows = 0, cols = 0, type_ = CV_8U, channels_ = 1;
    size_t step = 0;  // bytes per row
    uint8_t* data = nullptr;

    Mat() = default;
    Mat(int r, int c, int type, int channels = 1) { create(r, c, type, channels); }
    void create(int r, int c, int type, int channels = 1) {
        rows = r; cols = c; type_ = type; channels_ = channels;
        step = (size_t)c * channels * elem_size(type);
        buf_ = std::make_shared<std::vector<uint8_t>>(step * r);
        data = buf_->data();
    }
    bool empty() const { return rows == 0 || cols == 0; }
    int type() const { return type_; }
    int channels() const { return channels_; }
    size_t elemSize() const { return (size_t)channels_ * elem_size(type_); }
    template <class T> T* ptr(int r = 0) { return reinterpret_cast<T*>(data + step * r); }
    template <class T> const T* ptr(int r = 0) const { return reinterpret_cast<const T*>(data + step * r); }
    template <class T> T& at(int r, int c = 0) { return ptr<T>(r)[c]; }
    template <class T> const T& at(int r, int c = 0) const { return ptr<T>(r)[c]; }
    Mat clone() const {
        Mat m(rows, cols, type_, channels_);
        if (!empty()) std::memcpy(m.data, data, step * rows);
        return m;
    }

   private:
    std::shared_ptr<std::vector<uint8_t>> buf_;
};

}  // namespace cv
