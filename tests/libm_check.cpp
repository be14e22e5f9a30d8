// Host build of sp-slam_amd/csrc/libm_restated.h for tests/test_libm_restated.py.
#include "../sp-slam_amd/csrc/libm_restated.h"

extern "C" {
void check_atan2f(const float* y, const float* x, float* out, long n) {
    for (long i = 0; i < n; i++) out[i] = spslam::libm::atan2f_(y[i], x[i]);
}
void check_sincosf(const float* t, float* s, float* c, long n) {
    for (long i = 0; i < n; i++) spslam::libm::sincosf_(t[i], &s[i], &c[i]);
}
}
