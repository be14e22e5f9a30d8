// Host build of sp-slam_amd/csrc/libm64_restated.h for tests/test_libm64_restated.py: each routine against
// the system libm (glibc) on the same arguments.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../sp-slam_amd/csrc/libm64_restated.h"

namespace {
int64_t ordered(double x) {  // monotone integer image of a double (ulp distance = difference)
    int64_t i;
    std::memcpy(&i, &x, sizeof i);
    return i < 0 ? INT64_MIN - i : i;
}
double ulps(double a, double b) {
    if (std::isnan(a) || std::isnan(b)) return (std::isnan(a) && std::isnan(b)) ? 0.0 : 1e300;
    return std::fabs((double)(ordered(a) - ordered(b)));
}
}  // namespace

extern "C" {
// kind 0 sin, 1 cos, 2 atan2(a, b), 3 cube vs pow(a, 3).  stats[0] = max ulp, stats[1] = arguments whose
// result differs from libm.
void check_libm64(int kind, const double* a, const double* b, long n, double* out, double* stats) {
    double mx = 0, ndiff = 0;
    for (long i = 0; i < n; i++) {
        double r, ref;
        switch (kind) {
            case 0: r = spslam::libm64::sin_(a[i]); ref = std::sin(a[i]); break;
            case 1: r = spslam::libm64::cos_(a[i]); ref = std::cos(a[i]); break;
            case 2: r = spslam::libm64::atan2_(a[i], b[i]); ref = std::atan2(a[i], b[i]); break;
            default: r = spslam::libm64::cube_(a[i]); ref = std::pow(a[i], 3.0); break;
        }
        out[i] = r;
        const double u = ulps(r, ref);
        if (u > mx) mx = u;
        if (u != 0) ndiff += 1;
    }
    stats[0] = mx;
    stats[1] = ndiff;
}
}
