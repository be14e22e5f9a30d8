// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// CPU restatement of the RGB-D Frame constructor's per-keypoint steps that
// follow ORB extraction (src/Frame.cc:130-181):
//   UndistortKeyPoints      (:504-534) -> cv::undistortPoints (OpenCV 3.4
//                           cvUndistortPointsInternal: 5 fixed-point
//                           iterations in double, k = k1 k2 p1 p2 k3, P = K);
//   ComputeImageBounds      (:536-564) (undistorted image corners);
//   ComputeStereoFromRGBD   (:743-764) (depth at the DISTORTED keypoint,
//                           truncated to int; uR = xUn - bf / d);
//   AssignFeaturesToGrid    (:326-341) with PosInGrid (:480-491), 64 x 48 cells.
// FP: double / float operations in source order, no contraction.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace oracle {
namespace frame {

constexpr int kGridCols = 64, kGridRows = 48;

struct Params {
    float fx, fy, cx, cy;
    float dist[5];  // k1 k2 p1 p2 k3 (mDistCoef)
    float bf;
};

// cv::undistortPoints(src, dst, K, D, noArray(), K) for one point.
void undistort_point(const Params& P, float u, float v, float* ou, float* ov) {
    const double fx = P.fx, fy = P.fy, cx = P.cx, cy = P.cy;
    const double ifx = 1. / fx, ify = 1. / fy;
    double k[14] = {P.dist[0], P.dist[1], P.dist[2], P.dist[3], P.dist[4], 0, 0, 0, 0, 0, 0, 0, 0, 0};
    double x = u, y = v;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    const double x0 = x, y0 = y;  // untilt with tau = 0: invProj = 1
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = P * I: [fx 0 cx; 0 fy cy; 0 0 1]
    const double xx = fx * x + 0. * y + cx;
    const double yy = 0. * x + fy * y + cy;
    const double ww = 1. / (0. * x + 0. * y + 1.);
    *ou = (float)(xx * ww);
    *ov = (float)(yy * ww);
}

// Frame::ComputeImageBounds -> mnMinX, mnMaxX, mnMinY, mnMaxY.
void image_bounds(const Params& P, int cols, int rows, float* b) {
    if (P.dist[0] != 0.0f) {
        float cu[4], cv[4];
        const float px[4] = {0.f, (float)cols, 0.f, (float)cols}, py[4] = {0.f, 0.f, (float)rows, (float)rows};
        for (int i = 0; i < 4; i++) undistort_point(P, px[i], py[i], &cu[i], &cv[i]);
        b[0] = std::min(cu[0], cu[2]);
        b[1] = std::max(cu[1], cu[3]);
        b[2] = std::min(cv[0], cv[1]);
        b[3] = std::max(cv[2], cv[3]);
    } else {
        b[0] = 0.0f; b[1] = (float)cols; b[2] = 0.0f; b[3] = (float)rows;
    }
}

struct Out {
    std::vector<float> xun, yun, depth, ur;
    std::vector<int> cell;            // x * 48 + y, or -1
    std::vector<int> grid_off, grid_idx;
    float bounds[4];
};

void frame_rgbd(const Params& P, const float* kx, const float* ky, int n, const float* depth, int w, int h,
                int stride, Out& O) {
    image_bounds(P, w, h, O.bounds);
    O.xun.resize(n); O.yun.resize(n); O.depth.assign(n, -1.f); O.ur.assign(n, -1.f); O.cell.assign(n, -1);
    for (int i = 0; i < n; i++) {
        if (P.dist[0] == 0.0f) { O.xun[i] = kx[i]; O.yun[i] = ky[i]; }
        else undistort_point(P, kx[i], ky[i], &O.xun[i], &O.yun[i]);
    }
    for (int i = 0; i < n; i++) {
        const float d = depth[(size_t)(int)ky[i] * stride + (int)kx[i]];
        if (d > 0) {
            O.depth[i] = d;
            O.ur[i] = O.xun[i] - P.bf / d;
        }
    }
    const float ginv_x = (float)kGridCols / (O.bounds[1] - O.bounds[0]);
    const float ginv_y = (float)kGridRows / (O.bounds[3] - O.bounds[2]);
    std::vector<std::vector<int>> grid(kGridCols * kGridRows);
    for (int i = 0; i < n; i++) {
        const int px = (int)std::round((O.xun[i] - O.bounds[0]) * ginv_x);
        const int py = (int)std::round((O.yun[i] - O.bounds[2]) * ginv_y);
        if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) continue;
        O.cell[i] = px * kGridRows + py;
        grid[O.cell[i]].push_back(i);
    }
    O.grid_off.assign(kGridCols * kGridRows + 1, 0);
    O.grid_idx.clear();
    for (int c = 0; c < kGridCols * kGridRows; c++) {
        O.grid_off[c] = (int)O.grid_idx.size();
        O.grid_idx.insert(O.grid_idx.end(), grid[c].begin(), grid[c].end());
    }
    O.grid_off[kGridCols * kGridRows] = (int)O.grid_idx.size();
}

}  // namespace frame
}  // namespace oracle

using namespace oracle::frame;

extern "C" {

// kxy: n (x, y) distorted keypoint coordinates.  Outputs: un (2n), depth (n),
// ur (n), cell (n), grid_off (64*48+1), grid_idx (n), bounds (4).
void oracle_frame_rgbd(const float* params10, const float* kxy, int n, const float* depth, int w, int h, int stride,
                       float* un, float* dep, float* ur, int* cell, int* grid_off, int* grid_idx, float* bounds) {
    Params P;
    P.fx = params10[0]; P.fy = params10[1]; P.cx = params10[2]; P.cy = params10[3];
    for (int k = 0; k < 5; k++) P.dist[k] = params10[4 + k];
    P.bf = params10[9];
    std::vector<float> kx(n), ky(n);
    for (int i = 0; i < n; i++) { kx[i] = kxy[2 * i]; ky[i] = kxy[2 * i + 1]; }
    Out O;
    frame_rgbd(P, kx.data(), ky.data(), n, depth, w, h, stride, O);
    for (int i = 0; i < n; i++) {
        un[2 * i] = O.xun[i]; un[2 * i + 1] = O.yun[i];
        dep[i] = O.depth[i]; ur[i] = O.ur[i]; cell[i] = O.cell[i];
    }
    std::memcpy(grid_off, O.grid_off.data(), O.grid_off.size() * 4);
    if (!O.grid_idx.empty()) std::memcpy(grid_idx, O.grid_idx.data(), O.grid_idx.size() * 4);
    std::memcpy(bounds, O.bounds, 16);
}

}  // extern "C"
