// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// CPU restatement of Frame::ComputePlanesFromOrganizedPointCloud
// (src/Frame.cc:854-936) and of the PCL 1.8.0 routines it calls (PCL is not
// vendored in the reference; build.sh:4-8 pins pcl-1.8.0):
//   pcl::IntegralImageNormalEstimation<PointXYZRGB, Normal>, AVERAGE_3D_GRADIENT,
//     setMaxDepthChangeFactor(0.05f), setNormalSmoothingSize(10.0f), default
//     BORDER_POLICY_IGNORE, no depth-dependent smoothing, viewpoint (0,0,0):
//     depth-change map, 2-pass chamfer distance map, diff images, double
//     IntegralImage2D<float,3>, computePointNormal, flipNormalTowardsViewpoint;
//   pcl::OrganizedMultiPlaneSegmentation::segmentAndRefine with the default
//     PlaneCoefficientComparator (depth-dependent distance 0.05 z^2, angle
//     cosf(3 deg)) and PlaneRefinementComparator (absolute 0.02 m), the
//     OrganizedConnectedComponentSegmentation labelling (run ids + findRoot),
//     computeMeanAndCovarianceMatrix (float, dense), pcl::eigen33 /
//     computeRoots (float), the curvature filter (maximum_curvature 0.001),
//     the two-pass refinement and findLabeledRegionBoundary (Moore tracing);
// then Frame's sign normalisation and PlaneNotSeen de-duplication.
// Parity: unpinned against PCL itself (absent); semantics listed in DESIGN.md.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

namespace oracle {
namespace planes {

struct P3 { float x, y, z; };

struct Params {
    int cloud_dis = 3;          // Cloud.Dis
    int min_size = 500;         // Plane.MinSize
    float angle_th_deg = 3.0f;  // Plane.AngleThreshold
    float dist_th = 0.05f;      // Plane.DistanceThreshold
    float fx, fy, cx, cy;
};

struct Result {
    int W = 0, H = 0;
    std::vector<P3> cloud;
    std::vector<float> nrm;      // 3 per point (NaN = invalid)
    std::vector<float> dist;     // chamfer distance map
    std::vector<uint32_t> labels_cc;     // after connected components
    std::vector<uint32_t> labels_ref;    // after refinement
    std::vector<std::vector<float>> models;       // segment() coefficients (pre-flip)
    std::vector<std::vector<int>> model_inliers;  // refined inlier indices per model
    std::vector<std::vector<int>> model_contour;  // boundary indices per model
    // Frame output (kept planes, in order)
    std::vector<std::vector<float>> coef;
    std::vector<int> kept_model;                  // model index of each kept plane
};

static bool isfin(float v) { return std::isfinite(v); }

// Eigen SSE predux order for a Vector4f dot: (a0 b0 + a2 b2) + (a1 b1 + a3 b3).
static float dot4(const float* a, const float* b) {
    float p0 = a[0] * b[0], p1 = a[1] * b[1], p2 = a[2] * b[2], p3 = a[3] * b[3];
    return (p0 + p2) + (p1 + p3);
}

// pcl::computeRoots2 / computeRoots (common/eigen.hpp), float.
static void compute_roots2(float b, float c, float* r) {
    r[0] = 0.f;
    float d = (float)(b * b - 4.0 * c);
    if (d < 0.0) d = 0.0;
    float sd = std::sqrt(d);
    r[2] = 0.5f * (b + sd);
    r[1] = 0.5f * (b - sd);
}
static void compute_roots(const float m[3][3], float* r) {
    float c0 = m[0][0] * m[1][1] * m[2][2] + 2.f * m[0][1] * m[0][2] * m[1][2] - m[0][0] * m[1][2] * m[1][2] -
               m[1][1] * m[0][2] * m[0][2] - m[2][2] * m[0][1] * m[0][1];
    float c1 = m[0][0] * m[1][1] - m[0][1] * m[0][1] + m[0][0] * m[2][2] - m[0][2] * m[0][2] + m[1][1] * m[2][2] -
               m[1][2] * m[1][2];
    float c2 = m[0][0] + m[1][1] + m[2][2];
    if (std::fabs(c0) < std::numeric_limits<float>::epsilon()) {
        compute_roots2(c2, c1, r);
        return;
    }
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
    if (r[0] <= 0) compute_roots2(c2, c1, r);
}
// pcl::eigen33(mat, eigenvalue, eigenvector): smallest eigenpair, float.
static void eigen33(const float mat[3][3], float* eval, float* evec) {
    float scale = 0.f;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) scale = std::max(scale, std::fabs(mat[i][j]));
    if (scale <= std::numeric_limits<float>::min()) scale = 1.f;
    float s[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) s[i][j] = mat[i][j] / scale;
    float r[3];
    compute_roots(s, r);
    *eval = r[0] * scale;
    for (int i = 0; i < 3; i++) s[i][i] -= r[0];
    auto cross = [](const float* a, const float* b, float* o) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    float v1[3], v2[3], v3[3];
    cross(s[0], s[1], v1);
    cross(s[0], s[2], v2);
    cross(s[1], s[2], v3);
    auto sq = [](const float* v) { return v[0] * v[0] + v[1] * v[1] + v[2] * v[2]; };
    float l1 = sq(v1), l2 = sq(v2), l3 = sq(v3);
    const float* v;
    float l;
    if (l1 >= l2 && l1 >= l3) { v = v1; l = l1; }
    else if (l2 >= l1 && l2 >= l3) { v = v2; l = l2; }
    else { v = v3; l = l3; }
    float sl = std::sqrt(l);
    for (int i = 0; i < 3; i++) evec[i] = v[i] / sl;
}

void extract(const float* depth, int w, int h, int stride_floats, const Params& P, Result& R) {
    // --- organized cloud (Frame.cc:855-874)
    const int ds = P.cloud_dis;
    const int W = (int)std::ceil(w / (float)ds), H = (int)std::ceil(h / (float)ds);
    R.W = W; R.H = H;
    const int N = W * H;
    R.cloud.resize(N);
    for (int m = 0, r = 0; m < h; m += ds, r++)
        for (int n = 0, c = 0; n < w; n += ds, c++) {
            const float d = depth[(size_t)m * stride_floats + n];
            P3 p;
            p.z = d;
            p.x = ((float)n - P.cx) * p.z / P.fx;
            p.y = ((float)m - P.cy) * p.z / P.fy;
            R.cloud[r * W + c] = p;
        }
    const std::vector<P3>& pc = R.cloud;

    // --- IntegralImageNormalEstimation::computeFeature
    std::vector<uint8_t> dcm(N, 255);
    const float mdcf = 0.05f;
    for (int ri = 0; ri < H - 1; ri++)
        for (int ci = 0; ci < W - 1; ci++) {
            const int idx = ri * W + ci;
            const float depth0 = pc[idx].z, depthR = pc[idx + 1].z, depthD = pc[idx + W].z;
            const float ddc = (mdcf * (std::fabs(depth0) + 1.0f) * 2.0f);
            if (std::fabs(depth0 - depthR) > ddc || !isfin(depth0) || !isfin(depthR)) { dcm[idx] = 0; dcm[idx + 1] = 0; }
            if (std::fabs(depth0 - depthD) > ddc || !isfin(depth0) || !isfin(depthD)) { dcm[idx] = 0; dcm[idx + W] = 0; }
        }
    // distance map (+1 element of slack: the reference reads one past the last row end)
    std::vector<float> dmv(N + 1, 0.f);
    float* dm = dmv.data();
    for (int i = 0; i < N; i++) dm[i] = dcm[i] == 0 ? 0.0f : (float)(W + H);
    {
        float* prev = dm;
        float* cur = prev + W;
        for (int ri = 1; ri < H; ++ri) {
            for (int ci = 1; ci < W; ++ci) {
                const float upLeft = prev[ci - 1] + 1.4f, up = prev[ci] + 1.0f, upRight = prev[ci + 1] + 1.4f;
                const float left = cur[ci - 1] + 1.0f, center = cur[ci];
                const float mv = std::min(std::min(upLeft, up), std::min(left, upRight));
                if (mv < center) cur[ci] = mv;
            }
            prev = cur;
            cur += W;
        }
        float* next = dm + W * (H - 1);
        cur = next - W;
        for (int ri = H - 2; ri >= 0; --ri) {
            for (int ci = W - 2; ci >= 0; --ci) {
                const float lowerLeft = next[ci - 1] + 1.4f, lower = next[ci] + 1.0f, lowerRight = next[ci + 1] + 1.4f;
                const float right = cur[ci + 1] + 1.0f, center = cur[ci];
                const float mv = std::min(std::min(lowerLeft, lower), std::min(right, lowerRight));
                if (mv < center) cur[ci] = mv;
            }
            next = cur;
            cur -= W;
        }
    }
    R.dist.assign(dm, dm + N);
    // diff images (initAverage3DGradientMethod) and double integral images
    std::vector<float> dx((size_t)N * 3, 0.f), dy((size_t)N * 3, 0.f);
    for (int ri = 1; ri < H - 1; ri++)
        for (int c = 1; c < W - 1; c++) {
            const int i = ri * W + c;
            dx[3 * i + 0] = pc[i + 1].x - pc[i - 1].x;
            dx[3 * i + 1] = pc[i + 1].y - pc[i - 1].y;
            dx[3 * i + 2] = pc[i + 1].z - pc[i - 1].z;
            dy[3 * i + 0] = pc[i + W].x - pc[i - W].x;
            dy[3 * i + 1] = pc[i + W].y - pc[i - W].y;
            dy[3 * i + 2] = pc[i + W].z - pc[i - W].z;
        }
    const int IW = W + 1;
    std::vector<double> IX((size_t)IW * (H + 1) * 3, 0.0), IY((size_t)IW * (H + 1) * 3, 0.0);
    std::vector<uint32_t> CX((size_t)IW * (H + 1), 0), CY((size_t)IW * (H + 1), 0);
    auto integral = [&](const std::vector<float>& d, std::vector<double>& I, std::vector<uint32_t>& Cn) {
        for (int r = 0; r < H; r++) {
            double* prev = &I[(size_t)r * IW * 3];
            double* cur = &I[(size_t)(r + 1) * IW * 3];
            uint32_t* cp = &Cn[(size_t)r * IW];
            uint32_t* cc = &Cn[(size_t)(r + 1) * IW];
            cur[0] = cur[1] = cur[2] = 0.0;
            cc[0] = 0;
            for (int c = 0; c < W; c++) {
                for (int k = 0; k < 3; k++) cur[3 * (c + 1) + k] = prev[3 * (c + 1) + k] + cur[3 * c + k] - prev[3 * c + k];
                cc[c + 1] = cp[c + 1] + cc[c] - cp[c];
                const float* e = &d[3 * ((size_t)r * W + c)];
                if (isfin(e[0] + e[1] + e[2])) {
                    for (int k = 0; k < 3; k++) cur[3 * (c + 1) + k] += (double)e[k];
                    ++cc[c + 1];
                }
            }
        }
    };
    integral(dx, IX, CX);
    integral(dy, IY, CY);
    const float bad = std::numeric_limits<float>::quiet_NaN();
    R.nrm.assign((size_t)N * 3, bad);
    const int border = 10;
    for (int ri = border; ri < H - border; ri++)
        for (int ci = border; ci < W - border; ci++) {
            const int idx = ri * W + ci;
            if (!isfin(pc[idx].z)) continue;
            const float smoothing = std::min(dm[idx], 10.0f);
            if (!(smoothing > 2.0f)) continue;
            const int rw = (int)smoothing, rh = (int)smoothing;
            const int sx = ci - rw / 2, sy = ri - rh / 2;
            auto cnt = [&](const std::vector<uint32_t>& Cn) {
                return Cn[(size_t)(sy + rh) * IW + sx + rw] + Cn[(size_t)sy * IW + sx] - Cn[(size_t)sy * IW + sx + rw] -
                       Cn[(size_t)(sy + rh) * IW + sx];
            };
            if (cnt(CX) == 0 || cnt(CY) == 0) continue;
            double gx[3], gy[3];
            for (int k = 0; k < 3; k++) {
                gx[k] = IX[((size_t)(sy + rh) * IW + sx + rw) * 3 + k] + IX[((size_t)sy * IW + sx) * 3 + k] -
                        IX[((size_t)sy * IW + sx + rw) * 3 + k] - IX[((size_t)(sy + rh) * IW + sx) * 3 + k];
                gy[k] = IY[((size_t)(sy + rh) * IW + sx + rw) * 3 + k] + IY[((size_t)sy * IW + sx) * 3 + k] -
                        IY[((size_t)sy * IW + sx + rw) * 3 + k] - IY[((size_t)(sy + rh) * IW + sx) * 3 + k];
            }
            double nv[3] = {gy[1] * gx[2] - gy[2] * gx[1], gy[2] * gx[0] - gy[0] * gx[2], gy[0] * gx[1] - gy[1] * gx[0]};
            const double len = nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2];
            if (len == 0.0f) continue;
            const double sl = std::sqrt(len);
            for (double& v : nv) v /= sl;
            float nx = (float)nv[0], ny = (float)nv[1], nz = (float)nv[2];
            const float vx = 0.f - pc[idx].x, vy = 0.f - pc[idx].y, vz = 0.f - pc[idx].z;
            const float cos_theta = (vx * nx + vy * ny + vz * nz);
            if (cos_theta < 0) { nx *= -1; ny *= -1; nz *= -1; }
            R.nrm[3 * idx] = nx; R.nrm[3 * idx + 1] = ny; R.nrm[3 * idx + 2] = nz;
        }
    const float* nrm = R.nrm.data();

    // --- OrganizedMultiPlaneSegmentation::segment
    std::vector<float> pd(N);
    for (int i = 0; i < N; i++) pd[i] = pc[i].x * nrm[3 * i] + pc[i].y * nrm[3 * i + 1] + pc[i].z * nrm[3 * i + 2];
    const float ang_th = std::cos((float)(0.017453 * P.angle_th_deg));
    const float dist_th = P.dist_th;
    auto compare = [&](int i1, int i2) {
        float threshold = dist_th;
        const float z = pc[i1].x * 0.f + pc[i1].y * 0.f + pc[i1].z * 1.f;
        threshold *= z * z;
        const float nd = nrm[3 * i1] * nrm[3 * i2] + nrm[3 * i1 + 1] * nrm[3 * i2 + 1] + nrm[3 * i1 + 2] * nrm[3 * i2 + 2];
        return (std::fabs(pd[i1] - pd[i2]) < threshold) && (nd > ang_th);
    };
    const uint32_t invalid = std::numeric_limits<uint32_t>::max();
    std::vector<uint32_t> lab(N, invalid);
    std::vector<uint32_t> run;
    uint32_t clust = 0;
    auto find_root = [&](uint32_t x) { while (run[x] != x) x = run[x]; return x; };
    if (isfin(pc[0].x)) { lab[0] = clust++; run.push_back(lab[0]); }
    for (int c = 1; c < W; c++) {
        if (!isfin(pc[c].x)) continue;
        if (compare(c, c - 1)) lab[c] = lab[c - 1];
        else { lab[c] = clust++; run.push_back(lab[c]); }
    }
    for (int r = 1; r < H; r++) {
        const int cr = r * W, pr = (r - 1) * W;
        if (isfin(pc[cr].x)) {
            if (compare(cr, pr)) lab[cr] = lab[pr];
            else { lab[cr] = clust++; run.push_back(lab[cr]); }
        }
        for (int c = 1; c < W; c++) {
            const int i = cr + c;
            if (!isfin(pc[i].x)) continue;
            if (compare(i, i - 1)) lab[i] = lab[i - 1];
            if (compare(i, pr + c)) {
                if (lab[i] == invalid) lab[i] = lab[pr + c];
                else if (lab[pr + c] != invalid) {
                    uint32_t r1 = find_root(lab[i]), r2 = find_root(lab[pr + c]);
                    if (r1 < r2) run[r2] = r1;
                    else run[r1] = r2;
                }
            }
            if (lab[i] == invalid) { lab[i] = clust++; run.push_back(lab[i]); }
        }
    }
    std::vector<uint32_t> map(clust);
    uint32_t max_id = 0;
    for (uint32_t k = 0; k < run.size(); ++k) {
        if (run[k] == k) map[k] = max_id++;
        else map[k] = map[find_root(k)];
    }
    std::vector<std::vector<int>> label_indices(max_id + 1);
    for (int i = 0; i < N; i++)
        if (lab[i] != invalid) { lab[i] = map[lab[i]]; label_indices[lab[i]].push_back(i); }
    R.labels_cc = lab;

    std::vector<std::vector<float>> models;
    std::vector<std::vector<int>> inl;
    float vp[4] = {0, 0, 0, 0};
    for (size_t li = 0; li < label_indices.size(); li++) {
        const std::vector<int>& ids = label_indices[li];
        if (!((unsigned)ids.size() > (unsigned)P.min_size)) continue;
        float accu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i : ids) {
            const P3& p = pc[i];
            accu[0] += p.x * p.x; accu[1] += p.x * p.y; accu[2] += p.x * p.z;
            accu[3] += p.y * p.y; accu[4] += p.y * p.z; accu[5] += p.z * p.z;
            accu[6] += p.x; accu[7] += p.y; accu[8] += p.z;
        }
        const float cnt = (float)ids.size();
        for (float& a : accu) a /= cnt;
        float cen[4] = {accu[6], accu[7], accu[8], 1.f};
        float cov[3][3];
        cov[0][0] = accu[0] - accu[6] * accu[6];
        cov[0][1] = accu[1] - accu[6] * accu[7];
        cov[0][2] = accu[2] - accu[6] * accu[8];
        cov[1][1] = accu[3] - accu[7] * accu[7];
        cov[1][2] = accu[4] - accu[7] * accu[8];
        cov[2][2] = accu[5] - accu[8] * accu[8];
        cov[1][0] = cov[0][1]; cov[2][0] = cov[0][2]; cov[2][1] = cov[1][2];
        float ev, evec[3];
        eigen33(cov, &ev, evec);
        float pp[4] = {evec[0], evec[1], evec[2], 0.f};
        pp[3] = -1 * dot4(pp, cen);
        for (int k = 0; k < 4; k++) vp[k] -= cen[k];
        const float cos_theta = dot4(vp, pp);
        if (cos_theta < 0) {
            for (float& v : pp) v *= -1;
            pp[3] = 0;
            pp[3] = -1 * dot4(pp, cen);
        }
        float curvature;
        const float eig_sum = cov[0][0] + cov[1][1] + cov[2][2];
        if (eig_sum != 0) curvature = std::fabs(ev / eig_sum);
        else curvature = 0;
        if (curvature < 0.001f) {
            models.push_back({pp[0], pp[1], pp[2], pp[3]});
            inl.push_back(ids);
        }
    }

    // --- refine (two raster passes, PlaneRefinementComparator)
    std::vector<char> grow(label_indices.size(), 0);
    std::vector<int> l2m(label_indices.size(), 0);
    for (size_t i = 0; i < models.size(); i++) {
        const uint32_t ml = lab[inl[i][0]];
        l2m[ml] = (int)i;
        grow[ml] = 1;
    }
    auto rcompare = [&](int i1, int i2) {
        const int cl = (int)lab[i1], nl = (int)lab[i2];
        if (!(grow[cl] && !grow[nl])) return false;
        const std::vector<float>& m = models[l2m[cl]];
        const P3& p = pc[i2];
        const double ptp = std::fabs(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3]);
        const float threshold = 0.02f;
        return ptp < threshold;
    };
    for (int r = 0; r < H - 1; r++) {
        const int cr = r * W, nr = cr + W;
        for (int c = 0; c < W - 1; c++) {
            const int cl = (int)lab[cr + c], rl = (int)lab[cr + c + 1];
            if (cl < 0 || rl < 0) continue;
            if (rcompare(cr + c, cr + c + 1)) {
                lab[cr + c + 1] = cl;
                inl[l2m[cl]].push_back(cr + c + 1);
            }
            const int ll = (int)lab[nr + c];
            if (ll < 0) continue;
            if (rcompare(cr + c, nr + c)) {
                lab[nr + c] = cl;
                inl[l2m[cl]].push_back(nr + c);
            }
        }
    }
    for (int r = H - 1; r >= 1; r--) {
        const int cr = r * W, pr = cr - W;
        for (int c = W - 1; c >= 0; c--) {
            const int cl = (int)lab[cr + c], ll = (int)lab[cr + c - 1];
            if (cl < 0 || ll < 0) continue;
            if (rcompare(cr + c, cr + c - 1)) {
                lab[cr + c - 1] = cl;
                inl[l2m[cl]].push_back(cr + c - 1);
            }
            const int ul = (int)lab[pr + c];
            if (ul < 0) continue;
            if (rcompare(cr + c, pr + c)) {
                lab[pr + c] = cl;
                inl[l2m[cl]].push_back(pr + c);
            }
        }
    }
    R.labels_ref = lab;

    // --- boundaries: segmentAndRefine traces findLabeledRegionBoundary from
    // inlier_indices[i].indices[max_inlier_idx], the model's LAST inlier (its
    // last grow event, else its last component member in raster order)
    std::vector<std::vector<int>> contours(models.size());
    const int ddx[8] = {-1, -1, 0, 1, 1, 1, 0, -1}, ddy[8] = {0, -1, -1, -1, 0, 1, 1, 1};
    for (size_t i = 0; i < models.size(); i++) {
        const int start = inl[i].back();
        int cur = start, cx = start % W, cy = start / W;
        const uint32_t label = lab[start];
        int dir = -1;
        for (int d = 0; d < 8; ++d) {
            const int x = cx + ddx[d], y = cy + ddy[d];
            if (x >= 0 && x < W && y >= 0 && y < H && lab[y * W + x] != label) { dir = d; break; }
        }
        if (dir == -1) continue;
        std::vector<int>& b = contours[i];
        b.push_back(start);
        do {
            int nIdx = 0;
            for (int d = 1; d <= 8; ++d) {
                nIdx = (dir + d) & 7;
                const int x = cx + ddx[nIdx], y = cy + ddy[nIdx];
                if (x >= 0 && x < W && y >= 0 && y < H && lab[y * W + x] == label) break;
            }
            dir = (nIdx + 4) & 7;
            cx += ddx[nIdx];
            cy += ddy[nIdx];
            cur = cy * W + cx;
            b.push_back(cur);
        } while (cur != start && b.size() < (size_t)8 * N);
    }
    R.models = models;
    R.model_inliers = inl;
    R.model_contour = contours;

    // --- Frame.cc:912-934: sign normalisation + PlaneNotSeen
    R.coef.clear();
    R.kept_model.clear();
    for (size_t i = 0; i < models.size(); i++) {
        std::vector<float> cf = models[i];
        if (cf[3] < 0)
            for (float& v : cf) v = -v;
        bool seen = false;
        for (const auto& pm : R.coef) {
            const float d = pm[3] - cf[3];
            const float angle = std::fmaf(pm[2], cf[2], std::fmaf(pm[1], cf[1], pm[0] * cf[0]));  // GCC -O3 -march=native
            if ((double)d > 0.2 || (double)d < -0.2) continue;
            if ((double)angle < 0.9397 && (double)angle > -0.9397) continue;
            seen = true;
            break;
        }
        if (seen) continue;
        R.coef.push_back(cf);
        R.kept_model.push_back((int)i);
    }
}

}  // namespace planes
}  // namespace oracle

// ---------------------------------------------------------------------------
// C API.  The result of the last call is kept in a handle for stage access.
using namespace oracle::planes;

extern "C" {

void* oracle_planes_new() { return new Result(); }
void oracle_planes_free(void* h) { delete (Result*)h; }

// depth: float meters (W x H, row stride in floats).  Returns the number of
// kept planes.
int oracle_planes_extract(void* h, const float* depth, int w, int hgt, int stride, float fx, float fy, float cx,
                          float cy, int cloud_dis, int min_size, float angle_th, float dist_th) {
    Params P;
    P.fx = fx; P.fy = fy; P.cx = cx; P.cy = cy;
    P.cloud_dis = cloud_dis; P.min_size = min_size; P.angle_th_deg = angle_th; P.dist_th = dist_th;
    Result* R = (Result*)h;
    extract(depth, w, hgt, stride, P, *R);
    return (int)R->coef.size();
}
int oracle_planes_dims(void* h, int* W, int* H, int* n_models) {
    Result* R = (Result*)h;
    *W = R->W; *H = R->H; *n_models = (int)R->models.size();
    return (int)R->coef.size();
}
void oracle_planes_cloud(void* h, float* xyz) { std::memcpy(xyz, ((Result*)h)->cloud.data(), ((Result*)h)->cloud.size() * 12); }
void oracle_planes_normals(void* h, float* n) { std::memcpy(n, ((Result*)h)->nrm.data(), ((Result*)h)->nrm.size() * 4); }
void oracle_planes_distance(void* h, float* d) { std::memcpy(d, ((Result*)h)->dist.data(), ((Result*)h)->dist.size() * 4); }
void oracle_planes_labels(void* h, int refined, uint32_t* out) {
    Result* R = (Result*)h;
    const auto& v = refined ? R->labels_ref : R->labels_cc;
    std::memcpy(out, v.data(), v.size() * 4);
}
// model i: coefficients (pre-flip), inlier / contour counts
void oracle_planes_model(void* h, int i, float* coef, int* n_inliers, int* n_contour) {
    Result* R = (Result*)h;
    for (int k = 0; k < 4; k++) coef[k] = R->models[i][k];
    *n_inliers = (int)R->model_inliers[i].size();
    *n_contour = (int)R->model_contour[i].size();
}
void oracle_planes_model_inliers(void* h, int i, int* out) {
    const auto& v = ((Result*)h)->model_inliers[i];
    std::memcpy(out, v.data(), v.size() * 4);
}
void oracle_planes_model_contour(void* h, int i, int* out) {
    const auto& v = ((Result*)h)->model_contour[i];
    std::memcpy(out, v.data(), v.size() * 4);
}
// kept plane k: coefficients after the Frame sign flip, and its model index
int oracle_planes_kept(void* h, int k, float* coef) {
    Result* R = (Result*)h;
    for (int j = 0; j < 4; j++) coef[j] = R->coef[k][j];
    return R->kept_model[k];
}

}  // extern "C"
