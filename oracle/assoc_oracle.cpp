// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// CPU restatement of Map::AssociatePlanesByBoundary (src/Map.cc:196-340) and
// Map::PointDistanceFromPlane (src/Map.cc:343-359) for one frame:
//   pM = Frame::ComputePlaneWorldCoeff(i) = Tcw^T * coef   (src/Frame.cc:1146-1150;
//        cv::Mat float gemm, accumulated in double and rounded once -- OpenCV's
//        GEMMSingleMul<float,double>; OpenCV is absent here, so this rounding is
//        parity-unpinned)
//   for every map plane in mspMapPlanes order (a std::set<MapPlane*>, i.e. by
//   pointer; the build iterates by mnId):
//     angle = pM . pW (float);
//     |angle| > AssociationAngRef -> dis = min_p |pM . (p, 1)| over the map
//        plane's boundary cloud (float per point, double minimum starting at
//        100); dis < ldTh -> match, ldTh = dis, next map plane;
//     |angle| < lverTh -> vertical, lverTh = |angle|, next map plane;
//     |angle| > lparTh -> parallel, lparTh = |angle|.
//   mbNewPlane = some frame plane has no match.
// The frame's mvpMapPlanes / mvpParallelPlanes / mvpVerticalPlanes are never
// cleared by the reference, only overwritten when a candidate is found
// (:230-252): with carry != 0 the match / parallel / vertical arrays hold the
// frame's current associations on entry (TrackLocalMap's call after
// TrackWithMotionModel's outlier discard, src/Tracking.cc:1004-1028, 1058).
// The not-seen branches (:259-337) are dead (mvNotSeenPlaneCoefficients is
// never written, SURVEY.md §8 notes) and are not restated.
//
// FP: the reference is built with -O3 -march=native, where GCC contracts the
// float dot products a0*b0 + a1*b1 + a2*b2 (+ a3) into
// fma(a2, b2, fma(a0, b0, a1*b1)) (+ a3); written out here with explicit fmaf
// (tests/test_oracle_assoc.py checks that against g++ on this host).
#include <cmath>
#include <cstdint>

namespace oracle {
namespace assoc {

struct MapPlane {
    float world[4];
    int32_t id, boundary_offset, n_boundary, pad;
};

struct Params {
    float dis_th, angle_th, ver_th, par_th;  // Plane.AssociationDisRef / AngRef / VerticalThreshold / ParallelThreshold
};

inline float dot3(const float* a, const float* b) { return std::fmaf(a[2], b[2], std::fmaf(a[0], b[0], a[1] * b[1])); }

// Frame::ComputePlaneWorldCoeff: transpose(Tcw) * coef
void world_coeff(const float* Tcw, const float* coef, float* pM) {
    for (int j = 0; j < 4; j++) {
        double s = 0.0;
        for (int k = 0; k < 4; k++) s += (double)Tcw[4 * k + j] * (double)coef[k];
        pM[j] = (float)s;
    }
}

// Map::PointDistanceFromPlane
double point_distance_from_plane(const float* pM, const float* xyz, int n) {
    double res = 100;
    for (int i = 0; i < n; i++) {
        const float* p = xyz + 3 * i;
        const float dis = std::fabs(dot3(pM, p) + pM[3]);
        if (dis < res) res = dis;
    }
    return res;
}

}  // namespace assoc
}  // namespace oracle

extern "C" {

// Map planes must be given in mnId order.  Outputs per frame plane: index of the
// matched / parallel / vertical map plane (-1 if none; read first when carry != 0),
// the world coefficients and the min boundary distance to every map plane (-1
// where the angle test failed).
int oracle_planes_associate(const float* Tcw, const float* coefs, int n_planes, const void* map_planes, int n_map,
                            const float* boundary_xyz, const float* params, int32_t* match, int32_t* parallel,
                            int32_t* vertical, float* world, double* dist, int carry) {
    using namespace oracle::assoc;
    const MapPlane* M = (const MapPlane*)map_planes;
    const Params P{params[0], params[1], params[2], params[3]};
    int new_plane = 0;
    for (int i = 0; i < n_planes; i++) {
        float pM[4];
        world_coeff(Tcw, coefs + 4 * i, pM);
        if (world)
            for (int k = 0; k < 4; k++) world[4 * i + k] = pM[k];
        float ldTh = P.dis_th, lverTh = P.ver_th, lparTh = P.par_th;
        if (!carry) match[i] = parallel[i] = vertical[i] = -1;
        for (int j = 0; j < n_map; j++) {
            const float angle = dot3(pM, M[j].world);
            double dis = -1.0;
            if (angle > P.angle_th || angle < -P.angle_th) {
                dis = point_distance_from_plane(pM, boundary_xyz + 3 * (size_t)M[j].boundary_offset, M[j].n_boundary);
                if (dist) dist[(size_t)i * n_map + j] = dis;
                if (dis < ldTh) {
                    ldTh = (float)dis;
                    match[i] = j;
                    continue;
                }
            } else if (dist) {
                dist[(size_t)i * n_map + j] = -1.0;
            }
            if (angle < lverTh && angle > -lverTh) {
                lverTh = std::fabs(angle);
                vertical[i] = j;
                continue;
            }
            if (angle > lparTh || angle < -lparTh) {
                lparTh = std::fabs(angle);
                parallel[i] = j;
            }
        }
        if (match[i] < 0) new_plane = 1;
    }
    return new_plane;
}

}  // extern "C"
