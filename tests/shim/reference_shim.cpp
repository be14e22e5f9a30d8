// Reference-side shim, compiled: INTEGRATION.md sections 1-7 as C++ at the reference's call sites.
//
// The classes below carry the members of SP-SLAM's ORBextractor / Frame / KeyFrame / MapPoint / MapPlane
// that the hot path reads and writes (include/ORBextractor.h, include/Frame.h, include/KeyFrame.h,
// include/MapPoint.h, include/MapPlane.h), with cv::Mat / cv::KeyPoint from cv_lite.h (OpenCV is not in this
// image).  The member functions are the reference's call sites re-implemented over the C ABI
// (include/spslam_gpu.h):
//   ORBextractor::operator()                       src/ORBextractor.cc:1043-1105          
//   Frame RGB-D constructor: planes, keypoint steps src/Frame.cc:130-197, 854-936, 938-1144 (2, 4, 5)
//   Optimizer::PoseOptimization                    src/Optimizer.cc:519-1152             (3)
//   Optimizer::LocalBundleAdjustment               src/Optimizer.cc:1154-1977            (6)
//   Tracking::GrabImageRGBD                        src/Tracking.cc:208-229               (7)
//   Map::AssociatePlanesByBoundary                 src/Map.cc:196-359                    (8, f1)
//   ORBmatcher::SearchByProjection (motion model)  src/ORBmatcher.cc:1328-1470, Tracking.cc:951-975 (9, f2)
//   Frame/KeyFrame::ComputeBoW, ORBmatcher::SearchByBoW  src/Frame.cc:495-502, ORBmatcher.cc:159-288 (11, f4)
// extern "C" entry points at the end let tests/test_gpu_shim.py drive them from flat arrays and compare with
// the oracle.  TEST INFRASTRUCTURE: built by `make` into tests/shim/libreference_shim.so, never part of the
// product library.
#include <algorithm>
#include <array>
#include <cmath>
#include <list>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/spslam_gpu.h"
#include "cv_lite.h"

namespace ORB_SLAM2 {

static void check(spslam_ctx* ctx, int rc, const char* what) {
    if (rc != SPSLAM_OK) throw std::runtime_error(std::string(what) + ": " + (ctx ? spslam_last_error(ctx) : "?"));
}

// ---------------------------------------------------------------------------------------------------- 1
class ORBextractor {
   public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int width, int height) {
        spslam_orb_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, width, height, /*max_batch*/ 1};
        check(nullptr, spslam_create(0, &p, &mGpu), "spslam_create");
        nlevels_ = nlevels;
        mvInvLevelSigma2.resize(nlevels);
        check(mGpu, spslam_orb_tables(mGpu, nullptr, nullptr, nullptr, nullptr, mvInvLevelSigma2.data(), nullptr),
              "spslam_orb_tables");
    }
    ~ORBextractor() { spslam_destroy(mGpu); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // ORBextractor::operator()(InputArray image, InputArray mask, vector<KeyPoint>&, OutputArray descriptors)
    void operator()(const cv::Mat& image, const cv::Mat& /*mask*/, std::vector<cv::KeyPoint>& kps, cv::Mat& desc) {
        if (image.empty()) return;
        const int cap = spslam_orb_max_keypoints(mGpu);
        std::vector<cv::KeyPoint> tmp(cap);  // spslam_keypoint is bit-compatible with cv::KeyPoint
        cv::Mat d(cap, 32, cv::CV_8U);
        int n = 0;
        check(mGpu, spslam_orb_extract(mGpu, image.data, image.cols, image.rows, (int)image.step,
                                       reinterpret_cast<spslam_keypoint*>(tmp.data()), d.data, cap, &n),
              "spslam_orb_extract");
        kps.assign(tmp.begin(), tmp.begin() + n);
        desc = cv::Mat(n, 32, cv::CV_8U);
        if (n) std::memcpy(desc.data, d.data, (size_t)n * 32);
    }
    const std::vector<float>& GetInverseScaleSigmaSquares() const { return mvInvLevelSigma2; }
    spslam_ctx* mGpu = nullptr;  // the one GPU context of this tracker (ORB, frame steps, planes, optimizers)

   private:
    int nlevels_ = 8;
    std::vector<float> mvInvLevelSigma2;
};

class KeyFrame;
struct ById {  // id order replaces the reference's pointer-ordered std::map / std::set
    template <class T> bool operator()(const T* a, const T* b) const { return a->mnId < b->mnId; }
};

class MapPoint {
   public:
    long unsigned int mnId = 0;
    cv::Mat mWorldPos{3, 1, cv::CV_32F};
    cv::Mat mDescriptor{1, 32, cv::CV_8U};
    int nObs = 0;  // kept by AddObservation / EraseObservation in the reference
    cv::Mat GetDescriptor() const { return mDescriptor.clone(); }
    int Observations() const { return nObs; }
    std::map<KeyFrame*, size_t, ById> mObservations;
    long unsigned int mnBALocalForKF = 0;
    bool mbBad = false;
    cv::Mat GetWorldPos() const { return mWorldPos.clone(); }
    void SetWorldPos(const float* x) { for (int i = 0; i < 3; i++) mWorldPos.at<float>(i) = x[i]; }
    bool isBad() const { return mbBad; }
    const std::map<KeyFrame*, size_t, ById>& GetObservations() const { return mObservations; }
    void EraseObservation(KeyFrame* pKF) { mObservations.erase(pKF); }
};

struct PointXYZ { float x, y, z; };
struct BoundaryCloud { std::vector<PointXYZ> points; };  // pcl::PointCloud<PointT> stand-in

class MapPlane {
   public:
    long unsigned int mnId = 0;
    cv::Mat mWorldPos{4, 1, cv::CV_32F};
    BoundaryCloud mvBoundaryPoints;
    std::map<KeyFrame*, int, ById> mObservations, mVerObservations, mParObservations;
    long unsigned int mnBALocalForKF = 0;
    cv::Mat GetWorldPos() const { return mWorldPos.clone(); }
    void SetWorldPos(const float* x) { for (int i = 0; i < 4; i++) mWorldPos.at<float>(i) = x[i]; }
};

class KeyFrame {
   public:
    long unsigned int mnId = 0;
    cv::Mat mTcw{4, 4, cv::CV_32F};
    float fx = 0, fy = 0, cx = 0, cy = 0, mbf = 0;
    int N = 0;
    std::vector<cv::KeyPoint> mvKeysUn;
    cv::Mat mDescriptors;
    std::map<unsigned int, double> mBowVec;                       // DBoW2::BowVector
    std::map<unsigned int, std::vector<unsigned int>> mFeatVec;   // DBoW2::FeatureVector
    std::vector<float> mvuRight;
    std::vector<float> mvInvLevelSigma2;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<std::array<float, 4>> mvPlaneCoefficients;
    std::vector<MapPlane*> mvpMapPlanes;  // size mnPlaneNum
    int mnPlaneNum = 0;
    std::vector<KeyFrame*> mvpOrderedConnectedKeyFrames;
    long unsigned int mnBALocalForKF = 0, mnBAFixedForKF = 0;
    bool mbBad = false;
    bool isBad() const { return mbBad; }
    std::vector<KeyFrame*> GetVectorCovisibleKeyFrames() const { return mvpOrderedConnectedKeyFrames; }
    std::vector<MapPoint*> GetMapPointMatches() const { return mvpMapPoints; }
    cv::Mat GetPose() const { return mTcw.clone(); }
    void SetPose(const float* T) { std::memcpy(mTcw.data, T, 64); }
    void EraseMapPointMatch(size_t idx) { mvpMapPoints[idx] = nullptr; }
};

// ---------------------------------------------------------------------------------------------------- 2, 4, 5
struct CameraConfig {  // the Camera.* / Plane.* / Line.* keys the RGB-D Frame reads
    float fx, fy, cx, cy, dist[5], bf;
    int cloud_dis, min_size;
    float angle_threshold, distance_threshold;
    double line_ratio;
    float line_distance_threshold;
};

class Frame {
   public:
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    cv::Mat mDescriptors;
    std::vector<float> mvuRight, mvDepth;
    std::vector<float> mvInvLevelSigma2;
    std::vector<std::vector<std::size_t>> mGrid;  // 64 x 48 cells, column major as FRAME_GRID_COLS x ROWS
    std::vector<std::array<float, 4>> mvPlaneCoefficients;
    std::vector<std::vector<int32_t>> mvPlanePointIdx, mvBoundaryPointIdx;  // organized-cloud indices (PCL clouds)
    int mnPlaneNum = 0, mnRealPlaneNum = 0;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    std::vector<MapPlane*> mvpMapPlanes, mvpParallelPlanes, mvpVerticalPlanes;
    std::vector<bool> mvbPlaneOutlier, mvbParPlaneOutlier, mvbVerPlaneOutlier;
    bool mbNewPlane = false;
    std::map<unsigned int, double> mBowVec;                       // DBoW2::BowVector
    std::map<unsigned int, std::vector<unsigned int>> mFeatVec;   // DBoW2::FeatureVector
    cv::Mat mTcw{4, 4, cv::CV_32F};
    float fx = 0, fy = 0, cx = 0, cy = 0, mbf = 0;
    ORBextractor* mpORBextractorLeft = nullptr;

    Frame() = default;
    // Frame::Frame(imGray, imDepth, timeStamp, extractor, voc, K, distCoef, bf, thDepth) (src/Frame.cc:130-197):
    // ORB (1), then -- N > 0 -- UndistortKeyPoints + ComputeStereoFromRGBD + AssignFeaturesToGrid (4),
    // ComputePlanesFromOrganizedPointCloud (2) and GeneratePlanesFromBoundries (5).
    Frame(const cv::Mat& imGray, const cv::Mat& imDepth, ORBextractor* extractor, const CameraConfig& K) {
        spslam_ctx* ctx = extractor->mGpu;
        mpORBextractorLeft = extractor;
        fx = K.fx; fy = K.fy; cx = K.cx; cy = K.cy; mbf = K.bf;
        (*extractor)(imGray, cv::Mat(), mvKeys, mDescriptors);
        N = (int)mvKeys.size();
        mvInvLevelSigma2 = extractor->GetInverseScaleSigmaSquares();
        if (N == 0) return;  // src/Frame.cc:148-149
        // mbInitialComputations (Frame.cc:162-177): image bounds and grid scale (every Frame here; the context
        // keeps them, so a tracker would call this once)
        spslam_frame_params fp{K.fx, K.fy, K.cx, K.cy, {K.dist[0], K.dist[1], K.dist[2], K.dist[3], K.dist[4]},
                               K.bf, imGray.cols, imGray.rows};
        float bounds[4];
        check(ctx, spslam_frame_configure(ctx, &fp, bounds, nullptr), "spslam_frame_configure");
        std::vector<int32_t> goff(64 * 48 + 1), gidx(N);
        mvKeysUn.resize(N);
        mvDepth.resize(N);
        mvuRight.resize(N);
        check(ctx, spslam_frame_rgbd(ctx, reinterpret_cast<const spslam_keypoint*>(mvKeys.data()), N,
                                     imDepth.ptr<float>(), imDepth.cols, imDepth.rows, (int)(imDepth.step / 4),
                                     reinterpret_cast<spslam_keypoint*>(mvKeysUn.data()), mvDepth.data(),
                                     mvuRight.data(), goff.data(), gidx.data()),
              "spslam_frame_rgbd");
        mGrid.assign(64 * 48, {});
        for (int c = 0; c < 64 * 48; ++c) mGrid[c].assign(gidx.begin() + goff[c], gidx.begin() + goff[c + 1]);
        mvpMapPoints.assign(N, nullptr);
        mvbOutlier.assign(N, false);

        // 2: ComputePlanesFromOrganizedPointCloud
        spslam_plane_params pp{K.cloud_dis, K.min_size, K.angle_threshold, K.distance_threshold, K.fx, K.fy, K.cx, K.cy,
                               imDepth.cols, imDepth.rows, K.line_ratio, K.line_distance_threshold,
                               {bounds[0], bounds[1], bounds[2], bounds[3]}};
        check(ctx, spslam_planes_configure(ctx, &pp), "spslam_planes_configure");
        int pcap, icap, ccap, n = 0;
        check(ctx, spslam_planes_capacity(ctx, &pcap, &icap, &ccap), "spslam_planes_capacity");
        std::vector<spslam_plane> pl(pcap);
        std::vector<int32_t> inl(icap), con(ccap);
        check(ctx, spslam_planes_extract(ctx, imDepth.ptr<float>(), imDepth.cols, imDepth.rows, (int)(imDepth.step / 4),
                                         pl.data(), pcap, &n, inl.data(), con.data()),
              "spslam_planes_extract");
        for (int k = 0; k < n; ++k) {
            mvPlanePointIdx.emplace_back(inl.begin() + pl[k].inlier_offset,
                                         inl.begin() + pl[k].inlier_offset + pl[k].n_inliers);
            mvBoundaryPointIdx.emplace_back(con.begin() + pl[k].contour_offset,
                                            con.begin() + pl[k].contour_offset + pl[k].n_contour);
            mvPlaneCoefficients.push_back({pl[k].coef[0], pl[k].coef[1], pl[k].coef[2], pl[k].coef[3]});
        }
        mnRealPlaneNum = n;
        // 5: GeneratePlanesFromBoundries (src/Frame.cc:186-194), on the same frame
        int scap, lcap, npatch, m = 0;
        check(ctx, spslam_supposed_capacity(ctx, &scap, &lcap, &npatch), "spslam_supposed_capacity");
        std::vector<spslam_supposed_plane> sp(scap);
        std::vector<int32_t> lidx(lcap);
        std::vector<float> patch((size_t)scap * npatch * 3);
        check(ctx, spslam_planes_generate_from_boundaries(ctx, imDepth.ptr<float>(), imDepth.cols, imDepth.rows,
                                                          (int)(imDepth.step / 4), sp.data(), scap, &m, lidx.data(),
                                                          patch.data()),
              "spslam_planes_generate_from_boundaries");
        for (int k = 0; k < m && k < scap; ++k) {
            mvBoundaryPointIdx.emplace_back(lidx.begin() + sp[k].line_offset,
                                            lidx.begin() + sp[k].line_offset + sp[k].n_line);
            mvPlanePointIdx.push_back(mvBoundaryPointIdx.back());  // + the synthetic patch (points, not indices)
            mvPlaneCoefficients.push_back({sp[k].coef[0], sp[k].coef[1], sp[k].coef[2], sp[k].coef[3]});
        }
        mnPlaneNum = (int)mvPlaneCoefficients.size();
        mvpMapPlanes.assign(mnPlaneNum, nullptr);
        mvpParallelPlanes.assign(mnPlaneNum, nullptr);
        mvpVerticalPlanes.assign(mnPlaneNum, nullptr);
        mvbPlaneOutlier.assign(mnPlaneNum, false);
        mvbParPlaneOutlier.assign(mnPlaneNum, false);
        mvbVerPlaneOutlier.assign(mnPlaneNum, false);
    }
    void SetPose(const float* T) { std::memcpy(mTcw.data, T, 64); }
    void ComputeBoW();
};

// ---------------------------------------------------------------------------------------------------- 11 (f4)
// The vocabulary is loaded into the tracker's context once, where System loads ORBvoc.txt (src/System.cc:59-71).
inline void LoadVocabulary(spslam_ctx* ctx, const std::string& text) {
    check(ctx, spslam_bow_load_vocabulary(ctx, text.data(), text.size(), nullptr, nullptr, nullptr, nullptr),
          "spslam_bow_load_vocabulary");
}
// Frame::ComputeBoW / KeyFrame::ComputeBoW (src/Frame.cc:495-502, src/KeyFrame.cc:64-72): transform(desc, mBowVec,
// mFeatVec, 4)
inline void ComputeBoW(spslam_ctx* ctx, const cv::Mat& desc, std::map<unsigned int, double>& bowVec,
                       std::map<unsigned int, std::vector<unsigned int>>& featVec) {
    if (!bowVec.empty()) return;
    const int n = desc.rows;
    std::vector<uint32_t> bw(std::max(n, 1)), fvn(std::max(n, 1));
    std::vector<double> bv(std::max(n, 1));
    std::vector<int32_t> fvs(n + 1), fvf(std::max(n, 1));
    int nb = 0, nfv = 0;
    check(ctx, spslam_bow_transform(ctx, desc.data, n, 4, bw.data(), bv.data(), &nb, fvn.data(), fvs.data(),
                                    fvf.data(), &nfv),
          "spslam_bow_transform");
    for (int i = 0; i < nb; ++i) bowVec[bw[i]] = bv[i];
    for (int j = 0; j < nfv; ++j) featVec[fvn[j]].assign(fvf.begin() + fvs[j], fvf.begin() + fvs[j + 1]);
}
inline void Frame::ComputeBoW() { ORB_SLAM2::ComputeBoW(mpORBextractorLeft->mGpu, mDescriptors, mBowVec, mFeatVec); }

// ---------------------------------------------------------------------------------------------------- 9, 11
class ORBmatcher {
   public:
    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

    // SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono) (src/ORBmatcher.cc:1328-1470):
    // the last frame's map points (mvpMapPoints[i] && !mvbOutlier[i], in i order) against the current frame's
    // grid; the assignments go into CurrentFrame.mvpMapPoints
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, float th, bool bMono) const {
        spslam_ctx* ctx = CurrentFrame.mpORBextractorLeft->mGpu;
        std::vector<spslam_proj_point> pts;
        std::vector<MapPoint*> src;
        for (int i = 0; i < LastFrame.N; ++i) {
            MapPoint* pMP = LastFrame.mvpMapPoints[i];
            if (!pMP || LastFrame.mvbOutlier[i]) continue;
            const cv::Mat x = pMP->GetWorldPos(), d = pMP->GetDescriptor();
            spslam_proj_point p{};
            for (int k = 0; k < 3; ++k) p.xw[k] = x.at<float>(k);
            p.angle = LastFrame.mvKeysUn[i].angle;
            p.octave = LastFrame.mvKeys[i].octave;
            p.n_obs = pMP->Observations();
            p.last_index = i;
            p.id = (int)pMP->mnId;
            std::memcpy(p.desc, d.data, 32);
            pts.push_back(p);
            src.push_back(pMP);
        }
        spslam_proj_frame fr{};
        std::memcpy(fr.Tcw, CurrentFrame.mTcw.data, 64);
        std::memcpy(fr.Tlw, LastFrame.mTcw.data, 64);
        fr.n_points = (int)pts.size();
        std::vector<int32_t> goff(1, 0), gidx;
        for (const auto& cell : CurrentFrame.mGrid) {
            for (size_t k : cell) gidx.push_back((int32_t)k);
            goff.push_back((int32_t)gidx.size());
        }
        gidx.push_back(0);
        const spslam_match_params prm{th, bMono ? 1 : 0, mbCheckOrientation ? 1 : 0, /*retry_below*/ 0};
        std::vector<int32_t> match(std::max(CurrentFrame.N, 1));
        int n = 0;
        check(ctx, spslam_search_by_projection(ctx, &fr, pts.data(),
                                               reinterpret_cast<const spslam_keypoint*>(CurrentFrame.mvKeysUn.data()),
                                               CurrentFrame.mDescriptors.data, CurrentFrame.mvuRight.data(),
                                               CurrentFrame.N, goff.data(), gidx.data(), &prm, match.data(), &n),
              "spslam_search_by_projection");
        for (int i = 0; i < CurrentFrame.N; ++i)
            if (match[i] >= 0) CurrentFrame.mvpMapPoints[i] = src[match[i]];
        return n;
    }

    // SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches) (src/ORBmatcher.cc:159-288)
    int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) const {
        spslam_ctx* ctx = F.mpORBextractorLeft->mGpu;
        const std::vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
        std::vector<uint8_t> has(std::max(pKF->N, 1));
        for (int i = 0; i < pKF->N; ++i) has[i] = vpMapPointsKF[i] && !vpMapPointsKF[i]->isBad();
        std::vector<uint32_t> kn, fn;
        std::vector<int32_t> ks, kf, fs, ff;
        const int nk = flat(pKF->mFeatVec, kn, ks, kf), nf = flat(F.mFeatVec, fn, fs, ff);
        const spslam_bow_params prm{mfNNratio, mbCheckOrientation ? 1 : 0};
        std::vector<int32_t> match(std::max(F.N, 1));
        int nmatches = 0;
        check(ctx, spslam_search_by_bow(ctx, pKF->mDescriptors.data,
                                        reinterpret_cast<const spslam_keypoint*>(pKF->mvKeysUn.data()), has.data(),
                                        pKF->N, kn.data(), ks.data(), kf.data(), nk, F.mDescriptors.data,
                                        reinterpret_cast<const spslam_keypoint*>(F.mvKeys.data()), F.N, fn.data(),
                                        fs.data(), ff.data(), nf, &prm, match.data(), &nmatches),
              "spslam_search_by_bow");
        vpMapPointMatches = std::vector<MapPoint*>(F.N, static_cast<MapPoint*>(nullptr));
        for (int i = 0; i < F.N; ++i)
            if (match[i] >= 0) vpMapPointMatches[i] = vpMapPointsKF[match[i]];
        return nmatches;
    }

    float mfNNratio;
    bool mbCheckOrientation;

   private:
    // a FeatureVector (std::map: ascending node id) as the ABI's CSR; returns its node count
    static int flat(const std::map<unsigned int, std::vector<unsigned int>>& fv, std::vector<uint32_t>& nodes,
                    std::vector<int32_t>& start, std::vector<int32_t>& feats) {
        for (const auto& kv : fv) {
            nodes.push_back(kv.first);
            start.push_back((int32_t)feats.size());
            feats.insert(feats.end(), kv.second.begin(), kv.second.end());
        }
        start.push_back((int32_t)feats.size());
        nodes.push_back(0);  // (non-empty buffers)
        feats.push_back(0);
        return (int)fv.size();
    }
};

// ---------------------------------------------------------------------------------------------------- 8 (f1)
class Map {
   public:
    std::set<MapPlane*, ById> mspMapPlanes;  // id order replaces the pointer order
    float mfDisTh = 0, mfAngleTh = 0, mfVerTh = 0, mfParTh = 0;
    spslam_ctx* mGpu = nullptr;

    // Map::AssociatePlanesByBoundary(Frame& pF, bool out) (src/Map.cc:196-359): the map planes flattened in
    // mnId order; pF's current associations handed in (the reference only overwrites them, :230-252)
    void AssociatePlanesByBoundary(Frame& pF, bool /*out*/ = false) {
        std::vector<spslam_map_plane> mp;
        std::vector<float> bxyz;
        std::vector<MapPlane*> byIndex;
        std::map<unsigned long, int> indexById;
        for (MapPlane* p : mspMapPlanes) {
            const cv::Mat w = p->GetWorldPos();
            indexById[p->mnId] = (int)mp.size();
            byIndex.push_back(p);
            mp.push_back({{w.at<float>(0), w.at<float>(1), w.at<float>(2), w.at<float>(3)}, (int)p->mnId,
                          (int)(bxyz.size() / 3), (int)p->mvBoundaryPoints.points.size(), 0});
            for (const PointXYZ& q : p->mvBoundaryPoints.points) {
                bxyz.push_back(q.x);
                bxyz.push_back(q.y);
                bxyz.push_back(q.z);
            }
        }
        spslam_assoc_frame f{};
        std::memcpy(f.Tcw, pF.mTcw.data, 64);
        f.n_map = (int)mp.size();
        f.carry = 1;
        const int n = pF.mnPlaneNum;
        std::vector<int32_t> m(std::max(n, 1)), par(std::max(n, 1)), ver(std::max(n, 1));
        std::vector<float> coefs(4 * std::max(n, 1));
        auto idx = [&](MapPlane* p) { return p ? indexById.at(p->mnId) : -1; };
        for (int i = 0; i < n; ++i) {
            m[i] = idx(pF.mvpMapPlanes[i]);
            par[i] = idx(pF.mvpParallelPlanes[i]);
            ver[i] = idx(pF.mvpVerticalPlanes[i]);
            for (int q = 0; q < 4; ++q) coefs[4 * i + q] = pF.mvPlaneCoefficients[i][q];
        }
        const spslam_assoc_params prm{mfDisTh, mfAngleTh, mfVerTh, mfParTh};
        int newPlane = 0;
        bxyz.resize(std::max<size_t>(bxyz.size(), 3));
        check(mGpu, spslam_planes_associate(mGpu, &f, coefs.data(), n, mp.data(), (int)mp.size(), bxyz.data(),
                                            (int)(bxyz.size() / 3), &prm, m.data(), par.data(), ver.data(), &newPlane),
              "spslam_planes_associate");
        for (int i = 0; i < n; ++i) {
            pF.mvpMapPlanes[i] = m[i] < 0 ? nullptr : byIndex[m[i]];
            pF.mvpParallelPlanes[i] = par[i] < 0 ? nullptr : byIndex[par[i]];
            pF.mvpVerticalPlanes[i] = ver[i] < 0 ? nullptr : byIndex[ver[i]];
        }
        pF.mbNewPlane = newPlane != 0;
    }
};

// ---------------------------------------------------------------------------------------------------- 7
// Tracking::GrabImageRGBD's image preparation: cvtColor to gray + depth convertTo(CV_32F, mDepthMapFactor)
inline void GrabImageRGBD(spslam_ctx* ctx, const cv::Mat& imRGB, const cv::Mat& imD, bool mbRGB, float depthFactor,
                          cv::Mat& imGray, cv::Mat& imDepth) {
    spslam_grab_params gp{imRGB.channels(), mbRGB ? 1 : 0, imD.type() == cv::CV_16U ? 1 : 0, depthFactor};
    imGray.create(imRGB.rows, imRGB.cols, cv::CV_8U);
    imDepth.create(imD.rows, imD.cols, cv::CV_32F);
    check(ctx, spslam_grab_rgbd(ctx, imRGB.data, (int)imRGB.step, imD.data, (int)(imD.step / imD.elemSize()),
                                imRGB.cols, imRGB.rows, &gp, imGray.data, imDepth.ptr<float>()),
          "spslam_grab_rgbd");
}

// ---------------------------------------------------------------------------------------------------- 3, 6
class Optimizer {
   public:
    // Optimizer::PoseOptimization(Frame*): the graph's edges flattened in the reference's insertion order --
    // points by keypoint index (:561-647), then plane, parallel, vertical edges by plane index (:700-859)
    static int PoseOptimization(spslam_ctx* ctx, Frame* F, const spslam_plane_config& cfg) {
        std::vector<spslam_point_obs> pts;
        std::vector<int> ptIdx;
        for (int i = 0; i < F->N; ++i) {
            MapPoint* mp = F->mvpMapPoints[i];
            if (!mp) continue;
            const cv::Mat X = mp->GetWorldPos();
            const cv::KeyPoint& k = F->mvKeysUn[i];
            pts.push_back({k.pt.x, k.pt.y, F->mvuRight[i], F->mvInvLevelSigma2[k.octave],
                           {X.at<float>(0), X.at<float>(1), X.at<float>(2)}, i});
            ptIdx.push_back(i);
        }
        std::vector<spslam_plane_obs> pls;
        std::vector<int> plIdx;
        const std::vector<MapPlane*>* lists[3] = {&F->mvpMapPlanes, &F->mvpParallelPlanes, &F->mvpVerticalPlanes};
        for (int kind = 0; kind < 3; ++kind)
            for (int i = 0; i < F->mnPlaneNum; ++i) {
                MapPlane* p = (*lists[kind])[i];
                if (!p) continue;
                const cv::Mat w = p->GetWorldPos();
                spslam_plane_obs o{};
                for (int q = 0; q < 4; ++q) { o.meas[q] = F->mvPlaneCoefficients[i][q]; o.world[q] = w.at<float>(q); }
                o.kind = kind;
                o.plane_index = i;
                o.map_plane_id = (int)p->mnId;
                pls.push_back(o);
                plIdx.push_back(i);
            }
        spslam_pose_problem pr{};
        std::memcpy(pr.Tcw, F->mTcw.ptr<float>(), 64);
        pr.fx = F->fx; pr.fy = F->fy; pr.cx = F->cx; pr.cy = F->cy; pr.bf = F->mbf;
        pr.n_points = (int)pts.size();
        pr.n_planes = (int)pls.size();
        spslam_pose_result res;
        std::vector<uint8_t> po(std::max<size_t>(pts.size(), 1)), plo(std::max<size_t>(pls.size(), 1));
        check(ctx, spslam_pose_optimize(ctx, &pr, pts.data(), pls.data(), &cfg, &res, po.data(), plo.data()),
              "spslam_pose_optimize");
        for (size_t k = 0; k < pts.size(); ++k) F->mvbOutlier[ptIdx[k]] = po[k] != 0;
        for (size_t k = 0; k < pls.size(); ++k) {
            std::vector<bool>& flags = pls[k].kind == 0   ? F->mvbPlaneOutlier
                                       : pls[k].kind == 1 ? F->mvbParPlaneOutlier
                                                          : F->mvbVerPlaneOutlier;
            flags[plIdx[k]] = plo[k] != 0;
        }
        if (pts.size() < 3) return 0;  // nInitialCorrespondences < 3: no SetPose (:653)
        F->SetPose(res.Tcw);
        return res.n_inliers;
    }

    // The flattened problem of one LocalBundleAdjustment call (kept for the test's checks).
    struct LbaGraph {
        std::vector<KeyFrame*> kfs;          // local, then fixed
        std::vector<MapPoint*> points;
        std::vector<MapPlane*> planes;
        std::vector<std::pair<MapPoint*, KeyFrame*>> point_obs_src;
        std::vector<std::pair<MapPlane*, KeyFrame*>> plane_obs_src;
        spslam_lba_problem prob{};
        std::vector<spslam_lba_keyframe> k;
        std::vector<spslam_lba_point> p;
        std::vector<spslam_lba_point_obs> po;
        std::vector<spslam_lba_plane> q;
        std::vector<spslam_lba_plane_obs> qo;
        spslam_lba_result res{};
        std::vector<uint8_t> po_out, qo_out;
    };

    // Optimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap): the graph collection of :1156-1298 (local
    // keyframes, local map points / planes, fixed cameras), flattened for spslam_lba_optimize, and the result
    // application of :1896-1977 (outlier observations erased, poses and positions set).
    static void LocalBundleAdjustment(spslam_ctx* ctx, KeyFrame* pKF, bool* pbStopFlag, const spslam_plane_config& cfg,
                                      LbaGraph& G) {
        std::list<KeyFrame*> lLocalKeyFrames{pKF};
        pKF->mnBALocalForKF = pKF->mnId;
        for (KeyFrame* pKFi : pKF->GetVectorCovisibleKeyFrames()) {
            pKFi->mnBALocalForKF = pKF->mnId;
            if (!pKFi->isBad()) lLocalKeyFrames.push_back(pKFi);
        }
        std::list<MapPoint*> lLocalMapPoints;
        std::list<MapPlane*> lLocalMapPlanes;
        for (KeyFrame* pKFi : lLocalKeyFrames) {
            for (MapPoint* pMP : pKFi->GetMapPointMatches())
                if (pMP && !pMP->isBad() && pMP->mnBALocalForKF != pKF->mnId) {
                    lLocalMapPoints.push_back(pMP);
                    pMP->mnBALocalForKF = pKF->mnId;
                }
            for (int i = 0; i < pKFi->mnPlaneNum; ++i) {
                MapPlane* pMP = pKFi->mvpMapPlanes[i];
                if (pMP && pMP->mnBALocalForKF != pKF->mnId) {
                    lLocalMapPlanes.push_back(pMP);
                    pMP->mnBALocalForKF = pKF->mnId;
                }
            }
        }
        std::list<KeyFrame*> lFixedCameras;
        auto fixed = [&](KeyFrame* pKFi) {
            if (pKFi->mnBALocalForKF != pKF->mnId && pKFi->mnBAFixedForKF != pKF->mnId) {
                pKFi->mnBAFixedForKF = pKF->mnId;
                if (!pKFi->isBad()) lFixedCameras.push_back(pKFi);
            }
        };
        for (MapPoint* pMP : lLocalMapPoints)
            for (auto& o : pMP->GetObservations()) fixed(o.first);
        for (MapPlane* pMP : lLocalMapPlanes) {
            for (auto& o : pMP->mObservations) fixed(o.first);
            for (auto& o : pMP->mVerObservations) fixed(o.first);
            for (auto& o : pMP->mParObservations) fixed(o.first);
        }

        // flatten: keyframes (local, then fixed), points with their observations, planes with their
        // observation / vertical / parallel edges (the reference's edge insertion order, :1383-1613)
        std::map<KeyFrame*, int> kidx;
        for (KeyFrame* pKFi : lLocalKeyFrames) { kidx[pKFi] = (int)G.kfs.size(); G.kfs.push_back(pKFi); }
        const int nLocal = (int)G.kfs.size();
        for (KeyFrame* pKFi : lFixedCameras) { kidx[pKFi] = (int)G.kfs.size(); G.kfs.push_back(pKFi); }
        for (size_t i = 0; i < G.kfs.size(); ++i) {
            KeyFrame* f = G.kfs[i];
            spslam_lba_keyframe r{};
            std::memcpy(r.Tcw, f->mTcw.ptr<float>(), 64);
            r.fx = f->fx; r.fy = f->fy; r.cx = f->cx; r.cy = f->cy; r.bf = f->mbf;
            r.id = (int32_t)f->mnId;
            r.fixed = (int)i >= nLocal;
            G.k.push_back(r);
        }
        for (MapPoint* pMP : lLocalMapPoints) {
            spslam_lba_point r{};
            const cv::Mat X = pMP->GetWorldPos();
            for (int i = 0; i < 3; i++) r.xw[i] = X.at<float>(i);
            r.id = (int32_t)pMP->mnId;
            r.obs_offset = (int32_t)G.po.size();
            for (auto& o : pMP->GetObservations()) {
                KeyFrame* pKFi = o.first;
                if (pKFi->isBad() || !kidx.count(pKFi)) continue;
                const cv::KeyPoint& kp = pKFi->mvKeysUn[o.second];
                G.po.push_back({kidx[pKFi], kp.pt.x, kp.pt.y, pKFi->mvuRight[o.second],
                                pKFi->mvInvLevelSigma2[kp.octave]});
                G.point_obs_src.push_back({pMP, pKFi});
            }
            r.n_obs = (int32_t)G.po.size() - r.obs_offset;
            G.p.push_back(r);
            G.points.push_back(pMP);
        }
        for (MapPlane* pMP : lLocalMapPlanes) {
            spslam_lba_plane r{};
            const cv::Mat W = pMP->GetWorldPos();
            for (int i = 0; i < 4; i++) r.world[i] = W.at<float>(i);
            r.id = (int32_t)pMP->mnId;
            r.obs_offset = (int32_t)G.qo.size();
            const std::pair<const std::map<KeyFrame*, int, ById>*, int> kinds[3] = {
                {&pMP->mObservations, SPSLAM_PLANE_EDGE},
                {&pMP->mVerObservations, SPSLAM_VERTICAL_EDGE},
                {&pMP->mParObservations, SPSLAM_PARALLEL_EDGE}};
            for (auto& kd : kinds)
                for (auto& o : *kd.first) {
                    KeyFrame* pKFi = o.first;
                    if (pKFi->isBad() || !kidx.count(pKFi)) continue;
                    spslam_lba_plane_obs ob{};
                    ob.kf = kidx[pKFi];
                    ob.kind = kd.second;
                    for (int i = 0; i < 4; i++) ob.meas[i] = pKFi->mvPlaneCoefficients[o.second][i];
                    G.qo.push_back(ob);
                    G.plane_obs_src.push_back({pMP, pKFi});
                }
            r.n_obs = (int32_t)G.qo.size() - r.obs_offset;
            G.q.push_back(r);
            G.planes.push_back(pMP);
        }
        G.prob.n_kf = (int)G.k.size();
        G.prob.n_points = (int)G.p.size();
        G.prob.n_planes = (int)G.q.size();
        G.prob.n_point_obs = (int)G.po.size();
        G.prob.n_plane_obs = (int)G.qo.size();
        std::vector<float> kf_out(16 * G.k.size()), pt_out(3 * std::max<size_t>(G.p.size(), 1)),
            pl_out(4 * std::max<size_t>(G.q.size(), 1));
        G.po_out.assign(std::max<size_t>(G.po.size(), 1), 0);
        G.qo_out.assign(std::max<size_t>(G.qo.size(), 1), 0);
        check(ctx, spslam_lba_optimize(ctx, &G.prob, G.k.data(), G.p.data(), G.po.data(), G.q.data(), G.qo.data(), &cfg,
                                       kf_out.data(), pt_out.data(), pl_out.data(), G.po_out.data(), G.qo_out.data(),
                                       &G.res, reinterpret_cast<const volatile uint8_t*>(pbStopFlag)),
              "spslam_lba_optimize");
        if (G.res.stopped == 1) return;  // pbStopFlag before optimize(5): the reference returns unchanged

        // :1896-1920 -- erase the outlier observations (points; plane edges are only flagged)
        for (size_t i = 0; i < G.po.size(); ++i)
            if (G.po_out[i]) {
                MapPoint* pMP = G.point_obs_src[i].first;
                KeyFrame* pKFi = G.point_obs_src[i].second;
                pKFi->EraseMapPointMatch(pMP->GetObservations().at(pKFi));
                pMP->EraseObservation(pKFi);
            }
        // :1925-1977 -- recover the optimized data
        for (int i = 0; i < nLocal; ++i) G.kfs[i]->SetPose(&kf_out[16 * i]);
        for (size_t i = 0; i < G.points.size(); ++i) G.points[i]->SetWorldPos(&pt_out[3 * i]);
        for (size_t i = 0; i < G.planes.size(); ++i) G.planes[i]->SetWorldPos(&pl_out[4 * i]);
    }
};

}  // namespace ORB_SLAM2

// ================================================================================================== test harness
using namespace ORB_SLAM2;

namespace {
thread_local std::string g_err;
template <class F> int guarded(F&& f) {
    try {
        f();
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}
}  // namespace

extern "C" {

const char* shim_last_error() { return g_err.c_str(); }

// Tracking::GrabImageRGBD (7) + the RGB-D Frame constructor (1, 4, 2, 5) on one colour / u16 depth frame.
// Outputs: keypoints (mvKeys) + descriptors, mvKeysUn, mvuRight, and the plane coefficients (extracted, then
// supposed) with the extracted count.
int shim_track_frame(const uint8_t* rgb, const uint16_t* depth_u16, int w, int h, float depth_factor,
                     const float* cam /* fx fy cx cy k1 k2 p1 p2 k3 bf */, int nfeatures, int min_size,
                     cv::KeyPoint* kps, uint8_t* desc, cv::KeyPoint* keys_un, float* uright, int cap, int* n,
                     float* plane_coef, int plane_cap, int* n_planes, int* n_real_planes) {
    return guarded([&] {
        ORBextractor ex(nfeatures, 1.2f, 8, 20, 7, w, h);
        cv::Mat imRGB(h, w, cv::CV_8U, 3), imD(h, w, cv::CV_16U);
        std::memcpy(imRGB.data, rgb, (size_t)w * h * 3);
        std::memcpy(imD.data, depth_u16, (size_t)w * h * 2);
        cv::Mat gray, depth;
        GrabImageRGBD(ex.mGpu, imRGB, imD, /*mbRGB*/ true, 1.0f / depth_factor, gray, depth);
        CameraConfig K{cam[0], cam[1], cam[2], cam[3], {cam[4], cam[5], cam[6], cam[7], cam[8]}, cam[9],
                       /*Cloud.Dis*/ 3, min_size, /*AngleThreshold*/ 3.0f, /*DistanceThreshold*/ 0.05f,
                       /*Line.Ratio*/ 0.2, /*Line.DistanceThreshold*/ 0.01f};
        Frame F(gray, depth, &ex, K);
        if (F.N > cap || F.mnPlaneNum > plane_cap) throw std::runtime_error("shim_track_frame: capacity");
        *n = F.N;
        std::memcpy(kps, F.mvKeys.data(), sizeof(cv::KeyPoint) * F.N);
        if (F.N) std::memcpy(desc, F.mDescriptors.data, (size_t)F.N * 32);
        std::memcpy(keys_un, F.mvKeysUn.data(), sizeof(cv::KeyPoint) * F.N);
        std::memcpy(uright, F.mvuRight.data(), sizeof(float) * F.N);
        *n_planes = F.mnPlaneNum;
        *n_real_planes = F.mnRealPlaneNum;
        for (int k = 0; k < F.mnPlaneNum; ++k) std::memcpy(plane_coef + 4 * k, F.mvPlaneCoefficients[k].data(), 16);
    });
}

// PoseOptimization (3) on a Frame assembled from per-keypoint arrays: keypoint i has a map point when
// has_mp[i] (world position xw[3i..]); plane i of the frame (meas 4i..) is associated to map plane
// assoc[kind][i] >= 0 (world coefficients world[4 * that..]).
int shim_pose_optimization(int N, const cv::KeyPoint* keys_un, const float* uright, const float* inv_sigma2_levels,
                           const uint8_t* has_mp, const float* xw, int n_planes, const float* meas,
                           const int32_t* assoc /* [3][n_planes] */, const float* world, const float* Tcw,
                           const float* cam /* fx fy cx cy bf */, const double* cfg6, float* Tcw_out,
                           int* n_inliers, uint8_t* outlier, uint8_t* plane_outlier /* [3][n_planes] */) {
    return guarded([&] {
        spslam_orb_params p{1000, 1.2f, 8, 20, 7, 640, 480, 1};
        spslam_ctx* ctx = nullptr;
        check(nullptr, spslam_create(0, &p, &ctx), "spslam_create");
        std::unique_ptr<spslam_ctx, void (*)(spslam_ctx*)> hold(ctx, spslam_destroy);
        Frame F;
        F.N = N;
        F.mvKeysUn.assign(keys_un, keys_un + N);
        F.mvuRight.assign(uright, uright + N);
        F.mvInvLevelSigma2.assign(inv_sigma2_levels, inv_sigma2_levels + 8);
        std::vector<std::unique_ptr<MapPoint>> mps;
        F.mvpMapPoints.assign(N, nullptr);
        F.mvbOutlier.assign(N, false);
        for (int i = 0; i < N; ++i)
            if (has_mp[i]) {
                mps.emplace_back(new MapPoint);
                mps.back()->mnId = (unsigned long)i + 1;
                mps.back()->SetWorldPos(xw + 3 * i);
                F.mvpMapPoints[i] = mps.back().get();
            }
        F.mnPlaneNum = n_planes;
        std::vector<std::unique_ptr<MapPlane>> mpl;
        std::map<int, MapPlane*> byIdx;
        std::vector<MapPlane*>* lists[3] = {&F.mvpMapPlanes, &F.mvpParallelPlanes, &F.mvpVerticalPlanes};
        for (int kind = 0; kind < 3; ++kind) {
            lists[kind]->assign(n_planes, nullptr);
            for (int i = 0; i < n_planes; ++i) {
                const int a = assoc[kind * n_planes + i];
                if (a < 0) continue;
                if (!byIdx.count(a)) {
                    mpl.emplace_back(new MapPlane);
                    mpl.back()->mnId = (unsigned long)a + 1;
                    mpl.back()->SetWorldPos(world + 4 * a);
                    byIdx[a] = mpl.back().get();
                }
                (*lists[kind])[i] = byIdx[a];
            }
        }
        for (int i = 0; i < n_planes; ++i) F.mvPlaneCoefficients.push_back({meas[4 * i], meas[4 * i + 1], meas[4 * i + 2], meas[4 * i + 3]});
        F.mvbPlaneOutlier.assign(n_planes, false);
        F.mvbParPlaneOutlier.assign(n_planes, false);
        F.mvbVerPlaneOutlier.assign(n_planes, false);
        F.SetPose(Tcw);
        F.fx = cam[0]; F.fy = cam[1]; F.cx = cam[2]; F.cy = cam[3]; F.mbf = cam[4];
        const spslam_plane_config cfg{cfg6[0], cfg6[1], cfg6[2], cfg6[3], cfg6[4], cfg6[5]};
        *n_inliers = Optimizer::PoseOptimization(ctx, &F, cfg);
        std::memcpy(Tcw_out, F.mTcw.data, 64);
        for (int i = 0; i < N; ++i) outlier[i] = F.mvbOutlier[i];
        for (int i = 0; i < n_planes; ++i) {
            plane_outlier[i] = F.mvbPlaneOutlier[i];
            plane_outlier[n_planes + i] = F.mvbParPlaneOutlier[i];
            plane_outlier[2 * n_planes + i] = F.mvbVerPlaneOutlier[i];
        }
    });
}

// LocalBundleAdjustment (6) on a keyframe graph given as the flat records of spslam_lba (keyframes with ids;
// points / planes with their observations): the harness builds KeyFrame / MapPoint / MapPlane objects
// (keypoint slots, map point matches, plane coefficient slots, observation maps), makes keyframe 0 the
// current keyframe with the other non-fixed keyframes as its covisible keyframes, and runs the shim.
// Returns the shim's flattened problem (for the test to rebuild the oracle call) and, per INPUT record, the
// result after application: keyframe poses, point positions, plane coefficients, and per input point
// observation whether it was erased.
int shim_local_ba(int n_kf, const spslam_lba_keyframe* kfs, int n_points, const spslam_lba_point* points,
                  const spslam_lba_point_obs* point_obs, int n_planes, const spslam_lba_plane* planes,
                  const spslam_lba_plane_obs* plane_obs, const float* inv_sigma2_levels, const double* cfg6,
                  int stop, spslam_lba_problem* flat_prob, spslam_lba_keyframe* flat_kfs, spslam_lba_point* flat_pts,
                  spslam_lba_point_obs* flat_pobs, spslam_lba_plane* flat_pls, spslam_lba_plane_obs* flat_plobs,
                  int flat_cap_pobs, int flat_cap_plobs, float* kf_out, float* pt_out, float* pl_out,
                  uint8_t* pobs_erased, spslam_lba_result* result) {
    return guarded([&] {
        spslam_orb_params p{1000, 1.2f, 8, 20, 7, 640, 480, 1};
        spslam_ctx* ctx = nullptr;
        check(nullptr, spslam_create(0, &p, &ctx), "spslam_create");
        std::unique_ptr<spslam_ctx, void (*)(spslam_ctx*)> hold(ctx, spslam_destroy);
        std::vector<std::unique_ptr<KeyFrame>> K;
        for (int i = 0; i < n_kf; ++i) {
            K.emplace_back(new KeyFrame);
            KeyFrame& f = *K.back();
            f.mnId = (unsigned long)kfs[i].id;
            f.SetPose(kfs[i].Tcw);
            f.fx = kfs[i].fx; f.fy = kfs[i].fy; f.cx = kfs[i].cx; f.cy = kfs[i].cy; f.mbf = kfs[i].bf;
            f.mvInvLevelSigma2.assign(inv_sigma2_levels, inv_sigma2_levels + 8);
        }
        for (int i = 1; i < n_kf; ++i)
            if (!kfs[i].fixed) K[0]->mvpOrderedConnectedKeyFrames.push_back(K[i].get());
        auto octave_of = [&](float inv_s2) {
            for (int o = 0; o < 8; ++o)
                if (inv_sigma2_levels[o] == inv_s2) return o;
            throw std::runtime_error("shim_local_ba: inv_sigma2 not a level value");
        };
        std::vector<std::unique_ptr<MapPoint>> P;
        int n_pobs = 0;
        for (int j = 0; j < n_points; ++j) n_pobs = std::max(n_pobs, points[j].obs_offset + points[j].n_obs);
        std::vector<std::pair<KeyFrame*, size_t>> obs_slot(n_pobs, {nullptr, 0});
        for (int j = 0; j < n_points; ++j) {
            P.emplace_back(new MapPoint);
            MapPoint& m = *P.back();
            m.mnId = (unsigned long)points[j].id;
            m.SetWorldPos(points[j].xw);
            for (int o = points[j].obs_offset; o < points[j].obs_offset + points[j].n_obs; ++o) {
                KeyFrame* f = K[point_obs[o].kf].get();
                cv::KeyPoint kp;
                kp.pt.x = point_obs[o].u;
                kp.pt.y = point_obs[o].v;
                kp.octave = octave_of(point_obs[o].inv_sigma2);
                const size_t idx = f->mvKeysUn.size();
                f->mvKeysUn.push_back(kp);
                f->mvuRight.push_back(point_obs[o].ur);
                f->mvpMapPoints.push_back(&m);
                m.mObservations[f] = idx;
                obs_slot[o] = {f, idx};
            }
        }
        std::vector<std::unique_ptr<MapPlane>> Q;
        for (int j = 0; j < n_planes; ++j) {
            Q.emplace_back(new MapPlane);
            MapPlane& m = *Q.back();
            m.mnId = (unsigned long)planes[j].id;
            m.SetWorldPos(planes[j].world);
            for (int o = planes[j].obs_offset; o < planes[j].obs_offset + planes[j].n_obs; ++o) {
                KeyFrame* f = K[plane_obs[o].kf].get();
                const int idx = (int)f->mvPlaneCoefficients.size();
                f->mvPlaneCoefficients.push_back({plane_obs[o].meas[0], plane_obs[o].meas[1], plane_obs[o].meas[2],
                                                  plane_obs[o].meas[3]});
                f->mvpMapPlanes.push_back(plane_obs[o].kind == SPSLAM_PLANE_EDGE ? &m : nullptr);
                f->mnPlaneNum = idx + 1;
                if (plane_obs[o].kind == SPSLAM_PLANE_EDGE) m.mObservations[f] = idx;
                else if (plane_obs[o].kind == SPSLAM_VERTICAL_EDGE) m.mVerObservations[f] = idx;
                else m.mParObservations[f] = idx;
            }
        }
        const spslam_plane_config cfg{cfg6[0], cfg6[1], cfg6[2], cfg6[3], cfg6[4], cfg6[5]};
        bool stopFlag = stop != 0;
        Optimizer::LbaGraph G;
        Optimizer::LocalBundleAdjustment(ctx, K[0].get(), &stopFlag, cfg, G);
        if ((int)G.po.size() > flat_cap_pobs || (int)G.qo.size() > flat_cap_plobs || (int)G.k.size() > n_kf ||
            (int)G.p.size() > n_points || (int)G.q.size() > n_planes)
            throw std::runtime_error("shim_local_ba: capacity");
        *flat_prob = G.prob;
        std::copy(G.k.begin(), G.k.end(), flat_kfs);
        std::copy(G.p.begin(), G.p.end(), flat_pts);
        std::copy(G.po.begin(), G.po.end(), flat_pobs);
        std::copy(G.q.begin(), G.q.end(), flat_pls);
        std::copy(G.qo.begin(), G.qo.end(), flat_plobs);
        *result = G.res;
        for (int i = 0; i < n_kf; ++i) std::memcpy(kf_out + 16 * i, K[i]->mTcw.data, 64);
        for (int j = 0; j < n_points; ++j) std::memcpy(pt_out + 3 * j, P[j]->mWorldPos.data, 12);
        for (int j = 0; j < n_planes; ++j) std::memcpy(pl_out + 4 * j, Q[j]->mWorldPos.data, 16);
        for (size_t o = 0; o < obs_slot.size(); ++o) {
            KeyFrame* f = obs_slot[o].first;
            pobs_erased[o] = f && f->mvpMapPoints[obs_slot[o].second] == nullptr;
        }
    });
}


// Map::AssociatePlanesByBoundary (8) on a Frame with n_planes coefficients at pose Tcw against a map of n_map
// planes (spslam_map_plane records: world, id, boundary range in bxyz); params: dis, angle, ver, par thresholds.
// Outputs: map-plane array indices (-1 none) and mbNewPlane.
int shim_associate_planes(const float* Tcw, const float* coefs, int n_planes, const spslam_map_plane* map, int n_map,
                          const float* bxyz, const float* params, int32_t* match, int32_t* parallel,
                          int32_t* vertical, int* new_plane) {
    return guarded([&] {
        spslam_orb_params p{1000, 1.2f, 8, 20, 7, 640, 480, 1};
        spslam_ctx* ctx = nullptr;
        check(nullptr, spslam_create(0, &p, &ctx), "spslam_create");
        std::unique_ptr<spslam_ctx, void (*)(spslam_ctx*)> hold(ctx, spslam_destroy);
        std::vector<std::unique_ptr<MapPlane>> planes;
        Map M;
        M.mGpu = ctx;
        M.mfDisTh = params[0]; M.mfAngleTh = params[1]; M.mfVerTh = params[2]; M.mfParTh = params[3];
        std::map<unsigned long, int> index;
        for (int j = 0; j < n_map; ++j) {
            planes.emplace_back(new MapPlane);
            MapPlane* mp = planes.back().get();
            mp->mnId = (unsigned long)map[j].id;
            mp->SetWorldPos(map[j].world);
            for (int k = 0; k < map[j].n_boundary; ++k) {
                const float* q = bxyz + 3 * (map[j].boundary_offset + k);
                mp->mvBoundaryPoints.points.push_back({q[0], q[1], q[2]});
            }
            M.mspMapPlanes.insert(mp);
            index[mp->mnId] = j;
        }
        Frame F;
        F.SetPose(Tcw);
        F.mnPlaneNum = n_planes;
        for (int i = 0; i < n_planes; ++i) F.mvPlaneCoefficients.push_back({coefs[4 * i], coefs[4 * i + 1],
                                                                            coefs[4 * i + 2], coefs[4 * i + 3]});
        F.mvpMapPlanes.assign(n_planes, nullptr);  // a new Frame (src/Frame.cc:199-213)
        F.mvpParallelPlanes.assign(n_planes, nullptr);
        F.mvpVerticalPlanes.assign(n_planes, nullptr);
        M.AssociatePlanesByBoundary(F);
        auto out = [&](MapPlane* mp) { return mp ? index.at(mp->mnId) : -1; };
        for (int i = 0; i < n_planes; ++i) {
            match[i] = out(F.mvpMapPlanes[i]);
            parallel[i] = out(F.mvpParallelPlanes[i]);
            vertical[i] = out(F.mvpVerticalPlanes[i]);
        }
        *new_plane = F.mbNewPlane ? 1 : 0;
    });
}

// TrackWithMotionModel's matching (9; src/Tracking.cc:951-975): ORBmatcher(0.9, true), mvpMapPoints cleared,
// SearchByProjection at th, again at 2 th below 20 matches.  The last frame: one keypoint per point record
// (its map point, angle, octave; no outliers); the current frame: n_kp keypoints (mvKeysUn, descriptors,
// mvuRight, mGrid as CSR); cam: fx fy cx cy bf width height (the context's frame geometry).  Output per current
// keypoint: the index of its map point in `points`, -1 none; the returned nmatches.
int shim_track_motion_model_matching(const spslam_proj_frame* fr, const spslam_proj_point* points, int n_points,
                                     const cv::KeyPoint* keys_un, const uint8_t* desc, const float* uright, int n_kp,
                                     const int32_t* grid_off, const int32_t* grid_idx, const float* cam, float th,
                                     int32_t* match, int* nmatches) {
    return guarded([&] {
        ORBextractor ex(1000, 1.2f, 8, 20, 7, (int)cam[5], (int)cam[6]);
        spslam_frame_params fp{cam[0], cam[1], cam[2], cam[3], {0, 0, 0, 0, 0}, cam[4], (int)cam[5], (int)cam[6]};
        float bounds[4];
        check(ex.mGpu, spslam_frame_configure(ex.mGpu, &fp, bounds, nullptr), "spslam_frame_configure");
        std::vector<std::unique_ptr<MapPoint>> mps;
        Frame Last, Cur;
        Last.mpORBextractorLeft = Cur.mpORBextractorLeft = &ex;
        Last.N = n_points;
        Last.SetPose(fr->Tlw);
        Last.mvKeys.resize(n_points);
        Last.mvKeysUn.resize(n_points);
        Last.mvbOutlier.assign(n_points, false);
        for (int i = 0; i < n_points; ++i) {
            mps.emplace_back(new MapPoint);
            MapPoint* mp = mps.back().get();
            mp->mnId = (unsigned long)points[i].id;
            mp->SetWorldPos(points[i].xw);
            std::memcpy(mp->mDescriptor.data, points[i].desc, 32);
            mp->nObs = points[i].n_obs;
            Last.mvpMapPoints.push_back(mp);
            Last.mvKeysUn[i].angle = points[i].angle;
            Last.mvKeys[i].octave = points[i].octave;
        }
        Cur.N = n_kp;
        Cur.SetPose(fr->Tcw);  // mVelocity * mLastFrame.mTcw
        Cur.mvKeysUn.assign(keys_un, keys_un + n_kp);
        Cur.mDescriptors = cv::Mat(std::max(n_kp, 1), 32, cv::CV_8U);
        if (n_kp) std::memcpy(Cur.mDescriptors.data, desc, (size_t)n_kp * 32);
        Cur.mvuRight.assign(uright, uright + n_kp);
        Cur.mGrid.assign(64 * 48, {});
        for (int c = 0; c < 64 * 48; ++c) Cur.mGrid[c].assign(grid_idx + grid_off[c], grid_idx + grid_off[c + 1]);
        ORBmatcher matcher(0.9f, true);
        Cur.mvpMapPoints.assign(n_kp, nullptr);
        int n = matcher.SearchByProjection(Cur, Last, th, false);
        if (n < 20) {
            Cur.mvpMapPoints.assign(n_kp, nullptr);
            n = matcher.SearchByProjection(Cur, Last, 2 * th, false);
        }
        std::map<const MapPoint*, int> idx;
        for (int i = 0; i < n_points; ++i) idx[mps[i].get()] = i;
        for (int i = 0; i < n_kp; ++i) match[i] = Cur.mvpMapPoints[i] ? idx.at(Cur.mvpMapPoints[i]) : -1;
        *nmatches = n;
    });
}

// TrackReferenceKeyFrame's matching (11; src/Tracking.cc:797-802): the vocabulary into the context, ComputeBoW of
// the keyframe and the frame, ORBmatcher(nn_ratio, check_ori).SearchByBoW(pKF, F, vpMapPointMatches).  Keyframe
// feature i has a map point when has_mp[i].  Outputs: per frame feature the keyframe feature whose map point it
// received (-1 none), nmatches, and the frame's BowVector / FeatureVector (ascending ids; fv_start CSR).
int shim_bow_match(const char* vocab, size_t vocab_len, const uint8_t* kf_desc, const cv::KeyPoint* kf_keys_un,
                   const uint8_t* has_mp, int kf_n, const uint8_t* f_desc, const cv::KeyPoint* f_keys, int f_n,
                   float nn_ratio, int check_ori, int32_t* match, int* nmatches, uint32_t* bow_words,
                   double* bow_values, int* n_bow, uint32_t* fv_nodes, int32_t* fv_start, int32_t* fv_features,
                   int* n_fv) {
    return guarded([&] {
        ORBextractor ex(1000, 1.2f, 8, 20, 7, 640, 480);
        LoadVocabulary(ex.mGpu, std::string(vocab, vocab_len));
        std::vector<std::unique_ptr<MapPoint>> mps;
        KeyFrame KF;
        KF.N = kf_n;
        KF.mvKeysUn.assign(kf_keys_un, kf_keys_un + kf_n);
        KF.mDescriptors = cv::Mat(kf_n, 32, cv::CV_8U);
        if (kf_n) std::memcpy(KF.mDescriptors.data, kf_desc, (size_t)kf_n * 32);
        KF.mvpMapPoints.assign(kf_n, nullptr);
        for (int i = 0; i < kf_n; ++i)
            if (has_mp[i]) {
                mps.emplace_back(new MapPoint);
                mps.back()->mnId = (unsigned long)i;
                KF.mvpMapPoints[i] = mps.back().get();
            }
        ComputeBoW(ex.mGpu, KF.mDescriptors, KF.mBowVec, KF.mFeatVec);  // KeyFrame::ComputeBoW
        Frame F;
        F.mpORBextractorLeft = &ex;
        F.N = f_n;
        F.mvKeys.assign(f_keys, f_keys + f_n);
        F.mDescriptors = cv::Mat(f_n, 32, cv::CV_8U);
        if (f_n) std::memcpy(F.mDescriptors.data, f_desc, (size_t)f_n * 32);
        F.ComputeBoW();
        ORBmatcher matcher(nn_ratio, check_ori != 0);
        std::vector<MapPoint*> vpMapPointMatches;
        *nmatches = matcher.SearchByBoW(&KF, F, vpMapPointMatches);
        for (int i = 0; i < f_n; ++i) match[i] = vpMapPointMatches[i] ? (int32_t)vpMapPointMatches[i]->mnId : -1;
        int b = 0;
        for (const auto& kv : F.mBowVec) {
            bow_words[b] = kv.first;
            bow_values[b++] = kv.second;
        }
        *n_bow = b;
        int j = 0, o = 0;
        for (const auto& kv : F.mFeatVec) {
            fv_nodes[j] = kv.first;
            fv_start[j++] = o;
            for (unsigned int q : kv.second) fv_features[o++] = (int32_t)q;
        }
        fv_start[j] = o;
        *n_fv = j;
    });
}

}  // extern "C"
