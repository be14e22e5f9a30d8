/* spslam_gpu.h -- C ABI of the MI355X (gfx950) implementation of SP-SLAM's
 * per-frame RGB-D tracking hot path.
 *
 * Plain C: no C++/torch types cross this boundary; every buffer is
 * caller-owned (host pointers for the drop-in entry points, device pointers
 * for the *_device batch entry points).  Errors are returned as negative
 * status codes, the message is kept per context (spslam_last_error); nothing
 * throws across the ABI and nothing calls exit().
 *
 * Threading: one context per calling host thread.  A context owns its device
 * scratch and one HIP stream, mirroring the reference, where Tracking
 * (ORB/planes/pose) and LocalMapping (LBA) run on different threads
 * (src/System.cc:92-106).
 *
 * Reference interfaces replaced (paths relative to the reference tree):
 *   spslam_orb_*        ORB_SLAM2::ORBextractor (include/ORBextractor.h:45-111,
 *                       src/ORBextractor.cc:410-470, 1043-1132)
 *   spslam_pose_*       Optimizer::PoseOptimization (include/Optimizer.h:47,
 *                       src/Optimizer.cc:519-1152) with g2oAddition plane edges
 *   spslam_planes_extract*  Frame::ComputePlanesFromOrganizedPointCloud
 *                       (include/Frame.h:120, src/Frame.cc:854-936)
 *   spslam_planes_generate_from_boundaries*  Frame::GeneratePlanesFromBoundries
 *                       (include/Frame.h:121, src/Frame.cc:938-1144)
 *   spslam_frame_*      RGB-D Frame constructor keypoint steps (src/Frame.cc:146-181)
 *   spslam_lba_*        Optimizer::LocalBundleAdjustment (include/Optimizer.h:46,
 *                       src/Optimizer.cc:1154-1977)
 *   spslam_planes_associate*  Map::AssociatePlanesByBoundary (include/Map.h:69-74,
 *                       src/Map.cc:196-359)
 */
#ifndef SPSLAM_GPU_H
#define SPSLAM_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPSLAM_OK 0
#define SPSLAM_ERR_ARG (-1)        /* bad argument / shape */
#define SPSLAM_ERR_CAPACITY (-2)   /* caller buffer too small (count still written) */
#define SPSLAM_ERR_HIP (-3)        /* HIP runtime error */
#define SPSLAM_ERR_NOT_READY (-4)  /* stage data requested before it was computed */

typedef struct spslam_ctx spslam_ctx;

/* Bit-compatible with cv::KeyPoint {Point2f pt; float size, angle, response;
 * int octave, class_id;} (28 bytes), the element type of the reference's
 * std::vector<cv::KeyPoint> output (include/ORBextractor.h:59-61). */
typedef struct spslam_keypoint {
    float x, y;
    float size;
    float angle;
    float response;
    int32_t octave;
    int32_t class_id;
} spslam_keypoint;

/* ORBextractor constructor arguments (include/ORBextractor.h:51-52; values
 * come from ORBextractor.* keys of the YAML, src/Tracking.cc:113-119), plus the
 * image geometry and the largest batch the context must hold. */
typedef struct spslam_orb_params {
    int nfeatures;      /* ORBextractor.nFeatures (1000) */
    float scale_factor; /* ORBextractor.scaleFactor (1.2) */
    int nlevels;        /* ORBextractor.nLevels (8), <= SPSLAM_MAX_LEVELS */
    int ini_th_fast;    /* ORBextractor.iniThFAST (20) */
    int min_th_fast;    /* ORBextractor.minThFAST (7) */
    int width, height;  /* input image size */
    int max_batch;      /* frames per batched call */
} spslam_orb_params;

#define SPSLAM_MAX_LEVELS 8

/* Create a context on HIP device `device`.  Replaces `new ORBextractor(...)`
 * (src/Tracking.cc:119). */
int spslam_create(int device, const spslam_orb_params* params, spslam_ctx** out);
void spslam_destroy(spslam_ctx* ctx);
const char* spslam_last_error(const spslam_ctx* ctx);

/* Per-level tables: GetLevels / GetScaleFactor(s) / GetInverseScaleFactors /
 * GetScaleSigmaSquares / GetInverseScaleSigmaSquares
 * (include/ORBextractor.h:63-83).  Any output pointer may be NULL. */
int spslam_orb_tables(const spslam_ctx* ctx, int* nlevels, float* scale, float* inv_scale, float* sigma2,
                      float* inv_sigma2, int* features_per_level);

/* Upper bound on keypoints one frame can produce (size caller buffers with it). */
int spslam_orb_max_keypoints(const spslam_ctx* ctx);

/* Drop-in for ORBextractor::operator()(image, mask, keypoints, descriptors)
 * (include/ORBextractor.h:59-61, src/ORBextractor.cc:1043-1105): host gray
 * u8 image in, keypoints (level order) + n x 32 descriptor bytes out.
 * The mask is ignored by the reference and is not taken here.  An empty
 * image (w == 0 or h == 0) returns SPSLAM_OK with *n = 0 and buffers
 * untouched.  The image size must equal the context's width/height. */
int spslam_orb_extract(spslam_ctx* ctx, const uint8_t* gray, int w, int h, int stride, spslam_keypoint* kps,
                       uint8_t* desc, int cap, int* n);

/* Throughput entry: n_frames gray frames already resident in device memory
 * (frame f at d_gray + f*frame_stride, rows `stride` bytes apart).  Writes,
 * per frame f, counts[f] keypoints to d_kps + f*cap_per_frame and
 * descriptors to d_desc + f*cap_per_frame*32.  Asynchronous on `hip_stream`
 * (a hipStream_t).  In every *_batch_device call NULL means HIP's default
 * (NULL) stream -- the one PyTorch calls its default stream -- so device
 * buffers filled by the caller on that stream are ordered before the work;
 * the host-buffer drop-ins run on the context's own stream. */
int spslam_orb_extract_batch_device(spslam_ctx* ctx, const uint8_t* d_gray, int n_frames, size_t frame_stride,
                                    int stride, spslam_keypoint* d_kps, uint8_t* d_desc, int* d_counts,
                                    int cap_per_frame, void* hip_stream);

/* Stage access for parity tests (valid for frame `frame` of the last call).
 * stage: 0 = pyramid level image (w*h bytes), 1 = blurred level (w*h bytes),
 *        2 = FAST cell candidates of the level, as spslam_keypoint with
 *            coordinates relative to (minBorderX, minBorderY) like
 *            src/ORBextractor.cc:822-824 (count in *n),
 *        3 = DistributeOctTree output of the level (level coordinates, before
 *            orientation; count in *n). */
int spslam_orb_debug_stage(spslam_ctx* ctx, int frame, int level, int stage, void* out, int cap, int* n);
int spslam_orb_level_size(const spslam_ctx* ctx, int level, int* w, int* h);

/* ------------------------------------------------------------------------
 * PoseOptimization (src/Optimizer.cc:519-1152; include/Optimizer.h:47).
 *
 * The reference builds a g2o graph from Frame/MapPoint/MapPlane members; at
 * this boundary the caller passes those members flattened:
 *   - one spslam_point_obs per keypoint i with mvpMapPoints[i] != NULL, in
 *     increasing i (the reference's edge insertion order, :561-647);
 *   - one spslam_plane_obs per plane edge, all kind 0 (mvpMapPlanes) first,
 *     then kind 1 (mvpParallelPlanes), then kind 2 (mvpVerticalPlanes), each
 *     in increasing plane index (:700-859).  world = MapPlane::GetWorldPos(),
 *     meas = Frame::mvPlaneCoefficients[i]; map_plane_id = MapPlane::mnId
 *     (only used for the vertex-id bookkeeping the reference does).
 * Results: the optimized Tcw (what Frame::SetPose receives, :1149-1150), the
 * returned inlier count (:1151; 0 when fewer than 3 point correspondences,
 * :653), and the per-observation outlier flags (mvbOutlier, mvbPlaneOutlier,
 * mvbParPlaneOutlier, mvbVerPlaneOutlier). */
typedef struct spslam_point_obs {
    float u, v;        /* mvKeysUn[i].pt */
    float ur;          /* mvuRight[i]; < 0 -> monocular edge */
    float inv_sigma2;  /* mvInvLevelSigma2[mvKeysUn[i].octave] */
    float xw[3];       /* MapPoint::GetWorldPos() */
    int32_t kp_index;  /* i (informational) */
} spslam_point_obs;

#define SPSLAM_PLANE_EDGE 0      /* g2o::EdgePlane          (3-D error) */
#define SPSLAM_PARALLEL_EDGE 1   /* g2o::EdgeParallelPlane  (2-D error) */
#define SPSLAM_VERTICAL_EDGE 2   /* g2o::EdgeVerticalPlane  (2-D error) */

typedef struct spslam_plane_obs {
    float meas[4];     /* frame plane coefficients (a,b,c,d) */
    float world[4];    /* map plane world coefficients */
    int32_t kind;      /* SPSLAM_*_EDGE */
    int32_t plane_index;
    int32_t map_plane_id;
    int32_t pad;
} spslam_plane_obs;

/* Config keys read by PoseOptimization (src/Optimizer.cc:681-693; YAML
 * Plane.AngleInfo/DistanceInfo/ParallelInfo/VerticalInfo/Chi/VPChi). */
typedef struct spslam_plane_config {
    double angle_info, distance_info, parallel_info, vertical_info, chi, vp_chi;
} spslam_plane_config;

typedef struct spslam_pose_problem {
    float Tcw[16];      /* Frame::mTcw, row-major 4x4 */
    float fx, fy, cx, cy, bf;
    int32_t n_points;   /* observations [point_offset, point_offset + n_points) */
    int32_t n_planes;
    int32_t point_offset;
    int32_t plane_offset;
    int32_t pad;
} spslam_pose_problem;

typedef struct spslam_pose_result {
    float Tcw[16];      /* optimized pose (unchanged input if n_inliers == 0 by the <3 rule) */
    int32_t n_inliers;  /* PoseOptimization return value */
    int32_t lm_iterations;  /* total LM iterations run (diagnostic); -1 = the device gave up on a bounded
                               internal wait (never observed): invalid result, Tcw = input, n_inliers = 0,
                               every point / plane outlier flag set to 1 */
    int32_t trial_passes;   /* edge passes at trial poses (damping trials are evaluated 4 per pass; diagnostic) */
    int32_t trials;         /* damping trials the reference evaluated (computeActiveErrors calls; diagnostic) */
} spslam_pose_result;

/* Drop-in for Optimizer::PoseOptimization(Frame*) on host buffers, one frame.
 * point_outlier / plane_outlier (n_points / n_planes bytes) receive the
 * outlier flags. */
int spslam_pose_optimize(spslam_ctx* ctx, const spslam_pose_problem* problem, const spslam_point_obs* points,
                         const spslam_plane_obs* planes, const spslam_plane_config* cfg, spslam_pose_result* result,
                         uint8_t* point_outlier, uint8_t* plane_outlier);

/* Batched, device resident: n problems, one workgroup each.  Observation
 * arrays are indexed through each problem's point/plane offsets; the outlier
 * flag arrays share those offsets.  If d_init_from is non-NULL, problem p
 * starts from d_init_from[p].Tcw instead of its own Tcw (used to chain the
 * motion-model and local-map optimizations of one frame on the device).
 * Asynchronous on hip_stream (NULL = the default stream). */
int spslam_pose_optimize_batch_device(spslam_ctx* ctx, int n, const spslam_pose_problem* d_problems,
                                      const spslam_point_obs* d_points, const spslam_plane_obs* d_planes,
                                      const spslam_plane_config* cfg, const spslam_pose_result* d_init_from,
                                      spslam_pose_result* d_results, uint8_t* d_point_outlier,
                                      uint8_t* d_plane_outlier, void* hip_stream);

/* ------------------------------------------------------------------------
 * LocalBundleAdjustment (include/Optimizer.h:46, src/Optimizer.cc:1154-1977)
 * from the point where the local graph is known.  The caller (LocalMapping's
 * shim) flattens what the reference collects from the Map:
 *   keyframes  lLocalKeyFrames in list order (fixed = 0; mnId 0 is held fixed
 *              like the reference), then lFixedCameras (fixed = 1);
 *   points     lLocalMapPoints in list order, each with its observations in
 *              MapPoint::GetObservations() order (std::map<KeyFrame*>:
 *              pointer order in the reference, keyframe-id order here --
 *              SURVEY.md Appendix A.9), observations of bad keyframes dropped;
 *   planes     lLocalMapPlanes in list order, each with its GetObservations()
 *              edges (kind SPSLAM_PLANE_EDGE), then GetVerObservations()
 *              (SPSLAM_VERTICAL_EDGE), then GetParObservations()
 *              (SPSLAM_PARALLEL_EDGE), the reference's edge insertion order.
 * Results: poses of the local keyframes (KeyFrame::SetPose), point positions
 * (MapPoint::SetWorldPos), plane coefficients (MapPlane::SetWorldPos), and per
 * observation the outlier flag the reference acts on (point observations:
 * vToErase -> EraseMapPointMatch / EraseObservation; plane observations:
 * chi2 above Plane.Chi / VPChi, informational -- the reference's erase is
 * commented out, Optimizer.cc:1862-1870).  The not-seen plane branches are
 * dead in the reference (SURVEY.md 8 notes) and are not represented. */
typedef struct spslam_lba_keyframe {
    float Tcw[16];            /* KeyFrame::GetPose(), row-major */
    float fx, fy, cx, cy, bf; /* KeyFrame::fx..cy, mbf (edge intrinsics) */
    int32_t id;               /* KeyFrame::mnId (g2o vertex id) */
    int32_t fixed;            /* 1 = fixed camera */
    int32_t pad;
} spslam_lba_keyframe;

typedef struct spslam_lba_point {
    float xw[3];              /* MapPoint::GetWorldPos() */
    int32_t id;               /* MapPoint::mnId */
    int32_t obs_offset;       /* observations [obs_offset, obs_offset + n_obs) */
    int32_t n_obs;
} spslam_lba_point;

typedef struct spslam_lba_point_obs {
    int32_t kf;               /* index into the problem's keyframes */
    float u, v;               /* KeyFrame::mvKeysUn[idx].pt */
    float ur;                 /* KeyFrame::mvuRight[idx]; < 0 -> monocular edge */
    float inv_sigma2;         /* KeyFrame::mvInvLevelSigma2[octave] */
} spslam_lba_point_obs;

typedef struct spslam_lba_plane {
    float world[4];           /* MapPlane::GetWorldPos() */
    int32_t id;               /* MapPlane::mnId */
    int32_t obs_offset;
    int32_t n_obs;
    int32_t pad;
} spslam_lba_plane;

typedef struct spslam_lba_plane_obs {
    int32_t kf;
    int32_t kind;             /* SPSLAM_PLANE_EDGE / SPSLAM_VERTICAL_EDGE / SPSLAM_PARALLEL_EDGE */
    float meas[4];            /* KeyFrame::mvPlaneCoefficients[idx] */
} spslam_lba_plane_obs;

/* One problem of a batch: its keyframes / points / planes start at the given
 * offsets of the batch arrays; observation offsets inside points / planes are
 * absolute indices into the batch observation arrays. */
typedef struct spslam_lba_problem {
    int32_t n_kf, n_points, n_planes;
    int32_t kf_offset, point_offset, plane_offset;
    int32_t n_point_obs, n_plane_obs;   /* total observations of its points / planes */
} spslam_lba_problem;

typedef struct spslam_lba_result {
    int32_t iterations[2];    /* LM iterations of optimize(5) / optimize(10) */
    int32_t n_point_outliers; /* flagged point observations */
    int32_t n_plane_outliers;
    int32_t status;           /* 0 ok, < 0 capacity / numerical failure */
    int32_t trials;           /* LM trials (lambda steps) in total */
    int32_t stopped;          /* pbStopFlag: 0 not seen (or seen after the schedule ended), 1 seen before
                                 optimize(5) -- returned, outputs = inputs, no outliers -- 2 seen at a later
                                 check point: the schedule ended there (trials = trials run) */
    int32_t pad;
    float phase_us[8];        /* diagnostics: device time per phase (setup, errors, edge terms, block sums,
                                 Schur, factorisation, substitution, update), microseconds */
} spslam_lba_result;

/* Drop-in for Optimizer::LocalBundleAdjustment on host buffers, one problem
 * (offsets inside *problem are ignored; observation offsets index obs arrays).
 * stop_flag = pbStopFlag (NULL allowed): a bool another thread may raise while
 * the call runs (LocalMapping::InterruptBA); it is copied to the device at the
 * call and at every host poll of the schedule and honoured at g2o's check
 * points (result.stopped).
 * kf_out: 16 floats per keyframe (local keyframes optimised, fixed ones
 * copied), pt_out 3 per point, pl_out 4 per plane, outlier flags per
 * observation.  cfg = the Plane.* config keys (as for PoseOptimization). */
int spslam_lba_optimize(spslam_ctx* ctx, const spslam_lba_problem* problem, const spslam_lba_keyframe* kfs,
                        const spslam_lba_point* points, const spslam_lba_point_obs* point_obs,
                        const spslam_lba_plane* planes, const spslam_lba_plane_obs* plane_obs,
                        const spslam_plane_config* cfg, float* kf_out, float* pt_out, float* pl_out,
                        uint8_t* point_obs_outlier, uint8_t* plane_obs_outlier, spslam_lba_result* result,
                        const volatile uint8_t* stop_flag);

/* Summation order of the LocalBundleAdjustment entries (default SPSLAM_LBA_G2O_ORDER):
 *   SPSLAM_LBA_G2O_ORDER  g2o's own arithmetic, bit-exact to the reference-order oracle: edge-insertion-order
 *                         sums, the landmark-ordered Schur complement (block_solver.hpp:381-431), Eigen's
 *                         SimplicialLDLT with its AMD ordering (linear_solver_eigen.h:58-121); one workgroup per
 *                         problem, the whole schedule in one launch;
 *   SPSLAM_LBA_FAST_ORDER the grid-wide phase kernels (tree-ordered reductions, Schur sums on the f64 matrix
 *                         cores, natural-order LDL^T): the same algorithm to rounding (<= 1e-4 on the tested maps),
 *                         a throughput mode for maps that do not need the reference's bits. */
#define SPSLAM_LBA_G2O_ORDER 0
#define SPSLAM_LBA_FAST_ORDER 1
int spslam_lba_set_order(spslam_ctx* ctx, int order);

/* Test hook (deterministic LocalMapping::InterruptBA): the context's following
 * LocalBundleAdjustment calls see pbStopFlag raised once a problem has run
 * `trials` LM trials -- before optimize(5) when 0 -- at the same check points
 * as a raised flag; -1 turns the hook off (default). */
int spslam_lba_debug_stop_after(spslam_ctx* ctx, int trials);

/* Workgroups per problem of the SPSLAM_LBA_G2O_ORDER launch (1 .. 16; 0, the
 * default: as many as fill the device's compute units, at most 8).  Results do
 * not depend on it: every sum keeps g2o's order whatever the split. */
int spslam_lba_set_team(spslam_ctx* ctx, int workgroups);

/* Batched, device resident: n problems (host copy `problems` for sizing, the
 * same records on the device at d_problems), a team of workgroups each
 * (spslam_lba_set_team), the whole optimize(5) / relabel / optimize(10)
 * schedule on the device.  Outputs are indexed like the inputs (keyframe /
 * point / plane offsets of each problem, absolute observation indices).
 * SPSLAM_LBA_G2O_ORDER: at most 1024 keyframes per problem (local + fixed) of
 * which at most 128 free poses (local keyframes, id != 0, with an active
 * edge; batches whose windows all hold <= 64 keyframes run the narrow
 * instance, others the wide one); SPSLAM_LBA_FAST_ORDER: at most 64 keyframes; status -2 otherwise
 * (nothing else written for that problem).  d_stop_flags: one pbStopFlag per
 * problem in device-visible memory (device, or host-mapped coherent memory
 * another thread raises), nonzero = stop; NULL = no flags.  Results are
 * complete on hip_stream (SPSLAM_LBA_G2O_ORDER only enqueues one launch; the
 * fast order polls the device and returns once every problem is done).  One
 * LocalBundleAdjustment call per context is in flight at a time: a call on
 * another stream first waits (on the device) for the context's previous call,
 * whose scratch it reuses. */
int spslam_lba_optimize_batch_device(spslam_ctx* ctx, int n, const spslam_lba_problem* problems,
                                     const spslam_lba_problem* d_problems, const spslam_lba_keyframe* d_kfs,
                                     const spslam_lba_point* d_points, const spslam_lba_point_obs* d_point_obs,
                                     const spslam_lba_plane* d_planes, const spslam_lba_plane_obs* d_plane_obs,
                                     const spslam_plane_config* cfg, float* d_kf_out, float* d_pt_out,
                                     float* d_pl_out, uint8_t* d_point_obs_outlier, uint8_t* d_plane_obs_outlier,
                                     spslam_lba_result* d_results, const int32_t* d_stop_flags, void* hip_stream);

/* ------------------------------------------------------------------------
 * Plane extraction: Frame::ComputePlanesFromOrganizedPointCloud
 * (include/Frame.h:120, src/Frame.cc:854-936) with the PCL 1.8
 * IntegralImageNormalEstimation + OrganizedMultiPlaneSegmentation it calls.
 *
 * Input: the float depth image in meters the RGB-D Frame constructor
 * receives (imDepth, CV_32F, src/Tracking.cc:230-231).  Output per frame:
 * the planes Frame appends to mvPlaneCoefficients (d >= 0, PlaneNotSeen
 * de-duplicated, in the reference's order) with, per plane, the
 * organized-cloud indices of its inliers (mvPlanePoints) and of its contour
 * (mvBoundaryPoints).  The organized cloud itself (points (x, y, z), row-major
 * ceil(h/dis) x ceil(w/dis)) is available through spslam_planes_cloud. */
typedef struct spslam_plane_params {
    int cloud_dis;            /* Cloud.Dis (3) */
    int min_size;             /* Plane.MinSize (500) */
    float angle_threshold;    /* Plane.AngleThreshold, degrees (3.0) */
    float distance_threshold; /* Plane.DistanceThreshold (0.05) */
    float fx, fy, cx, cy;     /* static Frame::fx, fy, cx, cy */
    int width, height;        /* depth image size */
    /* GeneratePlanesFromBoundries (src/Frame.cc:938-998) */
    double line_ratio;             /* Line.Ratio (0.2) */
    float line_distance_threshold; /* Line.DistanceThreshold (0.01) */
    float image_bounds[4];         /* Frame::mnMinX, mnMaxX, mnMinY, mnMaxY; all 0 -> 0, width, 0, height
                                      (Frame::ComputeImageBounds without distortion, src/Frame.cc:557-563) */
} spslam_plane_params;

typedef struct spslam_plane {
    float coef[4];            /* mvPlaneCoefficients entry */
    int32_t n_inliers;        /* mvPlanePoints size */
    int32_t inlier_offset;    /* into the frame's inlier index buffer */
    int32_t n_contour;        /* mvBoundaryPoints size */
    int32_t contour_offset;   /* into the frame's contour index buffer */
} spslam_plane;

/* Configure (and allocate scratch for max_batch frames) the plane stage. */
int spslam_planes_configure(spslam_ctx* ctx, const spslam_plane_params* params);

/* Capacities the caller must provide per frame: planes, inlier indices,
 * contour indices. */
int spslam_planes_capacity(const spslam_ctx* ctx, int* planes_cap, int* inlier_cap, int* contour_cap);

/* Drop-in for one frame, host buffers.  *n_planes receives the plane count;
 * inliers / contours receive the index lists referenced by planes[]. */
int spslam_planes_extract(spslam_ctx* ctx, const float* depth, int w, int h, int stride_floats,
                          spslam_plane* planes, int planes_cap, int* n_planes, int32_t* inliers, int32_t* contours);

/* Batched, device resident: frame f's depth at d_depth + f*frame_stride
 * floats (rows stride_floats apart).  Per frame f: counts[f] planes at
 * d_planes + f*planes_cap, indices at d_inliers + f*inlier_cap and
 * d_contours + f*contour_cap (capacities from spslam_planes_capacity). */
int spslam_planes_extract_batch_device(spslam_ctx* ctx, const float* d_depth, int n_frames, size_t frame_stride,
                                       int stride_floats, spslam_plane* d_planes, int* d_counts,
                                       int32_t* d_inliers, int32_t* d_contours, void* hip_stream);

/* ------------------------------------------------------------------------
 * Supposed planes: Frame::GeneratePlanesFromBoundries (include/Frame.h:121,
 * src/Frame.cc:938-1144), run by the RGB-D Frame constructor right after
 * ComputePlanesFromOrganizedPointCloud (src/Frame.cc:186-194).  For each
 * plane boundary (last to first) up to 4 lines are fitted with PCL's
 * SACSegmentation (LINE, RANSAC, 1000 iterations, Line.DistanceThreshold,
 * optimized coefficients); a line that keeps >= Line.Ratio of the boundary,
 * lies >= 50 px inside the image (LineInRange) and runs along a depth border
 * (IsBorderLine) yields the plane through the line perpendicular to the source
 * plane (CaculatePlanes), appended when PlaneNotSeen.  Each appended plane
 * carries: its coefficients, the line, the source plane index, its line
 * points (organized-cloud indices; the new plane's mvBoundaryPoints and the
 * tail of its mvPlanePoints) and its synthetic patch (n_patch xyz points, the
 * head of its mvPlanePoints).  A source plane whose boundary was empty gets
 * mvBoundaryPoints = every 20th of its inliers (GenerateBoundaryPoints,
 * src/Frame.cc:1001-1011) -- an output-formatting step the caller's shim does
 * from the inlier list; it produces no lines. */
typedef struct spslam_supposed_plane {
    float coef[4];            /* appended mvPlaneCoefficients entry (d >= 0) */
    float line[6];            /* SACMODEL_LINE coefficients: point + unit direction */
    int32_t source_plane;     /* index i of the plane whose boundary gave the line */
    int32_t n_line;           /* line points */
    int32_t line_offset;      /* into the frame's line index buffer */
    int32_t n_patch;          /* synthetic patch points */
    int32_t patch_offset;     /* into the frame's patch buffer, in points (3 floats each) */
    int32_t pad;
} spslam_supposed_plane;

/* Per-frame capacities: appended planes, line indices, patch points per plane. */
int spslam_supposed_capacity(const spslam_ctx* ctx, int* supp_cap, int* line_cap, int* patch_points);

/* Drop-in for one frame on host buffers: runs on the planes of the last
 * spslam_planes_extract call of this context (the reference calls both on the
 * same Frame).  depth as passed to spslam_planes_extract.  *n receives the
 * number of appended planes; line_idx (line_cap ints) and patch_xyz
 * (supp_cap * patch_points * 3 floats) the data referenced by out[]. */
int spslam_planes_generate_from_boundaries(spslam_ctx* ctx, const float* depth, int w, int h, int stride_floats,
                                           spslam_supposed_plane* out, int cap, int* n, int32_t* line_idx,
                                           float* patch_xyz);

/* Batched, device resident: must follow spslam_planes_extract_batch_device
 * on the same frames (it reads that call's organized clouds) and takes its
 * outputs.  Per frame f: out_counts[f] appended planes at d_out + f*supp_cap,
 * line indices at d_line_idx + f*line_cap, patches at
 * d_patch + f*supp_cap*patch_points*3.  Counts beyond supp_cap are reported
 * but not stored. */
int spslam_planes_generate_from_boundaries_batch_device(spslam_ctx* ctx, const float* d_depth, int n_frames,
                                                        size_t frame_stride, int stride_floats,
                                                        const spslam_plane* d_planes, const int* d_counts,
                                                        const int32_t* d_contours, spslam_supposed_plane* d_out,
                                                        int* d_out_counts, int32_t* d_line_idx, float* d_patch,
                                                        void* hip_stream);

/* Pipelining (no reference counterpart; the reference runs both calls on one
 * Frame before the next): the organized cloud that
 * spslam_planes_extract_batch_device writes and
 * spslam_planes_generate_from_boundaries_batch_device reads is one of two sets,
 * chosen by this call for the calls enqueued after it (host order).  With
 * alternating sets, batch k+1's extraction may run on one stream while batch
 * k's supposed planes run on another; the caller orders a set's reuse after its
 * last reader (stream events).  Set 0 after spslam_planes_configure. */
int spslam_planes_select_cloud_set(spslam_ctx* ctx, int set);

/* Parity access: the line candidates fitted on boundary `plane` of frame
 * `frame` in the last call, in fit order (<= 4; the last may be the failing
 * one).  Per candidate: line[6], inlier count, RANSAC trials, flags (1 kept
 * >= Line.Ratio, 2 LineInRange, 4 IsBorderLine), offset of its points in idx
 * (organized-cloud indices, only for flag-1 candidates). */
typedef struct spslam_line_candidate {
    float line[6];
    int32_t n_inliers;
    int32_t iterations;
    int32_t flags;
    int32_t idx_offset;
} spslam_line_candidate;
int spslam_supposed_debug(spslam_ctx* ctx, int frame, int plane, spslam_line_candidate* cand, int* n_cand,
                          int32_t* idx, int idx_cap);

/* Stage access for parity tests, frame `frame` of the last batch:
 * what 0 = organized cloud (3*N floats, x,y,z per point), 1 = normals
 * (3*N floats, NaN = invalid), 2 = distance map (N floats), 3 = labels after
 * connected components (N uint32, PCL label ids), 4 = segmentation phase
 * timestamps (16 int64 ticks of the 100 MHz GPU real-time clock). */
int spslam_planes_debug(spslam_ctx* ctx, int frame, int what, void* out, int* n_points);

/* Test hook: keep = 1 makes the following plane extractions also store the connected-component labels that
 * spslam_planes_debug(what = 3) returns.  Off by default: frames whose union-find runs in LDS (16-bit labels)
 * then write no label map at all. */
int spslam_debug_plane_labels(spslam_ctx* ctx, int keep);

/* Test hook: Frame::PlaneNotSeen (src/Frame.cc:1116-1130) of each of n_coefs
 * candidate coefficient vectors against n_planes planes (4 floats each, host
 * buffers), evaluated by the device predicate the plane-extraction and
 * supposed-plane kernels use; not_seen[k] = 1 when candidate k would be kept. */
int spslam_debug_plane_not_seen(spslam_ctx* ctx, const float* planes, int n_planes, const float* coefs, int n_coefs,
                                int* not_seen);

/* Test hook: the device's double elementary functions (PoseOptimization and
 * LocalBundleAdjustment: SE3Quat::exp, Plane3D, AngleAxis -> std::sin /
 * std::cos / std::atan2 / std::pow(x, 3)), correctly rounded.
 * kind 0 sin(a), 1 cos(a), 2 atan2(a, b), 3 a^3; n host doubles each. */
int spslam_debug_libm64(spslam_ctx* ctx, int kind, const double* a, const double* b, int n, double* out);

/* Test hook: bound of PoseOptimization's internal waits (the chain wave and the compute waves hand edge rows over
 * through LDS; every wait gives up after `cap` polls).  0 restores the default (2^20 polls, never reached); -1
 * reports every problem as given up, deterministically.  A problem whose wait gave up reports lm_iterations = -1,
 * n_inliers = 0, Tcw = input, and every point and plane outlier flag set (nothing of it is kept). */
int spslam_debug_pose_spin_cap(spslam_ctx* ctx, int cap);

/* Test hook: the context's following PoseOptimization (spslam_pose_optimize*) and g2o-order
 * LocalBundleAdjustment calls treat the linear solve of LM trial q (0-based, counted over each
 * call) as failed when bit q of trial_mask is set -- what g2o does on a non-positive dense LDLT
 * (linear_solver_dense.h:107-112) or a zero SimplicialLDLT pivot (linear_solver_eigen.h:104-110):
 * the solution vector keeps its previous contents, which the update and computeScale then use
 * (optimization_algorithm_levenberg.cpp:110-127).  0 (default) turns it off. */
int spslam_debug_force_solve_failures(spslam_ctx* ctx, unsigned trial_mask);

/* ------------------------------------------------------------------------
 * RGB-D Frame per-keypoint steps (src/Frame.cc:146-181): UndistortKeyPoints
 * (:504-534, cv::undistortPoints with K and mDistCoef), ComputeStereoFromRGBD
 * (:743-764: mvDepth / mvuRight from the depth at the distorted keypoint) and
 * AssignFeaturesToGrid (:326-341: 64 x 48 cells over ComputeImageBounds).
 * Outputs per frame: mvKeysUn (keypoints with undistorted x, y), mvDepth,
 * mvuRight (-1 where no depth) and mGrid as CSR: cell (x, y) = x * 48 + y owns
 * grid_idx[grid_off[cell] .. grid_off[cell + 1]) in increasing keypoint index. */
#define SPSLAM_GRID_COLS 64
#define SPSLAM_GRID_ROWS 48

typedef struct spslam_frame_params {
    float fx, fy, cx, cy;   /* Camera.fx .. cy (mK) */
    float dist[5];          /* Camera.k1 k2 p1 p2 k3 (mDistCoef) */
    float bf;               /* Camera.bf (mbf) */
    int width, height;      /* image size (ComputeImageBounds) */
} spslam_frame_params;

/* Configure the frame stage; computes mnMinX/mnMaxX/mnMinY/mnMaxY and the grid
 * scale like the reference's first Frame (mbInitialComputations, Frame.cc:162-177).
 * bounds (4 floats) and grid_inv (2 floats) may be NULL. */
int spslam_frame_configure(spslam_ctx* ctx, const spslam_frame_params* params, float* bounds, float* grid_inv);

/* Drop-in for one frame on host buffers: kps = mvKeys (n keypoints), depth =
 * imDepth (float meters).  keys_un, mv_depth, mv_uright receive n entries,
 * grid_off 64*48+1 ints, grid_idx up to n ints. */
int spslam_frame_rgbd(spslam_ctx* ctx, const spslam_keypoint* kps, int n, const float* depth, int w, int h,
                      int stride_floats, spslam_keypoint* keys_un, float* mv_depth, float* mv_uright,
                      int32_t* grid_off, int32_t* grid_idx);

/* Batched, device resident, on the ORB batch outputs (frame f: counts[f]
 * keypoints at d_kps + f*cap_per_frame) and the depth frames.  Per frame f:
 * keys_un / depth / uright / grid_idx at f*cap_per_frame, grid_off at
 * f*(64*48+1).  d_plane_counts / d_supp_counts (may be NULL) are zeroed for
 * frames without keypoints: the reference's constructor returns before plane
 * extraction then (Frame.cc:148-149). */
int spslam_frame_rgbd_batch_device(spslam_ctx* ctx, const spslam_keypoint* d_kps, const int* d_counts,
                                   int cap_per_frame, const float* d_depth, int n_frames, size_t frame_stride,
                                   int stride_floats, spslam_keypoint* d_keys_un, float* d_mv_depth,
                                   float* d_mv_uright, int32_t* d_grid_off, int32_t* d_grid_idx,
                                   int* d_plane_counts, int* d_supp_counts, void* hip_stream);

/* ---------------------------------------------------------------- plane association
 * Map::AssociatePlanesByBoundary (src/Map.cc:196-340) with
 * Map::PointDistanceFromPlane (:343-359) and Frame::ComputePlaneWorldCoeff
 * (src/Frame.cc:1146-1150).  For every frame plane (mvPlaneCoefficients, the
 * extracted planes followed by the supposed planes) against the map planes in
 * mnId order (the reference iterates a std::set<MapPlane*> by pointer; the build
 * fixes id order):
 *   |angle| > angle_th and min boundary distance < running distance threshold
 *      -> mvpMapPlanes[i] (the last such map plane wins, thresholds tighten);
 *   else |angle| < running vertical threshold  -> mvpVerticalPlanes[i];
 *   else |angle| > running parallel threshold  -> mvpParallelPlanes[i].
 * Outputs are map-plane indices into the map-plane array (-1 = none) and
 * mbNewPlane (some frame plane without a match).  The reference never clears
 * mvpMapPlanes / mvpParallelPlanes / mvpVerticalPlanes (they are only
 * overwritten when a candidate is found), so the second call of a frame
 * (TrackLocalMap, src/Tracking.cc:1058) starts from what the first call left
 * after TrackWithMotionModel's plane-outlier discard (:1004-1028): with
 * spslam_assoc_frame.carry != 0 the match / parallel / vertical arrays are
 * read as that starting state and updated in place; with carry == 0 they start
 * at -1 (a new Frame, src/Frame.cc:199-213).  The not-seen branches
 * (:259-337) are dead in the reference and are not provided. */
typedef struct spslam_map_plane {
    float world[4];           /* MapPlane::GetWorldPos (a, b, c, d) */
    int32_t id;               /* mnId (informative: the array order is the iteration order) */
    int32_t boundary_offset;  /* first point of mvBoundaryPoints in the boundary xyz array */
    int32_t n_boundary;
    int32_t pad;
} spslam_map_plane;           /* 32 bytes */

typedef struct spslam_assoc_params {
    float dis_th;    /* Plane.AssociationDisRef (mfDisTh) */
    float angle_th;  /* Plane.AssociationAngRef (mfAngleTh) */
    float ver_th;    /* Plane.VerticalThreshold (mfVerTh) */
    float par_th;    /* Plane.ParallelThreshold (mfParTh) */
} spslam_assoc_params;

typedef struct spslam_assoc_frame {
    float Tcw[16];            /* Frame::mTcw, row-major float */
    int32_t map_offset;       /* this frame's map: planes [map_offset, map_offset + n_map) */
    int32_t n_map;
    int32_t carry;            /* != 0: match / parallel / vertical hold the frame's current associations */
    int32_t pad;
} spslam_assoc_frame;         /* 80 bytes */

/* Drop-in for one frame on host buffers.  coefs: n_planes x 4 floats; boundary_xyz:
 * float x, y, z per boundary point.  match / parallel / vertical: n_planes ints
 * (read first when frame->carry != 0); new_plane (may be NULL) receives mbNewPlane. */
int spslam_planes_associate(spslam_ctx* ctx, const spslam_assoc_frame* frame, const float* coefs, int n_planes,
                            const spslam_map_plane* map_planes, int n_map, const float* boundary_xyz,
                            int n_boundary, const spslam_assoc_params* params, int32_t* match, int32_t* parallel,
                            int32_t* vertical, int* new_plane);

/* Batched, device resident.  Frame f's planes are the first d_count_a[f] records of
 * source A (record r of frame f at d_planes_a + (f * cap_a + r) * stride_a bytes,
 * coefficients = its first 4 floats; spslam_plane / spslam_supposed_plane layouts)
 * followed by the first d_count_b[f] records of source B (may be NULL).  Outputs at
 * f * (cap_a + cap_b) + i; d_new_plane: one int per frame (may be NULL).  max_map
 * bounds every frame's n_map (host-known launch size). */
int spslam_planes_associate_batch_device(spslam_ctx* ctx, int n_frames, const spslam_assoc_frame* d_frames,
                                         const void* d_planes_a, int stride_a, const int* d_count_a, int cap_a,
                                         const void* d_planes_b, int stride_b, const int* d_count_b, int cap_b,
                                         const spslam_map_plane* d_map, const float* d_boundary_xyz, int max_map,
                                         const spslam_assoc_params* params, int32_t* d_match, int32_t* d_parallel,
                                         int32_t* d_vertical, int* d_new_plane, void* hip_stream);

/* ---------------------------------------------------------------- projection matching
 * ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame,
 * th, bMono) (src/ORBmatcher.cc:1328-1470) with Frame::GetFeaturesInArea
 * (src/Frame.cc:427-480), DescriptorDistance (src/ORBmatcher.cc:1647-1662) and
 * the rotation-consistency check (ComputeThreeMaxima, :1601-1642), as
 * Tracking::TrackWithMotionModel calls it (src/Tracking.cc:951-975: matcher
 * (0.9, checkOri = true), mvpMapPoints cleared, and when fewer than 20 matches
 * a second search at 2*th).  The last frame is given as its map points: one
 * spslam_proj_point per keypoint i with mvpMapPoints[i] && !mvbOutlier[i], in
 * increasing i.  The current frame is the frame stage's output (mvKeysUn,
 * mvuRight, mGrid) with the ORB descriptors; camera and grid geometry come
 * from spslam_frame_configure, the scale factors from the ORB tables.
 * Output per current keypoint: the index (into the frame's point list) of the
 * map point assigned to it (mvpMapPoints), -1 if none; and nmatches. */
typedef struct spslam_proj_point {
    float xw[3];          /* MapPoint::GetWorldPos */
    float angle;          /* LastFrame.mvKeysUn[i].angle */
    int32_t octave;       /* LastFrame.mvKeys[i].octave */
    int32_t n_obs;        /* MapPoint::Observations(): 0 (a visual-odometry point) does not block a keypoint */
    int32_t last_index;   /* i (informative) */
    int32_t id;           /* MapPoint::mnId (the caller's bookkeeping: seen stamps, next last frame) */
    uint8_t desc[32];     /* MapPoint::GetDescriptor */
} spslam_proj_point;      /* 64 bytes */

typedef struct spslam_proj_frame {
    float Tcw[16];        /* CurrentFrame.mTcw (motion-model prediction), row-major */
    float Tlw[16];        /* LastFrame.mTcw */
    int32_t point_offset; /* this frame's last-frame map points: [point_offset, point_offset + n_points) */
    int32_t n_points;
    int32_t pad[2];
} spslam_proj_frame;      /* 144 bytes */

typedef struct spslam_match_params {
    float th;                   /* window radius at level 0 (15 for RGB-D, Tracking.cc:963-967) */
    int32_t mono;               /* bMono */
    int32_t check_orientation;  /* ORBmatcher mbCheckOrientation */
    int32_t retry_below;        /* nmatches < retry_below -> clear and search at 2*th (20; 0 = no retry) */
} spslam_match_params;

/* Drop-in for one frame pair on host buffers.  keys_un / desc / uright: the
 * current frame's n_kp keypoints; grid_off (64*48+1) / grid_idx: its mGrid CSR.
 * match: n_kp ints.  *nmatches receives the return value of the (last) search. */
int spslam_search_by_projection(spslam_ctx* ctx, const spslam_proj_frame* frame, const spslam_proj_point* points,
                                const spslam_keypoint* keys_un, const uint8_t* desc, const float* uright, int n_kp,
                                const int32_t* grid_off, const int32_t* grid_idx, const spslam_match_params* params,
                                int32_t* match, int* nmatches);

/* Batched, device resident.  Frame f: d_frames[f]; its current frame at
 * d_keys_un / d_uright / d_match + f*cap, d_desc + f*cap*32, d_grid_off +
 * f*(64*48+1), d_grid_idx + f*cap, d_counts[f] keypoints (the ORB / frame-stage
 * batch layouts).  max_points bounds every frame's n_points (host-known launch
 * size).  d_nmatches: one int per frame. */
int spslam_search_by_projection_batch_device(spslam_ctx* ctx, int n_frames, const spslam_proj_frame* d_frames,
                                             const spslam_proj_point* d_points, int max_points,
                                             const spslam_keypoint* d_keys_un, const uint8_t* d_desc,
                                             const float* d_uright, const int32_t* d_grid_off,
                                             const int32_t* d_grid_idx, const int* d_counts, int cap,
                                             const spslam_match_params* params, int32_t* d_match, int* d_nmatches,
                                             void* hip_stream);

/* Local-map projection matching: Tracking::SearchLocalPoints (src/Tracking.cc:
 * 1375-1425) -- Frame::isInFrustum (src/Frame.cc:369-425, viewing-cosine
 * limit 0.5) with MapPoint::PredictScale (src/MapPoint.cc:402-417), then
 * ORBmatcher(nn_ratio).SearchByProjection(F, vpMapPoints, th)
 * (src/ORBmatcher.cc:45-130, RadiusByViewingCos :131-137).  The local map
 * points are given in mvpLocalMapPoints order without those the caller skips
 * (already matched in this frame, or bad).  d_taken (may be NULL) marks the
 * current keypoints whose mvpMapPoints entry is already set with
 * Observations() > 0.  Output per current keypoint: the index of the local
 * point newly assigned to it, -1 otherwise; nmatches; optionally
 * mbTrackInView per point. */
typedef struct spslam_local_point {
    float xw[3];          /* MapPoint::GetWorldPos */
    float normal[3];      /* MapPoint::GetNormal */
    float min_dist;       /* mfMinDistance (the invariance region is 0.8x .. 1.2x mfMaxDistance) */
    float max_dist;       /* mfMaxDistance */
    int32_t id;           /* mnId: index into the frame's seen-stamp array (batched form) */
    int32_t n_obs;        /* MapPoint::Observations() (carried into the next last frame) */
    int32_t pad[2];
    uint8_t desc[32];     /* MapPoint::GetDescriptor */
} spslam_local_point;     /* 80 bytes */

typedef struct spslam_local_frame {
    float Tcw[16];        /* CurrentFrame.mTcw after the motion-model PoseOptimization */
    int32_t point_offset; /* local points [point_offset, point_offset + n_points) */
    int32_t n_points;
    int32_t seen_offset;  /* batched form with d_seen: point p is skipped when d_seen[seen_offset + p.id] == stamp */
    int32_t stamp;        /*   (mnLastFrameSeen == mCurrentFrame.mnId, Tracking.cc:1380-1395) */
} spslam_local_frame;     /* 80 bytes */

typedef struct spslam_local_params {
    float th;             /* 3 for RGB-D, 5 right after relocalisation (Tracking.cc:1416-1422) */
    float nn_ratio;       /* ORBmatcher mfNNratio (0.8) */
    float view_cos_limit; /* isInFrustum limit (0.5) */
    int32_t pad;
} spslam_local_params;

int spslam_search_local_points(spslam_ctx* ctx, const spslam_local_frame* frame, const spslam_local_point* points,
                               const spslam_keypoint* keys_un, const uint8_t* desc, const float* uright, int n_kp,
                               const int32_t* grid_off, const int32_t* grid_idx, const uint8_t* taken,
                               const spslam_local_params* params, int32_t* match, int* nmatches, uint8_t* in_view);

/* Batched, device resident, same current-frame layout as
 * spslam_search_by_projection_batch_device; d_taken at f*cap (may be NULL),
 * d_in_view at the points' global index (may be NULL).  d_seen (may be NULL):
 * the frames' seen stamps (spslam_local_frame.seen_offset / stamp; the
 * SPSLAM_TRACK_DISCARD stage writes them), so the local map can be passed
 * whole and the points the frame already tracks are skipped on the device. */
int spslam_search_local_points_batch_device(spslam_ctx* ctx, int n_frames, const spslam_local_frame* d_frames,
                                            const spslam_local_point* d_points, int max_points,
                                            const spslam_keypoint* d_keys_un, const uint8_t* d_desc,
                                            const float* d_uright, const int32_t* d_grid_off,
                                            const int32_t* d_grid_idx, const int* d_counts, int cap,
                                            const uint8_t* d_taken, const spslam_local_params* params,
                                            int32_t* d_match, int* d_nmatches, uint8_t* d_in_view,
                                            const int32_t* d_seen, void* hip_stream);

/* ---------------------------------------------------------------- input images
 * Tracking::GrabImageRGBD's image preparation (src/Tracking.cc:208-229), the
 * first kernel of a step:
 *   gray  = cvtColor(imRGB, RGB2GRAY / BGR2GRAY / RGBA2GRAY / BGRA2GRAY by
 *           channels and mbRGB), OpenCV's 8U fixed point
 *           (R*4899 + G*9617 + B*1868 + 8192) >> 14; a 1-channel image is copied;
 *   depth = imD.convertTo(CV_32F, mDepthMapFactor) when the factor is not 1 or
 *           the depth is not CV_32F: float(d) * (float)factor; else copied.
 * mDepthMapFactor is the reciprocal of the YAML DepthMapFactor (Tracking.cc:142-146),
 * i.e. depth_scale = 1.0f / 5000.0f for TUM. */
typedef struct spslam_grab_params {
    int32_t channels;     /* 1, 3 or 4 (interleaved u8) */
    int32_t rgb;          /* mbRGB: 1 = R,G,B(,A) order, 0 = B,G,R(,A) */
    int32_t depth_u16;    /* 1 = CV_16U depth, 0 = CV_32F */
    float depth_scale;    /* mDepthMapFactor */
} spslam_grab_params;

/* Drop-in for one frame on host buffers: color (row stride color_stride bytes),
 * depth (row stride depth_stride elements); gray (w*h u8) and depth_out (w*h f32) dense. */
int spslam_grab_rgbd(spslam_ctx* ctx, const uint8_t* color, int color_stride, const void* depth, int depth_stride,
                     int w, int h, const spslam_grab_params* params, uint8_t* gray, float* depth_out);

/* Batched, device resident: frame f's color at d_color + f * color_frame_stride bytes,
 * depth at d_depth + f * depth_frame_stride elements; outputs dense, frame f at
 * d_gray + f*w*h and d_depth_out + f*w*h (the ORB / plane batch layouts). */
int spslam_grab_rgbd_batch_device(spslam_ctx* ctx, int n_frames, const uint8_t* d_color, size_t color_frame_stride,
                                  int color_stride, const void* d_depth, size_t depth_frame_stride, int depth_stride,
                                  int w, int h, const spslam_grab_params* params, uint8_t* d_gray, float* d_depth_out,
                                  void* hip_stream);

/* Fusion with the plane stage (no reference counterpart: Frame::ComputePlanesFromOrganizedPointCloud,
 * Frame.cc:857-874, samples the converted depth a second time).  With enable = 1 and
 * spslam_planes_configure called on the same context for the same image size, a
 * spslam_grab_rgbd_batch_device call also writes the organized cloud of its depth output into the
 * selected cloud set (spslam_planes_select_cloud_set) and tags the set with that depth output; the
 * set's next spslam_planes_extract_batch_device over exactly that depth (same pointer, dense layout,
 * no more frames) uses the cloud as it is instead of sampling the depth again (bit-identical cloud),
 * and clears the tag.  Any other extraction makes its own cloud.  The caller orders the grab before
 * the extraction (same stream or an event), as it already must for the depth.  Default 0: in the
 * pipelined batch step the grab is on the ORB stream's critical path and the fused pass measured 2 %
 * slower than a separate cloud kernel on the plane stream (profiles/r06/ab_grab_cloud_c2.txt); the
 * environment variable SPSLAM_GRAB_CLOUD=1 makes 1 the default. */
int spslam_grab_fuse_cloud(spslam_ctx* ctx, int enable);

/* ---------------------------------------------------------------- tracking graph glue
 * The Tracking-side bookkeeping between matching / plane association and
 * PoseOptimization, on the device, for a batch of frames (one stage per call):
 *
 * SPSLAM_TRACK_MOTION_MODEL -- TrackWithMotionModel's graph (src/Tracking.cc:
 *   951-981): mvpMapPoints[i] = the SearchByProjection match of keypoint i,
 *   mvpMapPlanes / mvpParallelPlanes / mvpVerticalPlanes = the first
 *   AssociatePlanesByBoundary; then Optimizer::PoseOptimization's edge loops
 *   (src/Optimizer.cc:561-640: one point edge per keypoint with a map point, in
 *   keypoint order, stereo iff mvuRight >= 0, information mvInvLevelSigma2
 *   [octave]; :681-860: plane edges over the frame planes in index order, then
 *   parallel, then vertical).  The initial pose is the motion-model prediction
 *   (proj_frames[f].Tcw).  edge_of_kp[i] receives keypoint i's edge index.
 * SPSLAM_TRACK_DISCARD -- the outlier discard after that PoseOptimization
 *   (src/Tracking.cc:986-1000: mvpMapPoints[i] = NULL where mvbOutlier[i];
 *   :1004-1028: mvpMapPlanes / mvpParallelPlanes / mvpVerticalPlanes[i] = NULL
 *   where the plane / parallel / vertical edge is an outlier -- written to
 *   next_match / next_parallel / next_vertical, the starting state of the
 *   second association (spslam_assoc_frame.carry), when those are given) and
 *   the SearchLocalPoints preconditions: taken[i] = keypoint i keeps a map point
 *   with Observations() > 0 (src/ORBmatcher.cc:95-97); the optimized pose is
 *   written into local_frames[f].Tcw and, if given, assoc_frames_next[f].Tcw
 *   (the second association runs at that pose, src/Tracking.cc:1066).
 *   With `seen` given it also stamps every map point the motion model matched
 *   (inliers and discarded outliers both get mnLastFrameSeen = the frame,
 *   Tracking.cc:997 and :1380-1390): seen[local_frames[f].seen_offset + id] =
 *   local_frames[f].stamp, which spslam_search_local_points_batch_device skips.
 * SPSLAM_TRACK_LOCAL_MAP -- TrackLocalMap's graph (src/Tracking.cc:1062-1068):
 *   mvpMapPoints = the surviving motion-model points, replaced by the
 *   SearchLocalPoints match where it assigned one (it may re-assign a keypoint
 *   whose point has no observations, src/ORBmatcher.cc:115); planes from the
 *   second association; initial pose = the motion-model result.
 *
 * Layouts: current frame f's keypoints / mvuRight / matches / taken /
 * edge_of_kp at f * cap (ORB and frame-stage batch layout); match indices are
 * relative to the frame's proj / local point_offset; plane association outputs
 * at f * (cap_a + cap_b) + i (spslam_planes_associate_batch_device layout) are
 * global map-plane indices.  The graphs are written with point_offset = f * cap
 * and plane_offset = f * 3 * (cap_a + cap_b), so the PoseOptimization outlier
 * flags of frame f are at the same offsets.  The motion model's failure test and the switch to
 * TrackReferenceKeyFrame: spslam_track_refkf_batch_device below; relocalisation is the caller's.
 *
 * Frame-to-frame state of a tracked sequence (Tracking::Track, src/Tracking.cc:
 * 443-505, TrackWithMotionModel :956-958), for batches that are consecutive
 * frames of their sequences:
 * SPSLAM_TRACK_MOTION_PRIOR -- mCurrentFrame.SetPose(mVelocity * mLastFrame.mTcw):
 *   proj_frames[f].Tcw = velocity[f] (4x4 row-major float) * proj_frames[f].Tlw
 *   (cv::Mat float product), also into assoc_frames_first[f].Tcw when given.
 *   The reference re-derives mLastFrame.mTcw through its reference keyframe
 *   (UpdateLastFrame, Tlr * Tref) first; with fixed keyframe poses that is the
 *   last pose up to float rounding, and is not restated.
 * SPSLAM_TRACK_LAST_FRAME -- after the local-map PoseOptimization (results /
 *   point_outlier = that optimisation's): mVelocity = mTcw * LastTwc (LastTwc =
 *   [Rlw^T | -Rlw^T tlw] of proj_frames[f].Tlw), the VO-match clean-up (points
 *   with Observations() < 1 dropped, :456-466) and the outlier drop (:484-488);
 *   the surviving map points (local-map match, else the kept motion-model
 *   match), in keypoint order, become the next frame's last-frame points:
 *   next_points at f * cap (xw, mvKeysUn angle, octave, n_obs, id, descriptor),
 *   next_frames[f] = {Tlw = mTcw, point_offset = f * cap, n_points}, velocity[f]. */
#define SPSLAM_TRACK_MOTION_MODEL 0
#define SPSLAM_TRACK_DISCARD 1
#define SPSLAM_TRACK_LOCAL_MAP 2
#define SPSLAM_TRACK_MOTION_PRIOR 3
#define SPSLAM_TRACK_LAST_FRAME 4

typedef struct spslam_track_batch {
    /* current frames */
    const spslam_keypoint* keys_un;  /* mvKeysUn */
    const float* uright;             /* mvuRight */
    const int* kp_counts;
    int32_t cap;
    /* motion model: last-frame map points and the SearchByProjection matches */
    const spslam_proj_frame* proj_frames;
    const spslam_proj_point* proj_points;
    const int32_t* proj_match;
    /* local map: SearchLocalPoints inputs / matches */
    spslam_local_frame* local_frames;     /* DISCARD writes Tcw */
    const spslam_local_point* local_points;
    const int32_t* local_match;           /* LOCAL_MAP */
    uint8_t* taken;                       /* DISCARD writes */
    /* frame planes (extracted, then supposed) and their association */
    const void* planes_a;
    const void* planes_b;
    const int* count_a;
    const int* count_b;
    int32_t stride_a, stride_b, cap_a, cap_b;
    const spslam_map_plane* map;
    const int32_t* assoc_match;
    const int32_t* assoc_parallel;
    const int32_t* assoc_vertical;
    spslam_assoc_frame* assoc_frames_next;  /* DISCARD writes Tcw (may be NULL) */
    const uint8_t* plane_outlier;           /* motion-model plane edge outlier flags (DISCARD, with next_*) */
    int32_t* next_match;                    /* DISCARD writes the surviving associations (may be NULL) */
    int32_t* next_parallel;
    int32_t* next_vertical;
    /* sequence state (MOTION_PRIOR, DISCARD stamps, LAST_FRAME) */
    spslam_assoc_frame* assoc_frames_first;  /* MOTION_PRIOR writes Tcw (may be NULL) */
    int32_t* seen;                        /* DISCARD stamps (may be NULL) */
    spslam_proj_frame* next_frames;       /* LAST_FRAME writes */
    spslam_proj_point* next_points;       /* LAST_FRAME writes, f * cap */
    float* velocity;                      /* 16 floats per frame: MOTION_PRIOR reads, LAST_FRAME writes */
    const uint8_t* point_outlier_local;   /* LAST_FRAME: the local-map PoseOptimization's point outlier flags */
    /* PoseOptimization graphs */
    spslam_pose_problem* problems;
    spslam_point_obs* points;             /* f * cap */
    spslam_plane_obs* planes;             /* f * 3 * (cap_a + cap_b) */
    int32_t* edge_of_kp;                  /* MOTION_MODEL writes, DISCARD / LOCAL_MAP read */
    const spslam_pose_result* results;    /* the motion-model PoseOptimization (DISCARD, LOCAL_MAP) */
    const uint8_t* point_outlier;         /* its point outlier flags (DISCARD, LOCAL_MAP) */
    float fx, fy, cx, cy, bf;
    int32_t pad;
} spslam_track_batch;

int spslam_track_graph_batch_device(spslam_ctx* ctx, int n_frames, int stage, const spslam_track_batch* batch,
                                    void* hip_stream);

/* TrackWithMotionModel's failure and the switch to TrackReferenceKeyFrame (src/Tracking.cc:318-324: bOK =
 * TrackWithMotionModel(); if (!bOK) bOK = TrackReferenceKeyFrame()), batched.  The motion model fails when
 * SearchByProjection (after the 2*th retry) finds fewer than 10 matches (:977, before the association and
 * PoseOptimization) or when fewer than 5 map points / map planes survive its discard (nmatchesMap, :986-1053).
 * For the frames that fail a caller runs ComputeBoW + SearchByBoW against the reference keyframe
 * (spslam_bow_transform_batch_device / spslam_search_by_bow_batch_device, :796-806); where that finds at least 10
 * matches the frame is re-tracked from the last frame's pose -- association, MOTION_MODEL graph, PoseOptimization
 * and DISCARD over the reference keyframe's map points (:808-882) -- into separate buffers that
 * spslam_masked_frame_copy_device then moves over the motion model's.
 *   SPSLAM_REFKF_PREPARE (after the motion model's DISCARD; mm = its spslam_track_batch): fallback[f], and
 *     refkf_counts[f] = kp_counts[f] where it failed, else 0 (the BoW transform's counts: it skips the others).
 *   SPSLAM_REFKF_SELECT (after SearchByBoW): apply[f] = fallback[f] && bow_nmatches[f] >= 10 (:806);
 *     state[f] = 0 (motion model), 1 (reference keyframe) or 2 (both failed: LOST, the motion model's result is
 *     kept); refkf_match = the BoW matches as rows of the keyframe's point set (-1 elsewhere and where !apply);
 *     refkf_frames[f] = {Tcw = Tlw = proj_frames[f].Tlw (SetPose(mLastFrame.mTcw)), point_offset / n_points =
 *     refkf_sets[2 f], [2 f + 1] (the keyframe's map points inside proj_points), 0 points where !apply};
 *     refkf_assoc[f] = assoc_frames[f] at Tcw = Tlw, n_map = 0 where !apply, carry = 1 (the association starts
 *     from the motion model's surviving planes, which the caller copies into its association arrays) unless the
 *     motion model stopped before associating (< 10 matches: carry = 0); and the seen stamps: the motion model's
 *     DISCARD stamped every one of its matches (mnLastFrameSeen); where the keyframe takes over only its discarded
 *     outliers keep the stamp (:990-997; none when it stopped at < 10 matches), the others get stamp - 1. */
#define SPSLAM_REFKF_PREPARE 0
#define SPSLAM_REFKF_SELECT 1

typedef struct spslam_refkf_batch {
    const int32_t* nmatches;                 /* SearchByProjection's count after the retry, per frame */
    uint8_t* fallback;                       /* PREPARE writes: the motion model failed */
    int32_t* refkf_counts;                   /* PREPARE writes */
    const int32_t* bow_nmatches;             /* SELECT: SearchByBoW's count per frame */
    const int32_t* bow_match;                /* SELECT: SearchByBoW's keyframe feature per keypoint (cap per frame) */
    const int32_t* refkf_rows;               /* SELECT: per keyframe feature its map point's row in the keyframe's
                                                point set or -1 (rows_stride per keyframe) */
    const int32_t* refkf_index;              /* SELECT: each frame's keyframe (row block of refkf_rows) */
    int32_t rows_stride, pad;
    const int32_t* refkf_sets;               /* SELECT: (point_offset, n_points) per frame */
    const spslam_assoc_frame* assoc_frames;  /* SELECT: the motion model's first-association frames */
    uint8_t* apply;                          /* SELECT writes */
    int8_t* state;                           /* SELECT writes (may be NULL) */
    int32_t* refkf_match;                    /* SELECT writes (cap per frame) */
    spslam_proj_frame* refkf_frames;         /* SELECT writes */
    spslam_assoc_frame* refkf_assoc;         /* SELECT writes */
} spslam_refkf_batch;

int spslam_track_refkf_batch_device(spslam_ctx* ctx, int n_frames, int stage, const spslam_track_batch* mm,
                                    const spslam_refkf_batch* rk, void* hip_stream);

/* The reference keyframe TrackReferenceKeyFrame uses (mpReferenceKF), per frame, batched.  TrackLocalMap's
 * UpdateLocalKeyFrames sets it to pKFmax, the keyframe that observes the most of the frame's map points after
 * TrackWithMotionModel's (or TrackReferenceKeyFrame's) discard, first maximum in keyframe order (src/Tracking.cc:
 * 1459-1570; the reference iterates a std::map<KeyFrame*, int> in pointer order: keyframe id order here, as
 * everywhere at this ABI); it is not run on a LOST frame (:406-409); CreateNewKeyFrame then makes the new keyframe
 * the reference (:1258).  mm = the first graph's spslam_track_batch after the discard (and after the masked copy
 * of a TrackReferenceKeyFrame re-tracking): the frame's map points are proj_points[point_offset +
 * proj_match[i]] for every keypoint i with an edge that is not an outlier; a point's keyframe is id / ids_per_kf
 * (each map point counted for the keyframe that created it).  Writes refkf_index[f] (kept where LOST or where no
 * map point remains: pKFmax stays NULL), refkf_sets[2 f .. 2 f + 1] = kf_sets of it and, when refkf_pairs is
 * given, the (keyframe, frame) pair of spslam_search_by_bow_batch_device. */
typedef struct spslam_refkf_vote {
    const int32_t* kf_base;     /* per frame: the index of its sequence's keyframe 0 in the keyframe tables */
    const int32_t* kf_sets;     /* per keyframe: (point_offset, n_points) of its map points inside proj_points */
    int32_t ids_per_kf;         /* map point id / ids_per_kf = the keyframe (of the sequence) that created it */
    int32_t n_kf;               /* keyframes per sequence, 1 .. 1024 */
    int32_t new_kf;             /* >= 0: the frames become keyframe new_kf of their sequence (CreateNewKeyFrame) */
    int32_t pad;
    const int8_t* state;        /* per frame: 2 = LOST (spslam_refkf_batch.state); may be NULL */
    int32_t* refkf_index;       /* in / out: each frame's reference keyframe (kf_base + its keyframe) */
    int32_t* refkf_sets;        /* out: (point_offset, n_points) of it */
    int32_t* refkf_pairs;       /* out (may be NULL): (refkf_index, f) */
} spslam_refkf_vote;

int spslam_track_refkf_vote_batch_device(spslam_ctx* ctx, int n_frames, const spslam_track_batch* mm,
                                         const spslam_refkf_vote* vote, void* hip_stream);

/* dst[f] = src[f] for every frame f with flags[f] != 0, region by region: frame f's bytes at dst + f * dst_stride
 * and src + f * src_stride (sizes and strides multiples of 4; at most 32 regions per call). */
typedef struct spslam_frame_region {
    void* dst;
    const void* src;
    int64_t frame_bytes;
    int64_t dst_stride;
    int64_t src_stride;
} spslam_frame_region;

int spslam_masked_frame_copy_device(spslam_ctx* ctx, int n_frames, const uint8_t* flags, int n_regions,
                                    const spslam_frame_region* regions, void* hip_stream);

/* ---------------------------------------------------------------- bag of words
 * DBoW2 (vendored Thirdparty/DBoW2) as the tracking path uses it:
 *   spslam_bow_load_vocabulary  TemplatedVocabulary::loadFromTextFile
 *                               (DBoW2/TemplatedVocabulary.h:1338-1424; System.cc:64 loads
 *                               ORBvoc.txt this way).  The text is "k L scoring weighting"
 *                               then one "parent isLeaf d0..d31 weight" line per node; an
 *                               empty line after a final newline becomes one more leaf under
 *                               the root with weight 0 (the reference's eof loop), whose
 *                               descriptor the reference leaves uninitialised (zero here).
 *                               One vocabulary per context, resident in HBM.
 *   spslam_bow_transform        Frame::ComputeBoW / KeyFrame::ComputeBoW (src/Frame.cc:495-502,
 *                               src/KeyFrame.cc:64-72): TemplatedVocabulary::transform(
 *                               descriptors, mBowVec, mFeatVec, levelsup = 4) (:1127-1194,
 *                               :1217-1259): BowVector = sorted (word id, value) pairs
 *                               (TF-IDF: summed idf weights, then L1-normalised for ORBvoc's
 *                               L1_NORM scoring), FeatureVector = sorted node ids (the node at
 *                               level L - levelsup on each feature's path) with the feature
 *                               indices of each node in increasing order (CSR: fv_start has
 *                               n_fv + 1 entries).  Stop words (weight 0) are in neither.
 *   spslam_search_by_bow        ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
 *                               (src/ORBmatcher.cc:159-288), as TrackReferenceKeyFrame
 *                               (matcher(0.7, true), Tracking.cc:797-802) and Relocalization
 *                               (0.75, Tracking.cc:1593-1609) call it: per shared FeatureVector
 *                               node, each keyframe feature with a good map point takes the
 *                               closest free frame feature if its distance <= TH_LOW (50) and
 *                               < nn_ratio x the second best; rotation-consistency filter
 *                               (HISTO_LENGTH 30, ComputeThreeMaxima).  Output per frame
 *                               feature: the keyframe feature whose map point it receives
 *                               (vpMapPointMatches), -1 if none; return value nmatches. */
typedef struct spslam_bow_params {
    float nn_ratio;           /* ORBmatcher mfNNratio (0.7 TrackReferenceKeyFrame, 0.75 Relocalization) */
    int32_t check_orientation;/* mbCheckOrientation */
} spslam_bow_params;

/* text: the vocabulary file's bytes (len of them).  Outputs (may be NULL): k, L, node and word counts. */
int spslam_bow_load_vocabulary(spslam_ctx* ctx, const char* text, size_t len, int* k, int* L, int* n_nodes,
                               int* n_words);

/* Drop-in for one frame on host buffers: desc n x 32 bytes.  bow_words / bow_values:
 * >= n entries, *n_bow receives the BowVector size; fv_nodes: >= n, fv_start: >= n + 1,
 * fv_features: >= n entries, *n_fv the FeatureVector size. */
int spslam_bow_transform(spslam_ctx* ctx, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words,
                         double* bow_values, int* n_bow, uint32_t* fv_nodes, int32_t* fv_start,
                         int32_t* fv_features, int* n_fv);

/* Batched, device resident: frame f's d_counts[f] descriptors at d_desc + f*cap*32 (the ORB
 * batch layout).  Outputs of frame f at f*cap (d_fv_start at f*(cap+1), relative to the
 * frame's f*cap); d_n_bow / d_n_fv one int per frame.  cap <= 8192. */
int spslam_bow_transform_batch_device(spslam_ctx* ctx, int n_frames, const uint8_t* d_desc, const int* d_counts,
                                      int cap, int levelsup, uint32_t* d_bow_words, double* d_bow_values,
                                      int* d_n_bow, uint32_t* d_fv_nodes, int32_t* d_fv_start,
                                      int32_t* d_fv_features, int* d_n_fv, void* hip_stream);

/* One side of SearchByBoW in the batch layout of spslam_bow_transform_batch_device:
 * slot f's features at f*cap (descriptors, keypoints -- only .angle is read -- and, on the
 * keyframe side, has_point[i] = GetMapPointMatches()[i] && !isBad()), its FeatureVector at
 * f*cap / f*(cap+1). */
typedef struct spslam_bow_side {
    const uint8_t* desc;
    const spslam_keypoint* keys;     /* keyframe: mvKeysUn; frame: mvKeys */
    const uint8_t* has_point;        /* keyframe side; ignored on the frame side */
    const int* counts;
    const uint32_t* fv_nodes;
    const int32_t* fv_start;
    const int32_t* fv_features;
    const int* n_fv;
    int32_t cap;
    int32_t pad;
} spslam_bow_side;

/* Drop-in for one (keyframe, frame) pair on host buffers (FeatureVectors as spslam_bow_transform
 * returns them).  match: f_n ints. */
int spslam_search_by_bow(spslam_ctx* ctx, const uint8_t* kf_desc, const spslam_keypoint* kf_keys,
                         const uint8_t* kf_has_point, int kf_n, const uint32_t* kf_fv_nodes,
                         const int32_t* kf_fv_start, const int32_t* kf_fv_features, int kf_n_fv,
                         const uint8_t* f_desc, const spslam_keypoint* f_keys, int f_n, const uint32_t* f_fv_nodes,
                         const int32_t* f_fv_start, const int32_t* f_fv_features, int f_n_fv,
                         const spslam_bow_params* params, int32_t* match, int* nmatches);

/* Batched, device resident: pair p = (keyframe slot, frame slot) = d_pairs[2p], d_pairs[2p+1];
 * d_match at p * frame.cap, d_nmatches one int per pair. */
int spslam_search_by_bow_batch_device(spslam_ctx* ctx, int n_pairs, const int32_t* d_pairs,
                                      const spslam_bow_side* keyframe, const spslam_bow_side* frame,
                                      const spslam_bow_params* params, int32_t* d_match, int* d_nmatches,
                                      void* hip_stream);

/* ---------------------------------------------------------------- the whole batched step
 * The throughput path as one call per step, for a C / C++ caller: GrabImageRGBD (Tracking.cc:208-229) ->
 * ORB extraction || ComputePlanesFromOrganizedPointCloud + GeneratePlanesFromBoundries (the RGB-D Frame
 * constructor) -> the tracking tail: Frame keypoint steps, SearchByProjection (TrackWithMotionModel,
 * Tracking.cc:951-975), AssociatePlanesByBoundary, the motion-model PoseOptimization graph and optimisation,
 * the outlier discard, SearchLocalPoints, the second association, the local-map graph and PoseOptimization
 * (TrackLocalMap, :1054-1068) -- the batched entry points above, enqueued on streams and events the step
 * object owns (the tail stream at high priority).  pipelined != 0: spslam_step_run(k) enqueues batch k+1's
 * extraction (grab + ORB on one stream, planes on another, into extraction set (k+1) % 2) beside batch k's
 * tail (set k % 2); a set is rewritten only after the tail that read it has finished.  spslam_step_prime
 * enqueues batch 0's extraction once before the first run.  pipelined == 0: each run is grab -> (planes ||
 * ORB) -> tail of `next`, set 0 only.  The context must be configured as for the single stages
 * (spslam_frame_configure, spslam_planes_configure; the vocabulary is not used).
 * Buffers: device memory; NULL members of the sets / tail are allocated by the step object (owned, freed by
 * spslam_step_destroy), others are the caller's; spslam_step_buffers returns all of them. */
typedef struct spslam_step_config {
    int32_t n_frames, width, height, kp_cap;      /* batch, image size, keypoint slots per frame */
    int32_t pipelined, tail_priority, orb_priority, planes_priority;
    spslam_grab_params grab;                      /* GrabImageRGBD: channels, mbRGB, depth type, mDepthMapFactor */
    spslam_match_params match;                    /* TrackWithMotionModel: th 15, checkOri, retry below 20 */
    spslam_local_params local;                    /* SearchLocalPoints: th 3, nn 0.8, viewing cos 0.5 */
    spslam_assoc_params assoc;                    /* Plane.Association* / Vertical / ParallelThreshold */
    spslam_plane_config pose;                     /* PoseOptimization Plane.* keys */
    float fx, fy, cx, cy, bf;                     /* camera (the graph's point edges) */
    int32_t pad;
} spslam_step_config;

typedef struct spslam_step_frames {               /* one batch of input frames (GrabImageRGBD's inputs) */
    const uint8_t* color;                         /* frame f at color + f * color_frame_stride bytes */
    size_t color_frame_stride;
    const void* depth;                            /* frame f at depth + f * depth_frame_stride elements */
    size_t depth_frame_stride;
    int32_t color_stride, depth_stride;           /* row strides: bytes / elements */
} spslam_step_frames;

typedef struct spslam_step_tracking {             /* one batch's tracking inputs (device) */
    const spslam_proj_frame* proj_frames;         /* last frames' map points (spslam_search_by_projection_batch_device) */
    const spslam_proj_point* proj_points;
    spslam_local_frame* local_frames;             /* local maps (spslam_search_local_points_batch_device; DISCARD writes Tcw) */
    const spslam_local_point* local_points;
    const spslam_assoc_frame* assoc_frames1;      /* first association (motion-model pose) */
    spslam_assoc_frame* assoc_frames2;            /* second (DISCARD writes Tcw), carry = 1 */
    const spslam_map_plane* map;
    const float* boundary_xyz;
    int32_t max_proj_points, max_local_points, max_map, pad;
} spslam_step_tracking;

typedef struct spslam_step_set {                  /* extraction outputs of one batch (the batch layouts above) */
    uint8_t* gray;
    float* depth;
    spslam_keypoint* kps;
    uint8_t* desc;
    int* counts;
    spslam_plane* planes;
    int* plane_counts;
    int32_t* inliers;
    int32_t* contours;
    spslam_supposed_plane* supposed;
    int* supposed_counts;
    int32_t* lines;
    float* patch;
} spslam_step_set;

typedef struct spslam_step_tail {                 /* the tracking tail's buffers and outputs */
    spslam_keypoint* keys_un;
    float* mv_depth;
    float* uright;
    int32_t* grid_off;
    int32_t* grid_idx;
    int32_t* match;
    int* nmatches;
    uint8_t* taken;
    int32_t* local_match;
    int* local_nmatches;
    int32_t* edge_of_kp;
    int32_t* assoc[2][3];                         /* [association][match, parallel, vertical] */
    int* new_plane[2];
    spslam_pose_problem* problems[2];             /* [0] motion model, [1] local map */
    spslam_point_obs* points[2];
    spslam_plane_obs* planes[2];
    uint8_t* point_outlier[2];
    uint8_t* plane_outlier[2];
    spslam_pose_result* results[2];
} spslam_step_tail;

typedef struct spslam_step spslam_step;
int spslam_step_create(spslam_ctx* ctx, const spslam_step_config* cfg, const spslam_step_set* sets /* [2], may be NULL */,
                       const spslam_step_tail* tail /* may be NULL */, spslam_step** out);
int spslam_step_buffers(const spslam_step* step, spslam_step_set* sets /* [2] */, spslam_step_tail* tail);
int spslam_step_prime(spslam_step* step, const spslam_step_frames* first);
int spslam_step_run(spslam_step* step, const spslam_step_frames* next, const spslam_step_tracking* tracking);
int spslam_step_sync(spslam_step* step);          /* host waits for every stream of the step */
void* spslam_step_stream(const spslam_step* step); /* the tail stream (hipStream_t) */
void spslam_step_destroy(spslam_step* step);

/* Measurement: when enabled, every kernel kind launched by this context is
 * bracketed by HIP events on its launch stream.  spslam_kernel_times returns,
 * per kind, the summed event time (ms) and number of timed launches since the
 * last spslam_set_timing call (it waits for the recorded events).  Returns the
 * number of kinds written; spslam_kernel_name(kind) names the kernel. */
int spslam_set_timing(spslam_ctx* ctx, int enable);
int spslam_kernel_times(spslam_ctx* ctx, double* total_ms, long long* launches, int max_kinds);
const char* spslam_kernel_name(int kind);

#ifdef __cplusplus
}
#endif

#endif /* SPSLAM_GPU_H */
