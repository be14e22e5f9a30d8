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
 * (a hipStream_t; NULL = the context's own stream). */
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
