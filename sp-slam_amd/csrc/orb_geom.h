// Level geometry of the ORB pyramid, shared by the host launcher and the
// gfx950 kernels.  All derived sizes follow src/ORBextractor.cc exactly:
// level size (:1111-1112), FAST cell grid (:769-787), per-level feature
// quota (:435-446), scaled patch size (:837).
#pragma once
#include <cstdint>

namespace spslam {

constexpr int kMaxLevels = 8;
constexpr int kEdgeThreshold = 19;     // src/ORBextractor.cc:74
constexpr int kMinBorder = kEdgeThreshold - 3;
constexpr int kCellCap = 512;          // max FAST survivors of one cell window (checked on host)
constexpr int kCellWinMax = 72;        // max cell window side (LDS tile pitch)
constexpr int kNodeCap = 1024;         // max DistributeOctTree list length (checked on host)
constexpr int kLevelTileW = 64;        // level_kernel output tile
constexpr int kLevelTileH = 32;

struct LevelGeom {
    int w, h;                 // level image size
    int stride;               // row pitch in bytes of the level image (levels >= 1: w rounded up to 64)
    int bpitch;               // row pitch of the blurred level and the FAST score map (w rounded up to 64)
    long long frame_stride;   // bytes between frames of this level
    const uint8_t* img;       // level image, frame 0
    uint8_t* blur;            // blurred level, frame 0 (pitch bpitch, frame stride blur_frame_stride)
    long long blur_frame_stride;
    int maxBorderX, maxBorderY;
    int nCols, nRows, wCell, hCell;
    int cell_base;            // first cell of this level in the per-frame cell array
    int nfeat;                // mnFeaturesPerLevel[level]
    int kp_cap;               // per-level keypoint slot capacity
    int kp_base;              // offset of the level's slot in the per-frame level-keypoint array
    int key_base;             // offset of the level's key scratch (in keys) per frame
    int patch_size;           // (int)(PATCH_SIZE * mvScaleFactor[level])
    float scale;              // mvScaleFactor[level]
    int tiles_x;              // level_kernel tiles per row
    uint8_t* score;           // FAST score map (pitch bpitch, frame stride blur_frame_stride), frame 0
    double rscale_x, rscale_y;  // resize from level-1: 1. / ((double)w / w_prev), as OpenCV computes it
};

struct OrbGeom {
    LevelGeom lv[kMaxLevels];
    int nlevels;
    int cells_per_frame;
    int lvl_kp_per_frame;     // sum of kp_cap over levels
    int keys_per_frame;       // sum of ncells*kCellCap over levels
    int level_tiles[kMaxLevels];  // level_kernel tiles per frame, per level
    int pad_[4];
};

// XCD-aware workgroup order.  MI355X dispatches consecutive workgroups of a
// launch round-robin over its 8 XCDs, each with its own L2.  xcd_remap turns
// the hardware id b of an n-workgroup 1-D launch into a logical id such that
// every XCD runs one contiguous range of logical ids -- a kernel that derives
// (frame, item) from the logical id then keeps each frame's reads on one L2.
constexpr int kXcds = 8;
#if defined(__HIPCC__)
__device__ __forceinline__ int xcd_remap(int b, int n) {
    const int x = b % kXcds, local = b / kXcds, q = n / kXcds, r = n % kXcds;
    return x * q + min(x, r) + local;  // XCD x owns q (+1 for x < r) consecutive logical ids
}
#endif

// Intermediate per-level keypoint (DistributeOctTree output, level coordinates).
struct LevelKp {
    uint16_t x, y;            // level pixel coordinates (integral in the reference)
    uint16_t response;        // FAST score
    uint16_t pad;
};

}  // namespace spslam
