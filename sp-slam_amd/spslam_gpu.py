"""ctypes binding of the C ABI in include/spslam_gpu.h (the gfx950 hot path).

This is the Python side of the drop-in boundary: the same entry points a
cgo/JNI/ctypes binding of the reference would call.  The
library is built in-tree (`make` -> sp-slam_amd/libspslam_gpu.so); there is
no CPU fallback -- if the library or a HIP device is missing, constructing
`OrbExtractor` raises.
"""
from __future__ import annotations

import ctypes
import os
import pathlib

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = _HERE / "libspslam_gpu.so"

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28


class OrbParams(ctypes.Structure):
    _fields_ = [("nfeatures", ctypes.c_int), ("scale_factor", ctypes.c_float), ("nlevels", ctypes.c_int),
                ("ini_th_fast", ctypes.c_int), ("min_th_fast", ctypes.c_int), ("width", ctypes.c_int),
                ("height", ctypes.c_int), ("max_batch", ctypes.c_int)]


EXPORTED = [
    "spslam_create", "spslam_destroy", "spslam_last_error", "spslam_orb_tables", "spslam_orb_max_keypoints",
    "spslam_orb_extract", "spslam_orb_extract_batch_device", "spslam_orb_debug_stage", "spslam_orb_level_size",
    "spslam_set_timing", "spslam_kernel_times", "spslam_kernel_name",
]

_lib = None


def load_library(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load libspslam_gpu.so (raises OSError if it was not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7.  If
    # torch is importable, load it first so our DT_NEEDED libamdhip64.so.7
    # binds to the already-loaded copy instead of a second runtime from
    # /opt/rocm (two runtimes in one process cannot share the device).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(str(path or os.environ.get("SPSLAM_GPU_LIB") or LIB_PATH))
    vp, ip, fp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_float)
    lib.spslam_create.argtypes = [ctypes.c_int, ctypes.POINTER(OrbParams), ctypes.POINTER(vp)]
    lib.spslam_destroy.argtypes = [vp]
    lib.spslam_destroy.restype = None
    lib.spslam_last_error.argtypes = [vp]
    lib.spslam_last_error.restype = ctypes.c_char_p
    lib.spslam_orb_tables.argtypes = [vp, ip, fp, fp, fp, fp, ip]
    lib.spslam_orb_max_keypoints.argtypes = [vp]
    lib.spslam_orb_extract.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int, ip]
    lib.spslam_orb_extract_batch_device.argtypes = [vp, vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, vp, vp, vp,
                                                    ctypes.c_int, vp]
    lib.spslam_orb_debug_stage.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ip]
    lib.spslam_orb_level_size.argtypes = [vp, ctypes.c_int, ip, ip]
    lib.spslam_set_timing.argtypes = [vp, ctypes.c_int]
    lib.spslam_kernel_times.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong),
                                        ctypes.c_int]
    lib.spslam_kernel_name.argtypes = [ctypes.c_int]
    lib.spslam_kernel_name.restype = ctypes.c_char_p
    if path is None:
        _lib = lib
    return lib


class SpslamError(RuntimeError):
    pass


class OrbExtractor:
    """GPU ORB extractor; mirrors ORB_SLAM2::ORBextractor (include/ORBextractor.h:45-111)."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th_fast=20, min_th_fast=7,
                 width=640, height=480, max_batch=1, device=0):
        self.lib = load_library()
        self.params = OrbParams(nfeatures, scale_factor, nlevels, ini_th_fast, min_th_fast, width, height, max_batch)
        self.ctx = ctypes.c_void_p()
        rc = self.lib.spslam_create(device, ctypes.byref(self.params), ctypes.byref(self.ctx))
        if rc != 0:
            raise SpslamError(f"spslam_create failed ({rc})")
        self.width, self.height, self.nlevels = width, height, nlevels
        self.max_kp = self.lib.spslam_orb_max_keypoints(self.ctx)

    def close(self):
        if self.ctx:
            self.lib.spslam_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise SpslamError(f"rc={rc}: {self.lib.spslam_last_error(self.ctx).decode()}")

    # --- ORBextractor getters (include/ORBextractor.h:63-83)
    def tables(self):
        n = ctypes.c_int()
        arr = [(ctypes.c_float * 8)() for _ in range(4)]
        fpl = (ctypes.c_int * 8)()
        self._check(self.lib.spslam_orb_tables(self.ctx, ctypes.byref(n), *arr, fpl))
        k = n.value
        return dict(nlevels=k, scale=np.array(arr[0][:k]), inv_scale=np.array(arr[1][:k]),
                    sigma2=np.array(arr[2][:k]), inv_sigma2=np.array(arr[3][:k]), features=np.array(fpl[:k]))

    def level_size(self, level):
        w, h = ctypes.c_int(), ctypes.c_int()
        self._check(self.lib.spslam_orb_level_size(self.ctx, level, ctypes.byref(w), ctypes.byref(h)))
        return w.value, h.value

    # --- ORBextractor::operator() (host buffers)
    def __call__(self, gray: np.ndarray):
        gray = np.ascontiguousarray(gray, dtype=np.uint8)
        h, w = gray.shape if gray.size else (0, 0)
        kps = np.zeros(self.max_kp, KEYPOINT_DTYPE)
        desc = np.zeros((self.max_kp, 32), np.uint8)
        n = ctypes.c_int()
        self._check(self.lib.spslam_orb_extract(self.ctx, gray.ctypes.data if gray.size else None, w, h, w,
                                                kps.ctypes.data, desc.ctypes.data, self.max_kp, ctypes.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    # --- batched, device resident
    def extract_batch_device(self, gray_ptr: int, n_frames: int, frame_stride: int, stride: int,
                             kps_ptr: int, desc_ptr: int, counts_ptr: int, cap_per_frame: int, stream: int = 0):
        self._check(self.lib.spslam_orb_extract_batch_device(self.ctx, gray_ptr, n_frames, frame_stride, stride,
                                                             kps_ptr, desc_ptr, counts_ptr, cap_per_frame,
                                                             stream or None))

    # --- measurement
    def set_timing(self, enable: bool):
        self._check(self.lib.spslam_set_timing(self.ctx, int(enable)))

    def kernel_times(self):
        """{kernel name: (total ms, launches)} since set_timing(True)."""
        tot = (ctypes.c_double * 32)()
        cnt = (ctypes.c_longlong * 32)()
        n = self.lib.spslam_kernel_times(self.ctx, tot, cnt, 32)
        return {self.lib.spslam_kernel_name(k).decode(): (tot[k], cnt[k]) for k in range(n)}

    # --- stage access for parity tests
    def debug_stage(self, frame: int, level: int, stage: int, cap: int | None = None):
        w, h = self.level_size(level)
        n = ctypes.c_int()
        if stage in (0, 1):
            out = np.zeros((h, w), np.uint8)
            self._check(self.lib.spslam_orb_debug_stage(self.ctx, frame, level, stage, out.ctypes.data, out.size,
                                                        ctypes.byref(n)))
            return out
        cap = cap or (1 << 20 if stage == 2 else 4096)
        out = np.zeros(cap, KEYPOINT_DTYPE)
        self._check(self.lib.spslam_orb_debug_stage(self.ctx, frame, level, stage, out.ctypes.data, cap,
                                                    ctypes.byref(n)))
        return out[:n.value].copy()


# ---------------------------------------------------------------------------
# PoseOptimization (include/spslam_gpu.h, spslam_pose_*)
POINT_OBS_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("ur", "<f4"), ("inv_sigma2", "<f4"), ("xw", "<f4", 3),
                            ("kp_index", "<i4")])
PLANE_OBS_DTYPE = np.dtype([("meas", "<f4", 4), ("world", "<f4", 4), ("kind", "<i4"), ("plane_index", "<i4"),
                            ("map_plane_id", "<i4"), ("pad", "<i4")])
POSE_PROBLEM_DTYPE = np.dtype([("Tcw", "<f4", 16), ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"),
                               ("bf", "<f4"), ("n_points", "<i4"), ("n_planes", "<i4"), ("point_offset", "<i4"),
                               ("plane_offset", "<i4"), ("pad", "<i4")])
POSE_RESULT_DTYPE = np.dtype([("Tcw", "<f4", 16), ("n_inliers", "<i4"), ("lm_iterations", "<i4"),
                              ("trial_passes", "<i4"), ("trials", "<i4")])
assert POINT_OBS_DTYPE.itemsize == 32 and PLANE_OBS_DTYPE.itemsize == 48
assert POSE_PROBLEM_DTYPE.itemsize == 104 and POSE_RESULT_DTYPE.itemsize == 80


class PlaneConfig(ctypes.Structure):
    """Plane.* YAML keys read by PoseOptimization (TUM1.yaml defaults)."""
    _fields_ = [("angle_info", ctypes.c_double), ("distance_info", ctypes.c_double),
                ("parallel_info", ctypes.c_double), ("vertical_info", ctypes.c_double), ("chi", ctypes.c_double),
                ("vp_chi", ctypes.c_double)]

    @classmethod
    def tum(cls):
        return cls(1.0, 100.0, 0.5, 0.5, 300.0, 300.0)


def _bind_pose(lib):
    vp = ctypes.c_void_p
    lib.spslam_pose_optimize.argtypes = [vp, vp, vp, vp, ctypes.POINTER(PlaneConfig), vp, vp, vp]
    lib.spslam_pose_optimize_batch_device.argtypes = [vp, ctypes.c_int, vp, vp, vp, ctypes.POINTER(PlaneConfig), vp,
                                                      vp, vp, vp, vp]


EXPORTED += ["spslam_pose_optimize", "spslam_pose_optimize_batch_device", "spslam_debug_libm64",
             "spslam_debug_pose_spin_cap", "spslam_debug_force_solve_failures"]


def debug_force_solve_failures(ex: "OrbExtractor", trial_mask: int):
    """Test hook: bit q set = LM trial q's linear solve (PoseOptimization, g2o-order LocalBundleAdjustment) reports
    failure, so g2o's stale-solution path runs (0 = off)."""
    ex.lib.spslam_debug_force_solve_failures.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    ex._check(ex.lib.spslam_debug_force_solve_failures(ex.ctx, int(trial_mask)))


def debug_pose_spin_cap(ex: "OrbExtractor", cap: int):
    """Test hook: bound of PoseOptimization's internal waits (0 = default); a tiny cap forces the give-up path."""
    ex.lib.spslam_debug_pose_spin_cap.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ex._check(ex.lib.spslam_debug_pose_spin_cap(ex.ctx, int(cap)))


def debug_libm64(ex: "OrbExtractor", kind: int, a, b=None):
    """The device's correctly rounded sin (kind 0) / cos (1) / atan2(a, b) (2) / cube (3) on host arrays."""
    lib = ex.lib
    vp = ctypes.c_void_p
    lib.spslam_debug_libm64.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_int, vp]
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(a if b is None else b, np.float64)
    out = np.zeros_like(a)
    ex._check(lib.spslam_debug_libm64(ex.ctx, int(kind), a.ctypes.data, b.ctypes.data, len(a), out.ctypes.data))
    return out


def pose_optimize(ex: OrbExtractor, problem, points, planes, cfg: PlaneConfig | None = None):
    """Optimizer::PoseOptimization drop-in on host arrays (one frame).

    Returns (result record, point outlier flags, plane outlier flags)."""
    _bind_pose(ex.lib)
    cfg = cfg or PlaneConfig.tum()
    problem = np.ascontiguousarray(problem, POSE_PROBLEM_DTYPE).reshape(())
    points = np.ascontiguousarray(points, POINT_OBS_DTYPE)
    planes = np.ascontiguousarray(planes, PLANE_OBS_DTYPE)
    res = np.zeros((), POSE_RESULT_DTYPE)
    po = np.zeros(max(len(points), 1), np.uint8)
    plo = np.zeros(max(len(planes), 1), np.uint8)
    ex._check(ex.lib.spslam_pose_optimize(ex.ctx, problem.ctypes.data, points.ctypes.data if len(points) else None,
                                          planes.ctypes.data if len(planes) else None, ctypes.byref(cfg),
                                          res.ctypes.data, po.ctypes.data, plo.ctypes.data))
    return res, po[:len(points)].astype(bool), plo[:len(planes)].astype(bool)


def pose_optimize_batch_device(ex: OrbExtractor, n, problems_ptr, points_ptr, planes_ptr, results_ptr,
                               pout_ptr, plout_ptr, init_from_ptr=0, cfg: PlaneConfig | None = None, stream=0):
    _bind_pose(ex.lib)
    cfg = cfg or PlaneConfig.tum()
    ex._check(ex.lib.spslam_pose_optimize_batch_device(ex.ctx, n, problems_ptr, points_ptr, planes_ptr,
                                                       ctypes.byref(cfg), init_from_ptr or None, results_ptr,
                                                       pout_ptr, plout_ptr, stream or None))
