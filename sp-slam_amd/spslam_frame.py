"""ctypes binding of the RGB-D Frame per-keypoint stage of include/spslam_gpu.h
(Frame::UndistortKeyPoints / ComputeStereoFromRGBD / AssignFeaturesToGrid on gfx950)."""
from __future__ import annotations

import ctypes

import numpy as np

import spslam_gpu

GRID_COLS, GRID_ROWS = 64, 48
N_CELLS = GRID_COLS * GRID_ROWS


class FrameParams(ctypes.Structure):
    _fields_ = [("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("dist", ctypes.c_float * 5), ("bf", ctypes.c_float), ("width", ctypes.c_int),
                ("height", ctypes.c_int)]


spslam_gpu.EXPORTED += ["spslam_frame_configure", "spslam_frame_rgbd", "spslam_frame_rgbd_batch_device"]


def _bind(lib):
    vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
    lib.spslam_frame_configure.argtypes = [vp, ctypes.POINTER(FrameParams), vp, vp]
    lib.spslam_frame_rgbd.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, vp,
                                      vp, vp]
    lib.spslam_frame_rgbd_batch_device.argtypes = [vp, vp, vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_size_t,
                                                   ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp]


class FrameStage:
    """GPU RGB-D Frame keypoint steps on a context (shares its stream/device)."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, fx, fy, cx, cy, dist=(0, 0, 0, 0, 0), bf=40.0, width=640,
                 height=480):
        self.ex = ex
        _bind(ex.lib)
        self.params = FrameParams(fx, fy, cx, cy, (ctypes.c_float * 5)(*dist), bf, width, height)
        b = np.zeros(4, np.float32)
        gi = np.zeros(2, np.float32)
        ex._check(ex.lib.spslam_frame_configure(ex.ctx, ctypes.byref(self.params), b.ctypes.data, gi.ctypes.data))
        self.bounds, self.grid_inv = b, gi

    def __call__(self, kps: np.ndarray, depth_f32: np.ndarray):
        """kps: spslam_keypoint records (mvKeys).  Returns dict(keys_un, depth, uright, grid_off, grid_idx)."""
        k = np.ascontiguousarray(kps).view(spslam_gpu.KEYPOINT_DTYPE)
        d = np.ascontiguousarray(depth_f32, np.float32)
        n = len(k)
        un = np.zeros(max(n, 1), spslam_gpu.KEYPOINT_DTYPE)
        dep = np.zeros(max(n, 1), np.float32)
        ur = np.zeros(max(n, 1), np.float32)
        go = np.zeros(N_CELLS + 1, np.int32)
        gi = np.zeros(max(n, 1), np.int32)
        self.ex._check(self.ex.lib.spslam_frame_rgbd(self.ex.ctx, k.ctypes.data if n else None, n, d.ctypes.data,
                                                     d.shape[1], d.shape[0], d.shape[1], un.ctypes.data,
                                                     dep.ctypes.data, ur.ctypes.data, go.ctypes.data, gi.ctypes.data))
        return dict(keys_un=un[:n], depth=dep[:n], uright=ur[:n], grid_off=go, grid_idx=gi[:go[-1]])

    def batch_device(self, kps_ptr, counts_ptr, cap, depth_ptr, n_frames, frame_stride, stride, keys_un_ptr,
                     depth_out_ptr, ur_ptr, grid_off_ptr, grid_idx_ptr, plane_counts_ptr=None, supp_counts_ptr=None,
                     stream=0):
        self.ex._check(self.ex.lib.spslam_frame_rgbd_batch_device(
            self.ex.ctx, kps_ptr, counts_ptr, cap, depth_ptr, n_frames, frame_stride, stride, keys_un_ptr,
            depth_out_ptr, ur_ptr, grid_off_ptr, grid_idx_ptr, plane_counts_ptr, supp_counts_ptr, stream or None))
