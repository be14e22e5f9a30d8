"""ctypes binding of the input-image part of include/spslam_gpu.h
(Tracking::GrabImageRGBD's cvtColor + depth convertTo, src/Tracking.cc:208-229, on gfx950)."""
from __future__ import annotations

import ctypes

import numpy as np

import spslam_gpu

spslam_gpu.EXPORTED += ["spslam_grab_rgbd", "spslam_grab_rgbd_batch_device", "spslam_grab_fuse_cloud"]


class GrabParams(ctypes.Structure):
    _fields_ = [("channels", ctypes.c_int32), ("rgb", ctypes.c_int32), ("depth_u16", ctypes.c_int32),
                ("depth_scale", ctypes.c_float)]


def _bind(lib):
    vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    lib.spslam_grab_rgbd.argtypes = [vp, vp, ci, vp, ci, ci, ci, vp, vp, vp]
    lib.spslam_grab_rgbd_batch_device.argtypes = [vp, ci, vp, sz, ci, vp, sz, ci, ci, ci, vp, vp, vp, vp]
    lib.spslam_grab_fuse_cloud.argtypes = [vp, ci]


class Grabber:
    """GPU GrabImageRGBD image preparation on a context.  depth_factor is the YAML DepthMapFactor
    (5000 for TUM); the conversion scale is its float reciprocal, as Tracking.cc:142-146 stores it."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, channels=3, rgb=True, depth_u16=True, depth_factor=5000.0):
        self.ex = ex
        _bind(ex.lib)
        f = np.float32(depth_factor)
        scale = np.float32(1.0) if abs(float(f)) < 1e-5 else np.float32(np.float32(1.0) / f)
        self.params = GrabParams(channels, int(bool(rgb)), int(bool(depth_u16)), float(scale))

    def __call__(self, color, depth):
        c = np.ascontiguousarray(color, np.uint8)
        h, w = c.shape[:2]
        d = np.ascontiguousarray(depth, np.uint16 if self.params.depth_u16 else np.float32)
        gray = np.zeros((h, w), np.uint8)
        z = np.zeros((h, w), np.float32)
        self.ex._check(self.ex.lib.spslam_grab_rgbd(self.ex.ctx, c.ctypes.data, w * self.params.channels,
                                                    d.ctypes.data, w, w, h, ctypes.byref(self.params),
                                                    gray.ctypes.data, z.ctypes.data))
        return gray, z

    def batch_device(self, n, d_color, color_frame_stride, color_stride, d_depth, depth_frame_stride, depth_stride,
                     w, h, d_gray, d_depth_out, stream=0):
        self.ex._check(self.ex.lib.spslam_grab_rgbd_batch_device(
            self.ex.ctx, n, d_color, color_frame_stride, color_stride, d_depth, depth_frame_stride, depth_stride,
            w, h, ctypes.byref(self.params), d_gray, d_depth_out, stream or None))

    def fuse_cloud(self, enable):
        """spslam_grab_fuse_cloud: batches on this context also make the plane stage's organized cloud."""
        self.ex._check(self.ex.lib.spslam_grab_fuse_cloud(self.ex.ctx, int(bool(enable))))
