"""ctypes binding of the plane-extraction part of include/spslam_gpu.h
(Frame::ComputePlanesFromOrganizedPointCloud on gfx950)."""
from __future__ import annotations

import ctypes

import numpy as np

import spslam_gpu

PLANE_DTYPE = np.dtype([("coef", "<f4", 4), ("n_inliers", "<i4"), ("inlier_offset", "<i4"), ("n_contour", "<i4"),
                        ("contour_offset", "<i4")])
assert PLANE_DTYPE.itemsize == 32


class PlaneParams(ctypes.Structure):
    _fields_ = [("cloud_dis", ctypes.c_int), ("min_size", ctypes.c_int), ("angle_threshold", ctypes.c_float),
                ("distance_threshold", ctypes.c_float), ("fx", ctypes.c_float), ("fy", ctypes.c_float),
                ("cx", ctypes.c_float), ("cy", ctypes.c_float), ("width", ctypes.c_int), ("height", ctypes.c_int)]


spslam_gpu.EXPORTED += ["spslam_planes_configure", "spslam_planes_capacity", "spslam_planes_extract",
                        "spslam_planes_extract_batch_device", "spslam_planes_debug"]


def _bind(lib):
    vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
    lib.spslam_planes_configure.argtypes = [vp, ctypes.POINTER(PlaneParams)]
    lib.spslam_planes_capacity.argtypes = [vp, ip, ip, ip]
    lib.spslam_planes_extract.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ip, vp,
                                          vp]
    lib.spslam_planes_extract_batch_device.argtypes = [vp, vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, vp, vp,
                                                       vp, vp, vp]
    lib.spslam_planes_debug.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ip]


class PlaneExtractor:
    """GPU Frame::ComputePlanesFromOrganizedPointCloud on a context (shares its stream/device)."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, fx, fy, cx, cy, width=640, height=480, cloud_dis=3,
                 min_size=500, angle_threshold=3.0, distance_threshold=0.05):
        self.ex = ex
        _bind(ex.lib)
        self.params = PlaneParams(cloud_dis, min_size, angle_threshold, distance_threshold, fx, fy, cx, cy, width,
                                  height)
        ex._check(ex.lib.spslam_planes_configure(ex.ctx, ctypes.byref(self.params)))
        pc, ic, cc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        ex._check(ex.lib.spslam_planes_capacity(ex.ctx, ctypes.byref(pc), ctypes.byref(ic), ctypes.byref(cc)))
        self.planes_cap, self.inlier_cap, self.contour_cap = pc.value, ic.value, cc.value
        self.W = -(-width // cloud_dis)
        self.H = -(-height // cloud_dis)

    def configure(self, **kw):
        """Change Plane.* parameters (min_size, angle_threshold, distance_threshold, ...) in place."""
        for k, v in kw.items():
            setattr(self.params, k, v)
        self.ex._check(self.ex.lib.spslam_planes_configure(self.ex.ctx, ctypes.byref(self.params)))

    def __call__(self, depth_f32: np.ndarray):
        """Returns dict(coef=[...], inliers=[...], contour=[...]) like the oracle."""
        d = np.ascontiguousarray(depth_f32, np.float32)
        planes = np.zeros(self.planes_cap, PLANE_DTYPE)
        inl = np.zeros(self.inlier_cap, np.int32)
        con = np.zeros(self.contour_cap, np.int32)
        n = ctypes.c_int()
        self.ex._check(self.ex.lib.spslam_planes_extract(self.ex.ctx, d.ctypes.data, d.shape[1], d.shape[0],
                                                         d.shape[1], planes.ctypes.data, self.planes_cap,
                                                         ctypes.byref(n), inl.ctypes.data, con.ctypes.data))
        out = dict(coef=[], inliers=[], contour=[])
        for p in planes[:n.value]:
            out["coef"].append(p["coef"].copy())
            out["inliers"].append(inl[p["inlier_offset"]:p["inlier_offset"] + p["n_inliers"]].copy())
            out["contour"].append(con[p["contour_offset"]:p["contour_offset"] + p["n_contour"]].copy())
        return out

    def extract_batch_device(self, depth_ptr, n_frames, frame_stride, stride, planes_ptr, counts_ptr, inliers_ptr,
                             contours_ptr, stream=0):
        self.ex._check(self.ex.lib.spslam_planes_extract_batch_device(
            self.ex.ctx, depth_ptr, n_frames, frame_stride, stride, planes_ptr, counts_ptr, inliers_ptr,
            contours_ptr, stream or None))

    def debug(self, frame, what):
        N = self.W * self.H
        shape, dt = {0: ((N, 3), np.float32), 1: ((N, 3), np.float32), 2: (N, np.float32), 3: (N, np.uint32)}[what]
        out = np.zeros(shape, dt)
        n = ctypes.c_int()
        self.ex._check(self.ex.lib.spslam_planes_debug(self.ex.ctx, frame, what, out.ctypes.data, ctypes.byref(n)))
        return out
