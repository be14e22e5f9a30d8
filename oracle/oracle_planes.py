"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of the plane-extraction restatement in oracle/plane_oracle.cpp
(Frame::ComputePlanesFromOrganizedPointCloud + PCL 1.8 normals/segmentation).
"""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_ctypes


def depth_to_float(depth_u16: np.ndarray, factor: float = 5000.0) -> np.ndarray:
    """Tracking::GrabImageRGBD depth conversion (src/Tracking.cc:230-231):
    convertTo(CV_32F, 1.0f/DepthMapFactor) == float(u16) * float(1/factor)."""
    return depth_u16.astype(np.float32) * np.float32(np.float32(1.0) / np.float32(factor))


class PlaneOracle:
    def __init__(self):
        L = oracle_ctypes.lib()
        vp = ctypes.c_void_p
        L.oracle_planes_new.restype = vp
        L.oracle_planes_free.argtypes = [vp]
        L.oracle_planes_extract.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int] + \
            [ctypes.c_float] * 4 + [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float]
        L.oracle_planes_dims.argtypes = [vp] + [ctypes.POINTER(ctypes.c_int)] * 3
        for n in ("oracle_planes_cloud", "oracle_planes_normals", "oracle_planes_distance"):
            getattr(L, n).argtypes = [vp, vp]
        L.oracle_planes_labels.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_planes_model.argtypes = [vp, ctypes.c_int, vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.oracle_planes_model_inliers.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_planes_model_contour.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_planes_kept.argtypes = [vp, ctypes.c_int, vp]
        self.L = L
        self.h = L.oracle_planes_new()

    def __del__(self):
        try:
            self.L.oracle_planes_free(self.h)
        except Exception:
            pass

    def extract(self, depth_f32: np.ndarray, fx, fy, cx, cy, cloud_dis=3, min_size=500, angle_th=3.0,
                dist_th=0.05):
        d = np.ascontiguousarray(depth_f32, np.float32)
        n = self.L.oracle_planes_extract(self.h, d.ctypes.data, d.shape[1], d.shape[0], d.shape[1], fx, fy, cx, cy,
                                         cloud_dis, min_size, angle_th, dist_th)
        W, H, M = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.L.oracle_planes_dims(self.h, ctypes.byref(W), ctypes.byref(H), ctypes.byref(M))
        self.W, self.H, self.n_models = W.value, H.value, M.value
        out = dict(coef=[], model=[], inliers=[], contour=[])
        for k in range(n):
            c = np.zeros(4, np.float32)
            m = self.L.oracle_planes_kept(self.h, k, c.ctypes.data)
            out["coef"].append(c)
            out["model"].append(m)
            out["inliers"].append(self.model_inliers(m))
            out["contour"].append(self.model_contour(m))
        return out

    def _arr(self, fn, shape, dtype, *args):
        a = np.zeros(shape, dtype)
        fn(self.h, *args, a.ctypes.data)
        return a

    def cloud(self):
        return self._arr(self.L.oracle_planes_cloud, (self.H * self.W, 3), np.float32)

    def normals(self):
        return self._arr(self.L.oracle_planes_normals, (self.H * self.W, 3), np.float32)

    def distance(self):
        return self._arr(self.L.oracle_planes_distance, self.H * self.W, np.float32)

    def labels(self, refined: bool):
        return self._arr(self.L.oracle_planes_labels, self.H * self.W, np.uint32, int(refined))

    def model(self, i):
        c = np.zeros(4, np.float32)
        a, b = ctypes.c_int(), ctypes.c_int()
        self.L.oracle_planes_model(self.h, i, c.ctypes.data, ctypes.byref(a), ctypes.byref(b))
        return c, a.value, b.value

    def model_inliers(self, i):
        _, n, _ = self.model(i)
        return self._arr(self.L.oracle_planes_model_inliers, n, np.int32, i)

    def model_contour(self, i):
        _, _, n = self.model(i)
        return self._arr(self.L.oracle_planes_model_contour, n, np.int32, i)
