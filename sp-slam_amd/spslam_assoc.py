"""ctypes binding of the plane-association part of include/spslam_gpu.h
(Map::AssociatePlanesByBoundary, src/Map.cc:196-359, on gfx950)."""
from __future__ import annotations

import ctypes

import numpy as np

import spslam_gpu

MAP_PLANE_DTYPE = np.dtype([("world", "<f4", 4), ("id", "<i4"), ("boundary_offset", "<i4"),
                            ("n_boundary", "<i4"), ("pad", "<i4")])
assert MAP_PLANE_DTYPE.itemsize == 32
ASSOC_FRAME_DTYPE = np.dtype([("Tcw", "<f4", 16), ("map_offset", "<i4"), ("n_map", "<i4"), ("carry", "<i4"),
                              ("pad", "<i4")])
assert ASSOC_FRAME_DTYPE.itemsize == 80


class AssocParams(ctypes.Structure):
    _fields_ = [("dis_th", ctypes.c_float), ("angle_th", ctypes.c_float), ("ver_th", ctypes.c_float),
                ("par_th", ctypes.c_float)]


# TUM1/2/3.yaml, ICL.yaml: Plane.AssociationDisRef, AssociationAngRef, VerticalThreshold, ParallelThreshold
DEFAULT_PARAMS = (0.2, 0.8, 0.08716, 0.9962)

spslam_gpu.EXPORTED += ["spslam_planes_associate", "spslam_planes_associate_batch_device"]


def _bind(lib):
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.spslam_planes_associate.argtypes = [vp, vp, vp, ci, vp, ci, vp, ci, vp, vp, vp, vp, vp]
    lib.spslam_planes_associate_batch_device.argtypes = [vp, ci, vp, vp, ci, vp, ci, vp, ci, vp, ci, vp, vp, ci, vp,
                                                         vp, vp, vp, vp, vp]


class PlaneAssociator:
    """GPU Map::AssociatePlanesByBoundary on a context (shares its device/stream)."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, params=DEFAULT_PARAMS):
        self.ex = ex
        _bind(ex.lib)
        self.params = AssocParams(*params)

    def __call__(self, Tcw, coefs, map_planes, boundary_xyz, init=None):
        """One frame against one map (map planes in id order).  Returns match /
        parallel / vertical map-plane indices (-1 = none) and mbNewPlane.  init: the
        frame's current associations (dict match / parallel / vertical) that the
        reference keeps where no candidate is found; None = a new Frame."""
        fr = np.zeros((), ASSOC_FRAME_DTYPE)
        fr["Tcw"] = np.asarray(Tcw, np.float32).reshape(16)
        c = np.ascontiguousarray(coefs, np.float32).reshape(-1, 4)
        m = np.ascontiguousarray(map_planes, MAP_PLANE_DTYPE)
        b = np.ascontiguousarray(boundary_xyz, np.float32).reshape(-1, 3)
        n = len(c)
        out = np.zeros((3, max(n, 1)), np.int32)
        if init is not None:
            fr["carry"] = 1
            for k, key in enumerate(("match", "parallel", "vertical")):
                out[k, :n] = init[key]
        new = ctypes.c_int(0)
        ptr = lambda a: a.ctypes.data if a.size else None  # noqa: E731
        self.ex._check(self.ex.lib.spslam_planes_associate(
            self.ex.ctx, fr.ctypes.data, ptr(c), n, ptr(m), len(m), ptr(b), len(b), ctypes.byref(self.params),
            out[0].ctypes.data, out[1].ctypes.data, out[2].ctypes.data, ctypes.byref(new)))
        return dict(match=out[0, :n], parallel=out[1, :n], vertical=out[2, :n], new_plane=bool(new.value))

    def batch_device(self, n_frames, d_frames, planes_a, stride_a, count_a, cap_a, planes_b, stride_b, count_b,
                     cap_b, d_map, d_boundary, max_map, d_match, d_parallel, d_vertical, d_new_plane, stream=0):
        self.ex._check(self.ex.lib.spslam_planes_associate_batch_device(
            self.ex.ctx, n_frames, d_frames, planes_a, stride_a, count_a, cap_a, planes_b, stride_b, count_b, cap_b,
            d_map, d_boundary, max_map, ctypes.byref(self.params), d_match, d_parallel, d_vertical, d_new_plane,
            stream or None))
