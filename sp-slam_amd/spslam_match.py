"""ctypes binding of the projection-matching part of include/spslam_gpu.h
(ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono),
src/ORBmatcher.cc:1328-1470, as TrackWithMotionModel calls it, on gfx950)."""
from __future__ import annotations

import ctypes

import numpy as np

import spslam_gpu

PROJ_POINT_DTYPE = np.dtype([("xw", "<f4", 3), ("angle", "<f4"), ("octave", "<i4"), ("n_obs", "<i4"),
                             ("last_index", "<i4"), ("id", "<i4"), ("desc", "u1", 32)])
assert PROJ_POINT_DTYPE.itemsize == 64
PROJ_FRAME_DTYPE = np.dtype([("Tcw", "<f4", 16), ("Tlw", "<f4", 16), ("point_offset", "<i4"), ("n_points", "<i4"),
                             ("pad", "<i4", 2)])
assert PROJ_FRAME_DTYPE.itemsize == 144


class MatchParams(ctypes.Structure):
    _fields_ = [("th", ctypes.c_float), ("mono", ctypes.c_int), ("check_orientation", ctypes.c_int),
                ("retry_below", ctypes.c_int)]


# Tracking::TrackWithMotionModel for RGB-D: th = 15, not mono, checkOri, retry below 20 matches
MOTION_MODEL = (15.0, 0, 1, 20)

spslam_gpu.EXPORTED += ["spslam_search_by_projection", "spslam_search_by_projection_batch_device"]


def _bind(lib):
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.spslam_search_by_projection.argtypes = [vp, vp, vp, vp, vp, vp, ci, vp, vp, vp, vp, vp]
    lib.spslam_search_by_projection_batch_device.argtypes = [vp, ci, vp, vp, ci, vp, vp, vp, vp, vp, vp, ci, vp, vp,
                                                             vp, vp]


class Matcher:
    """GPU SearchByProjection on a context configured with spslam_frame_configure."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, params=MOTION_MODEL):
        self.ex = ex
        _bind(ex.lib)
        self.params = MatchParams(*params)

    def __call__(self, frame, points, keys_un, desc, uright, grid_off, grid_idx):
        fr = np.ascontiguousarray(frame, PROJ_FRAME_DTYPE).reshape(())
        pts = np.ascontiguousarray(points, PROJ_POINT_DTYPE)
        k = np.ascontiguousarray(keys_un, spslam_gpu.KEYPOINT_DTYPE)
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        ur = np.ascontiguousarray(uright, np.float32)
        go = np.ascontiguousarray(grid_off, np.int32)
        gi = np.ascontiguousarray(grid_idx, np.int32)
        n = len(k)
        match = np.zeros(max(n, 1), np.int32)
        nm = ctypes.c_int(0)
        ptr = lambda a: a.ctypes.data if a.size else None  # noqa: E731
        self.ex._check(self.ex.lib.spslam_search_by_projection(
            self.ex.ctx, fr.ctypes.data, ptr(pts), ptr(k), ptr(d), ptr(ur), n, go.ctypes.data, ptr(gi),
            ctypes.byref(self.params), match.ctypes.data, ctypes.byref(nm)))
        return match[:n], nm.value

    def batch_device(self, n_frames, d_frames, d_points, max_points, d_keys_un, d_desc, d_uright, d_grid_off,
                     d_grid_idx, d_counts, cap, d_match, d_nmatches, stream=0):
        self.ex._check(self.ex.lib.spslam_search_by_projection_batch_device(
            self.ex.ctx, n_frames, d_frames, d_points, max_points, d_keys_un, d_desc, d_uright, d_grid_off,
            d_grid_idx, d_counts, cap, ctypes.byref(self.params), d_match, d_nmatches, stream or None))


LOCAL_POINT_DTYPE = np.dtype([("xw", "<f4", 3), ("normal", "<f4", 3), ("min_dist", "<f4"), ("max_dist", "<f4"),
                              ("id", "<i4"), ("n_obs", "<i4"), ("pad", "<i4", 2), ("desc", "u1", 32)])
assert LOCAL_POINT_DTYPE.itemsize == 80
LOCAL_FRAME_DTYPE = np.dtype([("Tcw", "<f4", 16), ("point_offset", "<i4"), ("n_points", "<i4"), ("seen_offset", "<i4"),
                              ("stamp", "<i4")])
assert LOCAL_FRAME_DTYPE.itemsize == 80


class LocalParams(ctypes.Structure):
    _fields_ = [("th", ctypes.c_float), ("nn_ratio", ctypes.c_float), ("view_cos_limit", ctypes.c_float),
                ("pad", ctypes.c_int)]


# Tracking::SearchLocalPoints for RGB-D: th = 3, ORBmatcher(0.8), isInFrustum(pMP, 0.5)
SEARCH_LOCAL = (3.0, 0.8, 0.5, 0)

spslam_gpu.EXPORTED += ["spslam_search_local_points", "spslam_search_local_points_batch_device"]


class LocalMatcher:
    """GPU Tracking::SearchLocalPoints on a context configured with spslam_frame_configure."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, params=SEARCH_LOCAL):
        self.ex = ex
        vp, ci = ctypes.c_void_p, ctypes.c_int
        ex.lib.spslam_search_local_points.argtypes = [vp, vp, vp, vp, vp, vp, ci, vp, vp, vp, vp, vp, vp, vp]
        ex.lib.spslam_search_local_points_batch_device.argtypes = [vp, ci, vp, vp, ci, vp, vp, vp, vp, vp, vp, ci,
                                                                   vp, vp, vp, vp, vp, vp, vp]
        self.params = LocalParams(*params)

    def __call__(self, frame, points, keys_un, desc, uright, grid_off, grid_idx, taken=None):
        fr = np.ascontiguousarray(frame, LOCAL_FRAME_DTYPE).reshape(())
        pts = np.ascontiguousarray(points, LOCAL_POINT_DTYPE)
        k = np.ascontiguousarray(keys_un, spslam_gpu.KEYPOINT_DTYPE)
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        ur = np.ascontiguousarray(uright, np.float32)
        go = np.ascontiguousarray(grid_off, np.int32)
        gi = np.ascontiguousarray(grid_idx, np.int32)
        tk = None if taken is None else np.ascontiguousarray(taken, np.uint8)
        n = len(k)
        match = np.zeros(max(n, 1), np.int32)
        inv = np.zeros(max(len(pts), 1), np.uint8)
        nm = ctypes.c_int(0)
        ptr = lambda a: a.ctypes.data if a is not None and a.size else None  # noqa: E731
        self.ex._check(self.ex.lib.spslam_search_local_points(
            self.ex.ctx, fr.ctypes.data, ptr(pts), ptr(k), ptr(d), ptr(ur), n, go.ctypes.data, ptr(gi), ptr(tk),
            ctypes.byref(self.params), match.ctypes.data, ctypes.byref(nm), inv.ctypes.data))
        return match[:n], nm.value, inv[:len(pts)].astype(bool)

    def batch_device(self, n_frames, d_frames, d_points, max_points, d_keys_un, d_desc, d_uright, d_grid_off,
                     d_grid_idx, d_counts, cap, d_taken, d_match, d_nmatches, d_in_view=0, stream=0, d_seen=0):
        self.ex._check(self.ex.lib.spslam_search_local_points_batch_device(
            self.ex.ctx, n_frames, d_frames, d_points, max_points, d_keys_un, d_desc, d_uright, d_grid_off,
            d_grid_idx, d_counts, cap, d_taken or None, ctypes.byref(self.params), d_match, d_nmatches,
            d_in_view or None, d_seen or None, stream or None))
