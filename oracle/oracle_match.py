"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/match_oracle.cpp (ORBmatcher::SearchByProjection
frame-to-frame + GetFeaturesInArea + DescriptorDistance + ComputeThreeMaxima,
src/ORBmatcher.cc:1328-1470,1601-1662, src/Frame.cc:427-480; the
TrackWithMotionModel retry, src/Tracking.cc:968-975)."""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_ctypes

PROJ_POINT_DTYPE = np.dtype([("xw", "<f4", 3), ("angle", "<f4"), ("octave", "<i4"), ("n_obs", "<i4"),
                             ("last_index", "<i4"), ("id", "<i4"), ("desc", "u1", 32)])
PROJ_FRAME_DTYPE = np.dtype([("Tcw", "<f4", 16), ("Tlw", "<f4", 16), ("point_offset", "<i4"), ("n_points", "<i4"),
                             ("pad", "<i4", 2)])
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                           ("octave", "<i4"), ("class_id", "<i4")])


def search_by_projection(frame, points, keys_un, desc, uright, grid_off, grid_idx, geometry,
                         params=(15.0, 0, 1, 20)):
    """geometry: fx fy cx cy bf min_x max_x min_y max_y ginv_x ginv_y scale[8].
    Returns (match per current keypoint, nmatches, passes)."""
    L = oracle_ctypes.lib()
    vp = ctypes.c_void_p
    L.oracle_search_by_projection.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int, vp, vp, vp, vp, vp, vp]
    L.oracle_search_by_projection.restype = ctypes.c_int
    fr = np.ascontiguousarray(frame, PROJ_FRAME_DTYPE).reshape(())
    pts = np.ascontiguousarray(points, PROJ_POINT_DTYPE)
    k = np.ascontiguousarray(keys_un, KEYPOINT_DTYPE)
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    ur = np.ascontiguousarray(uright, np.float32)
    go = np.ascontiguousarray(grid_off, np.int32)
    gi = np.ascontiguousarray(grid_idx, np.int32)
    g = np.ascontiguousarray(geometry, np.float32)
    assert g.size == 19
    prm = np.zeros(4, np.int32)
    prm[0:1] = np.array([params[0]], np.float32).view(np.int32)
    prm[1:] = params[1:]
    n = len(k)
    match = np.zeros(max(n, 1), np.int32)
    passes = ctypes.c_int(0)
    nm = L.oracle_search_by_projection(fr.ctypes.data, pts.ctypes.data if len(pts) else None, k.ctypes.data,
                                       d.ctypes.data, ur.ctypes.data, n, go.ctypes.data, gi.ctypes.data,
                                       g.ctypes.data, prm.ctypes.data, match.ctypes.data, ctypes.byref(passes))
    return match[:n], nm, passes.value


def descriptor_distance(a, b):
    """ORBmatcher::DescriptorDistance in numpy (popcount of the XOR, 256 bits)."""
    x = np.bitwise_xor(np.asarray(a, np.uint8), np.asarray(b, np.uint8))
    return int(np.unpackbits(x).sum())


LOCAL_POINT_DTYPE = np.dtype([("xw", "<f4", 3), ("normal", "<f4", 3), ("min_dist", "<f4"), ("max_dist", "<f4"),
                              ("id", "<i4"), ("n_obs", "<i4"), ("pad", "<i4", 2), ("desc", "u1", 32)])
LOCAL_FRAME_DTYPE = np.dtype([("Tcw", "<f4", 16), ("point_offset", "<i4"), ("n_points", "<i4"), ("seen_offset", "<i4"),
                              ("stamp", "<i4")])


def search_local_points(frame, points, keys_un, desc, uright, grid_off, grid_idx, geometry, taken=None,
                        params=(3.0, 0.8, 0.5), scale_factor=1.2, n_levels=8):
    """Tracking::SearchLocalPoints (isInFrustum + PredictScale + SearchByProjection(F, points, th)).
    Returns (match per current keypoint, nmatches, in_view per point)."""
    L = oracle_ctypes.lib()
    vp = ctypes.c_void_p
    L.oracle_search_local_points.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp]
    L.oracle_search_local_points.restype = ctypes.c_int
    fr = np.ascontiguousarray(frame, LOCAL_FRAME_DTYPE).reshape(())
    pts = np.ascontiguousarray(points, LOCAL_POINT_DTYPE)
    k = np.ascontiguousarray(keys_un, KEYPOINT_DTYPE)
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    ur = np.ascontiguousarray(uright, np.float32)
    go = np.ascontiguousarray(grid_off, np.int32)
    gi = np.ascontiguousarray(grid_idx, np.int32)
    g = np.ascontiguousarray(geometry, np.float32)
    libm = ctypes.CDLL("libm.so.6")
    libm.logf.restype, libm.logf.argtypes = ctypes.c_float, [ctypes.c_float]
    lsf = np.float32(libm.logf(np.float32(scale_factor)))  # Frame::mfLogScaleFactor = log(mfScaleFactor), glibc logf
    prm = np.zeros(8, np.int32)
    prm[:4] = np.array([params[0], params[1], params[2], lsf], np.float32).view(np.int32)
    prm[4] = n_levels
    tk = None if taken is None else np.ascontiguousarray(taken, np.uint8)
    n = len(k)
    match = np.zeros(max(n, 1), np.int32)
    inv = np.zeros(max(len(pts), 1), np.uint8)
    nm = L.oracle_search_local_points(fr.ctypes.data, pts.ctypes.data if len(pts) else None, k.ctypes.data,
                                      d.ctypes.data, ur.ctypes.data, n, go.ctypes.data, gi.ctypes.data,
                                      g.ctypes.data, prm.ctypes.data, tk.ctypes.data if tk is not None else None,
                                      match.ctypes.data, inv.ctypes.data)
    return match[:n], nm, inv[:len(pts)].astype(bool)
