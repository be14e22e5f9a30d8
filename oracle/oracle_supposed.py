"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/supposed_oracle.cpp (Frame::GeneratePlanesFromBoundries,
src/Frame.cc:938-1144, with PCL 1.8 SACSegmentation LINE/RANSAC).
"""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_ctypes

FLAG_FITTED, FLAG_IN_RANGE, FLAG_BORDER, FLAG_ADDED = 1, 2, 4, 8


def _lib():
    L = oracle_ctypes.lib()
    if getattr(L, "_supposed_bound", False):
        return L
    vp, ip, fp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_float
    L.oracle_supposed_new.restype = vp
    L.oracle_supposed_free.argtypes = [vp]
    L.oracle_supposed_generate.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, fp, fp, fp, fp,
                                           ctypes.c_int, vp, vp, vp, vp, ctypes.c_double, fp, vp]
    L.oracle_supposed_n_candidates.argtypes = [vp]
    L.oracle_supposed_candidate.argtypes = [vp, ctypes.c_int, vp, vp, vp, ctypes.c_int]
    L.oracle_supposed_plane.argtypes = [vp, ctypes.c_int, vp]
    L.oracle_supposed_patch.argtypes = [vp, vp, vp, vp, ctypes.c_int]
    L.oracle_supposed_coef.argtypes = [vp, vp, vp]
    L.oracle_segment_line.argtypes = [vp, ctypes.c_int, ctypes.c_double, vp, vp, vp]
    L._supposed_bound = True
    return L


def segment_line(xyz: np.ndarray, threshold=0.01):
    """pcl::SACSegmentation LINE/RANSAC/optimize on an (n, 3) float32 cloud."""
    L = _lib()
    p = np.ascontiguousarray(xyz, np.float32)
    coef = np.zeros(6, np.float32)
    inl = np.zeros(max(len(p), 1), np.int32)
    info = np.zeros(2, np.int64)
    n = L.oracle_segment_line(p.ctypes.data, len(p), threshold, coef.ctypes.data, inl.ctypes.data, info.ctypes.data)
    return dict(ok=n >= 0, coef=coef, inliers=inl[:max(n, 0)].copy(), iterations=int(info[0]), draws=int(info[1]))


def patch(src_coef, line6, coef):
    L = _lib()
    a, b, c = (np.ascontiguousarray(x, np.float32) for x in (src_coef, line6, coef))
    n = L.oracle_supposed_patch(a.ctypes.data, b.ctypes.data, c.ctypes.data, None, 0)
    out = np.zeros((n, 3), np.float32)
    L.oracle_supposed_patch(a.ctypes.data, b.ctypes.data, c.ctypes.data, out.ctypes.data, n)
    return out


def supposed_coef(src_coef, line6):
    """Frame::CaculatePlanes' plane through the line, perpendicular to the source plane (d >= 0)."""
    L = _lib()
    a, b = (np.ascontiguousarray(x, np.float32) for x in (src_coef, line6))
    out = np.zeros(4, np.float32)
    L.oracle_supposed_coef(a.ctypes.data, b.ctypes.data, out.ctypes.data)
    return out


def generate(depth_f32, cloud_xyz, coefs, contours, fx, fy, cx, cy, line_ratio=0.2, dis_th=0.01, bounds=None):
    """GeneratePlanesFromBoundries over planes given as coefficient rows + contour
    index lists.  Returns dict(coef=[...], line=[...], source=[...], line_idx=[...],
    candidates=[dict(plane, j, n_inliers, iterations, flags, line, cloud_idx)])."""
    L = _lib()
    h = L.oracle_supposed_new()
    try:
        d = np.ascontiguousarray(depth_f32, np.float32)
        cl = np.ascontiguousarray(cloud_xyz, np.float32)
        cf = np.ascontiguousarray(np.asarray(coefs, np.float32).reshape(-1, 4))
        n_pl = len(cf)
        con_n = np.array([len(c) for c in contours], np.int32)
        con_off = np.concatenate([[0], np.cumsum(con_n)[:-1]]).astype(np.int32) if n_pl else np.zeros(0, np.int32)
        con = np.ascontiguousarray(np.concatenate(contours).astype(np.int32)) if n_pl and con_n.sum() else \
            np.zeros(1, np.int32)
        bd = None if bounds is None else np.asarray(bounds, np.float32)
        n = L.oracle_supposed_generate(h, d.ctypes.data, d.shape[1], d.shape[0], d.shape[1], cl.ctypes.data, fx, fy,
                                       cx, cy, n_pl, cf.ctypes.data, con_off.ctypes.data, con_n.ctypes.data,
                                       con.ctypes.data, line_ratio, dis_th, None if bd is None else bd.ctypes.data)
        cands = []
        for k in range(L.oracle_supposed_n_candidates(h)):
            info = np.zeros(5, np.int32)
            line = np.zeros(6, np.float32)
            m = L.oracle_supposed_candidate(h, k, info.ctypes.data, line.ctypes.data, None, 0)
            idx = np.zeros(max(m, 1), np.int32)
            L.oracle_supposed_candidate(h, k, info.ctypes.data, line.ctypes.data, idx.ctypes.data, m)
            cands.append(dict(plane=int(info[0]), j=int(info[1]), n_inliers=int(info[2]), iterations=int(info[3]),
                              flags=int(info[4]), line=line, cloud_idx=idx[:m].copy()))
        out = dict(coef=[], line=[], source=[], line_idx=[], candidates=cands)
        for k in range(n):
            c = np.zeros(4, np.float32)
            ci = L.oracle_supposed_plane(h, k, c.ctypes.data)
            out["coef"].append(c)
            out["line"].append(cands[ci]["line"])
            out["source"].append(cands[ci]["plane"])
            out["line_idx"].append(cands[ci]["cloud_idx"])
        return out
    finally:
        L.oracle_supposed_free(h)
