"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/lba_oracle.cpp (Optimizer::LocalBundleAdjustment,
src/Optimizer.cc:1154-1977)."""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_ctypes
import spslam_lba as L

PLANE_CONFIG = np.array([1.0, 100.0, 0.5, 0.5, 1000.0, 200.0], np.float64)  # ICL.yaml Plane.* keys (Chi 1000, VPChi 200)


def lba_optimize(prob, kfs, points, point_obs, planes, plane_obs, cfg=PLANE_CONFIG, stop_after=-1):
    """stop_after: pbStopFlag raised after that many LM trials (0 = set before the call, -1 = never)."""
    lib = oracle_ctypes.lib()
    vp = ctypes.c_void_p
    lib.oracle_lba_optimize_stop.argtypes = [vp] * 13 + [ctypes.c_int]
    arrs = [np.ascontiguousarray(a) for a in (prob, kfs, points, point_obs, planes, plane_obs)]
    c = np.ascontiguousarray(cfg, np.float64)
    kf_out = np.zeros((len(kfs), 16), np.float32)
    pt_out = np.zeros((max(len(points), 1), 3), np.float32)
    pl_out = np.zeros((max(len(planes), 1), 4), np.float32)
    po = np.zeros(max(len(point_obs), 1), np.uint8)
    plo = np.zeros(max(len(plane_obs), 1), np.uint8)
    res = np.zeros((), L.LBA_RESULT_DTYPE)
    lib.oracle_lba_optimize_stop(*[a.ctypes.data for a in arrs], c.ctypes.data, kf_out.ctypes.data,
                                 pt_out.ctypes.data, pl_out.ctypes.data, po.ctypes.data, plo.ctypes.data,
                                 res.ctypes.data, int(stop_after))
    return dict(Tcw=kf_out, points=pt_out[:len(points)], planes=pl_out[:len(planes)],
                point_outlier=po[:len(point_obs)], plane_outlier=plo[:len(plane_obs)], result=res)


def eigen_ldlt(A_upper_pattern, A, b):
    """Eigen SimplicialLDLT<Upper> restatement (oracle/eigen_simplicial_restated.h) on a dense matrix A whose
    structural upper pattern is the boolean matrix A_upper_pattern.  Returns (x, perm) or (None, perm) on a zero
    pivot."""
    lib = oracle_ctypes.lib()
    vp = ctypes.c_void_p
    lib.oracle_eigen_ldlt.argtypes = [ctypes.c_int] + [vp] * 6
    lib.oracle_eigen_ldlt.restype = ctypes.c_int
    n = A.shape[0]
    Ap, Ai, Ax = [0], [], []
    for c in range(n):
        for r in range(c + 1):
            if A_upper_pattern[r, c]:
                Ai.append(r)
                Ax.append(A[r, c])
        Ap.append(len(Ai))
    Ap = np.asarray(Ap, np.int32)
    Ai = np.asarray(Ai if Ai else [0], np.int32)
    Ax = np.asarray(Ax if Ax else [0.0], np.float64)
    b = np.ascontiguousarray(b, np.float64)
    x = np.zeros(n, np.float64)
    perm = np.zeros(n, np.int32)
    rc = lib.oracle_eigen_ldlt(n, Ap.ctypes.data, Ai.ctypes.data, Ax.ctypes.data, b.ctypes.data, x.ctypes.data,
                               perm.ctypes.data)
    return (None if rc else x), perm
