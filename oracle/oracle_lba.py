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
