"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/frame_oracle.cpp (RGB-D Frame: UndistortKeyPoints,
ComputeImageBounds, ComputeStereoFromRGBD, AssignFeaturesToGrid;
src/Frame.cc:130-181, 326-341, 480-564, 743-764)."""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_ctypes

N_CELLS = 64 * 48


def frame_rgbd(kxy, depth_f32, fx, fy, cx, cy, dist=(0, 0, 0, 0, 0), bf=40.0):
    L = oracle_ctypes.lib()
    vp = ctypes.c_void_p
    L.oracle_frame_rgbd.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [vp] * 7
    p = np.array([fx, fy, cx, cy, *dist, bf], np.float32)
    k = np.ascontiguousarray(kxy, np.float32).reshape(-1, 2)
    d = np.ascontiguousarray(depth_f32, np.float32)
    n = len(k)
    un = np.zeros((max(n, 1), 2), np.float32)
    dep = np.zeros(max(n, 1), np.float32)
    ur = np.zeros(max(n, 1), np.float32)
    cell = np.zeros(max(n, 1), np.int32)
    go = np.zeros(N_CELLS + 1, np.int32)
    gi = np.zeros(max(n, 1), np.int32)
    b = np.zeros(4, np.float32)
    L.oracle_frame_rgbd(p.ctypes.data, k.ctypes.data, n, d.ctypes.data, d.shape[1], d.shape[0], d.shape[1],
                        un.ctypes.data, dep.ctypes.data, ur.ctypes.data, cell.ctypes.data, go.ctypes.data,
                        gi.ctypes.data, b.ctypes.data)
    return dict(un=un[:n], depth=dep[:n], uright=ur[:n], cell=cell[:n], grid_off=go, grid_idx=gi[:go[-1]], bounds=b)
