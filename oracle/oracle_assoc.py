"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/assoc_oracle.cpp (Map::AssociatePlanesByBoundary +
PointDistanceFromPlane, src/Map.cc:196-359; Frame::ComputePlaneWorldCoeff,
src/Frame.cc:1146-1150)."""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_ctypes

MAP_PLANE_DTYPE = np.dtype([("world", "<f4", 4), ("id", "<i4"), ("boundary_offset", "<i4"),
                            ("n_boundary", "<i4"), ("pad", "<i4")])
# TUM1/2/3.yaml, ICL.yaml: Plane.AssociationDisRef, AssociationAngRef, VerticalThreshold, ParallelThreshold
ASSOC_PARAMS = np.array([0.2, 0.8, 0.08716, 0.9962], np.float32)


def associate(Tcw, coefs, map_planes, boundary_xyz, params=ASSOC_PARAMS, init=None):
    """One frame against one map (map planes in id order).  Returns match / parallel /
    vertical map-plane indices (-1 = none), world coefficients, the per-pair boundary
    distances (-1 where the angle test failed) and mbNewPlane.  init: the frame's
    current associations (dict of match / parallel / vertical), which the reference
    keeps wherever no candidate is found (src/Map.cc:230-252); None = a new Frame."""
    L = oracle_ctypes.lib()
    vp = ctypes.c_void_p
    L.oracle_planes_associate.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_int] + [vp] * 7 + [ctypes.c_int]
    L.oracle_planes_associate.restype = ctypes.c_int
    T = np.ascontiguousarray(Tcw, np.float32).reshape(16)
    c = np.ascontiguousarray(coefs, np.float32).reshape(-1, 4)
    m = np.ascontiguousarray(map_planes, MAP_PLANE_DTYPE)
    b = np.ascontiguousarray(boundary_xyz, np.float32).reshape(-1, 3)
    p = np.ascontiguousarray(params, np.float32)
    n, nm = len(c), len(m)
    match = np.zeros(max(n, 1), np.int32)
    par = np.zeros(max(n, 1), np.int32)
    ver = np.zeros(max(n, 1), np.int32)
    if init is not None:
        match[:n], par[:n], ver[:n] = init["match"], init["parallel"], init["vertical"]
    world = np.zeros((max(n, 1), 4), np.float32)
    dist = np.zeros((max(n, 1), max(nm, 1)), np.float64)
    new = L.oracle_planes_associate(T.ctypes.data, c.ctypes.data, n, m.ctypes.data if nm else None, nm,
                                    b.ctypes.data if len(b) else None, p.ctypes.data, match.ctypes.data,
                                    par.ctypes.data, ver.ctypes.data, world.ctypes.data, dist.ctypes.data,
                                    int(init is not None))
    return dict(match=match[:n], parallel=par[:n], vertical=ver[:n], world=world[:n], dist=dist[:n, :nm],
                new_plane=bool(new))
