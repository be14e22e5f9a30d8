"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/step_oracle.cpp: the benchmarked step's whole CPU
chain in C++ (GrabImageRGBD through the local-map PoseOptimization, the same
stages and parameters as oracle_step.run) and its timed multi-thread loop --
bench.py's cpu_baseline times this, so no Python runs between the stages.
Inputs are oracle_step.FrameInputs carrying the raw frame (rgb, depth_raw,
depth_scale)."""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_ctypes

vp = ctypes.c_void_p


class StepFrame(ctypes.Structure):
    _fields_ = [("rgb", vp), ("depth_raw", vp), ("w", ctypes.c_int32), ("h", ctypes.c_int32),
                ("depth_scale", ctypes.c_float), ("cam", ctypes.c_float * 5), ("geometry", vp), ("inv_sigma2", vp),
                ("proj_frame", vp), ("proj_points", vp), ("local_frame", vp), ("local_points", vp),
                ("map_planes", vp), ("n_map", ctypes.c_int32), ("min_size", ctypes.c_int32), ("boundary_xyz", vp),
                ("pose_cfg", vp), ("local_seen", ctypes.c_int32), ("supp_cap", ctypes.c_int32)]


class StepOut(ctypes.Structure):
    _fields_ = [("Tcw1", ctypes.c_float * 16), ("Tcw2", ctypes.c_float * 16), ("n_kps", ctypes.c_int32),
                ("n_planes", ctypes.c_int32), ("n_supposed", ctypes.c_int32), ("nmatches", ctypes.c_int32),
                ("local_nmatches", ctypes.c_int32), ("inliers1", ctypes.c_int32), ("inliers2", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


class LbaSet(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("lba_every", ctypes.c_int32), ("prob", vp), ("kfs", vp), ("pts", vp),
                ("pobs", vp), ("pls", vp), ("plobs", vp), ("cfg", vp)]


def _lib():
    L = oracle_ctypes.lib()
    if not getattr(L, "_step_bound", False):
        L.oracle_step_frame_run.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_step_bench.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp,
                                        vp, vp, ctypes.c_int]
        L._step_bound = True
    return L


class Frames:
    """C records of a list of FrameInputs (the numpy arrays they point at are kept alive here)."""

    def __init__(self, inputs, supp_cap=None):
        import spslam_gpu as G
        self.keep = []
        self.recs = (StepFrame * len(inputs))()
        for r, fi in zip(self.recs, inputs):
            a = lambda x, dt=None: self._arr(x, dt)  # noqa: E731
            rgb = a(fi.rgb, np.uint8)
            r.rgb, r.depth_raw = rgb.ctypes.data, a(fi.depth_raw, np.uint16).ctypes.data
            r.h, r.w = rgb.shape[:2]
            r.depth_scale = float(fi.depth_scale)
            r.cam[:] = [float(x) for x in fi.cam]
            r.geometry = a(fi.geometry, np.float32).ctypes.data
            r.inv_sigma2 = a(fi.inv_sigma2, np.float32).ctypes.data
            pfr, P = fi.proj
            lfr, LP = fi.local
            r.proj_frame, r.proj_points = a(pfr).ctypes.data, a(P).ctypes.data if len(P) else None
            r.local_frame, r.local_points = a(lfr).ctypes.data, a(LP).ctypes.data if len(LP) else None
            r.map_planes = a(fi.map_planes).ctypes.data if len(fi.map_planes) else None
            r.n_map = len(fi.map_planes)
            r.min_size = int(fi.min_size)
            r.boundary_xyz = a(fi.boundary, np.float32).ctypes.data if len(fi.boundary) else None
            cfg = fi.pose_cfg or G.PlaneConfig.tum()
            self.keep.append(cfg)
            r.pose_cfg = ctypes.addressof(cfg)
            r.local_seen = int(bool(fi.local_seen))
            r.supp_cap = -1 if supp_cap is None else int(supp_cap)

    def _arr(self, x, dt=None):
        x = np.ascontiguousarray(x if dt is None else np.asarray(x, dt))
        self.keep.append(x)
        return x


def run_frame(fi, nfeatures=1000, supp_cap=None):
    """One frame through the C++ chain: dict(Tcw1, Tcw2, n_kps, n_planes, n_supposed, nmatches, local_nmatches,
    inliers1, inliers2)."""
    fr = Frames([fi], supp_cap)
    o = StepOut()
    _lib().oracle_step_frame_run(ctypes.addressof(fr.recs[0]), nfeatures, ctypes.byref(o))
    return _out(o)


def _out(o):
    d = {k: getattr(o, k) for k, _ in StepOut._fields_ if k != "pad"}
    d["Tcw1"] = np.array(o.Tcw1, np.float32).reshape(4, 4)
    d["Tcw2"] = np.array(o.Tcw2, np.float32).reshape(4, 4)
    return d


def bench(inputs, nfeatures, warmup, timed, threads, supp_cap=None, lba=None, libm=0):
    """Timed loop (oracle_step_bench).  lba: (problems, lba_every, spslam_plane_config) with problems a list of
    synth.lba_problem tuples; libm: the workers' elementary functions (oracle_ctypes.LIBM_*).  Returns
    (per-thread timed seconds, thread 0's outputs per distinct frame)."""
    fr = Frames(inputs, supp_cap)
    n = len(inputs)
    outs = (StepOut * n)()
    el = np.zeros(threads, np.float64)
    ls = None
    if lba:
        probs, every, cfg = lba
        keep = []
        cols = []
        for j in range(6):
            arrs = [np.ascontiguousarray(p[j]) for p in probs]
            keep += arrs
            cols.append((vp * len(arrs))(*[x.ctypes.data if x.size else None for x in arrs]))
        keep.append(cfg)
        ls = LbaSet(len(probs), every, *[ctypes.addressof(c) for c in cols], ctypes.addressof(cfg))
        fr.keep += keep + cols
    rc = _lib().oracle_step_bench(ctypes.addressof(fr.recs), n, nfeatures, warmup, timed, threads,
                                  ctypes.byref(ls) if ls is not None else None, ctypes.addressof(outs),
                                  el.ctypes.data, int(libm))
    assert rc == 0
    return el, [_out(o) for o in outs]
