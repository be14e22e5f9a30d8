"""ctypes binding of the LocalBundleAdjustment part of include/spslam_gpu.h
(Optimizer::LocalBundleAdjustment on gfx950) and the numpy record types of
its flattened graph."""
from __future__ import annotations

import ctypes

import numpy as np

import spslam_gpu

LBA_KEYFRAME_DTYPE = np.dtype([("Tcw", "<f4", 16), ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"),
                               ("bf", "<f4"), ("id", "<i4"), ("fixed", "<i4"), ("pad", "<i4")])
LBA_POINT_DTYPE = np.dtype([("xw", "<f4", 3), ("id", "<i4"), ("obs_offset", "<i4"), ("n_obs", "<i4")])
LBA_POINT_OBS_DTYPE = np.dtype([("kf", "<i4"), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"), ("inv_sigma2", "<f4")])
LBA_PLANE_DTYPE = np.dtype([("world", "<f4", 4), ("id", "<i4"), ("obs_offset", "<i4"), ("n_obs", "<i4"),
                            ("pad", "<i4")])
LBA_PLANE_OBS_DTYPE = np.dtype([("kf", "<i4"), ("kind", "<i4"), ("meas", "<f4", 4)])
LBA_PROBLEM_DTYPE = np.dtype([("n_kf", "<i4"), ("n_points", "<i4"), ("n_planes", "<i4"), ("kf_offset", "<i4"),
                              ("point_offset", "<i4"), ("plane_offset", "<i4"), ("n_point_obs", "<i4"),
                              ("n_plane_obs", "<i4")])
LBA_RESULT_DTYPE = np.dtype([("iterations", "<i4", 2), ("n_point_outliers", "<i4"), ("n_plane_outliers", "<i4"),
                             ("status", "<i4"), ("trials", "<i4"), ("stopped", "<i4"), ("pad", "<i4"),
                             ("phase_us", "<f4", 8)])
assert LBA_KEYFRAME_DTYPE.itemsize == 96 and LBA_POINT_DTYPE.itemsize == 24
assert LBA_POINT_OBS_DTYPE.itemsize == 20 and LBA_PLANE_DTYPE.itemsize == 32
assert LBA_PLANE_OBS_DTYPE.itemsize == 24 and LBA_PROBLEM_DTYPE.itemsize == 32 and LBA_RESULT_DTYPE.itemsize == 64


spslam_gpu.EXPORTED += ["spslam_lba_optimize", "spslam_lba_optimize_batch_device", "spslam_lba_debug_stop_after",
                        "spslam_lba_set_order", "spslam_lba_set_team"]
G2O_ORDER, FAST_ORDER = 0, 1  # SPSLAM_LBA_G2O_ORDER (default, bit-exact to the oracle) / SPSLAM_LBA_FAST_ORDER

PLANE_CONFIG = np.array([1.0, 100.0, 0.5, 0.5, 1000.0, 200.0], np.float64)  # ICL.yaml Plane.* keys (Chi 1000, VPChi 200)


def _bind(lib):
    vp = ctypes.c_void_p
    lib.spslam_lba_optimize.argtypes = [vp] * 15
    lib.spslam_lba_optimize_batch_device.argtypes = [vp, ctypes.c_int] + [vp] * 16
    lib.spslam_lba_debug_stop_after.argtypes = [vp, ctypes.c_int]
    lib.spslam_lba_set_order.argtypes = [vp, ctypes.c_int]
    lib.spslam_lba_set_team.argtypes = [vp, ctypes.c_int]


def _addr(flag):
    if flag is None:
        return None
    if isinstance(flag, np.ndarray):
        assert flag.dtype == np.uint8 and flag.size >= 1
        return flag.ctypes.data
    return ctypes.addressof(flag)


class LocalBA:
    """GPU Optimizer::LocalBundleAdjustment on a context (shares its stream/device)."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, cfg=PLANE_CONFIG):
        self.ex = ex
        _bind(ex.lib)
        self.cfg = np.ascontiguousarray(cfg, np.float64)
        self.team = 0

    def __call__(self, prob, kfs, points, point_obs, planes, plane_obs, stop_flag=None):
        """stop_flag: pbStopFlag -- a one-byte buffer (ctypes.c_uint8 or numpy u8) another thread may set while
        the call runs (ctypes releases the GIL for the call)."""
        arrs = [np.ascontiguousarray(a) for a in (prob, kfs, points, point_obs, planes, plane_obs)]
        kf_out = np.zeros((max(len(kfs), 1), 16), np.float32)
        pt_out = np.zeros((max(len(points), 1), 3), np.float32)
        pl_out = np.zeros((max(len(planes), 1), 4), np.float32)
        po = np.zeros(max(len(point_obs), 1), np.uint8)
        plo = np.zeros(max(len(plane_obs), 1), np.uint8)
        res = np.zeros((), LBA_RESULT_DTYPE)
        ptr = lambda a: a.ctypes.data if a.size else None  # noqa: E731
        self.ex._check(self.ex.lib.spslam_lba_optimize(
            self.ex.ctx, *[ptr(a) for a in arrs], self.cfg.ctypes.data, kf_out.ctypes.data, pt_out.ctypes.data,
            pl_out.ctypes.data, po.ctypes.data, plo.ctypes.data, res.ctypes.data, _addr(stop_flag)))
        return dict(Tcw=kf_out[:len(kfs)], points=pt_out[:len(points)], planes=pl_out[:len(planes)],
                    point_outlier=po[:len(point_obs)], plane_outlier=plo[:len(plane_obs)], result=res)

    def set_order(self, order: int):
        """G2O_ORDER (default): g2o's summation order, bit-exact to the oracle; FAST_ORDER: the phase kernels."""
        self.ex._check(self.ex.lib.spslam_lba_set_order(self.ex.ctx, int(order)))

    def set_team(self, workgroups: int):
        """Workgroups per problem of the g2o-order launch (0 = fill the chip, at most 8); results do not depend on
        it."""
        self.ex._check(self.ex.lib.spslam_lba_set_team(self.ex.ctx, int(workgroups)))
        self.team = int(workgroups)

    def debug_stop_after(self, trials: int):
        """Test hook: the following calls see pbStopFlag raised after `trials` LM trials (-1 = off)."""
        self.ex._check(self.ex.lib.spslam_lba_debug_stop_after(self.ex.ctx, int(trials)))

    def batch_device(self, n, problems_host, d_problems, d_kfs, d_points, d_point_obs, d_planes, d_plane_obs,
                     d_kf_out, d_pt_out, d_pl_out, d_po, d_plo, d_res, stream=0, d_stop=None):
        ph = np.ascontiguousarray(problems_host)
        self.ex._check(self.ex.lib.spslam_lba_optimize_batch_device(
            self.ex.ctx, n, ph.ctypes.data, d_problems, d_kfs, d_points, d_point_obs, d_planes, d_plane_obs,
            self.cfg.ctypes.data, d_kf_out, d_pt_out, d_pl_out, d_po, d_plo, d_res, d_stop or None, stream or None))
