"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/liboracle.so, the CPU restatement of the reference
hot path.  Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg (as the checker / CPU baseline, never as the product).
Parity status: unpinned against the reference binary -- see orb_oracle.h.
"""
from __future__ import annotations

import contextlib
import ctypes
import pathlib

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = ctypes.CDLL(str(LIB_PATH))
        vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
        L.oracle_orb_new.restype = vp
        L.oracle_orb_new.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_orb_free.argtypes = [vp]
        for name in ("oracle_orb_features_per_level", "oracle_orb_umax"):
            getattr(L, name).argtypes = [vp, ip]
        L.oracle_orb_scale_tables.argtypes = [vp] + [ctypes.POINTER(ctypes.c_float)] * 4
        L.oracle_orb_extract.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int, ip]
        L.oracle_orb_pyramid.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_orb_level_size.argtypes = [vp, ctypes.c_int, ip, ip]
        L.oracle_orb_level_image.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_orb_level_blurred.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_orb_level_candidates.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, ip]
        L.oracle_orb_level_keypoints.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, ip]
        L.oracle_resize_linear.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int]
        L.oracle_gaussian_blur.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
        L.oracle_fast.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ip]
        for name in ("oracle_fast_atan2",):
            getattr(L, name).restype = ctypes.c_float
            getattr(L, name).argtypes = [ctypes.c_float, ctypes.c_float]
        for name in ("oracle_sinf", "oracle_cosf"):
            getattr(L, name).restype = ctypes.c_float
            getattr(L, name).argtypes = [ctypes.c_float]
        L.oracle_descriptor.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                        ctypes.c_float, vp]
        _lib = L
    return _lib


class OrbOracle:
    """CPU restatement of ORB_SLAM2::ORBextractor (src/ORBextractor.cc)."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th_fast=20, min_th_fast=7):
        self.L = lib()
        self.h = self.L.oracle_orb_new(nfeatures, scale_factor, nlevels, ini_th_fast, min_th_fast)
        self.nlevels = nlevels

    def __del__(self):
        try:
            self.L.oracle_orb_free(self.h)
        except Exception:
            pass

    def features_per_level(self):
        out = (ctypes.c_int * self.nlevels)()
        self.L.oracle_orb_features_per_level(self.h, out)
        return np.array(out[:])

    def scale_tables(self):
        arrs = [(ctypes.c_float * self.nlevels)() for _ in range(4)]
        self.L.oracle_orb_scale_tables(self.h, *arrs)
        return [np.array(a[:]) for a in arrs]

    def umax(self):
        out = (ctypes.c_int * 16)()
        self.L.oracle_orb_umax(self.h, out)
        return np.array(out[:])

    def extract(self, gray: np.ndarray, cap: int = 8192):
        gray = np.ascontiguousarray(gray, np.uint8)
        h, w = gray.shape if gray.size else (0, 0)
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int()
        rc = self.L.oracle_orb_extract(self.h, gray.ctypes.data if gray.size else None, w, h, w, kps.ctypes.data,
                                       desc.ctypes.data, cap, ctypes.byref(n))
        assert rc == 0
        return kps[:n.value].copy(), desc[:n.value].copy()

    def pyramid(self, gray: np.ndarray):
        gray = np.ascontiguousarray(gray, np.uint8)
        self.L.oracle_orb_pyramid(self.h, gray.ctypes.data, gray.shape[1], gray.shape[0], gray.shape[1])

    def level_size(self, level):
        w, h = ctypes.c_int(), ctypes.c_int()
        self.L.oracle_orb_level_size(self.h, level, ctypes.byref(w), ctypes.byref(h))
        return w.value, h.value

    def level_image(self, level):
        w, h = self.level_size(level)
        out = np.zeros((h, w), np.uint8)
        self.L.oracle_orb_level_image(self.h, level, out.ctypes.data)
        return out

    def level_blurred(self, level):
        w, h = self.level_size(level)
        out = np.zeros((h, w), np.uint8)
        self.L.oracle_orb_level_blurred(self.h, level, out.ctypes.data)
        return out

    def _kps(self, fn, level, cap=1 << 20):
        out = np.zeros(cap, KEYPOINT_DTYPE)
        n = ctypes.c_int()
        assert fn(self.h, level, out.ctypes.data, cap, ctypes.byref(n)) == 0
        return out[:n.value].copy()

    def level_candidates(self, level):
        return self._kps(self.L.oracle_orb_level_candidates, level)

    def level_keypoints(self, level):
        return self._kps(self.L.oracle_orb_level_keypoints, level, 8192)


def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros((dh, dw), np.uint8)
    lib().oracle_resize_linear(src.ctypes.data, src.shape[1], src.shape[0], out.ctypes.data, dw, dh)
    return out


def gaussian_blur(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros_like(src)
    lib().oracle_gaussian_blur(src.ctypes.data, src.shape[1], src.shape[0], out.ctypes.data)
    return out


def fast(img: np.ndarray, thr: int, cap: int = 1 << 16):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros(cap, KEYPOINT_DTYPE)
    n = ctypes.c_int()
    assert lib().oracle_fast(img.ctypes.data, img.shape[1], img.shape[0], thr, out.ctypes.data, cap,
                             ctypes.byref(n)) == 0
    return out[:n.value].copy()


def fast_atan2(y: float, x: float) -> float:
    return lib().oracle_fast_atan2(y, x)


def sinf(x: float) -> float:
    return lib().oracle_sinf(x)


def cosf(x: float) -> float:
    return lib().oracle_cosf(x)


def descriptor(img: np.ndarray, x: float, y: float, angle: float) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros(32, np.uint8)
    lib().oracle_descriptor(img.ctypes.data, img.shape[1], img.shape[0], x, y, angle, out.ctypes.data)
    return out


LIBM_CR, LIBM_GLIBC = 0, 1


def libm_cr(kind: int, a, b=None):
    """The oracle's correctly rounded sin (0) / cos (1) / atan2(a, b) (2) / cube (3) (oracle/libm_cr_oracle.h)."""
    L = lib()
    L.oracle_libm_cr.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p]
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(a if b is None else b, np.float64)
    out = np.zeros_like(a)
    L.oracle_libm_cr(int(kind), a.ctypes.data, b.ctypes.data, len(a), out.ctypes.data)
    return out


@contextlib.contextmanager
def g2o_fma(on: bool = True):
    """FMA diagnostic mode of the pose / LBA oracle inside the block, for the calling thread: the same restatement
    compiled with GCC's FP contraction (oracle/Makefile FMA_FLAGS), the arithmetic a -march=native build of the
    reference's g2o gets (Thirdparty/g2o/CMakeLists.txt:57).  Off (default): the pinned uncontracted semantics."""
    L = lib()
    L.oracle_get_g2o_fma.restype = ctypes.c_int
    L.oracle_set_g2o_fma.argtypes = [ctypes.c_int]
    prev = L.oracle_get_g2o_fma()
    L.oracle_set_g2o_fma(int(bool(on)))
    try:
        yield
    finally:
        L.oracle_set_g2o_fma(prev)


@contextlib.contextmanager
def libm(mode: int):
    """Elementary functions of the pose / LBA oracle inside the block, for the calling thread
    (oracle/g2o_restated.h libm_mode): LIBM_CR (default: correctly rounded, the path's pinned semantics,
    DESIGN.md section 3.3) or LIBM_GLIBC (the host glibc's double sin / cos / atan2 / pow)."""
    L = lib()
    L.oracle_get_libm.restype = ctypes.c_int
    L.oracle_set_libm.argtypes = [ctypes.c_int]
    prev = L.oracle_get_libm()
    L.oracle_set_libm(int(mode))
    try:
        yield
    finally:
        L.oracle_set_libm(prev)


@contextlib.contextmanager
def solve_failures(trial_mask: int):
    """Inside the block (calling thread): bit q set = LM trial q's linear solve of every pose / LBA oracle call
    reports failure (oracle_set_solve_fail_mask; the device hook is spslam_debug_force_solve_failures)."""
    L = lib()
    L.oracle_get_solve_fail_mask.restype = ctypes.c_uint
    L.oracle_set_solve_fail_mask.argtypes = [ctypes.c_uint]
    prev = L.oracle_get_solve_fail_mask()
    L.oracle_set_solve_fail_mask(int(trial_mask))
    try:
        yield
    finally:
        L.oracle_set_solve_fail_mask(prev)


def pose_optimize(problem, points, planes, cfg=None):
    """Oracle Optimizer::PoseOptimization.  Same arrays/dtypes as spslam_gpu.pose_optimize."""
    import spslam_gpu as G  # dtypes/config only (no GPU call)
    L = lib()
    L.oracle_pose_optimize.argtypes = [ctypes.c_void_p] * 7
    cfg = cfg or G.PlaneConfig.tum()
    problem = np.ascontiguousarray(problem, G.POSE_PROBLEM_DTYPE).reshape(())
    points = np.ascontiguousarray(points, G.POINT_OBS_DTYPE)
    planes = np.ascontiguousarray(planes, G.PLANE_OBS_DTYPE)
    res = np.zeros((), G.POSE_RESULT_DTYPE)
    po = np.zeros(max(len(points), 1), np.uint8)
    plo = np.zeros(max(len(planes), 1), np.uint8)
    L.oracle_pose_optimize(problem.ctypes.data, points.ctypes.data, planes.ctypes.data, ctypes.addressof(cfg),
                           res.ctypes.data, po.ctypes.data, plo.ctypes.data)
    return res, po[:len(points)].astype(bool), plo[:len(planes)].astype(bool)
