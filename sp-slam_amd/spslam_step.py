"""ctypes binding of the whole batched step (include/spslam_gpu.h "the whole batched step",
csrc/spslam_step.cpp): GrabImageRGBD -> ORB || planes -> tracking tail enqueued by the library on streams and
events it owns -- the throughput path a C / C++ caller drives with one call per step.  pipeline.HotPath(...,
native=True) drives it with the HotPath's own device buffers, so the two forms are compared buffer for buffer
(tests/test_gpu_pipeline.py::test_native_step_matches_python)."""
from __future__ import annotations

import ctypes

import spslam_assoc
import spslam_gpu
import spslam_grab
import spslam_match

vp = ctypes.c_void_p
spslam_gpu.EXPORTED += ["spslam_step_create", "spslam_step_buffers", "spslam_step_prime", "spslam_step_run",
                       "spslam_step_sync", "spslam_step_stream", "spslam_step_destroy"]


class StepConfig(ctypes.Structure):
    _fields_ = [("n_frames", ctypes.c_int32), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("kp_cap", ctypes.c_int32), ("pipelined", ctypes.c_int32), ("tail_priority", ctypes.c_int32),
                ("orb_priority", ctypes.c_int32), ("planes_priority", ctypes.c_int32),
                ("grab", spslam_grab.GrabParams), ("match", spslam_match.MatchParams),
                ("local", spslam_match.LocalParams), ("assoc", spslam_assoc.AssocParams),
                ("pose", spslam_gpu.PlaneConfig),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("bf", ctypes.c_float), ("pad", ctypes.c_int32)]


class StepFrames(ctypes.Structure):
    _fields_ = [("color", vp), ("color_frame_stride", ctypes.c_size_t), ("depth", vp),
                ("depth_frame_stride", ctypes.c_size_t), ("color_stride", ctypes.c_int32),
                ("depth_stride", ctypes.c_int32)]


class StepTracking(ctypes.Structure):
    _fields_ = [("proj_frames", vp), ("proj_points", vp), ("local_frames", vp), ("local_points", vp),
                ("assoc_frames1", vp), ("assoc_frames2", vp), ("map", vp), ("boundary_xyz", vp),
                ("max_proj_points", ctypes.c_int32), ("max_local_points", ctypes.c_int32),
                ("max_map", ctypes.c_int32), ("pad", ctypes.c_int32)]


SET_FIELDS = ("gray", "depth", "kps", "desc", "counts", "planes", "plane_counts", "inliers", "contours", "supposed",
              "supposed_counts", "lines", "patch")


class StepSet(ctypes.Structure):
    _fields_ = [(k, vp) for k in SET_FIELDS]


class StepTail(ctypes.Structure):
    _fields_ = [(k, vp) for k in ("keys_un", "mv_depth", "uright", "grid_off", "grid_idx", "match", "nmatches",
                                  "taken", "local_match", "local_nmatches", "edge_of_kp")] + \
               [("assoc", (vp * 3) * 2), ("new_plane", vp * 2), ("problems", vp * 2), ("points", vp * 2),
                ("planes", vp * 2), ("point_outlier", vp * 2), ("plane_outlier", vp * 2), ("results", vp * 2)]


def _bind(lib):
    if getattr(lib, "_step_bound", False):
        return
    lib.spslam_step_create.argtypes = [vp, ctypes.POINTER(StepConfig), ctypes.POINTER(StepSet),
                                       ctypes.POINTER(StepTail), ctypes.POINTER(vp)]
    lib.spslam_step_buffers.argtypes = [vp, ctypes.POINTER(StepSet), ctypes.POINTER(StepTail)]
    lib.spslam_step_prime.argtypes = [vp, ctypes.POINTER(StepFrames)]
    lib.spslam_step_run.argtypes = [vp, ctypes.POINTER(StepFrames), ctypes.POINTER(StepTracking)]
    lib.spslam_step_sync.argtypes = [vp]
    lib.spslam_step_stream.argtypes = [vp]
    lib.spslam_step_stream.restype = vp
    lib.spslam_step_destroy.argtypes = [vp]
    lib.spslam_step_destroy.restype = None
    lib._step_bound = True


class Step:
    """One step object on an OrbExtractor's context.  sets: two dicts of device pointers (SET_FIELDS), tail: a
    StepTail (0 members are allocated by the library)."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, cfg: StepConfig, sets=None, tail: StepTail | None = None):
        self.ex = ex
        _bind(ex.lib)
        arr = (StepSet * 2)()
        for j, d in enumerate(sets or ({}, {})):
            for k in SET_FIELDS:
                setattr(arr[j], k, d.get(k) or None)
        self.h = vp()
        self.ex._check(ex.lib.spslam_step_create(ex.ctx, ctypes.byref(cfg), arr, ctypes.byref(tail or StepTail()),
                                                 ctypes.byref(self.h)))

    def prime(self, frames: StepFrames):
        self.ex._check(self.ex.lib.spslam_step_prime(self.h, ctypes.byref(frames)))

    def run(self, frames: StepFrames, tracking: StepTracking):
        self.ex._check(self.ex.lib.spslam_step_run(self.h, ctypes.byref(frames), ctypes.byref(tracking)))

    def sync(self):
        self.ex._check(self.ex.lib.spslam_step_sync(self.h))

    def stream(self) -> int:
        return self.ex.lib.spslam_step_stream(self.h) or 0

    def close(self):
        if self.h:
            self.ex.lib.spslam_step_destroy(self.h)
            self.h = vp()
