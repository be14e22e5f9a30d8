"""ctypes binding of the tracking-graph part of include/spslam_gpu.h
(spslam_track_graph_batch_device: TrackWithMotionModel / TrackLocalMap's
bookkeeping between matching and Optimizer::PoseOptimization,
src/Tracking.cc:951-1000, 1055-1068; src/Optimizer.cc:561-640, 681-860;
spslam_track_refkf_batch_device + spslam_masked_frame_copy_device: the
motion model's failure test and the TrackReferenceKeyFrame switch,
src/Tracking.cc:318-324, 791-882; spslam_track_refkf_vote_batch_device: the
reference keyframe, UpdateLocalKeyFrames' pKFmax, :1459-1570)."""
from __future__ import annotations

import ctypes

import spslam_gpu

MOTION_MODEL, DISCARD, LOCAL_MAP, MOTION_PRIOR, LAST_FRAME = 0, 1, 2, 3, 4
REFKF_PREPARE, REFKF_SELECT = 0, 1

spslam_gpu.EXPORTED += ["spslam_track_graph_batch_device", "spslam_track_refkf_batch_device",
                        "spslam_track_refkf_vote_batch_device", "spslam_masked_frame_copy_device"]

_P = ctypes.c_void_p


class TrackBatch(ctypes.Structure):
    """struct spslam_track_batch (device pointers as ints)."""
    _fields_ = [("keys_un", _P), ("uright", _P), ("kp_counts", _P), ("cap", ctypes.c_int32),
                ("proj_frames", _P), ("proj_points", _P), ("proj_match", _P),
                ("local_frames", _P), ("local_points", _P), ("local_match", _P), ("taken", _P),
                ("planes_a", _P), ("planes_b", _P), ("count_a", _P), ("count_b", _P),
                ("stride_a", ctypes.c_int32), ("stride_b", ctypes.c_int32), ("cap_a", ctypes.c_int32),
                ("cap_b", ctypes.c_int32),
                ("map", _P), ("assoc_match", _P), ("assoc_parallel", _P), ("assoc_vertical", _P),
                ("assoc_frames_next", _P), ("plane_outlier", _P), ("next_match", _P), ("next_parallel", _P),
                ("next_vertical", _P), ("assoc_frames_first", _P), ("seen", _P), ("next_frames", _P),
                ("next_points", _P), ("velocity", _P), ("point_outlier_local", _P),
                ("problems", _P), ("points", _P), ("planes", _P), ("edge_of_kp", _P), ("results", _P),
                ("point_outlier", _P),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("bf", ctypes.c_float), ("pad", ctypes.c_int32)]


class RefkfBatch(ctypes.Structure):
    """struct spslam_refkf_batch (device pointers as ints)."""
    _fields_ = [("nmatches", _P), ("fallback", _P), ("refkf_counts", _P), ("bow_nmatches", _P), ("bow_match", _P),
                ("refkf_rows", _P), ("refkf_index", _P), ("rows_stride", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("refkf_sets", _P), ("assoc_frames", _P), ("apply", _P), ("state", _P), ("refkf_match", _P),
                ("refkf_frames", _P), ("refkf_assoc", _P)]


class RefkfVote(ctypes.Structure):
    """struct spslam_refkf_vote (device pointers as ints)."""
    _fields_ = [("kf_base", _P), ("kf_sets", _P), ("ids_per_kf", ctypes.c_int32), ("n_kf", ctypes.c_int32),
                ("new_kf", ctypes.c_int32), ("pad", ctypes.c_int32), ("state", _P), ("refkf_index", _P),
                ("refkf_sets", _P), ("refkf_pairs", _P)]


class FrameRegion(ctypes.Structure):
    """struct spslam_frame_region."""
    _fields_ = [("dst", _P), ("src", _P), ("frame_bytes", ctypes.c_int64), ("dst_stride", ctypes.c_int64),
                ("src_stride", ctypes.c_int64)]


def _bind(lib):
    lib.spslam_track_graph_batch_device.argtypes = [_P, ctypes.c_int, ctypes.c_int, _P, _P]
    lib.spslam_track_refkf_batch_device.argtypes = [_P, ctypes.c_int, ctypes.c_int, _P, _P, _P]
    lib.spslam_masked_frame_copy_device.argtypes = [_P, ctypes.c_int, _P, ctypes.c_int, _P, _P]
    lib.spslam_track_refkf_vote_batch_device.argtypes = [_P, ctypes.c_int, _P, _P, _P]


class TrackGraph:
    """GPU tracking-graph bookkeeping on a context (its ORB tables give mvInvLevelSigma2)."""

    def __init__(self, ex: spslam_gpu.OrbExtractor):
        self.ex = ex
        _bind(ex.lib)

    def batch_device(self, n_frames: int, stage: int, batch: TrackBatch, stream=0):
        self.ex._check(self.ex.lib.spslam_track_graph_batch_device(self.ex.ctx, n_frames, stage,
                                                                    ctypes.byref(batch), stream or None))

    def refkf_device(self, n_frames: int, stage: int, mm: TrackBatch, rk: RefkfBatch, stream=0):
        self.ex._check(self.ex.lib.spslam_track_refkf_batch_device(self.ex.ctx, n_frames, stage, ctypes.byref(mm),
                                                                    ctypes.byref(rk), stream or None))

    def refkf_vote_device(self, n_frames: int, mm: TrackBatch, vote: RefkfVote, stream=0):
        self.ex._check(self.ex.lib.spslam_track_refkf_vote_batch_device(self.ex.ctx, n_frames, ctypes.byref(mm),
                                                                         ctypes.byref(vote), stream or None))

    def masked_copy_device(self, n_frames: int, flags: int, regions, stream=0):
        """regions: [(dst tensor, src tensor)] of n_frames equal rows each (contiguous, byte sizes multiple of 4)."""
        arr = (FrameRegion * len(regions))()
        for k, (d, sv) in enumerate(regions):
            fb = d.numel() * d.element_size() // n_frames
            assert d.is_contiguous() and sv.is_contiguous() and sv.numel() * sv.element_size() == fb * n_frames
            arr[k] = FrameRegion(d.data_ptr(), sv.data_ptr(), fb, fb, fb)
        self.ex._check(self.ex.lib.spslam_masked_frame_copy_device(self.ex.ctx, n_frames, flags, len(regions), arr,
                                                                    stream or None))
