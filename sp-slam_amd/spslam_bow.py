"""ctypes binding of the bag-of-words part of include/spslam_gpu.h: DBoW2
TemplatedVocabulary::loadFromTextFile / transform (Frame::ComputeBoW,
src/Frame.cc:495-502) and ORBmatcher::SearchByBoW (src/ORBmatcher.cc:159-288)
on gfx950."""
from __future__ import annotations

import ctypes
import gzip
import pathlib

import numpy as np

import spslam_gpu

spslam_gpu.EXPORTED += ["spslam_bow_load_vocabulary", "spslam_bow_transform", "spslam_bow_transform_batch_device",
                        "spslam_search_by_bow", "spslam_search_by_bow_batch_device"]

_P = ctypes.c_void_p
VOCAB = pathlib.Path(__file__).resolve().parents[1] / "tests" / "golden" / "vocab_k6_l6.txt.gz"


class BowParams(ctypes.Structure):
    _fields_ = [("nn_ratio", ctypes.c_float), ("check_orientation", ctypes.c_int32)]


class BowSide(ctypes.Structure):
    """struct spslam_bow_side (device pointers as ints)."""
    _fields_ = [("desc", _P), ("keys", _P), ("has_point", _P), ("counts", _P), ("fv_nodes", _P), ("fv_start", _P),
                ("fv_features", _P), ("n_fv", _P), ("cap", ctypes.c_int32), ("pad", ctypes.c_int32)]


def read_vocabulary_text(path=VOCAB) -> bytes:
    path = pathlib.Path(path)
    return gzip.open(path, "rb").read() if path.suffix == ".gz" else path.read_bytes()


def _bind(lib):
    ci, ip = ctypes.c_int, ctypes.POINTER(ctypes.c_int)
    lib.spslam_bow_load_vocabulary.argtypes = [_P, ctypes.c_char_p, ctypes.c_size_t, ip, ip, ip, ip]
    lib.spslam_bow_transform.argtypes = [_P, _P, ci, ci, _P, _P, ip, _P, _P, _P, ip]
    lib.spslam_bow_transform_batch_device.argtypes = [_P, ci, _P, _P, ci, ci, _P, _P, _P, _P, _P, _P, _P, _P]
    lib.spslam_search_by_bow.argtypes = [_P, _P, _P, _P, ci, _P, _P, _P, ci, _P, _P, ci, _P, _P, _P, ci,
                                         ctypes.POINTER(BowParams), _P, ip]
    lib.spslam_search_by_bow_batch_device.argtypes = [_P, ci, _P, ctypes.POINTER(BowSide), ctypes.POINTER(BowSide),
                                                      ctypes.POINTER(BowParams), _P, _P, _P]


class Vocabulary:
    """A DBoW2 vocabulary loaded into a context's HBM."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, text: bytes | None = None):
        self.ex = ex
        _bind(ex.lib)
        text = read_vocabulary_text() if text is None else text
        k, L, nn, nw = (ctypes.c_int() for _ in range(4))
        ex._check(ex.lib.spslam_bow_load_vocabulary(ex.ctx, text, len(text), ctypes.byref(k), ctypes.byref(L),
                                                    ctypes.byref(nn), ctypes.byref(nw)))
        self.k, self.L, self.n_nodes, self.n_words = k.value, L.value, nn.value, nw.value

    def transform(self, desc, levelsup=4):
        """Frame::ComputeBoW on host arrays: (BowVector words, values, FeatureVector nodes, starts, features)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        c = max(n, 1)
        bw, bv = np.zeros(c, np.uint32), np.zeros(c, np.float64)
        fn, fs, ff = np.zeros(c, np.uint32), np.zeros(c + 1, np.int32), np.zeros(c, np.int32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        self.ex._check(self.ex.lib.spslam_bow_transform(self.ex.ctx, d.ctypes.data if n else None, n, levelsup,
                                                        bw.ctypes.data, bv.ctypes.data, ctypes.byref(nb),
                                                        fn.ctypes.data, fs.ctypes.data, ff.ctypes.data,
                                                        ctypes.byref(nf)))
        b, f = nb.value, nf.value
        return dict(words=bw[:b], values=bv[:b], nodes=fn[:f], start=fs[:f + 1], features=ff[:fs[f]])

    def transform_batch_device(self, n_frames, d_desc, d_counts, cap, levelsup, d_words, d_values, d_n_bow, d_nodes,
                               d_start, d_features, d_n_fv, stream=0):
        self.ex._check(self.ex.lib.spslam_bow_transform_batch_device(
            self.ex.ctx, n_frames, d_desc, d_counts, cap, levelsup, d_words, d_values, d_n_bow, d_nodes, d_start,
            d_features, d_n_fv, stream or None))


def search_by_bow(ex: spslam_gpu.OrbExtractor, kf_desc, kf_keys, kf_has_point, kf_fv, f_desc, f_keys, f_fv,
                  nn_ratio=0.7, check_orientation=True):
    """ORBmatcher::SearchByBoW(KeyFrame*, Frame&) on host arrays; kf_fv / f_fv as Vocabulary.transform returns
    them.  Returns (match per frame feature: keyframe feature index or -1, nmatches)."""
    _bind(ex.lib)
    kd = np.ascontiguousarray(kf_desc, np.uint8).reshape(-1, 32)
    fd = np.ascontiguousarray(f_desc, np.uint8).reshape(-1, 32)
    kk = np.ascontiguousarray(kf_keys, spslam_gpu.KEYPOINT_DTYPE)
    fk = np.ascontiguousarray(f_keys, spslam_gpu.KEYPOINT_DTYPE)
    hp = np.ascontiguousarray(kf_has_point, np.uint8)
    arrs = [np.ascontiguousarray(kf_fv[k], t) for k, t in (("nodes", np.uint32), ("start", np.int32),
                                                           ("features", np.int32))]
    arrf = [np.ascontiguousarray(f_fv[k], t) for k, t in (("nodes", np.uint32), ("start", np.int32),
                                                          ("features", np.int32))]
    ptr = lambda a: a.ctypes.data if a.size else None  # noqa: E731
    match = np.zeros(max(len(fd), 1), np.int32)
    nm = ctypes.c_int()
    p = BowParams(nn_ratio, int(check_orientation))
    ex._check(ex.lib.spslam_search_by_bow(ex.ctx, ptr(kd), ptr(kk), ptr(hp), len(kd), ptr(arrs[0]), arrs[1].ctypes.data,
                                          ptr(arrs[2]), len(arrs[0]), ptr(fd), ptr(fk), len(fd), ptr(arrf[0]),
                                          arrf[1].ctypes.data, ptr(arrf[2]), len(arrf[0]), ctypes.byref(p),
                                          match.ctypes.data, ctypes.byref(nm)))
    return match[:len(fd)], nm.value


def search_by_bow_batch_device(ex: spslam_gpu.OrbExtractor, n_pairs, d_pairs, kf: BowSide, fr: BowSide, d_match,
                               d_nmatches, nn_ratio=0.7, check_orientation=True, stream=0):
    _bind(ex.lib)
    p = BowParams(nn_ratio, int(check_orientation))
    ex._check(ex.lib.spslam_search_by_bow_batch_device(ex.ctx, n_pairs, d_pairs, ctypes.byref(kf), ctypes.byref(fr),
                                                       ctypes.byref(p), d_match, d_nmatches, stream or None))
