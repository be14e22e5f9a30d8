"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/bow_oracle.cpp: DBoW2 TemplatedVocabulary::
loadFromTextFile / transform (Frame::ComputeBoW, src/Frame.cc:495-502) and
ORBmatcher::SearchByBoW (src/ORBmatcher.cc:159-288)."""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_ctypes

_P = ctypes.c_void_p


def _lib():
    L = oracle_ctypes.lib()
    ci, ip = ctypes.c_int, ctypes.POINTER(ctypes.c_int)
    L.oracle_bow_load.argtypes = [ctypes.c_char_p, ctypes.c_longlong, ip, ip, ip, ip]
    L.oracle_bow_load.restype = _P
    L.oracle_bow_free.argtypes = [_P]
    L.oracle_bow_words.argtypes = [_P, _P, ci, ci, _P, _P, _P]
    L.oracle_bow_transform.argtypes = [_P, _P, ci, ci, _P, _P, ip, _P, _P, _P, ip]
    L.oracle_bow_transform.restype = ci
    L.oracle_search_by_bow.argtypes = [_P, _P, _P, _P, _P, _P, ci, _P, _P, ci, _P, _P, _P, ci, ctypes.c_float, ci, _P]
    L.oracle_search_by_bow.restype = ci
    return L


class Vocabulary:
    def __init__(self, text: bytes):
        L = _lib()
        k, l_, nn, nw = (ctypes.c_int() for _ in range(4))
        self.h = L.oracle_bow_load(text, len(text), ctypes.byref(k), ctypes.byref(l_), ctypes.byref(nn),
                                   ctypes.byref(nw))
        if not self.h:
            raise ValueError("not a DBoW2 text vocabulary")
        self.k, self.L, self.n_nodes, self.n_words = k.value, l_.value, nn.value, nw.value

    def __del__(self):
        if getattr(self, "h", None):
            _lib().oracle_bow_free(self.h)

    def words(self, desc, levelsup=4):
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        w, wt, nid = np.zeros(n, np.uint32), np.zeros(n, np.float64), np.zeros(n, np.uint32)
        _lib().oracle_bow_words(self.h, d.ctypes.data, n, levelsup, w.ctypes.data, wt.ctypes.data, nid.ctypes.data)
        return w, wt, nid

    def transform(self, desc, levelsup=4):
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        c = max(n, 1)
        bw, bv = np.zeros(c, np.uint32), np.zeros(c, np.float64)
        fn, fs, ff = np.zeros(c, np.uint32), np.zeros(c + 1, np.int32), np.zeros(c, np.int32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        _lib().oracle_bow_transform(self.h, d.ctypes.data, n, levelsup, bw.ctypes.data, bv.ctypes.data,
                                    ctypes.byref(nb), fn.ctypes.data, fs.ctypes.data, ff.ctypes.data,
                                    ctypes.byref(nf))
        b, f = nb.value, nf.value
        return dict(words=bw[:b], values=bv[:b], nodes=fn[:f], start=fs[:f + 1], features=ff[:fs[f]])


def search_by_bow(kf_desc, kf_angle, kf_has_point, kf_fv, f_desc, f_angle, f_fv, nn_ratio=0.7,
                  check_orientation=True):
    """Returns (match per frame feature: keyframe feature index or -1, nmatches)."""
    kd = np.ascontiguousarray(kf_desc, np.uint8).reshape(-1, 32)
    fd = np.ascontiguousarray(f_desc, np.uint8).reshape(-1, 32)
    ka = np.ascontiguousarray(kf_angle, np.float32)
    fa = np.ascontiguousarray(f_angle, np.float32)
    hp = np.ascontiguousarray(kf_has_point, np.uint8)
    k = [np.ascontiguousarray(kf_fv[x], t) for x, t in (("nodes", np.uint32), ("start", np.int32),
                                                        ("features", np.int32))]
    f = [np.ascontiguousarray(f_fv[x], t) for x, t in (("nodes", np.uint32), ("start", np.int32),
                                                       ("features", np.int32))]
    match = np.zeros(max(len(fd), 1), np.int32)
    n = _lib().oracle_search_by_bow(kd.ctypes.data, ka.ctypes.data, hp.ctypes.data, k[0].ctypes.data,
                                    k[1].ctypes.data, k[2].ctypes.data, len(k[0]), fd.ctypes.data, fa.ctypes.data,
                                    len(fd), f[0].ctypes.data, f[1].ctypes.data, f[2].ctypes.data, len(f[0]),
                                    float(nn_ratio), int(check_orientation), match.ctypes.data)
    return match[:len(fd)], n
