"""CPU checks of the plane-association oracle (oracle/assoc_oracle.cpp,
Map::AssociatePlanesByBoundary + PointDistanceFromPlane, src/Map.cc:196-359).

Parity anchors (the reference needs OpenCV + PCL and cannot be built here, and
its tests hold no fixtures for this path -- SURVEY.md §8c):
  * the float expressions (angle = pM . pW, |pM . p + d|) match what g++
    -O3 -march=native (the reference's flags) makes of the same source lines
    on this host, FMA contraction included;
  * an independent Python transcription of the decision loop (running
    distance / vertical / parallel thresholds, `continue` semantics) agrees
    with the oracle on the oracle's own angles and distances;
  * ground-truth semantics on synthetic rooms: a frame plane that is a noisy
    view of a map face is associated with a face lying in that plane."""
import ctypes
import pathlib
import subprocess

import numpy as np
import pytest

import oracle_assoc as OA
import synth

PROBE = r"""
#include <cmath>
#include <cstdlib>
using namespace std;
extern "C" float probe_angle(const float* pM, const float* pW) {
    float angle = pM[0] * pW[0] +
                  pM[1] * pW[1] +
                  pM[2] * pW[2];
    return angle;
}
extern "C" double probe_dist(const float* plane, const float* xyz, int n) {
    double res = 100;
    for (int i = 0; i < n; i++) {
        double dis = abs(plane[0] * xyz[3 * i] + plane[1] * xyz[3 * i + 1] + plane[2] * xyz[3 * i + 2] + plane[3]);
        if (dis < res) res = dis;
    }
    return res;
}
"""


def _map(rng, scene, **kw):
    mp, b = synth.map_planes(scene, rng, **kw)
    m = np.zeros(len(mp["world"]), OA.MAP_PLANE_DTYPE)
    for k, v in mp.items():
        m[k] = v
    return m, b


def test_float_expressions_match_gcc_march_native(tmp_path):
    if "fma" not in pathlib.Path("/proc/cpuinfo").read_text():
        pytest.skip("host CPU without FMA: -march=native does not contract")
    src = tmp_path / "probe.cpp"
    src.write_text(PROBE)
    so = tmp_path / "probe.so"
    subprocess.run(["g++", "-O3", "-march=native", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    L = ctypes.CDLL(str(so))
    vp = ctypes.c_void_p
    L.probe_angle.argtypes = [vp, vp]
    L.probe_angle.restype = ctypes.c_float
    L.probe_dist.argtypes = [vp, vp, ctypes.c_int]
    L.probe_dist.restype = ctypes.c_double
    rng = np.random.default_rng(11)
    sc = synth.Scene(2)
    m, b = _map(rng, sc)
    T = np.eye(4, dtype=np.float32)
    for trial in range(40):
        coefs = rng.normal(size=(4, 4)).astype(np.float32)
        coefs[:, :3] /= np.linalg.norm(coefs[:, :3], axis=1, keepdims=True)
        coefs[:, 3] = np.abs(coefs[:, 3])
        r = OA.associate(T, coefs, m, b, params=np.array([0.2, 0.0, 0.0, 2.0], np.float32))  # every pair measured
        for i in range(4):
            pM = np.ascontiguousarray(r["world"][i])
            for j in range(len(m)):
                pW = np.ascontiguousarray(m["world"][j])
                ang = L.probe_angle(pM.ctypes.data, pW.ctypes.data)
                assert OA_angle(pM, pW) == ang, (trial, i, j)
                pts = np.ascontiguousarray(b[m["boundary_offset"][j]:m["boundary_offset"][j] + m["n_boundary"][j]])
                d = L.probe_dist(pM.ctypes.data, pts.ctypes.data, len(pts))
                if ang != 0.0:  # angle_th 0: every pair with a nonzero angle is measured
                    assert r["dist"][i, j] == d, (trial, i, j)


def _decide(world, m, dist, P, init=None):
    """Independent transcription of the Map.cc:207-257 loop over precomputed distances; init = the
    frame's current associations (the reference only overwrites them)."""
    n = len(world)
    out = np.full((3, n), -1, np.int32)
    if init is not None:
        out[:] = np.stack([init["match"], init["parallel"], init["vertical"]])
    for i in range(n):
        ld, lv, lp = np.float32(P[0]), np.float32(P[2]), np.float32(P[3])
        for j in range(len(m)):
            a = OA_angle(world[i], m["world"][j])
            if a > P[1] or a < -P[1]:
                if dist[i, j] < ld:
                    ld = np.float32(dist[i, j])
                    out[0, i] = j
                    continue
            if -lv < a < lv:
                lv = np.float32(abs(a))
                out[2, i] = j
                continue
            if a > lp or a < -lp:
                lp = np.float32(abs(a))
                out[1, i] = j
    return out


def OA_angle(a, b):
    """fma(a2, b2, fma(a0, b0, a1*b1)) in float: products are exact in double, and
    one double add of an exact product and a float rounds at most once before the
    float rounding (checked against the oracle below)."""
    f = np.float32
    t = f(np.float64(a[1]) * np.float64(b[1]))
    t = f(np.float64(a[0]) * np.float64(b[0]) + np.float64(t))
    return f(np.float64(a[2]) * np.float64(b[2]) + np.float64(t))


def test_decision_loop_matches_transcription():
    rng = np.random.default_rng(3)
    for seq in range(3):
        sc = synth.Scene(seq, n_boxes=3)
        m, b = _map(rng, sc)
        for fr in range(0, 120, 15):
            T, c, _ = synth.assoc_frame_planes(sc, fr, rng)
            r = OA.associate(T, c, m, b)
            got = np.stack([r["match"], r["parallel"], r["vertical"]])
            assert np.array_equal(got, _decide(r["world"], m, r["dist"], OA.ASSOC_PARAMS)), (seq, fr)
            assert r["new_plane"] == bool((r["match"] < 0).any())
            # a carried call (TrackLocalMap's) at a shifted pose keeps what it does not overwrite
            init = {k: rng.integers(-1, len(m), len(c)).astype(np.int32) for k in ("match", "parallel", "vertical")}
            T2 = T.copy()
            T2[:3, 3] += np.float32(0.1)
            r2 = OA.associate(T2, c, m, b, init=init)
            got = np.stack([r2["match"], r2["parallel"], r2["vertical"]])
            assert np.array_equal(got, _decide(r2["world"], m, r2["dist"], OA.ASSOC_PARAMS, init)), (seq, fr)
            assert r2["new_plane"] == bool((r2["match"] < 0).any())


def test_ground_truth_association():
    rng = np.random.default_rng(5)
    sc = synth.Scene(1, n_boxes=2)
    m, b = _map(rng, sc, coef_noise_deg=0.2, coef_noise_d=0.005)
    hits = total = 0
    for fr in range(0, 150, 10):
        T, c, src = synth.assoc_frame_planes(sc, fr, rng, far_frac=0.0, noise_deg=0.5, noise_d=0.01, n_random=0)
        r = OA.associate(T, c, m, b)
        for i, f in enumerate(src):
            total += 1
            j = r["match"][i]
            if j < 0:
                continue
            # the matched map plane lies in the same world plane as the source face
            pf, pj = synth.face_plane(sc.faces[f]), synth.face_plane(sc.faces[j])
            hits += abs(abs(pf[:3] @ pj[:3]) - 1) < 1e-6 and abs(abs(pf[3]) - abs(pj[3])) < 0.05
    assert hits >= 0.9 * total, (hits, total)


def test_empty_inputs():
    rng = np.random.default_rng(0)
    m, b = _map(rng, synth.Scene(0, n_boxes=0))
    T = np.eye(4, dtype=np.float32)
    r = OA.associate(T, np.zeros((0, 4), np.float32), m, b)
    assert len(r["match"]) == 0 and not r["new_plane"]
    c = np.array([[0, 1, 0, 1.3]], np.float32)
    r = OA.associate(T, c, m[:0], b[:0])
    assert r["match"][0] == -1 and r["new_plane"]
    # a map plane without boundary points never matches (distance stays 100)
    m2 = m.copy()
    m2["n_boundary"] = 0
    r = OA.associate(T, c, m2, b)
    assert r["match"][0] == -1 and (r["dist"][0][r["dist"][0] >= 0] == 100.0).all()
