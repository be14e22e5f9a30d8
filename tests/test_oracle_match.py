"""CPU checks of the projection-matching oracle (oracle/match_oracle.cpp:
ORBmatcher::SearchByProjection frame-to-frame, src/ORBmatcher.cc:1328-1470,
with Frame::GetFeaturesInArea, DescriptorDistance, ComputeThreeMaxima and the
TrackWithMotionModel retry, src/Tracking.cc:968-975).

Anchors (the reference needs OpenCV and has no fixtures for this path,
SURVEY.md §8c): an independent pure-Python transcription of the reference's
loops agrees with the oracle on real synthetic frame pairs; the float
projection expressions match g++ -O3 -march=native on the same source lines;
ground-truth semantics (matches are the keypoints of the same scene points)."""
import ctypes
import pathlib
import subprocess

import numpy as np
import pytest

import oracle_ctypes
import oracle_frame
import oracle_match as OM
import synth

K = synth.TUM3


def _f(x):
    return np.float32(x)


def _fma(a, b, c):
    return _f(np.float64(_f(a)) * np.float64(_f(b)) + np.float64(_f(c)))


def _mat3(T, x, c=None, transpose=False, sign=1.0):
    T = np.asarray(T, np.float32).reshape(4, 4)
    out = []
    for r in range(3):
        s = 0.0
        for k in range(3):
            s += float(T[k, r] if transpose else T[r, k]) * float(x[k])
        s *= sign
        if c is not None:
            s += float(c[r])
        out.append(_f(s))
    return out


def py_search(fr, P, kun, desc, ur, go, gi, geo, th, mono=False, check_ori=True):
    """Transcription of ORBmatcher.cc:1328-1470 + Frame.cc:427-480 in Python."""
    fx, fy, cx, cy, bf, minx, maxx, miny, maxy, gix, giy = [_f(v) for v in geo[:11]]
    scale = [_f(v) for v in geo[11:]]
    n = len(kun)
    match, blocking = [-1] * n, [False] * n
    Tcw, Tlw = fr["Tcw"].reshape(4, 4), fr["Tlw"].reshape(4, 4)
    tcw, tlw = Tcw[:3, 3], Tlw[:3, 3]
    twc = _mat3(Tcw, tcw, transpose=True, sign=-1.0)
    tlc = _mat3(Tlw, twc, c=tlw)
    mb = _f(bf / fx)
    fwd = tlc[2] > mb and not mono
    bwd = -tlc[2] > mb and not mono
    hist = [[] for _ in range(30)]
    nm = 0
    for i, p in enumerate(P):
        x3 = _mat3(Tcw, p["xw"], c=tcw)
        invz = _f(1.0 / float(x3[2]))
        if invz < 0:
            continue
        u, v = _fma(_f(fx * x3[0]), invz, cx), _fma(_f(fy * x3[1]), invz, cy)
        if u < minx or u > maxx or v < miny or v > maxy:
            continue
        o = int(p["octave"])
        r = _f(_f(th) * scale[o])
        lo, hi = (o, -1) if fwd else ((0, o) if bwd else (o - 1, o + 1))
        x0 = max(0, int(np.floor(_f(_f(_f(u - minx) - r) * gix))))
        x1 = min(63, int(np.ceil(_f(_f(_f(u - minx) + r) * gix))))
        y0 = max(0, int(np.floor(_f(_f(_f(v - miny) - r) * giy))))
        y1 = min(47, int(np.ceil(_f(_f(_f(v - miny) + r) * giy))))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        cand = []
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                c = ix * 48 + iy
                for j in range(go[c], go[c + 1]):
                    k = gi[j]
                    if (lo > 0 or hi >= 0) and (kun[k]["octave"] < lo or (hi >= 0 and kun[k]["octave"] > hi)):
                        continue
                    if abs(_f(kun[k]["x"] - u)) < r and abs(_f(kun[k]["y"] - v)) < r:
                        cand.append(k)
        best, bi = 256, -1
        for k in cand:
            if match[k] >= 0 and blocking[k]:
                continue
            if ur[k] > 0:
                urp = _fma(-bf, invz, u)
                if abs(_f(urp - ur[k])) > r:
                    continue
            d = OM.descriptor_distance(p["desc"], desc[k])
            if d < best:
                best, bi = d, k
        if best <= 100:
            match[bi] = i
            blocking[bi] = p["n_obs"] > 0
            nm += 1
            if check_ori:
                rot = _f(p["angle"] - kun[bi]["angle"])
                if rot < 0.0:
                    rot = _f(rot + _f(360.0))
                b = int(np.round(np.float64(_f(rot * _f(1.0 / 30)))))  # half-way cases away from zero below
                x = float(_f(rot * _f(_f(1.0) / _f(30))))
                b = int(np.floor(x + 0.5)) if x >= 0 else -int(np.floor(-x + 0.5))
                hist[0 if b == 30 else b].append(bi)
    if check_ori:
        m = [0, 0, 0]
        ind = [-1, -1, -1]
        for b in range(30):
            s = len(hist[b])
            if s > m[0]:
                m = [s, m[0], m[1]]
                ind = [b, ind[0], ind[1]]
            elif s > m[1]:
                m = [m[0], s, m[1]]
                ind = [ind[0], b, ind[1]]
            elif s > m[2]:
                m[2], ind[2] = s, b
        if m[1] < _f(_f(0.1) * _f(m[0])):
            ind[1] = ind[2] = -1
        elif m[2] < _f(_f(0.1) * _f(m[0])):
            ind[2] = -1
        for b in range(30):
            if b not in ind:
                for k in hist[b]:
                    match[k] = -1
                    nm -= 1
    return np.array(match, np.int32), nm


@pytest.fixture(scope="module")
def pairs():
    return make_pairs()


def make_pairs(specs=((0, 10, 12), (1, 30, 31), (2, 50, 53)), seed=4):
    """Frame pairs (last, current) of synthetic sequences with oracle ORB + frame-stage outputs."""
    orb = oracle_ctypes.OrbOracle()
    geo_scale = orb.scale_tables()[0]
    out = []
    rng = np.random.default_rng(seed)
    for seq, l, c in specs:
        sc = synth.Scene(seq)
        gl, dl, _ = sc.render(sc.pose(l), noise_seed=l)
        gc, dc, _ = sc.render(sc.pose(c), noise_seed=c)
        kl, desl = orb.extract(gl)
        kc, desc = orb.extract(gc)
        depth_c = dc.astype(np.float32) * np.float32(np.float32(1.0) / np.float32(5000.0))
        fo = oracle_frame.frame_rgbd(np.stack([kc["x"], kc["y"]], 1), depth_c, K["fx"], K["fy"], K["cx"], K["cy"],
                                     bf=K["bf"])
        kun = kc.copy()
        kun["x"], kun["y"] = fo["un"][:, 0], fo["un"][:, 1]
        b = fo["bounds"]
        geo = np.concatenate([[K["fx"], K["fy"], K["cx"], K["cy"], K["bf"], b[0], b[1], b[2], b[3],
                               np.float32(64) / np.float32(b[1] - b[0]), np.float32(48) / np.float32(b[3] - b[2])],
                              geo_scale]).astype(np.float32)
        fr, P = synth.proj_problem(sc, l, c, kl, desl, dl, rng)
        out.append(dict(fr=fr, P=P, kun=kun, desc=desc, ur=fo["uright"], go=fo["grid_off"], gi=fo["grid_idx"],
                        geo=geo, sc=sc, c=c))
    return out


def test_oracle_matches_python_transcription(pairs):
    for k, q in enumerate(pairs):
        for th, ori in ((15.0, 1), (7.0, 0), (30.0, 1)):
            mo, nmo, passes = OM.search_by_projection(q["fr"], q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"],
                                                      q["geo"], params=(th, 0, ori, 0))
            mp, nmp = py_search(q["fr"], q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"], q["geo"], th,
                                check_ori=bool(ori))
            assert passes == 1
            assert nmo == nmp, (k, th, nmo, nmp)
            assert np.array_equal(mo, mp), (k, th, np.nonzero(mo != mp)[0][:10])


def test_matches_are_true_correspondences(pairs):
    for q in pairs:
        m, nm, _ = OM.search_by_projection(q["fr"], q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"], q["geo"])
        # nmatches counts every accepted match; a keypoint taken by a point without observations can be
        # taken again later (the reference overwrites mvpMapPoints[i2]), so it may exceed the assigned count
        assert nm >= int((m >= 0).sum())
        assert nm > 0.5 * len(q["P"]), (nm, len(q["P"]))
        # a matched keypoint sees (nearly) the map point: reprojection with the true pose within a few pixels
        Tcw = np.linalg.inv(q["sc"].pose(q["c"]))
        good = 0
        for k in np.nonzero(m >= 0)[0]:
            X = np.append(q["P"][m[k]]["xw"], 1.0)
            pc = Tcw @ X
            u = K["fx"] * pc[0] / pc[2] + K["cx"]
            v = K["fy"] * pc[1] / pc[2] + K["cy"]
            good += np.hypot(u - q["kun"][k]["x"], v - q["kun"][k]["y"]) < 4.0 * 1.2 ** q["kun"][k]["octave"]
        assert good >= 0.9 * nm, (good, nm)


def test_retry_at_twice_the_radius(pairs):
    q = pairs[0]
    fr = q["fr"].copy()
    T = fr["Tcw"].reshape(4, 4).copy()
    T[0, 3] += 0.08  # a poor motion-model prediction: few matches inside the th=15 windows
    fr["Tcw"] = T.reshape(16)
    m1, n1, p1 = OM.search_by_projection(fr, q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"], q["geo"],
                                         params=(15.0, 0, 1, 0))
    m2, n2, p2 = OM.search_by_projection(fr, q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"], q["geo"],
                                         params=(15.0, 0, 1, max(n1 + 1, 20)))
    m3, n3, _ = OM.search_by_projection(fr, q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"], q["geo"],
                                        params=(30.0, 0, 1, 0))
    assert p1 == 1 and p2 == 2
    assert n2 == n3 and np.array_equal(m2, m3)


PROBE = r"""
extern "C" void probe_proj(float fx, float fy, float cx, float cy, float bf, float xc, float yc, float invzc,
                           float* out) {
    float u = fx*xc*invzc+cx;
    float v = fy*yc*invzc+cy;
    const float ur = u - bf*invzc;
    out[0] = u; out[1] = v; out[2] = ur;
}
"""


def test_projection_expressions_match_gcc_march_native(tmp_path):
    if "fma" not in pathlib.Path("/proc/cpuinfo").read_text():
        pytest.skip("host CPU without FMA: -march=native does not contract")
    src = tmp_path / "probe.cpp"
    src.write_text(PROBE)
    so = tmp_path / "probe.so"
    subprocess.run(["g++", "-O3", "-march=native", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    L = ctypes.CDLL(str(so))
    f = ctypes.c_float
    L.probe_proj.argtypes = [f] * 8 + [ctypes.c_void_p]
    rng = np.random.default_rng(9)
    out = np.zeros(3, np.float32)
    for _ in range(2000):
        xc, yc = rng.normal(size=2).astype(np.float32)
        invz = np.float32(1.0 / rng.uniform(0.3, 6.0))
        L.probe_proj(K["fx"], K["fy"], K["cx"], K["cy"], K["bf"], xc, yc, invz, out.ctypes.data)
        u = _fma(_f(_f(K["fx"]) * xc), invz, K["cx"])
        v = _fma(_f(_f(K["fy"]) * yc), invz, K["cy"])
        assert out[0] == u and out[1] == v
        assert out[2] == _fma(-_f(K["bf"]), invz, u)


# ---------------------------------------------------------------- SearchLocalPoints
_libm = ctypes.CDLL("libm.so.6")
_libm.logf.restype, _libm.logf.argtypes = ctypes.c_float, [ctypes.c_float]


def py_search_local(fr, P, kun, desc, ur, go, gi, geo, taken, th=3.0, nn=0.8, vcl=0.5):
    """Transcription of Frame::isInFrustum, MapPoint::PredictScale and ORBmatcher.cc:45-130."""
    fx, fy, cx, cy, bf, minx, maxx, miny, maxy, gix, giy = [_f(v) for v in geo[:11]]
    scale = [_f(v) for v in geo[11:]]
    lsf = _f(_libm.logf(_f(1.2)))
    n = len(kun)
    match, tk = [-1] * n, [bool(t) for t in taken]
    Tcw = fr["Tcw"].reshape(4, 4)
    tcw = Tcw[:3, 3]
    Ow = _mat3(Tcw, tcw, transpose=True, sign=-1.0)
    nm = 0
    inview = []
    for i, p in enumerate(P):
        Pc = _mat3(Tcw, p["xw"], c=tcw)
        ok = False
        if Pc[2] >= 0:
            invz = _f(_f(1.0) / Pc[2])
            u, v = _fma(_f(fx * Pc[0]), invz, cx), _fma(_f(fy * Pc[1]), invz, cy)
            if minx <= u <= maxx and miny <= v <= maxy:
                PO = [_f(p["xw"][k] - Ow[k]) for k in range(3)]
                s = _f(PO[0] * PO[0])
                s = _f(s + _f(PO[1] * PO[1]))
                s = _f(s + _f(PO[2] * PO[2]))
                dist = _f(np.sqrt(np.float64(s)))
                if not (dist < _f(_f(0.8) * p["min_dist"]) or dist > _f(_f(1.2) * p["max_dist"])):
                    dot = float(PO[0]) * float(p["normal"][0]) + float(PO[1]) * float(p["normal"][1])
                    dot += float(PO[2]) * float(p["normal"][2])
                    vc = _f(dot / float(dist))
                    if not vc < vcl:
                        ok = True
                        lvl = int(np.ceil(_f(_f(_libm.logf(_f(p["max_dist"] / dist))) / lsf)))
                        lvl = min(max(lvl, 0), 7)
        inview.append(ok)
        if not ok:
            continue
        r = _f(2.5) if vc > _f(0.998) else _f(4.0)
        if th != 1.0:
            r = _f(r * _f(th))
        rs = _f(r * scale[lvl])
        urp = _fma(-bf, invz, u)
        x0 = max(0, int(np.floor(_f(_f(_f(u - minx) - rs) * gix))))
        x1 = min(63, int(np.ceil(_f(_f(_f(u - minx) + rs) * gix))))
        y0 = max(0, int(np.floor(_f(_f(_f(v - miny) - rs) * giy))))
        y1 = min(47, int(np.ceil(_f(_f(_f(v - miny) + rs) * giy))))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                c = ix * 48 + iy
                for j in range(go[c], go[c + 1]):
                    k = gi[j]
                    o = kun[k]["octave"]
                    if o < lvl - 1 or o > lvl:
                        continue
                    if not (abs(_f(kun[k]["x"] - u)) < rs and abs(_f(kun[k]["y"] - v)) < rs):
                        continue
                    if tk[k]:
                        continue
                    if ur[k] > 0 and abs(_f(urp - ur[k])) > rs:
                        continue
                    d = OM.descriptor_distance(p["desc"], desc[k])
                    if d < bd:
                        bd2, bl2, bd, bl, bi = bd, bl, d, o, k
                    elif d < bd2:
                        bd2, bl2 = d, o
        if bd <= 100:
            if bl == bl2 and _f(bd) > _f(_f(nn) * _f(bd2)):
                continue
            match[bi] = i
            tk[bi] = True
            nm += 1
    return np.array(match, np.int32), nm, np.array(inview)


def local_problems(pairs_list, seed=6):
    """Local-map problems on the current frames of `pairs_list` (keyframe 4 frames earlier)."""
    orb = oracle_ctypes.OrbOracle()
    rng = np.random.default_rng(seed)
    out = []
    for q in pairs_list:
        sc, c = q["sc"], q["c"]
        gk, dk, _ = sc.render(sc.pose(c - 4), noise_seed=c + 900)
        kk, dsk = orb.extract(gk)
        fr, P = synth.local_problem(sc, c - 4, c, kk, dsk, dk, rng)
        taken = (rng.uniform(size=len(q["kun"])) < 0.3).astype(np.uint8)
        out.append(dict(q, lfr=fr, LP=P, taken=taken))
    return out


def test_local_oracle_matches_python_transcription(pairs):
    for k, q in enumerate(local_problems(pairs)):
        for taken in (q["taken"], np.zeros_like(q["taken"])):
            mo, nmo, ivo = OM.search_local_points(q["lfr"], q["LP"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"],
                                                  q["geo"], taken=taken)
            mp, nmp, ivp = py_search_local(q["lfr"], q["LP"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"],
                                           q["geo"], taken)
            assert np.array_equal(ivo, ivp), k
            assert nmo == nmp and np.array_equal(mo, mp), (k, nmo, nmp)
            assert nmo > 0.3 * ivo.sum(), (nmo, ivo.sum())
            assert not (mo[taken.astype(bool)] >= 0).any()
