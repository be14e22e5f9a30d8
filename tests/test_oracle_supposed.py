"""CPU pins of the supposed-plane oracle (oracle/supposed_oracle.cpp):

* its SACSegmentation LINE/RANSAC/optimize restatement against an independent
  pure-Python transcription of the same published PCL 1.8 / boost algorithms
  (mt19937(12345) >> 1 draws, partial Fisher-Yates sampling with isSampleGood,
  adaptive-k RANSAC, Eigen SSE lane order, PCL eigen33) on small clouds;
* known answers: points on a line are recovered, degenerate clouds (all z
  equal, < 2 points) yield no model after exactly 1000 sample checks;
* Frame.cc's own float expressions: the explicit-FMA restatement equals the
  same expressions compiled by this host's g++ -O3 -march=native;
* CaculatePlanes' patch loop length.
"""
import ctypes
import ctypes.util
import math
import pathlib
import subprocess

import numpy as np
import pytest

import oracle_supposed

f32 = np.float32
ROOT = pathlib.Path(__file__).resolve().parents[1]
LIBM = ctypes.CDLL(ctypes.util.find_library("m"))
for _n, _a in (("atan2f", 2), ("sinf", 1), ("cosf", 1), ("sqrtf", 1)):
    getattr(LIBM, _n).argtypes = [ctypes.c_float] * _a
    getattr(LIBM, _n).restype = ctypes.c_float


class MT19937:
    """std::mt19937 / boost::mt19937 (32-bit seed init_genrand)."""

    def __init__(self, seed):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            self.mt[i] = (1812433253 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.i = 624

    def __call__(self):
        if self.i >= 624:
            mt = self.mt
            for k in range(624):
                y = (mt[k] & 0x80000000) | (mt[(k + 1) % 624] & 0x7FFFFFFF)
                mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            self.i = 0
        y = self.mt[self.i]
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y


def test_mt19937_matches_numpy_legacy_seeding():
    rs = np.random.RandomState(12345)  # init_genrand(12345), raw 32-bit outputs
    ref = rs.randint(0, 2 ** 32, size=1000, dtype=np.uint64)
    g = MT19937(12345)
    assert [g() for _ in range(1000)] == [int(v) for v in ref]


def _normalize4(d):
    sq = (d[0] * d[0] + d[2] * d[2]) + (d[1] * d[1] + f32(0))
    if sq > 0:
        s = f32(LIBM.sqrtf(float(sq)))
        d = [d[0] / s, d[1] / s, d[2] / s]
    return d


def _sqd(c, P):
    lp = [f32(c[0]), f32(c[1]), f32(c[2])]
    ld = _normalize4([f32(c[3]), f32(c[4]), f32(c[5])])
    ax, ay, az = lp[0] - P[:, 0], lp[1] - P[:, 1], lp[2] - P[:, 2]
    cx = ay * ld[2] - az * ld[1]
    cy = az * ld[0] - ax * ld[2]
    cz = ax * ld[1] - ay * ld[0]
    return (cx * cx + cz * cz) + (cy * cy + f32(0))


def _roots2(b, c):
    d = f32(float(b * b) - 4.0 * float(c))
    if d < 0.0:
        d = f32(0)
    sd = f32(LIBM.sqrtf(float(d)))
    return [f32(0), f32(0.5) * (b - sd), f32(0.5) * (b + sd)]


def _roots3(m):
    c0 = m[0][0] * m[1][1] * m[2][2] + f32(2) * m[0][1] * m[0][2] * m[1][2] - m[0][0] * m[1][2] * m[1][2] - \
        m[1][1] * m[0][2] * m[0][2] - m[2][2] * m[0][1] * m[0][1]
    c1 = m[0][0] * m[1][1] - m[0][1] * m[0][1] + m[0][0] * m[2][2] - m[0][2] * m[0][2] + m[1][1] * m[2][2] - \
        m[1][2] * m[1][2]
    c2 = m[0][0] + m[1][1] + m[2][2]
    if abs(c0) < np.finfo(np.float32).eps:
        return _roots2(c2, c1)
    s_inv3 = f32(1.0 / 3.0)
    s_sqrt3 = f32(LIBM.sqrtf(3.0))
    c2_over_3 = c2 * s_inv3
    a_over_3 = (c1 - c2 * c2_over_3) * s_inv3
    if a_over_3 > 0:
        a_over_3 = f32(0)
    half_b = f32(0.5) * (c0 + c2_over_3 * (f32(2) * c2_over_3 * c2_over_3 - c1))
    q = half_b * half_b + a_over_3 * a_over_3 * a_over_3
    if q > 0:
        q = f32(0)
    rho = f32(LIBM.sqrtf(float(-a_over_3)))
    theta = f32(LIBM.atan2f(float(f32(LIBM.sqrtf(float(-q)))), float(half_b))) * s_inv3
    ct, st = f32(LIBM.cosf(float(theta))), f32(LIBM.sinf(float(theta)))
    r = [c2_over_3 + f32(2) * rho * ct, c2_over_3 - rho * (ct + s_sqrt3 * st), c2_over_3 - rho * (ct - s_sqrt3 * st)]
    if r[0] >= r[1]:
        r[0], r[1] = r[1], r[0]
    if r[1] >= r[2]:
        r[1], r[2] = r[2], r[1]
        if r[0] >= r[1]:
            r[0], r[1] = r[1], r[0]
    if r[0] <= 0:
        r = _roots2(c2, c1)
    return r


def _line_direction(cov):
    def scale_of(m):
        s = max(abs(v) for row in m for v in row)
        return f32(1) if s <= np.finfo(np.float32).tiny else f32(s)
    sc = scale_of(cov)
    r = _roots3([[cov[i][j] / sc for j in range(3)] for i in range(3)])
    eval2 = r[2] * sc
    sc2 = scale_of(cov)
    s = [[cov[i][j] / sc2 for j in range(3)] for i in range(3)]
    sub = eval2 / sc2
    for i in range(3):
        s[i][i] = s[i][i] - sub
    vs, ls = [], []
    for a, b in ((s[0], s[1]), (s[0], s[2]), (s[1], s[2])):
        v = [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]
        vs.append(v)
        ls.append(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    k = 0 if (ls[0] >= ls[1] and ls[0] >= ls[2]) else (1 if (ls[1] >= ls[0] and ls[1] >= ls[2]) else 2)
    sl = f32(LIBM.sqrtf(float(ls[k])))
    return [vs[k][j] / sl for j in range(3)]


def py_segment_line(P, threshold=0.01):
    """pcl::SACSegmentation<PointXYZRGB> LINE + RANSAC + optimize, independently transcribed."""
    n = len(P)
    if n < 2:
        return None
    P = P.astype(np.float32)
    mt = MT19937(12345)
    sh = list(range(n))
    sqr_th = float(np.float64(np.float32(threshold))) ** 2
    it, best, k, have, draws = 0, -(2 ** 31 - 1), 1.0, False, 0
    best_c = None
    while it < k:
        got = False
        for _ in range(1000):
            for i in (0, 1):
                r = mt() >> 1
                draws += 1
                j = i + r % (n - i)
                sh[i], sh[j] = sh[j], sh[i]
            a, b = P[sh[0]], P[sh[1]]
            if a[0] != b[0] and a[1] != b[1] and a[2] != b[2]:
                got = True
                break
        if not got:
            break
        d = [b[0] - a[0], b[1] - a[1], b[2] - a[2]]
        sq = d[0] * d[0] + d[1] * d[1] + d[2] * d[2]
        if sq > 0:
            s = f32(LIBM.sqrtf(float(sq)))
            d = [d[0] / s, d[1] / s, d[2] / s]
        c = [a[0], a[1], a[2]] + d
        cnt = int(np.count_nonzero(_sqd(c, P).astype(np.float64) < sqr_th))
        if cnt > best:
            best, best_c, have = cnt, c, True
            w = best * (1.0 / n)
            p = max(np.finfo(np.float64).eps, min(1.0 - np.finfo(np.float64).eps, 1.0 - w ** 2.0))
            k = math.log(1.0 - 0.99) / math.log(p)
        it += 1
        if it > 1000:
            break
    if not have:
        return dict(ok=False, iterations=it, draws=draws)
    inl = np.nonzero(_sqd(best_c, P).astype(np.float64) < sqr_th)[0]
    if len(inl) <= 2:
        ref = best_c
    else:
        cen = [f32(0), f32(0), f32(0)]
        for i in inl:
            cen = [cen[0] + P[i, 0], cen[1] + P[i, 1], cen[2] + P[i, 2]]
        cen = [v / f32(len(inl)) for v in cen]
        acc = [f32(0)] * 6
        for i in inl:
            x, y, z = P[i, 0] - cen[0], P[i, 1] - cen[1], P[i, 2] - cen[2]
            acc = [acc[0] + y * y, acc[1] + y * z, acc[2] + z * z, acc[3] + x * x, acc[4] + y * x, acc[5] + z * x]
        cov = [[acc[3], acc[4], acc[5]], [acc[4], acc[0], acc[1]], [acc[5], acc[1], acc[2]]]
        ref = cen + _line_direction(cov)
    inl = np.nonzero(_sqd(ref, P).astype(np.float64) < sqr_th)[0]
    return dict(ok=True, coef=np.array(ref, np.float32), inliers=inl.astype(np.int32), iterations=it, draws=draws)


def _cloud(rng, n_line, n_out, noise):
    t = rng.uniform(-0.5, 0.5, n_line)
    p0, d = np.array([0.3, -0.2, 2.0]), np.array([0.6, 0.3, -0.74])
    d /= np.linalg.norm(d)
    line = p0 + t[:, None] * d + rng.normal(0, noise, (n_line, 3))
    out = rng.uniform([-1, -1, 1], [1, 1, 3], (n_out, 3))
    P = np.concatenate([line, out]).astype(np.float32)
    return P[rng.permutation(len(P))]


@pytest.mark.parametrize("seed", range(6))
def test_segment_line_matches_python_transcription(seed):
    rng = np.random.default_rng(seed)
    P = _cloud(rng, n_line=int(rng.integers(10, 60)), n_out=int(rng.integers(5, 60)), noise=0.004)
    a = oracle_supposed.segment_line(P)
    b = py_segment_line(P)
    assert a["ok"] and b["ok"]
    assert a["iterations"] == b["iterations"] and a["draws"] == b["draws"]
    assert np.array_equal(a["coef"], b["coef"]), (a["coef"], b["coef"])
    assert np.array_equal(a["inliers"], b["inliers"])


def test_segment_line_recovers_line():
    rng = np.random.default_rng(11)
    P = _cloud(rng, n_line=80, n_out=40, noise=0.0005)
    r = oracle_supposed.segment_line(P)
    d = np.array([0.6, 0.3, -0.74]) / np.linalg.norm([0.6, 0.3, -0.74])
    assert len(r["inliers"]) >= 80
    assert abs(abs(float(np.dot(r["coef"][3:], d))) - 1.0) < 1e-5
    assert r["iterations"] < 100  # adaptive k stops early on a 2/3-inlier cloud


def test_degenerate_clouds_have_no_model():
    # all z equal -> isSampleGood (x, y AND z must differ) never holds: 1000 checks, 2000 draws, no model
    P = np.stack([np.linspace(0, 1, 40), np.linspace(0, 2, 40), np.full(40, 1.5)], 1).astype(np.float32)
    r = oracle_supposed.segment_line(P)
    assert not r["ok"] and r["iterations"] == 0 and r["draws"] == 2000
    assert py_segment_line(P)["draws"] == 2000
    r = oracle_supposed.segment_line(P[:1])
    assert not r["ok"] and r["draws"] == 0


def test_patch_loop_length():
    n, v = 0, np.float32(-0.25)
    while v < np.float32(0.25):
        n += 1
        v = np.float32(float(v) + 0.01)
    pts = oracle_supposed.patch(np.array([0, 0, 1, 1], np.float32), np.array([0, 0, 2, 1, 0, 0], np.float32),
                                np.array([0, 1, 0, 0.5], np.float32))
    assert len(pts) == n * n and n in (50, 51)


FMA_PROBE = r"""
// Frame.cc's CaculatePlanes / LineInRange float expressions, compiled like the reference (-O3 -march=native).
#include <cmath>
extern "C" void probe_coef(const float* ip, const float* il, float* out) {
    float a, b, c, d;
    a = ip[1]*il[5] - ip[2]*il[4];
    b = ip[2]*il[3] - ip[0]*il[5];
    c = ip[0]*il[4] - ip[1]*il[3];
    d = a*il[0] + b*il[1] + c*il[2];
    float v = sqrt(a*a + b*b + c*c);
    out[0] = a/v; out[1] = b/v; out[2] = c/v; out[3] = -d/v;
    if (out[3] < 0) for (int k = 0; k < 4; k++) out[k] = -out[k];
}
extern "C" void probe_patch(const float* ip, const float* il, const float* coef, float i, float j, float* o) {
    o[0] = il[0] + i * il[3] + j * ip[0];
    o[1] = il[1] + i * il[4] + j * ip[1];
    o[2] = (coef[0]*o[0] + coef[1]*o[1] + coef[3]) / (-coef[2]);
}
"""


def test_frame_expressions_match_gcc_march_native(tmp_path):
    if "fma" not in pathlib.Path("/proc/cpuinfo").read_text():
        pytest.skip("host CPU without FMA: -march=native does not contract")
    src = tmp_path / "probe.cpp"
    src.write_text(FMA_PROBE)
    so = tmp_path / "probe.so"
    subprocess.run(["g++", "-O3", "-march=native", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    L = ctypes.CDLL(str(so))
    vp = ctypes.c_void_p
    L.probe_coef.argtypes = [vp, vp, vp]
    L.probe_patch.argtypes = [vp, vp, vp, ctypes.c_float, ctypes.c_float, vp]
    rng = np.random.default_rng(5)
    for _ in range(300):
        ip = rng.normal(size=4).astype(np.float32)
        ip[:3] /= np.linalg.norm(ip[:3])
        il = rng.normal(size=6).astype(np.float32)
        il[3:] /= np.linalg.norm(il[3:])
        ref = np.zeros(4, np.float32)
        L.probe_coef(ip.ctypes.data, il.ctypes.data, ref.ctypes.data)
        assert np.array_equal(oracle_supposed.supposed_coef(ip, il), ref)
        pts = oracle_supposed.patch(ip, il, ref)
        o = np.zeros(3, np.float32)
        for idx in (0, len(pts) // 2 + 7):
            n = int(round(math.sqrt(len(pts))))
            vals = [np.float32(-0.25)]
            while len(vals) < n:
                vals.append(np.float32(float(vals[-1]) + 0.01))
            L.probe_patch(ip.ctypes.data, il.ctypes.data, ref.ctypes.data, float(vals[idx // n]), float(vals[idx % n]),
                          o.ctypes.data)
            assert np.array_equal(o, pts[idx])
