"""The correctly rounded double sin / cos / atan2 the GPU's PoseOptimization and LocalBundleAdjustment run
(sp-slam_amd/csrc/libm64_cr.h, host build of the same source, contraction off like the device build)
against the oracle's independent correctly rounded routines (oracle/libm_cr_oracle.h: x87 long double with a
quad-precision fallback): bit-identical on every argument.  The oracle itself is checked against exact
decimal arithmetic on a sample, and the host glibc 2.35 is shown to misround a small fraction of arguments
(the reason the path pins correct rounding)."""
import ctypes
import math
import pathlib
import subprocess
from decimal import Decimal as D, getcontext
from fractions import Fraction as F

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    so = tmp_path_factory.mktemp("libm64cr") / "libm64_cr_check.so"
    subprocess.run(["g++", "-O2", "-march=x86-64-v3", "-ffp-contract=off", "-std=c++17", "-shared", "-fPIC",
                    "-o", str(so), str(ROOT / "tests" / "libm64_cr_check.cpp"), "-lquadmath"], check=True)
    L = ctypes.CDLL(str(so))
    vp = ctypes.c_void_p
    L.check_libm64_cr.argtypes = [ctypes.c_int, vp, vp, ctypes.c_long, vp, vp]
    L.oracle_libm_cr.argtypes = [ctypes.c_int, vp, vp, ctypes.c_long, vp]
    return L


def _check(L, kind, a, b=None):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(a if b is None else b, np.float64)
    out = np.zeros_like(a)
    st = np.zeros(2, np.int64)
    L.check_libm64_cr(kind, a.ctypes.data, b.ctypes.data, len(a), out.ctypes.data, st.ctypes.data)
    return out, int(st[0]), int(st[1])


def _angles(rng, n):
    k = np.arange(-40, 41)
    near = (k * (math.pi / 2))[:, None] + rng.standard_normal((81, n // 200)) * 10.0 ** rng.uniform(-12, -1, (81, n // 200))
    return np.concatenate([
        rng.uniform(-math.pi, math.pi, n),                 # half angles, azimuth / elevation
        rng.uniform(-math.pi / 4, math.pi / 4, n),
        rng.uniform(-1e-3, 1e-3, n),                       # LM update rotations
        rng.standard_normal(n) * 10.0 ** rng.uniform(-9, -1, n),
        rng.uniform(-100, 100, n // 4),
        near.ravel(),                                      # near multiples of pi/2
        np.arange(-64, 65) / 64.0, np.arange(-64, 65) * (math.pi / 128),
        [0.0, -0.0, math.pi / 2, -math.pi / 2, math.pi / 4, math.pi, 3 * math.pi / 4, 1e-300, 5e-324,
         7.450580596923828e-09, 7.450580596923829e-09, 1.4901161193847656e-08, 1e5, -3e5, 2.0 ** 19],
    ])


@pytest.mark.parametrize("kind,name", [(0, "sin"), (1, "cos")])
def test_sin_cos_match_oracle(lib, kind, name):
    a = _angles(np.random.default_rng(21 + kind), 300_000)
    _, nd, ng = _check(lib, kind, a)
    assert nd == 0, (name, nd)
    assert 0 < ng < 0.01 * len(a), (name, ng)  # glibc 2.35 misrounds a few arguments per thousand


def test_atan2_matches_oracle(lib):
    rng = np.random.default_rng(7)
    n = 400_000
    y = np.concatenate([rng.standard_normal(n) * 10.0 ** rng.uniform(-8, 3, n), rng.standard_normal(n),
                        rng.uniform(-1e-3, 1e-3, n)])
    x = np.concatenate([rng.standard_normal(n) * 10.0 ** rng.uniform(-8, 3, n), np.abs(rng.standard_normal(n)),
                        rng.uniform(-1, 1, n)])
    x[::17] = 1.0
    x[::19] = y[::19]              # |y| == |x|
    x[::23] = -y[::23]
    y[::29] = y[::29] * 1e-200     # tiny ratios
    # extreme magnitudes: 1 / max(|x|, |y|) is not a normal double there (the quick path's reciprocal), and
    # ratios beyond 2^-900
    ext = np.array([1e300, -3e305, 2.0 ** 1000, 2.0 ** 1001, 2.0 ** -1000, 2.0 ** -1001, -7e-302, 1e-250, 3e-200])
    ye, xe = np.meshgrid(ext, np.concatenate([ext, [1.0, -2.5, 0.3]]))
    y = np.concatenate([y, ye.ravel(), xe.ravel()])
    x = np.concatenate([x, xe.ravel(), ye.ravel()])
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, 1e-310, 5e-324, np.nan])
    ys, xs = np.meshgrid(sp, sp)
    y = np.concatenate([y, ys.ravel()])
    x = np.concatenate([x, xs.ravel()])
    out, nd, ng = _check(lib, 2, y, x)
    assert nd == 0, nd
    # C99 special values
    for yy, xx, want in [(0.0, -0.0, math.pi), (-0.0, -1.0, -math.pi), (-0.0, 1.0, -0.0), (1.0, 0.0, math.pi / 2),
                         (np.inf, -np.inf, 3 * math.pi / 4), (-np.inf, np.inf, -math.pi / 4), (1.0, -np.inf, math.pi),
                         (-1.0, np.inf, -0.0)]:
        i = np.nonzero((y == yy) & (x == xx) & (np.signbit(y) == np.signbit(yy)) & (np.signbit(x) == np.signbit(xx)))[0][0]
        assert out[i] == want and np.signbit(out[i]) == np.signbit(want), (yy, xx, out[i])


def _dsin(x):
    x = D(x)
    t = s = x
    k = 1
    while abs(t) > D(10) ** -70:
        t = -t * x * x / ((2 * k) * (2 * k + 1))
        s += t
        k += 1
    return s


def test_oracle_against_exact_arithmetic(lib):
    """The oracle's sin rounds the exact value: 60-digit decimal Taylor series, rounded with exact rationals."""
    getcontext().prec = 70
    rng = np.random.default_rng(3)
    a = np.concatenate([rng.uniform(-1.6, 1.6, 4000), rng.uniform(-1e-3, 1e-3, 1000)])
    out = np.zeros_like(a)
    lib.oracle_libm_cr(0, a.ctypes.data, a.ctypes.data, len(a), out.ctypes.data)
    for x, r in zip(a, out):
        assert r == float(F(_dsin(float(x)))), x


def test_cube_matches_oracle(lib):
    """x^3 (SE3Quat::exp's pow(theta, 3), the LM damping update's pow(2 rho - 1, 3)): correctly rounded, special
    values (+-0, +-inf, NaN, overflow, underflow) like pow; glibc 2.35's pow misrounds ~0.1 %."""
    rng = np.random.default_rng(8)
    a = np.concatenate([rng.uniform(-1, 1, 300_000), rng.standard_normal(100_000) * 10.0 ** rng.uniform(-5, 5, 100_000),
                        [0.0, -0.0, np.inf, -np.inf, np.nan, 1e103, -1e103, 1e-110, 5e-324, 5.6e102]])
    out, nd, ng = _check(lib, 3, a)
    assert nd == 0, nd
    assert 0 < ng < 0.01 * len(a)
    for x, r in zip(a[:2000], out[:2000]):
        assert r == float(F(float(x)) ** 3), x
