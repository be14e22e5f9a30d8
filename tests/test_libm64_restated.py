"""The double-precision sin / cos / atan2 / cube that PoseOptimization uses on the GPU and in the oracle's
device-order mode (sp-slam_amd/csrc/libm64_restated.h) against the system libm the reference calls through
g2o / Eigen: within 1 ulp everywhere tested (mostly identical), cube identical to pow(x, 3).  The header is
built for the host with contraction off, like the device build."""
import ctypes
import math
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def chk(tmp_path_factory):
    so = tmp_path_factory.mktemp("libm64") / "libm64_check.so"
    subprocess.run(["g++", "-O2", "-march=x86-64-v3", "-ffp-contract=off", "-std=c++17", "-shared", "-fPIC",
                    "-o", str(so), str(ROOT / "tests" / "libm64_check.cpp")], check=True)
    lib = ctypes.CDLL(str(so))
    vp = ctypes.c_void_p
    lib.check_libm64.argtypes = [ctypes.c_int, vp, vp, ctypes.c_long, vp, vp]
    return lib


def _run(lib, kind, a, b=None):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(a if b is None else b, np.float64)
    out = np.zeros_like(a)
    st = np.zeros(2)
    lib.check_libm64(kind, a.ctypes.data, b.ctypes.data, len(a), out.ctypes.data, st.ctypes.data)
    return out, st[0], int(st[1])


def _angles(rng, n):
    return np.concatenate([
        rng.uniform(-math.pi, math.pi, n),             # azimuth / elevation / half angles
        rng.uniform(-1e-3, 1e-3, n),                   # LM update rotations
        rng.standard_normal(n) * 10.0 ** rng.uniform(-12, -5, n),
        rng.uniform(-20, 20, n),
        [0.0, -0.0, math.pi / 2, -math.pi / 2, math.pi / 4, math.pi, 3 * math.pi / 4, 2.356194490192345,
         1e-300, 5e-324, 1.5707963267948966, 4.71238898038469],
    ])


@pytest.mark.parametrize("kind,name", [(0, "sin"), (1, "cos")])
def test_sin_cos_within_one_ulp(chk, kind, name):
    a = _angles(np.random.default_rng(11 + kind), 200_000)
    _, mx, nd = _run(chk, kind, a)
    assert mx <= 1.0, (name, mx)
    assert nd < 0.05 * len(a), (name, nd)   # glibc's IBM routines are correctly rounded; fdlibm is within 1 ulp


def test_atan2_within_one_ulp(chk):
    rng = np.random.default_rng(5)
    n = 200_000
    y = np.concatenate([rng.standard_normal(n) * 10.0 ** rng.uniform(-8, 3, n), rng.standard_normal(n),
                        [0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, 1e-310, 3.0]])
    x = np.concatenate([rng.standard_normal(n) * 10.0 ** rng.uniform(-8, 3, n), np.abs(rng.standard_normal(n)),
                        [1.0, -1.0, 0.0, -0.0, np.inf, -np.inf, -2.0, 1.0]])
    x[::17] = 1.0
    _, mx, nd = _run(chk, 2, y, x)
    assert mx <= 1.0, mx
    assert nd < 0.25 * len(y), nd


def test_cube_correctly_rounded(chk):
    """cube_ is x^3 rounded once (checked against exact rational arithmetic); glibc's pow(x, 3.0) is within
    1 ulp of it (it misses the correct rounding for ~0.1 % of arguments)."""
    from fractions import Fraction
    rng = np.random.default_rng(3)
    a = np.concatenate([rng.uniform(1e-5, 1.0, 300_000), rng.standard_normal(100_000) * 10.0 ** rng.uniform(-5, 5, 100_000)])
    out, mx, nd = _run(chk, 3, a)
    assert mx <= 1.0 and nd < 0.005 * len(a), (mx, nd)
    for x, r in zip(a[::20], out[::20]):
        assert r == float(Fraction(float(x)) ** 3), x
