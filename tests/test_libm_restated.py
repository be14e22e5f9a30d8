"""The device restatement of glibc atan2f / sinf / cosf (sp-slam_amd/csrc/
libm_restated.h) against the system libm the oracle and the reference call
(pcl::computeRoots uses std::atan2 / std::cos / std::sin on floats).  The
header is compiled for the host with contraction off, like the device build
(-ffp-contract=off), and compared bit for bit."""
import ctypes
import ctypes.util
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def libs(tmp_path_factory):
    so = tmp_path_factory.mktemp("libm") / "libm_check.so"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-shared", "-fPIC", "-o", str(so),
                    str(ROOT / "tests" / "libm_check.cpp")], check=True)
    chk = ctypes.CDLL(str(so))
    vp = ctypes.c_void_p
    chk.check_atan2f.argtypes = [vp, vp, vp, ctypes.c_long]
    chk.check_sincosf.argtypes = [vp, vp, vp, ctypes.c_long]
    libm = ctypes.CDLL(ctypes.util.find_library("m"))
    for f in ("atan2f",):
        getattr(libm, f).argtypes = [ctypes.c_float, ctypes.c_float]
        getattr(libm, f).restype = ctypes.c_float
    return chk, libm


def _libm_vec(libm, name, *args):
    # numpy's float32 ufuncs do not call glibc; go through a tiny C loop instead
    fn = getattr(libm, name)
    return np.array([fn(*a) for a in zip(*args)], np.float32)


def test_atan2f_matches_glibc(libs):
    chk, libm = libs
    rng = np.random.default_rng(7)
    n = 20000
    # computeRoots: atan2(sqrt(-q) >= 0, half_b of either sign), plus general and special arguments
    y = np.concatenate([np.abs(rng.standard_normal(n)) * 10.0 ** rng.uniform(-20, 5, n),
                        rng.standard_normal(n) * 10.0 ** rng.uniform(-5, 5, n),
                        [0.0, -0.0, np.inf, -np.inf, 1.0, 1e-40]]).astype(np.float32)
    x = np.concatenate([rng.standard_normal(n) * 10.0 ** rng.uniform(-20, 5, n),
                        rng.standard_normal(n) * 10.0 ** rng.uniform(-5, 5, n),
                        [1.0, -1.0, np.inf, -np.inf, 0.0, -2.0]]).astype(np.float32)
    x[::13] = 1.0
    out = np.zeros_like(y)
    chk.check_atan2f(y.ctypes.data, x.ctypes.data, out.ctypes.data, len(y))
    ref = _libm_vec(libm, "atan2f", y.tolist(), x.tolist())
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_sincosf_matches_glibc(libs):
    chk, libm = libs
    for f in ("sinf", "cosf"):
        getattr(libm, f).argtypes = [ctypes.c_float]
        getattr(libm, f).restype = ctypes.c_float
    rng = np.random.default_rng(3)
    # theta = atan2(...)/3 in [0, pi/3] for computeRoots; ORB angles up to 2 pi
    t = np.concatenate([rng.uniform(0, np.pi / 3, 20000), rng.uniform(-7, 7, 20000),
                        [0.0, 1e-8, 0.7853982, 1.0471976]]).astype(np.float32)
    s = np.zeros_like(t)
    c = np.zeros_like(t)
    chk.check_sincosf(t.ctypes.data, s.ctypes.data, c.ctypes.data, len(t))
    assert np.array_equal(s.view(np.uint32), _libm_vec(libm, "sinf", t.tolist()).view(np.uint32))
    assert np.array_equal(c.view(np.uint32), _libm_vec(libm, "cosf", t.tolist()).view(np.uint32))


PREDICT_SCALE_C = r"""
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <stdint.h>
int main(void) {
    uint32_t lo, hi; float a = 0.05f, b = 64.0f;
    memcpy(&lo, &a, 4); memcpy(&hi, &b, 4);
    const float lsf = logf(1.2f);
    long bad = 0, fragile = 0;
    for (uint32_t u = lo; u < hi; u++) {
        float x; memcpy(&x, &u, 4);
        const double d = log((double)x);
        const int g = (int)ceilf(logf(x) / lsf);
        const int c = (int)ceilf((float)d / lsf);
        if (g != c) bad++;
        if ((int)ceilf((float)nextafter(d, INFINITY) / lsf) != c || (int)ceilf((float)nextafter(d, -INFINITY) / lsf) != c)
            fragile++;
    }
    printf("%ld %ld\n", bad, fragile);
    return 0;
}
"""


def test_predict_scale_with_rounded_log_equals_glibc_logf(tmp_path):
    """MapPoint::PredictScale (src/MapPoint.cc:402-417) computes ceil(logf(ratio) / logf(1.2f)).
    The GPU evaluates the log as (float)log((double)ratio): glibc's logf is not correctly rounded
    (it differs in ~0.7% of inputs), but the resulting level is identical for every float ratio in
    [0.05, 64) (the isInFrustum range is [1/1.2, 1.2^7/0.8]), also with a 1-ulp error in the double
    log (the device's log is within 1 ulp)."""
    src = tmp_path / "ps.c"
    src.write_text(PREDICT_SCALE_C)
    exe = tmp_path / "ps"
    subprocess.run(["gcc", "-O2", str(src), "-o", str(exe), "-lm"], check=True)
    bad, fragile = map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split())
    assert bad == 0 and fragile == 0
