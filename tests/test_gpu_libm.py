"""GPU parity of the double elementary functions PoseOptimization and LocalBundleAdjustment run
(sp-slam_amd/csrc/libm64_cr.h on gfx950, through spslam_debug_libm64) against the oracle's independent
correctly rounded routines (oracle/libm_cr_oracle.h): bit-identical on every argument, including the
arguments near multiples of pi/2 and the C99 special values."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import spslam_gpu
    ex = spslam_gpu.OrbExtractor(max_batch=1)
    yield ex
    ex.close()


def test_sin_cos_cube_bit_exact(gpu):
    import oracle_ctypes
    import spslam_gpu
    rng = np.random.default_rng(5)
    n = 200_000
    k = np.arange(-20, 21)
    a = np.concatenate([rng.uniform(-math.pi, math.pi, n), rng.uniform(-1e-3, 1e-3, n),
                        rng.standard_normal(n) * 10.0 ** rng.uniform(-9, -1, n),
                        ((k * math.pi / 2)[:, None] + rng.standard_normal((41, 500)) * 1e-6).ravel(),
                        [0.0, -0.0, math.pi / 2, math.pi, 1e-300, 5e-324, np.inf, -np.inf, np.nan]])
    # the constants g2o_device.h aa_apply_half_pi uses for sin / cos (M_PI / 2)
    assert oracle_ctypes.libm_cr(0, np.array([math.pi / 2]))[0] == 1.0
    assert oracle_ctypes.libm_cr(1, np.array([math.pi / 2]))[0] == 6.123233995736766e-17
    for kind in (0, 1, 3):
        d = spslam_gpu.debug_libm64(gpu, kind, a)
        o = oracle_ctypes.libm_cr(kind, a)
        bad = np.nonzero(~((d == o) | (np.isnan(d) & np.isnan(o))) | (np.signbit(d) != np.signbit(o)) & ~np.isnan(o))[0]
        assert len(bad) == 0, (kind, a[bad[:5]], d[bad[:5]], o[bad[:5]])


def test_atan2_bit_exact(gpu):
    import oracle_ctypes
    import spslam_gpu
    rng = np.random.default_rng(6)
    n = 200_000
    y = np.concatenate([rng.standard_normal(n) * 10.0 ** rng.uniform(-8, 3, n), rng.uniform(-1e-3, 1e-3, n)])
    x = np.concatenate([rng.standard_normal(n) * 10.0 ** rng.uniform(-8, 3, n), rng.uniform(-1, 1, n)])
    x[::19] = y[::19]
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, 1e-310, np.nan])
    ys, xs = np.meshgrid(sp, sp)
    y, x = np.concatenate([y, ys.ravel()]), np.concatenate([x, xs.ravel()])
    # extreme magnitudes (the quick path's reciprocal of max(|x|, |y|) leaves the normal range) and ratios
    # below 2^-900: the slow path decides
    ext = np.array([1e300, -3e305, 2.0 ** 1000, 2.0 ** 1001, 2.0 ** -1000, 2.0 ** -1001, -7e-302, 1e-250, 3e-200])
    ye, xe = np.meshgrid(ext, np.concatenate([ext, [1.0, -2.5, 0.3]]))
    y, x = np.concatenate([y, ye.ravel(), xe.ravel()]), np.concatenate([x, xe.ravel(), ye.ravel()])
    d = spslam_gpu.debug_libm64(gpu, 2, y, x)
    o = oracle_ctypes.libm_cr(2, y, x)
    bad = np.nonzero(~((d == o) | (np.isnan(d) & np.isnan(o))) | (np.signbit(d) != np.signbit(o)) & ~np.isnan(o))[0]
    assert len(bad) == 0, (y[bad[:5]], x[bad[:5]], d[bad[:5]], o[bad[:5]])
