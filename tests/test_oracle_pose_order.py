"""The pose oracle's two summation orders (oracle/pose_oracle.cpp): g2o's edge order with glibc, and the GPU
kernel's tree order with libm64_restated.h.  Same algorithm, so on the same problems the poses agree to the
north-star tolerance and the decisions (outlier flags, inlier count) coincide; they are not bitwise equal."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def problems():
    import oracle_ctypes
    import synth
    sc = synth.Scene(0)
    orb = oracle_ctypes.OrbOracle()
    invs2 = orb.scale_tables()[3]
    out = []
    for k, fi in enumerate((0, 19)):
        g, d, fid = sc.render(sc.pose(fi), noise_seed=fi)
        kps, _ = orb.extract(g)
        for variant in range(2):
            rng = np.random.default_rng(100 * k + variant)
            kw = [dict(), dict(match_frac=0.5, outlier_frac=0.2, rot_noise_deg=3.0, trans_noise=0.08)][variant]
            out.append(synth.pose_problem(sc, fi, kps, d, fid, invs2, rng, **kw))
    return out


def test_device_order_agrees_with_g2o_order(problems):
    import oracle_ctypes
    for k, (prob, pts, pls, _) in enumerate(problems):
        ra, pa, qa = oracle_ctypes.pose_optimize(prob, pts, pls)
        with oracle_ctypes.pose_order(oracle_ctypes.POSE_ORDER_DEVICE):
            rb, pb, qb = oracle_ctypes.pose_optimize(prob, pts, pls)
        Ta, Tb = ra["Tcw"].astype(np.float64), rb["Tcw"].astype(np.float64)
        assert np.abs(Ta - Tb).max() <= 1e-4, k
        assert int(ra["n_inliers"]) == int(rb["n_inliers"]) and np.array_equal(pa, pb) and np.array_equal(qa, qb), k


def test_pose_order_restored():
    import oracle_ctypes
    L = oracle_ctypes.lib()
    with oracle_ctypes.pose_order(oracle_ctypes.POSE_ORDER_DEVICE):
        assert L.oracle_get_pose_order() == 1
    assert L.oracle_get_pose_order() == 0
