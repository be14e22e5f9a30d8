"""GPU parity: LocalBundleAdjustment with local windows past the matrix-core Schur path (18 and 25 free poses),
against the CPU oracle with the bar of test_gpu_lba.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module")
def lba():
    import spslam_gpu
    import spslam_lba
    ex = spslam_gpu.OrbExtractor(max_batch=1)
    yield spslam_lba.LocalBA(ex)
    ex.close()


def _close(a, b):
    return np.abs(a - b).max() <= TOL * max(1.0, np.abs(b).max())


@pytest.mark.parametrize("n_kf,n_fixed", [(20, 2), (27, 2)])
def test_lba_large_windows_match_oracle(lba, n_kf, n_fixed):
    """Reduced systems past the matrix-core path: 18 free poses (n = 108: pose-pair Schur tasks, the
    register-resident factorization with two column registers) and 25 (n = 150: the global-memory factorization)."""
    import oracle_lba
    import synth
    rng = np.random.default_rng(300 + n_kf)
    P = synth.lba_problem(synth.Scene(4, n_boxes=4), list(range(0, 4 * n_kf, 4)), rng, n_fixed=n_fixed,
                          n_points=2000, first_kf_id=1, with_planes=True)
    o = oracle_lba.lba_optimize(*P[:6])
    g = lba(*P[:6])
    assert g["result"]["status"] == 0
    assert list(g["result"]["iterations"]) == list(o["result"]["iterations"])
    assert np.array_equal(g["point_outlier"], o["point_outlier"])
    assert np.array_equal(g["plane_outlier"], o["plane_outlier"])
    for i in range(len(P[1])):
        assert _close(g["Tcw"][i], o["Tcw"][i]), (i, g["Tcw"][i], o["Tcw"][i])
    assert _close(g["points"], o["points"])
