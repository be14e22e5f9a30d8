"""GPU parity: LocalBundleAdjustment with large local windows (18 and 25 free poses: reduced systems of 108 and
150 rows, factorised with L in global memory past the LDS-resident size), bit-exact to the CPU oracle as in
test_gpu_lba.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lba():
    import spslam_gpu
    import spslam_lba
    ex = spslam_gpu.OrbExtractor(max_batch=1)
    yield spslam_lba.LocalBA(ex)
    ex.close()


@pytest.mark.parametrize("n_kf,n_fixed", [(20, 2), (27, 2)])
def test_lba_large_windows_match_oracle(lba, n_kf, n_fixed):
    """18 free poses (n = 108, two registers of the factorisation wave per lane) and 25 (n = 150, three); both
    past the LDS-resident L (n <= 96); several Schur task rounds per lane."""
    import oracle_lba
    import synth
    rng = np.random.default_rng(300 + n_kf)
    P = synth.lba_problem(synth.Scene(4, n_boxes=4), list(range(0, 4 * n_kf, 4)), rng, n_fixed=n_fixed,
                          n_points=2000, first_kf_id=1, with_planes=True)
    import test_gpu_lba
    test_gpu_lba._assert_identical(lba(*P[:6]), oracle_lba.lba_optimize(*P[:6]), f"{n_kf} keyframes")
