"""GPU parity of tracked sequences (sp-slam_amd/sequence.py): every frame's
motion prior comes from the previous frame's optimised pose and velocity
(Tracking.cc:443-450, 958), its last-frame map points from the previous frame's
tracked matches (:456-505), and SearchLocalPoints skips the map points the
motion model already matched (mnLastFrameSeen).  The CPU oracle runs the same
loop (oracle/oracle_sequence.py); bar: every frame's local-map pose within 1e-4
(north star), ATE against the CPU trajectory <= 1e-4 m, the final last-frame
map points identical, and the pipelined step bit-identical to the serial one."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B, T, U = 4, 23, 2


@pytest.fixture(scope="module")
def tracked():
    import pipeline
    import sequence
    out = {}
    try:
        for mode in (False, True):
            sp = sequence.SequencePath(B, T, n_sequences=U, pipelined=mode, **pipeline.CONFIGS["c2"])
            out[mode] = (None, sp)
            for _ in range(T - 2):
                sp.step()
            out[mode] = (sp.trajectory(), sp)
        yield out
    finally:
        for _, sp in out.values():
            sp.close()


def _oracle(sp, slot, n):
    import oracle_ctypes
    import oracle_grab
    import oracle_planes
    import oracle_sequence
    import oracle_step
    frames, T0, P0, local_of = sp.oracle_inputs(slot)
    cam, geo, inv_s2 = oracle_step.camera_inputs(sp)
    return oracle_sequence.track(frames[:n], 1, T0, P0, local_of, cam, geo, inv_s2, sp.assoc_map, sp.assoc_boundary,
                                 oracle_ctypes.OrbOracle(nfeatures=sp.ex.params.nfeatures),
                                 oracle_planes.PlaneOracle(), supp_cap=sp.pe.supp_cap, min_size=sp.min_size,
                                 pose_cfg=sp.plane_cfg, depth_scale=oracle_grab.depth_scale(sp.depth_factor))


def test_pipelined_equals_serial(tracked):
    (ts, _), (tp, _) = tracked[False], tracked[True]
    assert ts.shape == tp.shape == (T - 1, B, 4, 4)
    assert ts.tobytes() == tp.tobytes()


def test_trajectory_matches_oracle(tracked):
    import trajectory
    from test_gpu_pose import pose_close
    tr, sp = tracked[False]
    n = T - 2
    for slot in range(U):
        cpu = _oracle(sp, slot, n)
        for k in range(n):
            ok, err = pose_close(tr[k + 1, slot].reshape(16), cpu[k].reshape(16))
            assert ok, (slot, k + 1, err)
        g = [trajectory.camera_center(tr[k + 1, slot].reshape(16)) for k in range(n)]
        c = [trajectory.camera_center(cpu[k].reshape(16)) for k in range(n)]
        assert trajectory.ate_rmse(g, c) <= 1e-4
        # and the tracking is real: within 2 cm of the synthetic ground truth
        gt = [np.linalg.inv(sp._true_pose(slot % U, k + 1))[:3, 3] for k in range(n)]
        assert trajectory.ate_rmse(g, gt) < 0.02
    # slots sharing a sequence track identically
    assert tr[:, 0].tobytes() == tr[:, U].tobytes()
