"""CPU check of the tracked-sequence oracle (oracle/oracle_sequence.py): the
motion-model loop of Tracking::Track (velocity, last-frame map points, seen
points skipped by SearchLocalPoints) on a synthetic sequence with a keyframe
map, run with the CPU oracle's own keypoints.  Sanity anchors (the reference
holds no trajectories): the tracked poses stay within 2 cm / 1 degree of the
synthetic ground truth, the velocity model predicts the next pose better than
the previous pose does, and every last-frame map point is a map point id."""
import numpy as np

import oracle_ctypes
import oracle_grab
import oracle_match as OM
import oracle_planes
import oracle_sequence
import oracle_track as OT
import synth


def test_motion_model_products():
    rng = np.random.default_rng(1)
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = synth._rot(rng.normal(size=3)).astype(np.float32)
    T[:3, 3] = rng.normal(size=3).astype(np.float32)
    W = OT.inverse_pose(T)
    np.testing.assert_allclose(OT.mat4(T, W), np.eye(4), atol=1e-6)
    np.testing.assert_array_equal(W[:3, :3], T[:3, :3].T)
    # a double sum rounded once: exact for small integers
    A = np.arange(16, dtype=np.float32).reshape(4, 4)
    np.testing.assert_array_equal(OT.mat4(A, A), (A.astype(np.float64) @ A).astype(np.float32))


def test_tracked_sequence_follows_ground_truth():
    K = synth.TUM3
    sc = synth.Scene(0, n_boxes=5)
    n = 12
    frames = synth.render_sequence_frames(0, n + 1, 640, 480, K, 5)
    orb = oracle_ctypes.OrbOracle()
    scale = oracle_grab.depth_scale(K["depth_factor"])
    kps0, desc0 = orb.extract(oracle_grab.cvt_gray(frames[0][0], rgb=True))
    kps10, desc10 = orb.extract(oracle_grab.cvt_gray(frames[10][0], rgb=True))
    cap = 1200
    L0 = synth.keyframe_points(sc, 0, kps0, desc0, frames[0][1], 0, K=K)
    L1 = synth.keyframe_points(sc, 10, kps10, desc10, frames[10][1], cap, K=K)
    P0 = synth.as_last_frame_points(L0, kps0, 0)
    T0 = np.linalg.inv(sc.pose(0)).astype(np.float32)
    local_of = lambda t: L0 if t <= 10 else np.concatenate([L0, L1])  # noqa: E731
    import spslam_frame  # noqa: F401  (dtypes only)
    fx, fy, cx, cy, bf = K["fx"], K["fy"], K["cx"], K["cy"], K["bf"]
    ginv = (64 / 640.0, 48 / 480.0)
    tab = orb.scale_tables()
    geo = np.concatenate([[fx, fy, cx, cy, bf, 0, 640, 0, 480, *ginv], tab[0]]).astype(np.float32)
    mp, bxyz = synth.map_planes(sc, np.random.default_rng(7))
    m = np.zeros(len(mp["world"]), np.dtype([("world", "<f4", 4), ("id", "<i4"), ("boundary_offset", "<i4"),
                                              ("n_boundary", "<i4"), ("pad", "<i4")]))
    for k, v in mp.items():
        m[k] = v
    seen_last = []
    poses = oracle_sequence.track(frames[1:n + 1], 1, T0, P0, local_of, (fx, fy, cx, cy, bf), geo, tab[3], m, bxyz,
                                  orb, oracle_planes.PlaneOracle(), supp_cap=32, depth_scale=scale,
                                  on_frame=lambda t, o, P: seen_last.append(P))
    ids = set(L0["id"]) | set(L1["id"])
    for t, Tcw in enumerate(poses, start=1):
        gt = np.linalg.inv(sc.pose(t))
        assert np.linalg.norm(np.linalg.inv(Tcw)[:3, 3] - np.linalg.inv(gt)[:3, 3]) < 0.02, t
        assert np.abs(Tcw[:3, :3] - gt[:3, :3]).max() < np.deg2rad(1.0), t
        P = seen_last[t - 1]
        assert len(P) > 200 and set(P["id"]) <= ids, t
        assert np.all(np.diff(P["last_index"]) > 0)
    # the constant-velocity prediction beats the previous pose from frame 3 on
    for t in range(3, n):
        V = OT.mat4(poses[t - 1], OT.inverse_pose(poses[t - 2]))
        pred = OT.mat4(V, poses[t - 1])
        gt = np.linalg.inv(sc.pose(t + 1))
        assert np.linalg.norm(pred[:3, 3] - gt[:3, 3]) <= np.linalg.norm(poses[t - 1][:3, 3] - gt[:3, 3]) + 1e-3
    assert OM.PROJ_POINT_DTYPE.names[5] == "id"
