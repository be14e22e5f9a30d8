"""CPU checks of the tracking-graph oracle (oracle/oracle_track.py: TrackWithMotionModel /
TrackLocalMap bookkeeping, src/Tracking.cc:951-1068, PoseOptimization's edge loops
src/Optimizer.cc:561-860) on hand-built cases with known answers, and of the
trajectory writer / ATE evaluator (sp-slam_amd/trajectory.py, System::SaveTrajectoryTUM
src/System.cc:329-384, Converter::toQuaternion)."""
import numpy as np

import oracle_track as OT

KP = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
               ("octave", "<i4"), ("class_id", "<i4")])
PP = np.dtype([("xw", "<f4", 3), ("angle", "<f4"), ("octave", "<i4"), ("n_obs", "<i4"), ("last_index", "<i4"),
               ("pad", "<i4"), ("desc", "u1", 32)])
LP = np.dtype([("xw", "<f4", 3), ("normal", "<f4", 3), ("min_dist", "<f4"), ("max_dist", "<f4"), ("id", "<i4"),
               ("pad", "<i4", 3), ("desc", "u1", 32)])
MP = np.dtype([("world", "<f4", 4), ("id", "<i4"), ("boundary_offset", "<i4"), ("n_boundary", "<i4"), ("pad", "<i4")])
PF = np.dtype([("Tcw", "<f4", 16), ("Tlw", "<f4", 16), ("point_offset", "<i4"), ("n_points", "<i4"),
               ("pad", "<i4", 2)])
INV_S2 = np.array([1.0, 0.69, 0.48, 0.33, 0.23, 0.16, 0.11, 0.08], np.float32)
CAM = (535.4, 539.2, 320.1, 247.6, 40.0)


def _case():
    kps = np.zeros(6, KP)
    kps["x"] = [10, 20, 30, 40, 50, 60]
    kps["y"] = [5, 6, 7, 8, 9, 10]
    kps["octave"] = [0, 1, 2, 3, 0, 7]
    ur = np.array([5, -1, 25, 35, -1, 55], np.float32)
    P = np.zeros(4, PP)
    P["xw"] = np.arange(12, dtype=np.float32).reshape(4, 3)
    P["n_obs"] = [2, 0, 1, 3]
    match = np.array([1, -1, 3, 0, -1, 2], np.int32)
    pf = np.zeros((), PF)
    pf["Tcw"] = np.eye(4, dtype=np.float32).reshape(16)
    maps = np.zeros(3, MP)
    maps["world"] = [[1, 0, 0, 1], [0, 1, 0, 2], [0, 0, 1, 3]]
    maps["id"] = [7, 8, 9]
    coefs = np.array([[1, 0, 0, 0.5], [0, 1, 0, 0.6]], np.float32)
    assoc = dict(match=np.array([2, -1]), parallel=np.array([-1, 0]), vertical=np.array([1, 1]))
    return kps, ur, P, match, pf, maps, coefs, assoc


def test_motion_model_graph_known_answer():
    kps, ur, P, match, pf, maps, coefs, assoc = _case()
    prob, pts, pls, edge = OT.motion_model_graph(pf, P, match, kps, ur, INV_S2, coefs, assoc, maps, CAM)
    # keypoint order, one edge per matched keypoint (Optimizer.cc:561-640)
    assert list(pts["kp_index"]) == [0, 2, 3, 5]
    assert list(edge) == [0, -1, 1, 2, -1, 3]
    np.testing.assert_array_equal(pts["xw"], P["xw"][[1, 3, 0, 2]])
    np.testing.assert_array_equal(pts["inv_sigma2"], INV_S2[[0, 2, 3, 7]])
    np.testing.assert_array_equal(pts["ur"], ur[[0, 2, 3, 5]])
    # plane edges, then parallel, then vertical, each in frame-plane order (Optimizer.cc:681-860)
    assert [(k, i, m) for k, i, m in zip(pls["kind"], pls["plane_index"], pls["map_plane_id"])] == \
        [(0, 0, 9), (1, 1, 7), (2, 0, 8), (2, 1, 8)]
    np.testing.assert_array_equal(pls["meas"][1], coefs[1])
    np.testing.assert_array_equal(pls["world"][0], maps["world"][2])
    assert prob["n_points"] == 4 and prob["n_planes"] == 4


def test_discard_and_local_map_graph_known_answer():
    kps, ur, P, match, pf, maps, coefs, assoc = _case()
    _, _, _, edge = OT.motion_model_graph(pf, P, match, kps, ur, INV_S2, coefs, assoc, maps, CAM)
    out = np.array([0, 1, 0, 0], bool)  # edge 1 (keypoint 2) is an outlier
    keep, taken = OT.discard_outliers(match, edge, out, P)
    assert list(keep) == [True, False, False, True, False, True]
    # keypoint 3 holds point 0 (2 obs) -> taken; keypoint 0 holds point 1 (0 obs) -> not taken
    assert list(taken) == [0, 0, 0, 1, 0, 1]
    L = np.zeros(3, LP)
    L["xw"] = 100 + np.arange(9, dtype=np.float32).reshape(3, 3)
    lmatch = np.array([2, 0, -1, -1, 1, -1], np.int32)  # replaces keypoint 0's 0-obs point, fills 1 and 4
    T1 = np.eye(4, dtype=np.float32)
    T1[0, 3] = 0.25
    prob, pts, pls = OT.local_map_graph(T1, P, match, keep, L, lmatch, kps, ur, INV_S2, coefs, assoc, maps, CAM)
    assert list(pts["kp_index"]) == [0, 1, 3, 4, 5]
    np.testing.assert_array_equal(pts["xw"], np.stack([L["xw"][2], L["xw"][0], P["xw"][0], L["xw"][1],
                                                       P["xw"][2]]))
    assert prob["Tcw"][3] == np.float32(0.25)


def test_quaternion_matches_rotation_matrix():
    from scipy.spatial.transform import Rotation

    import trajectory
    for R in Rotation.random(200, random_state=1).as_matrix():
        q = trajectory.quaternion_xyzw(R)
        want = Rotation.from_matrix(R).as_quat()  # x y z w
        assert np.allclose(q, want, atol=1e-12) or np.allclose(q, -want, atol=1e-12)
    # the trace <= 0 branches
    for axis in np.eye(3):
        R = Rotation.from_rotvec(np.pi * 0.999 * axis).as_matrix()
        q = trajectory.quaternion_xyzw(R)
        assert abs(np.linalg.norm(q) - 1) < 1e-12


def test_tum_lines_format_and_roundtrip(tmp_path):
    import trajectory
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = [0.5, -1.0, 2.0]
    lines = trajectory.tum_lines([1305031102.175304], [T])
    parts = lines[0].split()
    assert parts[0] == "1305031102.175304" and len(parts) == 8
    assert all(len(p.split(".")[1]) == 9 for p in parts[1:])
    np.testing.assert_allclose([float(p) for p in parts[1:4]], [-0.5, 1.0, -2.0])
    path = tmp_path / "CameraTrajectory.txt"
    trajectory.save_trajectory_tum(path, [0.0, 1.0], [T, T])
    ts, c, q = trajectory.load_trajectory_tum(path)
    assert len(ts) == 2 and np.allclose(q[:, 3], 1.0)


def test_ate_is_invariant_to_a_rigid_transform():
    from scipy.spatial.transform import Rotation

    import trajectory
    rng = np.random.default_rng(3)
    ref = rng.normal(size=(50, 3))
    R = Rotation.random(random_state=4).as_matrix()
    est = (R @ ref.T).T + np.array([1.0, -2.0, 0.5])
    assert trajectory.ate_rmse(est, ref) < 1e-12
    noisy = ref + rng.normal(0, 0.01, ref.shape)
    assert 0.005 < trajectory.ate_rmse(noisy, ref) < 0.02
    assert trajectory.ate_rmse(est, ref, align=False) > 0.5


def test_discard_planes_known_answer():
    """Tracking.cc:1004-1028: associations whose edge is an outlier are dropped; the rest carry into
    TrackLocalMap's association.  Edges: match (plane 0 -> 2), parallel (plane 1 -> 0), vertical (0 -> 1,
    1 -> 1)."""
    _, _, _, _, _, _, _, assoc = _case()
    kept = OT.discard_planes(assoc, np.array([0, 1, 0, 1], bool))
    assert list(kept["match"]) == [2, -1]
    assert list(kept["parallel"]) == [-1, -1]
    assert list(kept["vertical"]) == [1, -1]
    kept = OT.discard_planes(assoc, np.zeros(4, bool))
    for k in ("match", "parallel", "vertical"):
        assert list(kept[k]) == list(assoc[k])
