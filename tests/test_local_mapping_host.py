"""CPU checks of the LocalMapping host bookkeeping (sp-slam_amd/local_mapping.py) that both the GPU sequence loop
and the CPU oracle's loop run: the batched MapPoint::UpdateNormalAndDepth (MapPoint.cc:357-400) against the
per-point statement, and the local graph's point observations (Optimizer.cc:1156-1250) against records built one
observation at a time."""
import copy

import numpy as np

import local_mapping as LM
import spslam_assoc as SA
import spslam_lba as L
import spslam_match as SM

CAP = 64
CAM = (535.4, 539.2, 320.1, 247.6, 40.0)
SCALE = (1.2 ** np.arange(8)).astype(np.float32)
INV_S2 = (1.0 / (SCALE * SCALE)).astype(np.float32)


def _pose(rng):
    a = rng.normal(size=3) * 0.05
    c, s = np.cos(a[2]), np.sin(a[2])
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], np.float32)
    T[:3, 3] = rng.normal(size=3).astype(np.float32) * 0.2
    return T


def _map(seed=0, n_kf=5):
    rng = np.random.default_rng(seed)
    kf_points = []
    for j in range(n_kf):
        P = np.zeros(40, SM.LOCAL_POINT_DTYPE)
        P["id"] = j * CAP + rng.choice(CAP, 40, replace=False)
        P["xw"] = rng.normal(size=(40, 3)).astype(np.float32) + np.float32([0, 0, 4])
        kf_points.append(P)
    planes = np.zeros(3, SA.MAP_PLANE_DTYPE)
    planes["id"] = [7, 8, 9]
    planes["world"] = rng.normal(size=(3, 4)).astype(np.float32)
    m = LM.SeqMap(kf_points, CAP, CAM, SCALE, INV_S2, planes)
    for j in range(n_kf):
        keys = rng.uniform(0, 600, size=(CAP, 2)).astype(np.float32)
        ur = np.where(rng.random(CAP) < 0.7, keys[:, 0] - 20, -1).astype(np.float32)
        octave = rng.integers(0, 8, CAP).astype(np.int32)
        # matches to earlier keyframes' points: several observations per point
        earlier = [int(p) for k in range(j) for p in kf_points[k]["id"]]
        matched = {}
        if earlier:
            for kp in rng.choice(CAP, 20, replace=False):
                matched[int(kp)] = int(rng.choice(earlier))
        edges = [(0, 7, rng.normal(size=4).astype(np.float32)), (2, 8, rng.normal(size=4).astype(np.float32))]
        m.insert_keyframe(j, _pose(rng), keys, ur, octave, matched, edges if j else [])
    return m, rng


def test_point_observations_follow_the_keyframe_order():
    m, _ = _map()
    (prob, K, P, po, Q, qo), book = m.lba_problem(4)
    kidx = {k: n for n, k in enumerate(book["kfs"])}
    rec = []
    for pid in book["points"]:
        for i in sorted(m.obs[pid]):
            kp = m.obs[pid][i]
            kf = m.kfs[i]
            rec.append((kidx[i], kf["keys"][kp, 0], kf["keys"][kp, 1], kf["ur"][kp], INV_S2[kf["octave"][kp]]))
    want = np.array(rec, L.LBA_POINT_OBS_DTYPE)
    assert po.tobytes() == want.tobytes()
    assert int(prob["n_point_obs"]) == len(want) == len(book["src"])
    off = np.concatenate([[0], np.cumsum(P["n_obs"])[:-1]])
    assert np.array_equal(P["obs_offset"], off)
    assert np.array_equal(P["xw"], np.stack([m.table[m.row_of[p]]["xw"] for p in book["points"]]))


def test_batched_normal_and_depth_equals_the_per_point_statement():
    m, rng = _map(seed=3)
    (prob, K, P, po, Q, qo), book = m.lba_problem(4)
    ref = copy.deepcopy(m)
    kf_out = np.stack([_pose(rng).reshape(16) for _ in range(len(K))])
    pt_out = (P["xw"] + rng.normal(size=P["xw"].shape).astype(np.float32) * 0.01).astype(np.float32)
    pl_out = rng.normal(size=(len(Q), 4)).astype(np.float32)
    outl = (rng.random(len(po)) < 0.2).astype(np.uint8)
    rows = m.apply(book, kf_out, pt_out, pl_out, outl, 0)
    # the statement one point at a time (the erasures, poses and positions as apply makes them)
    for b in np.flatnonzero(outl):
        pid, i = book["src"][b]
        kp = ref.obs[pid].pop(i)
        ref.kfs[i]["mp"].pop(kp, None)
        if ref.ref.get(pid) == i and ref.obs[pid]:
            ref.ref[pid] = min(ref.obs[pid])
    for n in range(book["n_local"]):
        ref.kfs[book["kfs"][n]]["Tcw"] = kf_out[n].reshape(4, 4).copy()
    centers = {k: LM.camera_center(kf["Tcw"]) for k, kf in ref.kfs.items()}
    for n, pid in enumerate(book["points"]):
        r = ref.row_of[pid]
        ref.table[r]["xw"] = pt_out[n]
        ref.update_normal_and_depth(pid, r, centers)
    assert np.array_equal(rows, [ref.row_of[p] for p in book["points"]])
    assert m.table.tobytes() == ref.table.tobytes()
    assert m.obs == ref.obs and m.ref == ref.ref
