"""CPU checks of the LocalMapping host bookkeeping (sp-slam_amd/local_mapping.py) that both the GPU sequence loop
and the CPU oracle's loop run: the batched MapPoint::UpdateNormalAndDepth (MapPoint.cc:357-400) against the
per-point statement, and the local graph's point observations (Optimizer.cc:1156-1250) against records built one
observation at a time."""
import copy

import numpy as np
import pytest

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


def _twin_maps(seed, n_kf, n_match=20, ties=False):
    """The product's SeqMap and the oracle's KeyframeMap fed the same keyframes."""
    import oracle_local_map as OLM
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
    maps = (LM.SeqMap(kf_points, CAP, CAM, SCALE, INV_S2, planes), OLM.KeyframeMap(kf_points, CAP, CAM, SCALE, INV_S2, planes))
    for j in range(n_kf):
        keys = rng.uniform(0, 600, size=(CAP, 2)).astype(np.float32)
        ur = np.where(rng.random(CAP) < 0.7, keys[:, 0] - 20, -1).astype(np.float32)
        octave = rng.integers(0, 8, CAP).astype(np.int32)
        matched = {}
        if ties and j:  # the same number of shared points with every earlier keyframe (below the threshold)
            for k in range(j):
                for q, kp in enumerate(rng.choice(np.arange(k * 5, k * 5 + 5), 3, replace=False)):
                    matched[int(kp)] = int(kf_points[k]["id"][3 * j + q])
        elif j:
            earlier = [int(p) for k in range(j) for p in kf_points[k]["id"]]
            for kp in rng.choice(CAP, n_match, replace=False):
                matched[int(kp)] = int(rng.choice(earlier))
        kinds = [(0, 7), (2, 8), (1, 9), (0, 8)]
        edges = [(kd, pid, rng.normal(size=4).astype(np.float32)) for kd, pid in kinds[:int(rng.integers(0, 5))]]
        T = _pose(rng)
        for m in maps:
            m.insert_keyframe(j, T, keys, ur, octave, matched, edges if j else [])
    return maps, rng


def _same_problem(a, b):
    (pa, ba), (pb, bb) = a, b
    for x, y in zip(pa, pb):
        assert x.tobytes() == y.tobytes()
    assert ba == bb


@pytest.mark.parametrize("seed,n_kf,n_match,ties", [(0, 5, 20, False), (1, 7, 40, False), (2, 6, 6, False),
                                                    (3, 5, 20, True), (4, 9, 30, False)])
def test_local_mapping_matches_the_oracle_bookkeeping(seed, n_kf, n_match, ties):
    """The product's LocalMapping bookkeeping (covisibility, the local graph in the ABI's order, the write-back with
    UpdateNormalAndDepth) against oracle/oracle_local_map.py's independent statement, over three LocalBundleAdjustment
    rounds with random results (outliers included) -- bit-exact records, tables, planes and poses."""
    (prod, orc), rng = _twin_maps(seed, n_kf, n_match, ties)
    if ties:  # below the threshold everywhere, several keyframes at the maximum: the first one (KeyFrame.cc:353)
        j = n_kf - 1
        cnt = {}
        for pid in orc.kfs[j]["points"].values():
            for i in orc.observations[pid]:
                if i != j:
                    cnt[i] = cnt.get(i, 0) + 1
        best = max(cnt.values())
        assert best < 15 and sum(w == best for w in cnt.values()) > 1
        assert orc.covisible_keyframes(j) == prod.covisible(j) == [min(i for i, w in cnt.items() if w == best)]
    for j in range(n_kf):
        assert prod.covisible(j) == orc.covisible_keyframes(j)
    for rnd in range(3):
        j = n_kf - 1 - rnd
        a, b = prod.lba_problem(j), orc.lba_problem(j)
        _same_problem(a, b)
        (prob, K, P, po, Q, qo), book = a
        kf_out = np.stack([_pose(rng).reshape(16) for _ in range(len(K))])
        pt_out = (P["xw"] + rng.normal(size=P["xw"].shape).astype(np.float32) * 0.01).astype(np.float32)
        pl_out = rng.normal(size=(len(Q), 4)).astype(np.float32)
        outl = (rng.random(len(po)) < 0.25).astype(np.uint8)
        stopped = 1 if rnd == 2 else 0
        prod.apply(book, kf_out, pt_out, pl_out, outl, stopped)
        orc.apply(book, kf_out, pt_out, pl_out, outl, stopped)
        assert prod.table.tobytes() == orc.table.tobytes()
        assert prod.planes.tobytes() == orc.planes.tobytes()
        assert prod.obs == orc.observations and prod.ref == orc.ref_kf
        for k in prod.kfs:
            assert prod.kfs[k]["Tcw"].tobytes() == orc.kfs[k]["Tcw"].tobytes()
            assert prod.kfs[k]["mp"] == orc.kfs[k]["points"]
    for t in range(1, n_kf * 10, 7):
        assert prod.local_points(t).tobytes() == orc.local_points(t).tobytes()
    last = np.zeros(30, SM.PROJ_POINT_DTYPE) if hasattr(SM, "PROJ_POINT_DTYPE") else None
    if last is not None:
        last["id"] = rng.choice(prod.table["id"], 30)
        last["id"][:3] = -5  # not in the table
        assert prod.refresh_last_frame(last).tobytes() == orc.refresh_last_frame(last).tobytes()
