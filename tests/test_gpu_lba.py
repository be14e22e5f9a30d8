"""GPU parity: LocalBundleAdjustment (src/Optimizer.cc:1154-1977) vs the CPU
oracle (oracle/lba_oracle.cpp) on synthetic local maps (points + room / box
planes with observation, parallel and vertical edges; local and fixed
keyframes, keyframe id 0 held fixed).

Bar: bit equality.  The default SPSLAM_LBA_G2O_ORDER path sums every term in
g2o's order (edge-insertion-order quadratic forms and chi2, the Schur
complement landmark by landmark in vertex-id order, Eigen's SimplicialLDLT
after its AMD ordering), as the oracle does, so poses, points, planes, outlier
flags, LM iteration and trial counts must be identical, including on a weak
8-keyframe map, on a map whose point ids are not in list order, and on a
corridor map whose reduced system is genuinely sparse (AMD's elimination
loop).  The SPSLAM_LBA_FAST_ORDER phase kernels (tree / matrix-core order)
are held to the north-star 1e-4 relative bar."""
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


def _problems():
    import synth
    out = []
    for seq, frames, nfix, npts, first_id, planes in ((0, range(0, 60, 6), 2, 1500, 1, True),
                                                      (1, range(10, 70, 5), 3, 2500, 0, True),
                                                      (2, range(0, 45, 5), 1, 800, 5, False),
                                                      (3, range(0, 90, 6), 4, 3000, 0, True)):
        rng = np.random.default_rng(100 + seq)
        out.append(synth.lba_problem(synth.Scene(seq, n_boxes=4), list(frames), rng, n_fixed=nfix, n_points=npts,
                                     first_kf_id=first_id, with_planes=planes))
    return out


def _weak():
    """DESIGN section 3.9's weak map (8 keyframes, 400 points, short baselines): the golden fixture's problem."""
    import synth
    rng = np.random.default_rng(21)
    return synth.lba_problem(synth.Scene(1, n_boxes=3), list(range(0, 48, 6)), rng, n_fixed=2, n_points=400)


def _shuffled_ids(P, seed):
    """Point (and plane) ids permuted: g2o's landmark order (vertex id) differs from the edge-insertion order."""
    prob, kfs, pts, pobs, pls, plobs, gt = P
    rng = np.random.default_rng(seed)
    pts = pts.copy()
    pts["id"] = rng.permutation(pts["id"])
    pls = pls.copy()
    if len(pls):
        pls["id"] = rng.permutation(pls["id"])
    return prob, kfs, pts, pobs, pls, plobs, gt


def _corridor(P, reach=2):
    """Each point keeps the observations of keyframes within `reach` of its first observer (planes dropped: they
    see most keyframes): poses couple only to their neighbours, the reduced system is banded and not every scalar
    is above AMD's dense threshold."""
    prob, kfs, pts, pobs, pls, plobs, gt = P
    pls, plobs = pls[:0], plobs[:0]
    pts = pts.copy()
    keep_obs, keep_pts = [], []
    for i in range(len(pts)):
        o = pobs[pts[i]["obs_offset"]:pts[i]["obs_offset"] + pts[i]["n_obs"]]
        o = o[np.abs(o["kf"] - o["kf"][0]) <= reach]
        if len(o) < 2:
            continue
        p = pts[i].copy()
        p["obs_offset"] = sum(len(x) for x in keep_obs)
        p["n_obs"] = len(o)
        keep_obs.append(o)
        keep_pts.append(p)
    pts = np.array(keep_pts, pts.dtype)
    pobs = np.concatenate(keep_obs)
    prob = prob.copy()
    prob["n_points"], prob["n_point_obs"] = len(pts), len(pobs)
    prob["n_planes"], prob["n_plane_obs"] = 0, 0
    return prob, kfs, pts, pobs, pls, plobs, gt


def _assert_identical(g, o, tag):
    r, ro = g["result"], o["result"]
    assert r["status"] == 0, tag
    assert list(r["iterations"]) == list(ro["iterations"]), (tag, r, ro)
    assert r["trials"] == ro["trials"] and r["stopped"] == ro["stopped"], (tag, r, ro)
    assert np.array_equal(g["point_outlier"], o["point_outlier"]), \
        f"{tag}: {np.nonzero(g['point_outlier'] != o['point_outlier'])[0][:10]}"
    assert np.array_equal(g["plane_outlier"], o["plane_outlier"]), tag
    d = np.abs(g["Tcw"] - o["Tcw"]).max() if len(g["Tcw"]) else 0.0
    assert np.array_equal(g["Tcw"], o["Tcw"]), (tag, "poses differ by", d)
    assert np.array_equal(g["points"], o["points"]), (tag, np.abs(g["points"] - o["points"]).max())
    assert np.array_equal(g["planes"], o["planes"]), tag


def _close(a, b):
    return np.abs(a - b).max() <= TOL * max(1.0, np.abs(b).max())


def test_lba_bit_exact_to_oracle(lba):
    import oracle_lba
    for k, P in enumerate(_problems()):
        o = oracle_lba.lba_optimize(*P[:6])
        g = lba(*P[:6])
        _assert_identical(g, o, f"problem {k}")
        # the optimisation really moved the local keyframes toward the ground truth
        gt = P[6]["Tcw"]
        loc = P[1]["fixed"] == 0
        e0 = np.abs(P[1]["Tcw"].reshape(-1, 4, 4)[loc, :3, 3] - gt[loc, :3, 3]).mean()
        e1 = np.abs(g["Tcw"].reshape(-1, 4, 4)[loc, :3, 3] - gt[loc, :3, 3]).mean()
        assert e1 < 0.6 * e0, (k, e0, e1)


def test_lba_weak_map_bit_exact(lba):
    """The 8-keyframe short-baseline map where the matrix-core Schur order once left a point 4.7e-4 off."""
    import oracle_lba
    P = _weak()
    _assert_identical(lba(*P[:6]), oracle_lba.lba_optimize(*P[:6]), "weak")


def test_lba_landmark_order_is_vertex_id_order(lba):
    """Point and plane ids permuted (list order != id order): the Schur complement and x follow the id order,
    the edges their insertion order; the result changes with the ids and still matches the oracle bit for bit."""
    import oracle_lba
    P0 = _problems()[0]
    P = _shuffled_ids(P0, 5)
    o = oracle_lba.lba_optimize(*P[:6])
    _assert_identical(lba(*P[:6]), o, "shuffled ids")
    o0 = oracle_lba.lba_optimize(*P0[:6])
    assert not np.array_equal(o["points"], o0["points"])  # the order is observable in the bits


def test_lba_sparse_reduced_system_amd(lba):
    """Corridor maps: the reduced pose system is banded, AMD runs its elimination loop (a non-natural order),
    and the factorisation follows the elimination tree's row patterns."""
    import oracle_lba
    for k, P in enumerate(_problems()[1:4:2]):
        Pc = _corridor(P, reach=2)
        _assert_identical(lba(*Pc[:6]), oracle_lba.lba_optimize(*Pc[:6]), f"corridor {k}")


def _batch(lba, probs, flags=None, stream=None, sync=True):
    """One batch_device call over `probs` (optionally with per-problem stop flags preset in device memory); with
    sync=False the device buffers come back unsynchronised (a callable that finishes the call)."""
    import torch
    import spslam_lba as L
    hdr = np.zeros(len(probs), L.LBA_PROBLEM_DTYPE)
    kf, pt, po, pl, plo = [], [], [], [], []
    nk = npt = npo = npl = nplo = 0
    for i, P in enumerate(probs):
        prob, kfs, pts, pobs, pls, plobs, _ = P
        hdr[i] = prob
        hdr[i]["kf_offset"], hdr[i]["point_offset"], hdr[i]["plane_offset"] = nk, npt, npl
        pts = pts.copy(); pts["obs_offset"] += npo
        pls = pls.copy(); pls["obs_offset"] += nplo
        kf.append(kfs); pt.append(pts); po.append(pobs); pl.append(pls); plo.append(plobs)
        nk += len(kfs); npt += len(pts); npo += len(pobs); npl += len(pls); nplo += len(plobs)
    cat = lambda xs, dt: np.concatenate(xs) if sum(len(x) for x in xs) else np.zeros(1, dt)  # noqa: E731
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()  # noqa: E731
    d = [dev(hdr), dev(cat(kf, L.LBA_KEYFRAME_DTYPE)), dev(cat(pt, L.LBA_POINT_DTYPE)),
         dev(cat(po, L.LBA_POINT_OBS_DTYPE)), dev(cat(pl, L.LBA_PLANE_DTYPE)), dev(cat(plo, L.LBA_PLANE_OBS_DTYPE))]
    kf_out = torch.zeros((nk, 16), dtype=torch.float32, device="cuda")
    pt_out = torch.zeros((max(npt, 1), 3), dtype=torch.float32, device="cuda")
    pl_out = torch.zeros((max(npl, 1), 4), dtype=torch.float32, device="cuda")
    po_out = torch.zeros(max(npo, 1), dtype=torch.uint8, device="cuda")
    plo_out = torch.zeros(max(nplo, 1), dtype=torch.uint8, device="cuda")
    res = torch.zeros(len(probs) * L.LBA_RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    stop = None if flags is None else torch.tensor(flags, dtype=torch.int32, device="cuda")
    lba.batch_device(len(probs), hdr, *[x.data_ptr() for x in d], kf_out.data_ptr(), pt_out.data_ptr(),
                     pl_out.data_ptr(), po_out.data_ptr(), plo_out.data_ptr(), res.data_ptr(),
                     d_stop=None if stop is None else stop.data_ptr(),
                     stream=0 if stream is None else stream.cuda_stream)

    def finish():
        torch.cuda.synchronize()
        return (hdr, kf_out.cpu().numpy(), pt_out.cpu().numpy(), pl_out.cpu().numpy(), po_out.cpu().numpy(),
                plo_out.cpu().numpy(), res.cpu().numpy().view(L.LBA_RESULT_DTYPE), d)
    return finish()[:7] if sync else finish


def test_lba_batch_device_matches_single(lba):
    probs = _problems()[:3] + [_weak()]
    singles = [lba(*P[:6]) for P in probs]
    hdr, kf_out, pt_out, pl_out, po_out, plo_out, res = _batch(lba, probs)
    for i, s in enumerate(singles):
        h = hdr[i]
        assert np.array_equal(kf_out[h["kf_offset"]:h["kf_offset"] + h["n_kf"]], s["Tcw"])
        assert np.array_equal(pt_out[h["point_offset"]:h["point_offset"] + h["n_points"]], s["points"])
        assert np.array_equal(pl_out[h["plane_offset"]:h["plane_offset"] + h["n_planes"]], s["planes"])
        assert res[i]["trials"] == s["result"]["trials"]


def test_lba_two_streams_one_context(lba):
    """Two calls on one context, enqueued back to back on two streams without a host sync: the second
    waits on the device for the first (the context's scratch, offsets and team counters are reused), so both
    batches come back bit-identical to single calls."""
    import torch
    probs = _problems()
    a, b = probs[:2], probs[2:4]
    singles = [lba(*P[:6]) for P in probs[:4]]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    fa = _batch(lba, a, stream=s1, sync=False)
    fb = _batch(lba, b, stream=s2, sync=False)
    for f, ps, ss in ((fa, a, singles[:2]), (fb, b, singles[2:])):
        hdr, kf_out, pt_out, pl_out, po_out, plo_out, res = f()[:7]
        for i, sref in enumerate(ss):
            h = hdr[i]
            assert np.array_equal(kf_out[h["kf_offset"]:h["kf_offset"] + h["n_kf"]], sref["Tcw"])
            assert np.array_equal(pt_out[h["point_offset"]:h["point_offset"] + h["n_points"]], sref["points"])
            assert res[i]["trials"] == sref["result"]["trials"]


def test_lba_stop_flags_preset(lba):
    """pbStopFlag already raised at the call (Optimizer.cc:1757-1759): those problems return the map untouched and
    flag nothing; the other problems of the batch are unaffected (bit-identical to an unflagged run)."""
    probs = _problems()[:3]
    hdr, kf0, pt0, pl0, po0, plo0, res0 = _batch(lba, probs)
    hdr, kf1, pt1, pl1, po1, plo1, res1 = _batch(lba, probs, flags=[1, 0, 1])
    for i, P in enumerate(probs):
        h = hdr[i]
        ks, ps, qs = (slice(h["kf_offset"], h["kf_offset"] + h["n_kf"]),
                      slice(h["point_offset"], h["point_offset"] + h["n_points"]),
                      slice(h["plane_offset"], h["plane_offset"] + h["n_planes"]))
        if i == 1:
            assert res1[i]["stopped"] == 0 and res1[i]["trials"] == res0[i]["trials"]
            assert np.array_equal(kf1[ks], kf0[ks]) and np.array_equal(pt1[ps], pt0[ps])
            assert np.array_equal(pl1[qs], pl0[qs])
            continue
        assert res1[i]["stopped"] == 1 and res1[i]["trials"] == 0 and list(res1[i]["iterations"]) == [0, 0]
        assert np.array_equal(kf1[ks], P[1]["Tcw"]) and np.array_equal(pt1[ps], P[2]["xw"])
        assert np.array_equal(pl1[qs], P[4]["world"])
    assert not po1[:probs[0][0]["n_point_obs"]].any()


def test_lba_host_stop_flag_raised(lba):
    """The host-buffer entry's pbStopFlag (a bool another thread may raise) already set at the call: the
    reference returns before optimizing, the map comes back untouched."""
    P = _problems()[2]
    g = lba(*P[:6], stop_flag=np.ones(1, np.uint8))
    r = g["result"]
    assert r["stopped"] == 1 and r["trials"] == 0 and list(r["iterations"]) == [0, 0]
    assert np.array_equal(g["Tcw"], P[1]["Tcw"]) and np.array_equal(g["points"], P[2]["xw"])
    assert not g["point_outlier"].any()
    g0 = lba(*P[:6], stop_flag=np.zeros(1, np.uint8))
    assert g0["result"]["stopped"] == 0 and g0["result"]["trials"] > 0


def test_lba_stop_flag_raised_after_trial_k(lba):
    """LocalMapping::InterruptBA at a known point: the device's stop-after hook raises pbStopFlag once the
    problem has run k LM trials (k = 0: before optimize(5)).  For every k the map, outlier flags, trial and
    iteration counts equal the oracle's with the flag raised after trial k (no host timing involved)."""
    import oracle_lba
    P = _problems()[3]
    full = lba(*P[:6])
    n_trials = int(full["result"]["trials"])
    assert n_trials > 6
    try:
        for k in sorted({0, 1, 2, 3, n_trials // 3, n_trials // 2, n_trials - 1, n_trials, n_trials + 5}):
            lba.debug_stop_after(k)
            g = lba(*P[:6])
            r = g["result"]
            want_stopped = 1 if k == 0 else (2 if k < n_trials else 0)
            assert int(r["stopped"]) == want_stopped, (k, r)
            o = oracle_lba.lba_optimize(*P[:6], stop_after={0: -1, 1: 0, 2: k}[want_stopped])
            _assert_identical(g, o, f"stop after {k}")
            if want_stopped == 2:
                assert int(r["trials"]) == k
    finally:
        lba.debug_stop_after(-1)


def test_lba_shared_blocks_match_oracle(lba):
    """Points with two observations from one keyframe (the reference's MapPoint keeps one per keyframe, so this
    is outside its inputs; g2o itself accepts two edges between the same vertices): the (landmark, pose) block
    then sums two edges in edge order."""
    import oracle_lba
    prob, kfs, pts, pobs, pls, plobs, _ = _problems()[0]
    pts = pts.copy()
    new_obs = []
    for i in range(len(pts)):
        o = pobs[pts[i]["obs_offset"]:pts[i]["obs_offset"] + pts[i]["n_obs"]].copy()
        if i % 7 == 0 and len(o):
            d = o[:1].copy()
            d["u"] += 0.3
            d["v"] -= 0.2
            o = np.concatenate([o[:1], d, o[1:]])
        pts[i]["obs_offset"] = sum(len(x) for x in new_obs)
        pts[i]["n_obs"] = len(o)
        new_obs.append(o)
    pobs = np.concatenate(new_obs)
    prob = prob.copy()
    prob["n_point_obs"] = len(pobs)
    o = oracle_lba.lba_optimize(prob, kfs, pts, pobs, pls, plobs)
    _assert_identical(lba(prob, kfs, pts, pobs, pls, plobs), o, "shared blocks")


@pytest.mark.parametrize("mask", [0b1, 0b10, 0b1100, 0b100000, 0x3FF])
def test_lba_failed_solve_keeps_previous_solution(lba, mask):
    """g2o's failed-factorisation path (SimplicialLDLT's zero pivot, linear_solver_eigen.h:104-110): nothing of the
    solution vector is written (block_solver.hpp:447-457), yet update() applies it and computeScale() reads it
    (optimization_algorithm_levenberg.cpp:110-127) -- the previous solution, zeros before the first success, kept
    across the two optimize() passes -- and tempChi is DBL_MAX, so the trial is rejected and popped, its errors
    staying cached for the relabel.  Trials forced to fail (bit q = trial q) give the oracle's map, flags and counts
    bit for bit; 0x3FF makes a whole iteration's ten trials fail (qmax = 10)."""
    import oracle_ctypes
    import oracle_lba
    import spslam_gpu
    for k, P in enumerate(_problems()[:2]):
        try:
            spslam_gpu.debug_force_solve_failures(lba.ex, mask)
            g = lba(*P[:6])
        finally:
            spslam_gpu.debug_force_solve_failures(lba.ex, 0)
        with oracle_ctypes.solve_failures(mask):
            o = oracle_lba.lba_optimize(*P[:6])
        _assert_identical(g, o, f"mask {mask:#x} problem {k}")


def test_lba_fast_order_within_bar(lba):
    """SPSLAM_LBA_FAST_ORDER (the phase kernels): same decisions, values within 1e-4 relative."""
    import oracle_lba
    import spslam_lba
    lba.set_order(spslam_lba.FAST_ORDER)
    try:
        for k, P in enumerate(_problems()[:2]):
            o = oracle_lba.lba_optimize(*P[:6])
            g = lba(*P[:6])
            assert list(g["result"]["iterations"]) == list(o["result"]["iterations"]), k
            assert np.array_equal(g["point_outlier"], o["point_outlier"]), k
            assert _close(g["Tcw"], o["Tcw"]) and _close(g["points"], o["points"]), k
    finally:
        lba.set_order(spslam_lba.G2O_ORDER)
