"""CPU pins of the LocalBundleAdjustment oracle (oracle/lba_oracle.cpp):
known answers on synthetic local maps -- noise-free observations converge to
the ground truth, injected gross outliers are the observations flagged for
erasure, fixed keyframes are returned unchanged, and a problem without
edges is a no-op."""
import numpy as np

import oracle_lba
import synth


def _prob(seed, **kw):
    rng = np.random.default_rng(seed)
    return synth.lba_problem(synth.Scene(seed % 4, n_boxes=3), list(range(0, 60, 6)), rng, **kw)


def test_noise_free_converges_to_ground_truth():
    P = _prob(11, pix_noise=0.0, outlier_frac=0.0, plane_noise_deg=0.0, plane_noise_d=0.0, stereo_frac=0.0,
              n_points=1200)
    r = oracle_lba.lba_optimize(*P[:6])
    gt = P[6]["Tcw"]
    loc = P[1]["fixed"] == 0
    err0 = np.abs(P[1]["Tcw"].reshape(-1, 4, 4)[loc, :3, 3] - gt[loc, :3, 3]).max()
    err1 = np.abs(r["Tcw"].reshape(-1, 4, 4)[loc, :3, 3] - gt[loc, :3, 3]).max()
    assert err0 > 5e-3 and err1 < 2e-4, (err0, err1)
    assert r["point_outlier"].sum() == 0


def test_gross_outliers_are_flagged():
    rng = np.random.default_rng(5)
    P = list(synth.lba_problem(synth.Scene(1, n_boxes=3), list(range(0, 60, 6)), rng, outlier_frac=0.0,
                               n_points=1000, with_planes=False))
    pobs = P[3].copy()
    bad = rng.choice(len(pobs), len(pobs) // 25, replace=False)
    pobs["u"][bad] = (pobs["u"][bad] + 80.0) % 620.0 + 10.0  # 80 px off
    P[3] = pobs
    r = oracle_lba.lba_optimize(*P[:6])
    flagged = set(np.nonzero(r["point_outlier"])[0])
    assert len(set(bad) - flagged) <= len(bad) // 50
    assert len(flagged - set(bad)) <= len(pobs) // 100


def test_fixed_keyframes_unchanged_and_empty_problem():
    P = _prob(3, n_fixed=3, n_points=600)
    r = oracle_lba.lba_optimize(*P[:6])
    fixed = P[1]["fixed"] == 1
    assert np.array_equal(r["Tcw"][fixed], P[1]["Tcw"][fixed])
    prob, kfs = P[0].copy(), P[1]
    prob["n_points"] = prob["n_planes"] = prob["n_point_obs"] = prob["n_plane_obs"] = 0
    import spslam_lba as L
    e = np.zeros(0, L.LBA_POINT_DTYPE)
    r = oracle_lba.lba_optimize(prob, kfs, e, np.zeros(0, L.LBA_POINT_OBS_DTYPE), np.zeros(0, L.LBA_PLANE_DTYPE),
                                np.zeros(0, L.LBA_PLANE_OBS_DTYPE))
    assert list(r["result"]["iterations"]) == [0, 0]
    loc = kfs["fixed"] == 0
    # local keyframes go through Converter::toSE3Quat / toCvMat unchanged up to float rounding
    assert np.abs(r["Tcw"][loc] - kfs["Tcw"][loc]).max() < 1e-6


def test_stop_flag_schedule():
    """pbStopFlag (Optimizer.cc:1351-1352, 1757-1767; g2o SparseOptimizer::terminate): raised before the call the
    reference returns without touching the map; raised after trial T the schedule ends at the next check point
    (after that trial), so exactly T trials run, and a flag raised after the last trial changes nothing."""
    P = _prob(7, n_points=900)
    full = oracle_lba.lba_optimize(*P[:6])
    n = int(full["result"]["trials"])
    assert n >= 6 and full["result"]["stopped"] == 0
    r0 = oracle_lba.lba_optimize(*P[:6], stop_after=0)
    assert r0["result"]["stopped"] == 1 and r0["result"]["trials"] == 0
    assert np.array_equal(r0["Tcw"], P[1]["Tcw"]) and np.array_equal(r0["points"], P[2]["xw"])
    assert np.array_equal(r0["planes"], P[4]["world"]) and not r0["point_outlier"].any()
    late = oracle_lba.lba_optimize(*P[:6], stop_after=n)
    assert late["result"]["stopped"] == 0
    for k in ("Tcw", "points", "planes", "point_outlier", "plane_outlier"):
        assert np.array_equal(late[k], full[k]), k
    its_prev = 0
    pass2_seen = False
    for T in range(1, n):
        r = oracle_lba.lba_optimize(*P[:6], stop_after=T)
        res = r["result"]
        assert res["stopped"] == 2 and res["trials"] == T, (T, res)
        its = int(res["iterations"].sum())
        assert its_prev <= its <= int(full["result"]["iterations"].sum())
        its_prev = its
        pass2_seen |= res["iterations"][1] > 0
        again = oracle_lba.lba_optimize(*P[:6], stop_after=T)
        assert np.array_equal(again["points"], r["points"])
    assert pass2_seen


def _spd_with_pattern(pattern, rng):
    n = pattern.shape[0]
    M = np.where(pattern | pattern.T, rng.standard_normal((n, n)), 0.0)
    A = (M + M.T) / 2 + np.diag(np.abs(M).sum(1) + 1.0)  # diagonally dominant on the pattern
    return np.where(pattern | pattern.T | np.eye(n, dtype=bool), A, 0.0)


def test_eigen_ldlt_restatement_solves_and_orders():
    """oracle/eigen_simplicial_restated.h (Eigen SimplicialLDLT + AMD, parity unpinned: Eigen is absent): the
    result is a permutation, the factorisation solves the system, and the orderings forced by the algorithm come
    out -- a fully coupled pattern has every node above the dense threshold (natural order), an arrow pattern
    eliminates its leaves before the hub, a block-tridiagonal chain of pose blocks keeps each 6-scalar block
    contiguous."""
    rng = np.random.default_rng(7)
    # fully coupled 10-pose reduced system: every scalar's degree (60) exceeds dense = min(58, 77)
    n = 60
    pat = np.triu(np.ones((n, n), bool))
    A = _spd_with_pattern(pat, rng)
    b = rng.standard_normal(n)
    x, perm = oracle_lba.eigen_ldlt(pat, A, b)
    assert list(perm) == list(range(n))
    assert np.abs(A @ x - b).max() < 1e-10
    # arrow: hub 0 coupled to every leaf (hub degree 40 > dense 38), leaves to the hub only
    n = 40
    pat = np.eye(n, dtype=bool)
    pat[0, :] = True
    A = _spd_with_pattern(pat, rng)
    b = rng.standard_normal(n)
    x, perm = oracle_lba.eigen_ldlt(pat, A, b)
    assert sorted(perm) == list(range(n)) and perm[-1] == 0
    assert np.abs(A @ x - b).max() < 1e-10
    # block tridiagonal chain of 12 poses (each scalar coupled to <= 18 others, below dense = 26)
    P = 12
    n = 6 * P
    pat = np.zeros((n, n), bool)
    for p in range(P):
        for q in (p, p + 1):
            if q < P:
                pat[6 * p:6 * p + 6, 6 * q:6 * q + 6] = True
    pat = np.triu(pat)
    A = _spd_with_pattern(pat, rng)
    b = rng.standard_normal(n)
    x, perm = oracle_lba.eigen_ldlt(pat, A, b)
    assert sorted(perm) == list(range(n))
    assert np.abs(A @ x - b).max() < 1e-10
    blocks = perm // 6
    runs = [blocks[i] for i in range(n) if i == 0 or blocks[i] != blocks[i - 1]]
    assert sorted(runs) == list(range(P)), runs  # supervariables: each pose's 6 scalars eliminated together
    assert list(perm) != list(range(n))          # a genuine fill-reducing order, not the natural one


def test_fma_diagnostic_mode_is_contracted_and_scoped():
    """oracle_ctypes.g2o_fma: the LBA / pose restatement compiled with GCC's FP contraction (the reference's
    -march=native g2o) -- a different rounding of the same algorithm: close to the pinned result, not bit-equal,
    and only inside the block."""
    import oracle_ctypes
    P = _prob(7, n_points=800)
    a = oracle_lba.lba_optimize(*P[:6])
    with oracle_ctypes.g2o_fma(True):
        f = oracle_lba.lba_optimize(*P[:6])
    b = oracle_lba.lba_optimize(*P[:6])
    assert np.array_equal(a["Tcw"], b["Tcw"]) and np.array_equal(a["points"], b["points"])
    assert not np.array_equal(a["points"], f["points"])
    loc = P[1]["fixed"] == 0
    assert np.abs(a["Tcw"][loc] - f["Tcw"][loc]).max() < 1e-4
    assert np.array_equal(a["point_outlier"], f["point_outlier"])
