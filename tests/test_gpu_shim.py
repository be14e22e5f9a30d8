"""The compiled reference-side shim (tests/shim/reference_shim.cpp: INTEGRATION.md 1-7 as C++ at the
reference's call sites, over the C ABI) against the CPU oracle.

  * Tracking::GrabImageRGBD + the RGB-D Frame constructor (ORBextractor::operator(), UndistortKeyPoints /
    ComputeStereoFromRGBD, ComputePlanesFromOrganizedPointCloud, GeneratePlanesFromBoundries) on a colour +
    u16 depth frame: keypoints, descriptors, mvKeysUn, mvuRight and every plane coefficient bit-exact;
  * Optimizer::PoseOptimization(Frame*) on a Frame whose mvpMapPoints / mvpMapPlanes the shim builds from
    per-keypoint / per-plane arrays: the shim's graph equals the flattened problem the oracle receives, pose
    bit-exact to the oracle (g2o's order, correctly rounded libm), every outlier flag identical;
  * Optimizer::LocalBundleAdjustment(pKF, pbStopFlag) on a KeyFrame / MapPoint / MapPlane object graph: the
    shim's collection (local keyframes, local points and planes, fixed cameras) and flattening are checked
    against an independent Python restatement of Optimizer.cc:1156-1298, the GPU result against the oracle
    on that problem (poses, points and planes bit-identical: the default g2o-order LocalBundleAdjustment;
    identical iteration counts and outlier flags), and the applied result (SetPose / SetWorldPos /
    EraseMapPointMatch) against the optimizer's outputs;
  * Map::AssociatePlanesByBoundary (f1) on Frame / MapPlane objects: match / parallel / vertical and
    mbNewPlane identical to the oracle;
  * TrackWithMotionModel's SearchByProjection (f2, th then 2 th below 20 matches) on Frame / MapPoint objects:
    mvpMapPoints and nmatches identical;
  * KeyFrame / Frame::ComputeBoW and SearchByBoW (f4) with the vocabulary loaded into the context: the frame's
    BowVector / FeatureVector and the matches identical.
"""
import ctypes
import pathlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]
TOL = 1e-4


@pytest.fixture(scope="module")
def shim():
    import spslam_gpu
    spslam_gpu.load_library()  # the product library (and torch's HIP runtime) first
    lib = ctypes.CDLL(str(ROOT / "tests" / "shim" / "libreference_shim.so"))
    lib.shim_last_error.restype = ctypes.c_char_p
    return lib


def _close(a, b):  # 1e-4 relative, as tests/test_gpu_lba.py
    return np.abs(a - b).max() <= TOL * max(1.0, np.abs(b).max())


def _call(lib, fn, *args):
    rc = getattr(lib, fn)(*args)
    assert rc == 0, lib.shim_last_error().decode()


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def test_shim_track_frame_bit_exact(shim):
    import spslam_gpu as G
    import oracle_ctypes
    import oracle_frame
    import oracle_grab
    import oracle_planes
    import oracle_supposed
    import synth
    K = synth.TUM3
    sc = synth.Scene(2, n_boxes=5)
    for fi in (3, 17):
        g, d16, fid = sc.render(sc.pose(fi), noise_seed=fi)
        rgb = synth.colorize(g, fid)
        h, w = d16.shape
        cam = np.array([K["fx"], K["fy"], K["cx"], K["cy"], 0, 0, 0, 0, 0, K["bf"]], np.float32)
        cap, pcap = 20000, 256
        kps = np.zeros(cap, G.KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        kun = np.zeros(cap, G.KEYPOINT_DTYPE)
        ur = np.zeros(cap, np.float32)
        coef = np.zeros((pcap, 4), np.float32)
        n, npl, nreal = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _call(shim, "shim_track_frame", _p(np.ascontiguousarray(rgb)), _p(np.ascontiguousarray(d16)), w, h,
              ctypes.c_float(5000.0), _p(cam), 1000, 500, _p(kps), _p(desc), _p(kun), _p(ur), cap, ctypes.byref(n),
              _p(coef), pcap, ctypes.byref(npl), ctypes.byref(nreal))
        n = n.value
        # the oracle chain on the same frame
        gray = oracle_grab.cvt_gray(rgb, rgb=True)
        depth = oracle_grab.convert_depth(d16, oracle_grab.depth_scale(5000.0))
        ko, do = oracle_ctypes.OrbOracle().extract(gray, cap=cap)
        assert n == len(ko) and n > 500
        for f in ("x", "y", "size", "angle", "response", "octave"):
            assert np.array_equal(kps[:n][f], ko[f]), f
        assert np.array_equal(desc[:n], do)
        fo = oracle_frame.frame_rgbd(np.stack([ko["x"], ko["y"]], 1), depth, K["fx"], K["fy"], K["cx"], K["cy"],
                                     bf=K["bf"])
        assert np.array_equal(kun[:n]["x"], fo["un"][:, 0]) and np.array_equal(kun[:n]["y"], fo["un"][:, 1])
        assert np.array_equal(ur[:n].view(np.uint32), np.asarray(fo["uright"], np.float32).view(np.uint32))
        po = oracle_planes.PlaneOracle()
        r = po.extract(depth, K["fx"], K["fy"], K["cx"], K["cy"])
        so = oracle_supposed.generate(depth, po.cloud(), r["coef"], r["contour"], K["fx"], K["fy"], K["cx"], K["cy"])
        ref = np.concatenate([np.asarray(r["coef"], np.float32).reshape(-1, 4),
                              np.asarray(so["coef"], np.float32).reshape(-1, 4)])
        assert nreal.value == len(np.asarray(r["coef"]).reshape(-1, 4))
        assert npl.value == len(ref) and npl.value >= 3
        assert np.array_equal(coef[:npl.value].view(np.uint32), ref.view(np.uint32))


def _pose_problems():
    import oracle_ctypes
    import synth
    sc = synth.Scene(0)
    orb = oracle_ctypes.OrbOracle()
    invs2 = orb.scale_tables()[3]
    out = []
    for k, fi in enumerate((0, 19, 40)):
        g, d, fid = sc.render(sc.pose(fi), noise_seed=fi)
        kps, _ = orb.extract(g)
        rng = np.random.default_rng(7 + k)
        kw = [dict(), dict(match_frac=0.5, outlier_frac=0.2, rot_noise_deg=3.0, trans_noise=0.08), dict()][k]
        out.append((kps, np.asarray(invs2, np.float32)) + synth.pose_problem(sc, fi, kps, d, fid, invs2, rng, **kw))
    return out


def test_shim_pose_optimization(shim):
    """The shim's PoseOptimization(Frame*) builds its graph from Frame members; the test rebuilds those members
    from a flat problem (keypoint kp_index, plane_index, kind) so the shim's edge order can be checked against
    it: results must equal the oracle's on the flat problem."""
    import spslam_gpu as G
    import oracle_ctypes
    cfg = G.PlaneConfig.tum()
    cfg6 = np.array([cfg.angle_info, cfg.distance_info, cfg.parallel_info, cfg.vertical_info, cfg.chi, cfg.vp_chi])
    for kps, invs2, prob, pts, pls, _ in _pose_problems():
        N = len(kps)
        keys_un = np.zeros(N, G.KEYPOINT_DTYPE)
        keys_un["x"], keys_un["y"], keys_un["octave"] = kps["x"], kps["y"], kps["octave"]
        ur = np.full(N, -1.0, np.float32)
        has = np.zeros(N, np.uint8)
        xw = np.zeros((N, 3), np.float32)
        for o in pts:  # the frame's members behind each flat point observation
            i = int(o["kp_index"])
            keys_un[i]["x"], keys_un[i]["y"] = o["u"], o["v"]
            keys_un[i]["octave"] = int(np.nonzero(invs2 == o["inv_sigma2"])[0][0])
            ur[i], has[i], xw[i] = o["ur"], 1, o["xw"]
        npl = int(pls["plane_index"].max()) + 1 if len(pls) else 0
        meas = np.zeros((max(npl, 1), 4), np.float32)
        assoc = np.full((3, max(npl, 1)), -1, np.int32)
        world = np.zeros((max(len(pls), 1), 4), np.float32)
        for j, o in enumerate(pls):
            meas[o["plane_index"]] = o["meas"]
            assoc[o["kind"], o["plane_index"]] = j
            world[j] = o["world"]
        cam = np.array([prob["fx"], prob["fy"], prob["cx"], prob["cy"], prob["bf"]], np.float32)
        Tout = np.zeros(16, np.float32)
        nin = ctypes.c_int()
        pout = np.zeros(N, np.uint8)
        plout = np.zeros((3, max(npl, 1)), np.uint8)
        _call(shim, "shim_pose_optimization", N, _p(keys_un), _p(ur), _p(invs2), _p(has), _p(xw), npl, _p(meas),
              _p(np.ascontiguousarray(assoc[:, :max(npl, 1)])), _p(world), _p(np.ascontiguousarray(prob["Tcw"])),
              _p(cam), _p(cfg6), _p(Tout), ctypes.byref(nin), _p(pout), _p(plout))
        rd, pod, plod = oracle_ctypes.pose_optimize(prob, pts, pls)
        assert np.array_equal(Tout.view(np.uint32), rd["Tcw"].view(np.uint32))
        assert nin.value == int(rd["n_inliers"])
        assert np.array_equal(pout[pts["kp_index"]].astype(bool), pod)
        assert np.array_equal(plout[pls["kind"], pls["plane_index"]].astype(bool), plod)


def _collect_lba(kfs, points, pobs, planes, plobs):
    """Optimizer.cc:1156-1298 restated independently of the shim, on the same object graph: keyframe 0 and its
    covisible (non-fixed) keyframes; local points from their matches (keyframe order, slot order); local planes
    from their mvpMapPlanes; fixed cameras from the local points' then planes' observations (keyframe id order).
    Returns the flat problem in spslam_lba layout."""
    import spslam_lba as L
    n_kf = len(kfs)
    slots = [[] for _ in range(n_kf)]          # map point matches per keyframe, in slot order
    plane_slots = [[] for _ in range(n_kf)]    # (plane, kind) per plane coefficient slot
    for j, p in enumerate(points):
        for o in range(p["obs_offset"], p["obs_offset"] + p["n_obs"]):
            slots[pobs[o]["kf"]].append((j, o))
    for j, q in enumerate(planes):
        for o in range(q["obs_offset"], q["obs_offset"] + q["n_obs"]):
            plane_slots[plobs[o]["kf"]].append((j, o))
    local = [0] + [k for k in range(1, n_kf) if not kfs[k]["fixed"]]
    lp, seen = [], set()
    lq, seenq = [], set()
    for k in local:
        for j, _ in slots[k]:
            if j not in seen:
                seen.add(j)
                lp.append(j)
        for j, o in plane_slots[k]:
            if plobs[o]["kind"] == 0 and j not in seenq:
                seenq.add(j)
                lq.append(j)
    by_id = lambda ks: sorted(ks, key=lambda k: kfs[k]["id"])  # noqa: E731
    fixed, fset = [], set(local)
    for j in lp:
        for k in by_id({pobs[o]["kf"] for o in range(points[j]["obs_offset"], points[j]["obs_offset"] + points[j]["n_obs"])}):
            if k not in fset:
                fset.add(k)
                fixed.append(k)
    for j in lq:
        for kind in (0, 2, 1):
            for k in by_id({plobs[o]["kf"] for o in range(planes[j]["obs_offset"], planes[j]["obs_offset"] + planes[j]["n_obs"])
                            if plobs[o]["kind"] == kind}):
                if k not in fset:
                    fset.add(k)
                    fixed.append(k)
    order = local + fixed
    kidx = {k: i for i, k in enumerate(order)}
    fk = kfs[order].copy()
    fk["fixed"] = [0] * len(local) + [1] * len(fixed)
    fp, fpo = np.zeros(len(lp), L.LBA_POINT_DTYPE), []
    for i, j in enumerate(lp):
        fp[i] = points[j]
        fp[i]["obs_offset"] = len(fpo)
        obs = sorted(range(points[j]["obs_offset"], points[j]["obs_offset"] + points[j]["n_obs"]),
                     key=lambda o: kfs[pobs[o]["kf"]]["id"])
        for o in obs:
            r = pobs[o].copy()
            r["kf"] = kidx[int(r["kf"])]
            fpo.append(r)
        fp[i]["n_obs"] = len(fpo) - fp[i]["obs_offset"]
    fq, fqo = np.zeros(len(lq), L.LBA_PLANE_DTYPE), []
    for i, j in enumerate(lq):
        fq[i] = planes[j]
        fq[i]["obs_offset"] = len(fqo)
        for kind in (0, 2, 1):
            obs = sorted([o for o in range(planes[j]["obs_offset"], planes[j]["obs_offset"] + planes[j]["n_obs"])
                          if plobs[o]["kind"] == kind], key=lambda o: kfs[plobs[o]["kf"]]["id"])
            for o in obs:
                r = plobs[o].copy()
                r["kf"] = kidx[int(r["kf"])]
                fqo.append(r)
        fq[i]["n_obs"] = len(fqo) - fq[i]["obs_offset"]
    prob = np.zeros((), L.LBA_PROBLEM_DTYPE)
    prob["n_kf"], prob["n_points"], prob["n_planes"] = len(fk), len(fp), len(fq)
    prob["n_point_obs"], prob["n_plane_obs"] = len(fpo), len(fqo)
    return (prob, fk, fp, np.array(fpo, L.LBA_POINT_OBS_DTYPE), fq, np.array(fqo, L.LBA_PLANE_OBS_DTYPE), lp, lq,
            order)


def test_shim_local_bundle_adjustment(shim):
    import spslam_gpu as G
    import spslam_lba as L
    import oracle_lba
    import synth
    cfg = G.PlaneConfig.tum()
    cfg6 = np.array([cfg.angle_info, cfg.distance_info, cfg.parallel_info, cfg.vertical_info, cfg.chi, cfg.vp_chi])
    invs2 = np.array([1.0 / (1.2 ** (2 * o)) for o in range(8)], np.float32)
    rng = np.random.default_rng(100)  # tests/test_gpu_lba.py's first problem
    prob, kfs, pts, pobs, pls, plobs, _ = synth.lba_problem(synth.Scene(0, n_boxes=4), list(range(0, 60, 6)), rng,
                                                            n_fixed=2, n_points=1500, first_kf_id=1)
    n_kf, n_p, n_q = len(kfs), len(pts), len(pls)
    fprob = np.zeros((), L.LBA_PROBLEM_DTYPE)
    fk = np.zeros(n_kf, L.LBA_KEYFRAME_DTYPE)
    fp = np.zeros(max(n_p, 1), L.LBA_POINT_DTYPE)
    fpo = np.zeros(max(len(pobs), 1), L.LBA_POINT_OBS_DTYPE)
    fq = np.zeros(max(n_q, 1), L.LBA_PLANE_DTYPE)
    fqo = np.zeros(max(len(plobs), 1), L.LBA_PLANE_OBS_DTYPE)
    kf_out = np.zeros((n_kf, 16), np.float32)
    pt_out = np.zeros((max(n_p, 1), 3), np.float32)
    pl_out = np.zeros((max(n_q, 1), 4), np.float32)
    erased = np.zeros(max(len(pobs), 1), np.uint8)
    res = np.zeros((), L.LBA_RESULT_DTYPE)
    _call(shim, "shim_local_ba", n_kf, _p(kfs), n_p, _p(pts), _p(pobs), n_q, _p(pls), _p(plobs), _p(invs2),
          _p(cfg6), 0, _p(fprob), _p(fk), _p(fp), _p(fpo), _p(fq), _p(fqo), len(fpo), len(fqo), _p(kf_out),
          _p(pt_out), _p(pl_out), _p(erased), _p(res))
    # 1. the shim's collection + flattening == the restatement of Optimizer.cc:1156-1298
    xprob, xk, xp, xpo, xq, xqo, lp, lq, order = _collect_lba(kfs, pts, pobs, pls, plobs)
    for f in ("n_kf", "n_points", "n_planes", "n_point_obs", "n_plane_obs"):
        assert int(fprob[f]) == int(xprob[f]), f
    assert fk[:len(xk)].tobytes() == xk.tobytes()
    assert fp[:len(xp)].tobytes() == xp.tobytes()
    assert fpo[:len(xpo)].tobytes() == xpo.tobytes()
    assert fq[:len(xq)].tobytes() == xq.tobytes()
    assert fqo[:len(xqo)].tobytes() == xqo.tobytes()
    # 2. the GPU result behind the shim == the oracle on that problem
    ro = oracle_lba.lba_optimize(xprob, xk, xp, xpo, xq, xqo, cfg=cfg6)
    assert int(res["status"]) == 0 and list(res["iterations"]) == list(ro["result"]["iterations"])
    for i, k in enumerate(order):
        if xk[i]["fixed"]:
            assert np.array_equal(kf_out[k], kfs[k]["Tcw"]), k    # fixed cameras untouched
        else:
            assert np.array_equal(kf_out[k], ro["Tcw"][i]), k  # SetPose
    for i, j in enumerate(lp):
        assert np.array_equal(pt_out[j], ro["points"][i]), j  # SetWorldPos
    for i, j in enumerate(lq):
        assert np.array_equal(pl_out[j], ro["planes"][i]), j
    # 3. outlier observations erased (EraseMapPointMatch + EraseObservation, Optimizer.cc:1896-1920)
    flagged = set()
    for i, j in enumerate(lp):
        o0 = xp[i]["obs_offset"]
        for q in range(o0, o0 + xp[i]["n_obs"]):
            if ro["point_outlier"][q]:
                flagged.add((j, int(order[xpo[q]["kf"]])))
    got = {(j, int(pobs[o]["kf"])) for j, p in enumerate(pts)
           for o in range(p["obs_offset"], p["obs_offset"] + p["n_obs"]) if erased[o]}
    assert got == flagged and len(flagged) > 0


def test_shim_associate_planes(shim):
    import oracle_assoc as OA
    import synth
    rng = np.random.default_rng(23)
    n = 0
    for seq in range(3):
        sc = synth.Scene(seq, n_boxes=1 + seq)
        mp, bxyz = synth.map_planes(sc, rng)
        m = np.zeros(len(mp["world"]), OA.MAP_PLANE_DTYPE)
        for k, v in mp.items():
            m[k] = v
        b = np.ascontiguousarray(bxyz, np.float32).reshape(-1, 3)
        for fr in range(0, 120, 11):
            T, c, _ = synth.assoc_frame_planes(sc, fr, rng, n_faces=4 + fr % 6, n_random=fr % 4)
            o = OA.associate(T, c, m, b)
            T = np.ascontiguousarray(T, np.float32).reshape(16)
            c = np.ascontiguousarray(c, np.float32).reshape(-1, 4)
            k = len(c)
            out = [np.full(max(k, 1), -9, np.int32) for _ in range(3)]
            newp = ctypes.c_int(-1)
            _call(shim, "shim_associate_planes", _p(T), _p(c), k, _p(m), len(m), _p(b), _p(OA.ASSOC_PARAMS),
                  _p(out[0]), _p(out[1]), _p(out[2]), ctypes.byref(newp))
            for key, g in zip(("match", "parallel", "vertical"), out):
                assert np.array_equal(g[:k], o[key]), (seq, fr, key)
            assert bool(newp.value) == o["new_plane"], (seq, fr)
            n += 1
    assert n > 25


def test_shim_motion_model_matching(shim):
    import oracle_match as OM
    import synth
    from test_oracle_match import make_pairs
    K = synth.TUM3
    cam = np.array([K["fx"], K["fy"], K["cx"], K["cy"], K["bf"], 640, 480], np.float32)
    total = 0
    for q in make_pairs(((0, 10, 12), (1, 30, 31), (2, 50, 53), (3, 5, 9)), seed=17):
        mo, nmo, _ = OM.search_by_projection(q["fr"], q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"],
                                             q["geo"], params=(15.0, 0, 1, 20))
        fr = np.ascontiguousarray(q["fr"], OM.PROJ_FRAME_DTYPE).reshape(1)
        P = np.ascontiguousarray(q["P"], OM.PROJ_POINT_DTYPE)
        kun = np.ascontiguousarray(q["kun"])
        n = len(kun)
        match = np.full(max(n, 1), -9, np.int32)
        nm = ctypes.c_int(-1)
        _call(shim, "shim_track_motion_model_matching", _p(fr), _p(P), len(P), _p(kun),
              _p(np.ascontiguousarray(q["desc"])), _p(np.ascontiguousarray(q["ur"], np.float32)), n,
              _p(np.ascontiguousarray(q["go"], np.int32)), _p(np.ascontiguousarray(q["gi"], np.int32)), _p(cam),
              ctypes.c_float(15.0), _p(match), ctypes.byref(nm))
        assert nm.value == nmo
        assert np.array_equal(match[:n], mo), np.nonzero(match[:n] != mo)[0][:10]
        total += nmo
    assert total > 400


def test_shim_bow_match(shim):
    import bow_common as BC
    import oracle_bow
    text = BC.vocab_text()
    ov = oracle_bow.Vocabulary(text)
    feats = BC.frames(3)
    rng = np.random.default_rng(5)
    total = 0
    for a, b, nn, ori in ((0, 1, 0.7, 1), (1, 2, 0.7, 1), (0, 2, 0.75, 0)):
        (kk, kd), (fk, fd) = feats[a], feats[b]
        has = (rng.random(len(kd)) < 0.85).astype(np.uint8)
        ft = ov.transform(fd)
        om, on = oracle_bow.search_by_bow(kd, kk["angle"], has, ov.transform(kd), fd, fk["angle"], ft, nn, bool(ori))
        nf = len(fd)
        match = np.full(max(nf, 1), -9, np.int32)
        words, values = np.zeros(nf, np.uint32), np.zeros(nf, np.float64)
        nodes, start, feat = np.zeros(nf, np.uint32), np.zeros(nf + 1, np.int32), np.zeros(nf, np.int32)
        nm, nb, nfv = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        buf = ctypes.create_string_buffer(text, len(text))
        _call(shim, "shim_bow_match", buf, ctypes.c_size_t(len(text)), _p(np.ascontiguousarray(kd)),
              _p(np.ascontiguousarray(kk)), _p(has), len(kd), _p(np.ascontiguousarray(fd)),
              _p(np.ascontiguousarray(fk)), nf, ctypes.c_float(nn), ori, _p(match), ctypes.byref(nm), _p(words),
              _p(values), ctypes.byref(nb), _p(nodes), _p(start), _p(feat), ctypes.byref(nfv))
        assert nm.value == on and np.array_equal(match[:nf], om), (a, b)
        assert words[:nb.value].tobytes() == np.asarray(ft["words"], np.uint32).tobytes()
        assert values[:nb.value].tobytes() == np.asarray(ft["values"], np.float64).tobytes()
        assert nodes[:nfv.value].tobytes() == np.asarray(ft["nodes"], np.uint32).tobytes()
        assert start[:nfv.value + 1].tobytes() == np.asarray(ft["start"], np.int32).tobytes()
        assert feat[:start[nfv.value]].tobytes() == np.asarray(ft["features"], np.int32).tobytes()
        total += on
    assert total > 150
