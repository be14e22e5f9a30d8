"""GPU parity: ORBmatcher::SearchByProjection (frame to frame, with
GetFeaturesInArea, DescriptorDistance, the rotation check and
TrackWithMotionModel's retry; src/ORBmatcher.cc:1328-1470, src/Frame.cc:427-480,
src/Tracking.cc:968-975) on gfx950 vs the CPU oracle.  Bar: identical
mvpMapPoints assignment and nmatches (index work: bit-exact)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import spslam_frame
    import spslam_gpu
    import spslam_match
    import synth
    K = synth.TUM3
    ex = spslam_gpu.OrbExtractor(max_batch=1)
    spslam_frame.FrameStage(ex, K["fx"], K["fy"], K["cx"], K["cy"], (0,) * 5, K["bf"], 640, 480)
    yield ex, spslam_match
    ex.close()


@pytest.fixture(scope="module")
def pairs():
    from test_oracle_match import make_pairs
    return make_pairs(((0, 10, 12), (1, 30, 31), (2, 50, 53), (3, 5, 9), (4, 70, 71), (5, 0, 2)), seed=17)


def test_single_pairs_match_oracle(gpu, pairs):
    import oracle_match as OM
    ex, M = gpu
    for params in ((15.0, 0, 1, 20), (15.0, 0, 0, 0), (7.0, 0, 1, 0), (15.0, 1, 1, 20), (4.0, 0, 1, 400)):
        m = M.Matcher(ex, params)
        for k, q in enumerate(pairs):
            mo, nmo, _ = OM.search_by_projection(q["fr"], q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"],
                                                 q["geo"], params=params)
            mg, nmg = m(q["fr"], q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"])
            assert nmg == nmo, (params, k, nmg, nmo)
            assert np.array_equal(mg, mo), (params, k, np.nonzero(mg != mo)[0][:10])


def test_edge_cases(gpu, pairs):
    import oracle_match as OM
    ex, M = gpu
    m = M.Matcher(ex)
    q = pairs[0]
    cases = [q["P"][:0], q["P"][:1], q["P"]]
    behind = q["P"].copy()
    behind["xw"] = -behind["xw"] * 50  # far behind / outside the image
    cases.append(behind)
    zero_obs = q["P"].copy()
    zero_obs["n_obs"] = 0  # nothing blocks: later points may take the same keypoint
    cases.append(zero_obs)
    for P in cases:
        fr = q["fr"].copy()
        fr["n_points"] = len(P)
        mo, nmo, _ = OM.search_by_projection(fr, P, q["kun"], q["desc"], q["ur"], q["go"], q["gi"], q["geo"])
        mg, nmg = m(fr, P, q["kun"], q["desc"], q["ur"], q["go"], q["gi"])
        assert nmg == nmo and np.array_equal(mg, mo), len(P)


def test_batch_device_matches_single(gpu, pairs):
    import torch
    import spslam_gpu as G
    ex, M = gpu
    m = M.Matcher(ex)
    F, cap = len(pairs), max(len(q["kun"]) for q in pairs)
    frames = np.zeros(F, M.PROJ_FRAME_DTYPE)
    kun = np.zeros((F, cap), G.KEYPOINT_DTYPE)
    desc = np.zeros((F, cap, 32), np.uint8)
    ur = np.zeros((F, cap), np.float32)
    go = np.zeros((F, 64 * 48 + 1), np.int32)
    gi = np.zeros((F, cap), np.int32)
    counts = np.zeros(F, np.int32)
    pts, off = [], 0
    for f, q in enumerate(pairs):
        n = len(q["kun"])
        frames[f] = q["fr"]
        frames[f]["point_offset"] = off
        off += len(q["P"])
        pts.append(q["P"])
        kun[f, :n] = q["kun"]
        desc[f, :n] = q["desc"]
        ur[f, :n] = q["ur"]
        go[f] = q["go"]
        gi[f, :len(q["gi"])] = q["gi"]
        counts[f] = n
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()  # noqa
    d = [dev(frames), dev(np.concatenate(pts)), dev(kun), dev(desc), dev(ur), dev(go), dev(gi), dev(counts)]
    max_points = max(len(p) for p in pts)
    d_match = torch.full((F * cap,), -9, dtype=torch.int32, device="cuda")
    d_nm = torch.zeros(F, dtype=torch.int32, device="cuda")
    m.batch_device(F, d[0].data_ptr(), d[1].data_ptr(), max_points, d[2].data_ptr(), d[3].data_ptr(),
                   d[4].data_ptr(), d[5].data_ptr(), d[6].data_ptr(), d[7].data_ptr(), cap, d_match.data_ptr(),
                   d_nm.data_ptr())
    torch.cuda.synchronize()
    mb, nb = d_match.cpu().numpy().reshape(F, cap), d_nm.cpu().numpy()
    for f, q in enumerate(pairs):
        ms, ns = m(q["fr"], q["P"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"])
        assert nb[f] == ns and np.array_equal(mb[f, :len(q["kun"])], ms), f


@pytest.fixture(scope="module")
def local_pairs(pairs):
    from test_oracle_match import local_problems
    return local_problems(pairs, seed=23)


def test_local_points_match_oracle(gpu, local_pairs):
    import oracle_match as OM
    ex, M = gpu
    for params in ((3.0, 0.8, 0.5, 0), (5.0, 0.8, 0.5, 0), (1.0, 0.6, 0.5, 0), (3.0, 0.95, 0.9, 0)):
        lm = M.LocalMatcher(ex, params)
        for k, q in enumerate(local_pairs):
            for taken in (q["taken"], None):
                mo, nmo, ivo = OM.search_local_points(q["lfr"], q["LP"], q["kun"], q["desc"], q["ur"], q["go"],
                                                      q["gi"], q["geo"], taken=taken, params=params[:3])
                mg, nmg, ivg = lm(q["lfr"], q["LP"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"], taken)
                assert np.array_equal(ivg, ivo), (params, k)
                assert nmg == nmo, (params, k, nmg, nmo)
                assert np.array_equal(mg, mo), (params, k, np.nonzero(mg != mo)[0][:10])


def test_local_points_batch_matches_single(gpu, local_pairs):
    import torch
    import spslam_gpu as G
    ex, M = gpu
    lm = M.LocalMatcher(ex)
    F, cap = len(local_pairs), max(len(q["kun"]) for q in local_pairs)
    frames = np.zeros(F, M.LOCAL_FRAME_DTYPE)
    kun = np.zeros((F, cap), G.KEYPOINT_DTYPE)
    desc = np.zeros((F, cap, 32), np.uint8)
    ur = np.zeros((F, cap), np.float32)
    go = np.zeros((F, 64 * 48 + 1), np.int32)
    gi = np.zeros((F, cap), np.int32)
    tk = np.zeros((F, cap), np.uint8)
    counts = np.zeros(F, np.int32)
    pts, off = [], 0
    for f, q in enumerate(local_pairs):
        n = len(q["kun"])
        frames[f] = q["lfr"]
        frames[f]["point_offset"] = off
        off += len(q["LP"])
        pts.append(q["LP"])
        kun[f, :n], desc[f, :n], ur[f, :n], go[f] = q["kun"], q["desc"], q["ur"], q["go"]
        gi[f, :len(q["gi"])] = q["gi"]
        tk[f, :n] = q["taken"]
        counts[f] = n
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()  # noqa
    d = [dev(frames), dev(np.concatenate(pts)), dev(kun), dev(desc), dev(ur), dev(go), dev(gi), dev(counts), dev(tk)]
    max_points = max(len(p) for p in pts)
    d_match = torch.full((F * cap,), -9, dtype=torch.int32, device="cuda")
    d_nm = torch.zeros(F, dtype=torch.int32, device="cuda")
    d_iv = torch.zeros(off, dtype=torch.uint8, device="cuda")
    lm.batch_device(F, d[0].data_ptr(), d[1].data_ptr(), max_points, d[2].data_ptr(), d[3].data_ptr(),
                    d[4].data_ptr(), d[5].data_ptr(), d[6].data_ptr(), d[7].data_ptr(), cap, d[8].data_ptr(),
                    d_match.data_ptr(), d_nm.data_ptr(), d_iv.data_ptr())
    torch.cuda.synchronize()
    mb, nb, ivb = d_match.cpu().numpy().reshape(F, cap), d_nm.cpu().numpy(), d_iv.cpu().numpy().astype(bool)
    off = 0
    for f, q in enumerate(local_pairs):
        ms, ns, ivs = lm(q["lfr"], q["LP"], q["kun"], q["desc"], q["ur"], q["go"], q["gi"], q["taken"])
        assert nb[f] == ns and np.array_equal(mb[f, :len(q["kun"])], ms), f
        assert np.array_equal(ivb[off:off + len(q["LP"])], ivs), f
        off += len(q["LP"])
