"""GPU parity: bag of words on gfx950 (sp-slam_amd/csrc/bow_kernels.hip) vs the
CPU oracle (oracle/bow_oracle.cpp) -- Frame::ComputeBoW (DBoW2 transform with
levelsup 4, src/Frame.cc:495-502) and ORBmatcher::SearchByBoW
(src/ORBmatcher.cc:159-288).  Bar: bit-exact BowVector (word ids and fp64
values), FeatureVector (nodes, feature lists) and match lists / counts."""
import numpy as np
import pytest

import bow_common as BC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import oracle_bow
    import spslam_bow
    import spslam_gpu
    ex = spslam_gpu.OrbExtractor(max_batch=8)
    text = BC.vocab_text()
    yield ex, spslam_bow.Vocabulary(ex, text), oracle_bow.Vocabulary(text)
    ex.close()


@pytest.fixture(scope="module")
def feats():
    return BC.frames(4) + BC.frames(2, seq=3, n_boxes=6)


def _same(g, o, where):
    for k in ("words", "values", "nodes", "start", "features"):
        assert g[k].tobytes() == np.asarray(o[k], g[k].dtype).tobytes(), (where, k)


def test_vocabulary_loaded(ctx):
    _, gv, ov = ctx
    assert (gv.k, gv.L, gv.n_nodes, gv.n_words) == (ov.k, ov.L, ov.n_nodes, ov.n_words)


def test_transform_single(ctx, feats):
    _, gv, ov = ctx
    for f, (_, desc) in enumerate(feats):
        for ls in (4, 2, 6, 0):
            _same(gv.transform(desc, ls), ov.transform(desc, ls), (f, ls))
    _same(gv.transform(np.zeros((0, 32), np.uint8)), ov.transform(np.zeros((0, 32), np.uint8)), "empty")


def _batch(ctx, feats, cap):
    """Device-resident batch of the frames' descriptors in the ORB batch layout -> BoW outputs (host copies)."""
    import torch
    _, gv, _ = ctx
    F = len(feats)
    d = np.zeros((F, cap, 32), np.uint8)
    cnt = np.zeros(F, np.int32)
    for f, (_, desc) in enumerate(feats):
        d[f, :len(desc)] = desc
        cnt[f] = len(desc)
    dd, dc = torch.from_numpy(d).cuda(), torch.from_numpy(cnt).cuda()
    i32 = dict(dtype=torch.int32, device="cuda")
    bw, bv = torch.zeros((F, cap), **i32), torch.zeros((F, cap), dtype=torch.float64, device="cuda")
    nb, fn = torch.zeros(F, **i32), torch.zeros((F, cap), **i32)
    fs, ff, nf = torch.zeros((F, cap + 1), **i32), torch.zeros((F, cap), **i32), torch.zeros(F, **i32)
    gv.transform_batch_device(F, dd.data_ptr(), dc.data_ptr(), cap, 4, bw.data_ptr(), bv.data_ptr(), nb.data_ptr(),
                              fn.data_ptr(), fs.data_ptr(), ff.data_ptr(), nf.data_ptr())
    torch.cuda.synchronize()
    out = []
    for f in range(F):
        b, n = int(nb[f]), int(nf[f])
        st = fs[f, :n + 1].cpu().numpy()
        out.append(dict(words=bw[f, :b].cpu().numpy().view(np.uint32), values=bv[f, :b].cpu().numpy(),
                        nodes=fn[f, :n].cpu().numpy().view(np.uint32), start=st,
                        features=ff[f, :st[-1]].cpu().numpy()))
    return out, dict(desc=dd, counts=dc, nodes=fn, start=fs, features=ff, n_fv=nf)


def test_transform_batch_device(ctx, feats):
    _, _, ov = ctx
    for cap in (1200, 2048, 8192):  # 8192: the largest cap (128 KB of dynamic LDS in bow_vectors_kernel)
        out, _ = _batch(ctx, feats, cap)
        for f, (_, desc) in enumerate(feats):
            _same(out[f], ov.transform(desc), (cap, f))


def test_search_by_bow_single(ctx, feats):
    import oracle_bow
    import spslam_bow
    ex, gv, ov = ctx
    rng = np.random.default_rng(9)
    total = 0
    for a, b in ((0, 1), (1, 2), (0, 3), (4, 5), (2, 2)):
        (kk, kd), (fk, fd) = feats[a], feats[b]
        kfv, ffv = ov.transform(kd), ov.transform(fd)
        has = (rng.random(len(kd)) < 0.85).astype(np.uint8)
        for nn, ori in ((0.7, True), (0.75, True), (0.7, False)):
            om, on = oracle_bow.search_by_bow(kd, kk["angle"], has, kfv, fd, fk["angle"], ffv, nn, ori)
            gm, gn = spslam_bow.search_by_bow(ex, kd, kk, has, kfv, fd, fk, ffv, nn, ori)
            assert gn == on and np.array_equal(gm, om), (a, b, nn, ori)
            total += on
    assert total > 250


def test_search_by_bow_batch_device(ctx, feats):
    """Relocalization-shaped batch: every keyframe slot against every frame slot, device resident."""
    import torch
    import oracle_bow
    import spslam_bow
    ex, _, ov = ctx
    cap = 1200
    _, dev = _batch(ctx, feats, cap)
    F = len(feats)
    rng = np.random.default_rng(12)
    has = (rng.random((F, cap)) < 0.8).astype(np.uint8)
    keys = np.zeros((F, cap), feats[0][0].dtype)
    for f, (k, _) in enumerate(feats):
        keys[f, :len(k)] = k
    d_keys = torch.from_numpy(keys.view(np.uint8).reshape(F, -1).copy()).cuda()
    d_has = torch.from_numpy(has).cuda()
    side = lambda hp: spslam_bow.BowSide(  # noqa: E731
        dev["desc"].data_ptr(), d_keys.data_ptr(), hp, dev["counts"].data_ptr(), dev["nodes"].data_ptr(),
        dev["start"].data_ptr(), dev["features"].data_ptr(), dev["n_fv"].data_ptr(), cap, 0)
    pairs = np.array([(a, b) for a in range(F) for b in range(F)], np.int32)
    d_pairs = torch.from_numpy(pairs).cuda()
    d_match = torch.full((len(pairs), cap), -7, dtype=torch.int32, device="cuda")
    d_n = torch.zeros(len(pairs), dtype=torch.int32, device="cuda")
    spslam_bow.search_by_bow_batch_device(ex, len(pairs), d_pairs.data_ptr(), side(d_has.data_ptr()), side(0),
                                          d_match.data_ptr(), d_n.data_ptr(), nn_ratio=0.75)
    torch.cuda.synchronize()
    fv = [ov.transform(d) for _, d in feats]
    for p, (a, b) in enumerate(pairs):
        (kk, kd), (fk, fd) = feats[a], feats[b]
        om, on = oracle_bow.search_by_bow(kd, kk["angle"], has[a, :len(kd)], fv[a], fd, fk["angle"], fv[b], 0.75,
                                          True)
        assert int(d_n[p]) == on, (a, b)
        assert np.array_equal(d_match[p, :len(fd)].cpu().numpy(), om), (a, b)


# ---- ORBvoc.txt's shape: k = 10, L = 6, 10^6 words (bow_common.shape_vocab_text; the trained file is absent)

@pytest.fixture(scope="module")
def ctx10():
    import oracle_bow
    import spslam_bow
    import spslam_gpu
    ex = spslam_gpu.OrbExtractor(max_batch=8)
    text = BC.shape_vocab_text()
    yield ex, spslam_bow.Vocabulary(ex, text), oracle_bow.Vocabulary(text)
    ex.close()


def test_orbvoc_shape_loaded(ctx10):
    _, gv, ov = ctx10
    assert (gv.k, gv.L, gv.n_words) == (ov.k, ov.L, ov.n_words) == (10, 6, 10 ** 6)
    assert gv.n_nodes == ov.n_nodes == 1 + 1111110 + 1  # root, the tree, loadFromTextFile's phantom last node


def test_orbvoc_shape_transform(ctx10, feats):
    _, gv, ov = ctx10
    for f, (_, desc) in enumerate(feats):
        for ls in (4, 2):
            _same(gv.transform(desc, ls), ov.transform(desc, ls), (f, ls))
    out, _ = _batch(ctx10, feats, 1200)
    n_words = 0
    for f, (_, desc) in enumerate(feats):
        o = ov.transform(desc)
        _same(out[f], o, ("batch", f))
        n_words += len(o["words"])
        assert len(o["nodes"]) > 50  # the FeatureVector spreads over level 2's 100 nodes
    assert n_words > 0.8 * sum(len(d) for _, d in feats)  # 10^6 words: most features get a word of their own


def test_orbvoc_shape_search_by_bow(ctx10, feats):
    """SearchByBoW between consecutive frames of one sequence at ORBvoc's shape: identical matches."""
    import oracle_bow
    import spslam_bow
    ex, _, ov = ctx10
    rng = np.random.default_rng(4)
    total = 0
    for a, b in ((0, 1), (1, 2), (2, 3), (4, 5)):
        (kk, kd), (fk, fd) = feats[a], feats[b]
        kfv, ffv = ov.transform(kd), ov.transform(fd)
        has = (rng.random(len(kd)) < 0.9).astype(np.uint8)
        om, on = oracle_bow.search_by_bow(kd, kk["angle"], has, kfv, fd, fk["angle"], ffv, 0.7, True)
        gm, gn = spslam_bow.search_by_bow(ex, kd, kk, has, kfv, fd, fk, ffv, 0.7, True)
        assert gn == on and np.array_equal(gm, om), (a, b)
        total += on
    assert total > 250
