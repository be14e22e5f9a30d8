"""GPU parity: Map::AssociatePlanesByBoundary (src/Map.cc:196-359) on gfx950 vs
the CPU oracle (oracle/assoc_oracle.cpp).  Bar: identical match / parallel /
vertical map-plane indices and mbNewPlane (index work: bit-exact)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def assoc():
    import spslam_assoc
    import spslam_gpu
    ex = spslam_gpu.OrbExtractor(max_batch=1)
    yield spslam_assoc.PlaneAssociator(ex)
    ex.close()


def _map(rng, scene, **kw):
    import oracle_assoc as OA
    import synth
    mp, b = synth.map_planes(scene, rng, **kw)
    m = np.zeros(len(mp["world"]), OA.MAP_PLANE_DTYPE)
    for k, v in mp.items():
        m[k] = v
    return m, b


def test_single_frame_matches_oracle(assoc):
    import oracle_assoc as OA
    import synth
    rng = np.random.default_rng(21)
    n = 0
    for seq in range(4):
        sc = synth.Scene(seq, n_boxes=1 + seq)
        m, b = _map(rng, sc)
        for fr in range(0, 200, 9):
            T, c, _ = synth.assoc_frame_planes(sc, fr, rng, n_faces=4 + fr % 6, n_random=fr % 4)
            o = OA.associate(T, c, m, b)
            g = assoc(T, c, m, b)
            for k in ("match", "parallel", "vertical"):
                assert np.array_equal(g[k], o[k]), (seq, fr, k, g[k], o[k])
            assert g["new_plane"] == o["new_plane"]
            n += 1
    assert n > 80


def test_edge_cases(assoc):
    import oracle_assoc as OA
    import synth
    rng = np.random.default_rng(2)
    m, b = _map(rng, synth.Scene(0, n_boxes=0))
    T = np.eye(4, dtype=np.float32)
    c = np.array([[0, 1, 0, 1.3], [1, 0, 0, 2.5], [0, 0, 1, 0.1]], np.float32)
    for mm, bb, cc in ((m, b, c[:0]), (m[:0], b[:0], c), (m, b, c)):
        o, g = OA.associate(T, cc, mm, bb), assoc(T, cc, mm, bb)
        for k in ("match", "parallel", "vertical"):
            assert np.array_equal(g[k], o[k]), k
        assert g["new_plane"] == o["new_plane"]
    m2 = m.copy()
    m2["n_boundary"][::2] = 0  # map planes without boundary points never match
    o, g = OA.associate(T, c, m2, b), assoc(T, c, m2, b)
    assert np.array_equal(g["match"], o["match"])
    # thresholds exactly at the angle / distance limits
    m3 = m.copy()
    m3["world"][0] = [0.8, 0.6, 0, 1.0]
    c3 = np.array([[1, 0, 0, 1.0], [0.6, 0.8, 0, 1.0]], np.float32)
    o, g = OA.associate(T, c3, m3, b), assoc(T, c3, m3, b)
    for k in ("match", "parallel", "vertical"):
        assert np.array_equal(g[k], o[k]), k


def test_batch_two_sources_per_frame_maps(assoc):
    """Batched path: frames with their own maps (sequences), planes from two record
    sources (extracted spslam_plane + supposed spslam_supposed_plane layouts)."""
    import torch
    import oracle_assoc as OA
    import spslam_assoc as SA
    import spslam_planes as SP
    import synth
    rng = np.random.default_rng(8)
    F, cap_a, cap_b = 24, 8, 4
    maps, bounds, frames, expect = [], [], np.zeros(F, SA.ASSOC_FRAME_DTYPE), []
    A = np.zeros((F, cap_a), SP.PLANE_DTYPE)
    B = np.zeros((F, cap_b), SP.SUPPOSED_DTYPE)
    ca, cb = np.zeros(F, np.int32), np.zeros(F, np.int32)
    moff = boff = 0
    max_map = 0
    for f in range(F):
        sc = synth.Scene(f % 5, n_boxes=f % 4)
        m, b = _map(rng, sc)
        m = m.copy()
        m["boundary_offset"] += boff
        T, c, _ = synth.assoc_frame_planes(sc, 7 * f, rng, n_faces=5, n_random=f % 3)
        na = min(len(c), int(rng.integers(0, cap_a + 1)))
        nb = min(len(c) - na, cap_b)
        A[f, :na]["coef"], B[f, :nb]["coef"] = c[:na], c[na:na + nb]
        ca[f], cb[f] = na, nb
        frames[f]["Tcw"] = T.reshape(16)
        frames[f]["map_offset"], frames[f]["n_map"] = moff, len(m)
        mm = m.copy()
        mm["boundary_offset"] -= boff
        o = OA.associate(T, c[:na + nb], mm, b)
        expect.append((o, moff, na + nb))
        maps.append(m)
        bounds.append(b)
        moff += len(m)
        boff += len(b)
        max_map = max(max_map, len(m))
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()  # noqa
    d_fr, d_A, d_B = dev(frames), dev(A), dev(B)
    d_ca, d_cb = torch.from_numpy(ca).cuda(), torch.from_numpy(cb).cuda()
    d_m, d_b = dev(np.concatenate(maps)), dev(np.concatenate(bounds))
    P = cap_a + cap_b
    out = torch.full((3, F * P), -7, dtype=torch.int32, device="cuda")
    newp = torch.zeros(F, dtype=torch.int32, device="cuda")
    assoc.batch_device(F, d_fr.data_ptr(), d_A.data_ptr(), SP.PLANE_DTYPE.itemsize, d_ca.data_ptr(), cap_a,
                       d_B.data_ptr(), SP.SUPPOSED_DTYPE.itemsize, d_cb.data_ptr(), cap_b, d_m.data_ptr(),
                       d_b.data_ptr(), max_map, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                       newp.data_ptr())
    torch.cuda.synchronize()
    out, newp = out.cpu().numpy().reshape(3, F, P), newp.cpu().numpy()
    for f, (o, moff, n) in enumerate(expect):
        for k, key in enumerate(("match", "parallel", "vertical")):
            want = np.where(o[key] >= 0, o[key] + moff, -1)
            assert np.array_equal(out[k, f, :n], want), (f, key)
        assert bool(newp[f]) == o["new_plane"], f


def test_carried_associations(assoc):
    """TrackLocalMap's AssociatePlanesByBoundary starts from what TrackWithMotionModel's association left
    after the plane-outlier discard (src/Map.cc:230-252 never clears mvpMapPlanes; Tracking.cc:1004-1028):
    at a pose shifted so that some first-call matches miss the distance threshold, those matches are kept.
    GPU and oracle must agree entry for entry, and the carried state must change the result somewhere."""
    import oracle_assoc as OA
    import oracle_track as OT
    import synth
    rng = np.random.default_rng(33)
    n = n_kept = 0
    for seq in range(3):
        sc = synth.Scene(seq, n_boxes=2 + seq)
        m, b = _map(rng, sc)
        for fr in range(0, 150, 10):
            T, c, _ = synth.assoc_frame_planes(sc, fr, rng, n_faces=5, n_random=1)
            a0 = OA.associate(T, c, m, b)
            # a few first-call edges flagged as PoseOptimization outliers (edge order: match, parallel, vertical)
            n_edges = sum(int((a0[k] >= 0).sum()) for k in ("match", "parallel", "vertical"))
            kept = OT.discard_planes(a0, rng.random(n_edges) < 0.25)
            T2 = T.copy()
            T2[:3, 3] += rng.normal(0, 0.15, 3).astype(np.float32)  # the optimized pose, far enough to miss
            o = OA.associate(T2, c, m, b, init=kept)
            g = assoc(T2, c, m, b, init=kept)
            for k in ("match", "parallel", "vertical"):
                assert np.array_equal(g[k], o[k]), (seq, fr, k, g[k], o[k])
            assert g["new_plane"] == o["new_plane"]
            fresh = OA.associate(T2, c, m, b)
            n_kept += int(((fresh["match"] < 0) & (o["match"] >= 0)).sum())
            n += 1
    assert n >= 40 and n_kept > 0, (n, n_kept)


def test_large_map_two_kernel_path(assoc):
    """Maps with more planes than the fused kernel's LDS table holds ((cap_a + cap_b) x max_map floats > 48 KB)
    take the two-kernel path (per (frame, map plane) distance workgroups + the decision walk): same answers."""
    import torch
    import oracle_assoc as OA
    import spslam_assoc as SA
    import spslam_planes as SP
    import synth
    rng = np.random.default_rng(77)
    sc = synth.Scene(1, n_boxes=6)
    m0, b0 = _map(rng, sc)
    reps = -(-200 // len(m0))
    m = np.concatenate([m0] * reps)
    b = np.concatenate([b0] * reps)
    m["boundary_offset"] = np.concatenate([m0["boundary_offset"] + k * len(b0) for k in range(reps)])
    m["world"][len(m0):, 3] += rng.uniform(-0.3, 0.3, len(m) - len(m0)).astype(np.float32)
    F, cap_a, cap_b = 4, 64, 32  # 96 x 200+ x 4 B > 48 KB
    frames = np.zeros(F, SA.ASSOC_FRAME_DTYPE)
    A = np.zeros((F, cap_a), SP.PLANE_DTYPE)
    ca = np.zeros(F, np.int32)
    expect = []
    for f in range(F):
        T, c, _ = synth.assoc_frame_planes(sc, 25 * f, rng, n_faces=6, n_random=2)
        A[f, :len(c)]["coef"] = c
        ca[f] = len(c)
        frames[f]["Tcw"] = T.reshape(16)
        frames[f]["n_map"] = len(m)
        expect.append(OA.associate(T, c, m, b))
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()  # noqa
    d_fr, d_A, d_ca, d_m, d_b = dev(frames), dev(A), torch.from_numpy(ca).cuda(), dev(m), dev(b)
    d_cb = torch.zeros(F, dtype=torch.int32, device="cuda")
    d_B = torch.zeros(F * cap_b * SP.SUPPOSED_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    out = torch.full((3, F * (cap_a + cap_b)), -7, dtype=torch.int32, device="cuda")
    newp = torch.zeros(F, dtype=torch.int32, device="cuda")
    assoc.batch_device(F, d_fr.data_ptr(), d_A.data_ptr(), SP.PLANE_DTYPE.itemsize, d_ca.data_ptr(), cap_a,
                       d_B.data_ptr(), SP.SUPPOSED_DTYPE.itemsize, d_cb.data_ptr(), cap_b, d_m.data_ptr(),
                       d_b.data_ptr(), len(m), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                       newp.data_ptr())
    torch.cuda.synchronize()
    out = out.cpu().numpy().reshape(3, F, cap_a + cap_b)
    for f, o in enumerate(expect):
        n = int(ca[f])
        for k, key in enumerate(("match", "parallel", "vertical")):
            assert np.array_equal(out[k, f, :n], o[key]), (f, key)
        assert bool(newp[f]) == o["new_plane"], f
