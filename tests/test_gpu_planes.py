"""GPU parity: plane extraction (Frame::ComputePlanesFromOrganizedPointCloud,
src/Frame.cc:854-936, with PCL 1.8 IntegralImageNormalEstimation +
OrganizedMultiPlaneSegmentation) vs the CPU oracle.

Bar: organized cloud, chamfer distance map and normals bit-exact; labels,
inlier index lists and contours identical; plane coefficients within 1e-4.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
COEF_TOL = 1e-4


@pytest.fixture(scope="module")
def ctx():
    import spslam_gpu
    import spslam_planes
    import synth
    K = synth.TUM3
    ex = spslam_gpu.OrbExtractor(max_batch=4)
    pe = spslam_planes.PlaneExtractor(ex, K["fx"], K["fy"], K["cx"], K["cy"])
    pe.keep_labels()
    yield ex, pe
    ex.close()


@pytest.fixture(scope="module")
def depth_frames():
    import oracle_planes
    import synth
    out = []
    for seq, frames, boxes in ((0, (0, 20, 45), 3), (2, (10,), 6)):
        sc = synth.Scene(seq, n_boxes=boxes)
        for fi in frames:
            _, d, _ = sc.render(sc.pose(fi), noise_seed=fi)
            out.append(oracle_planes.depth_to_float(d))
    return out


def _oracle(depth, scale=1.0, min_size=500):
    import oracle_planes
    import synth
    K = synth.TUM3
    po = oracle_planes.PlaneOracle()
    res = po.extract(depth, K["fx"] * scale, K["fy"] * scale, K["cx"] * scale, K["cy"] * scale, min_size=min_size)
    return po, res


def _compare(pe, depth, k, scale=1.0, min_size=500):
    """Every stage and output of one frame against the oracle; returns (#planes, #models)."""
    po, ro = _oracle(depth, scale, min_size)
    rg = pe(depth)
    assert np.array_equal(pe.debug(0, 0), po.cloud(), equal_nan=True), f"frame {k}: cloud"
    assert np.array_equal(pe.debug(0, 2), po.distance(), equal_nan=True), f"frame {k}: distance map"
    ng, no = pe.debug(0, 1), po.normals()
    assert np.array_equal(np.isnan(ng), np.isnan(no)), f"frame {k}: normal validity"
    m = ~np.isnan(no)
    assert np.array_equal(ng[m], no[m]), f"frame {k}: normals"
    assert np.array_equal(pe.debug(0, 3), po.labels(False)), f"frame {k}: CC labels"
    assert len(rg["coef"]) == len(ro["coef"]), f"frame {k}: {len(rg['coef'])} vs {len(ro['coef'])} planes"
    for j in range(len(ro["coef"])):
        assert np.abs(rg["coef"][j] - ro["coef"][j]).max() <= COEF_TOL * max(1.0, abs(ro["coef"][j][3])), \
            f"frame {k} plane {j}: {rg['coef'][j]} vs {ro['coef'][j]}"
        assert np.array_equal(rg["coef"][j], ro["coef"][j]), f"frame {k} plane {j}: coef not bit-exact"
        assert np.array_equal(rg["inliers"][j], ro["inliers"][j]), f"frame {k} plane {j}: inliers"
        assert np.array_equal(rg["contour"][j], ro["contour"][j]), f"frame {k} plane {j}: contour"
    return len(ro["coef"]), po.n_models


def _refine_path(n_models):
    """Which refinement the kernel takes (plane_segment.hip phase K): fast narrow (<= 14 models, 16-bit
    descriptors), fast wide (<= 30, 32-bit descriptors) or the general 64-bit path."""
    return "narrow" if n_models <= 14 else "wide" if n_models <= 30 else "general"


def test_planes_many_models(ctx):
    """All three refinement paths at 640x480: small MinSize values give more candidate models per frame."""
    import oracle_planes
    import synth
    _, pe = ctx
    sc = synth.Scene(3, n_boxes=8)
    models = []
    for min_size in (500, 30, 15):
        pe.configure(min_size=min_size)
        for fi in (0, 15, 30):
            _, d, _ = sc.render(sc.pose(fi), noise_seed=fi)
            models.append(_compare(pe, oracle_planes.depth_to_float(d), fi, min_size=min_size)[1])
    pe.configure(min_size=500)
    assert {_refine_path(m) for m in models} == {"narrow", "wide", "general"}, models


def test_planes_c5_size():
    """1280x960 (BASELINE config C5): maps in global memory, 8 positions per lane; narrow and wide refinement."""
    import oracle_planes
    import spslam_gpu
    import spslam_planes
    import synth
    K = synth.TUM3
    ex = spslam_gpu.OrbExtractor(nfeatures=4000, width=1280, height=960, max_batch=1)
    try:
        for min_size, expect in ((500, "narrow"), (4000, "narrow"), (30, "wide")):
            pe = spslam_planes.PlaneExtractor(ex, K["fx"] * 2, K["fy"] * 2, K["cx"] * 2, K["cy"] * 2, 1280, 960,
                                              min_size=min_size)
            sc = synth.Scene(1, n_boxes=8)
            _, d, _ = sc.render(sc.pose(5), 1280, 960, noise_seed=5)
            n, nm = _compare(pe, oracle_planes.depth_to_float(d), 5, scale=2.0, min_size=min_size)
            assert n >= 2 and _refine_path(nm) == expect, (n, nm)
    finally:
        ex.close()


def test_planes_match_oracle(ctx, depth_frames):
    ex, pe = ctx
    total = 0
    for k, depth in enumerate(depth_frames):
        po, ro = _oracle(depth)
        rg = pe(depth)
        # stages
        assert np.array_equal(pe.debug(0, 0), po.cloud()), f"frame {k}: cloud"
        assert np.array_equal(pe.debug(0, 2), po.distance()), f"frame {k}: distance map"
        ng, no = pe.debug(0, 1), po.normals()
        assert np.array_equal(np.isnan(ng), np.isnan(no)), f"frame {k}: normal validity"
        m = ~np.isnan(no)
        assert np.array_equal(ng[m], no[m]), f"frame {k}: normals differ at {np.nonzero((ng != no) & m)[0][:5]}"
        assert np.array_equal(pe.debug(0, 3), po.labels(False)), f"frame {k}: CC labels"
        # outputs
        assert len(rg["coef"]) == len(ro["coef"]), f"frame {k}: {len(rg['coef'])} vs {len(ro['coef'])} planes"
        for j in range(len(ro["coef"])):
            assert np.abs(rg["coef"][j] - ro["coef"][j]).max() <= COEF_TOL * max(1.0, abs(ro["coef"][j][3])), \
                f"frame {k} plane {j}: {rg['coef'][j]} vs {ro['coef'][j]}"
            assert np.array_equal(rg["coef"][j], ro["coef"][j]), f"frame {k} plane {j}: coef not bit-exact"
            assert np.array_equal(rg["inliers"][j], ro["inliers"][j]), f"frame {k} plane {j}: inliers"
            assert np.array_equal(rg["contour"][j], ro["contour"][j]), f"frame {k} plane {j}: contour"
        total += len(ro["coef"])
    assert total >= 6


def test_zero_depth_frame(ctx):
    _, pe = ctx
    rg = pe(np.zeros((480, 640), np.float32))
    assert len(rg["coef"]) == 0


def test_batch_device(ctx, depth_frames):
    torch = pytest.importorskip("torch")
    import spslam_planes
    ex, pe = ctx
    n = 4
    d = torch.from_numpy(np.stack(depth_frames[:n])).cuda()
    planes = torch.zeros(n * pe.planes_cap * 8, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    inl = torch.zeros(n * pe.inlier_cap, dtype=torch.int32, device="cuda")
    con = torch.zeros(n * pe.contour_cap, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    pe.extract_batch_device(d.data_ptr(), n, 640 * 480, 640, planes.data_ptr(), cnt.data_ptr(), inl.data_ptr(),
                            con.data_ptr(), s)
    torch.cuda.synchronize()
    P = planes.cpu().numpy().view(spslam_planes.PLANE_DTYPE).reshape(n, pe.planes_cap)
    C, I = cnt.cpu().numpy(), inl.cpu().numpy().reshape(n, -1)
    for f in range(n):
        one = pe(depth_frames[f])
        assert C[f] == len(one["coef"])
        for j in range(C[f]):
            p = P[f, j]
            assert np.array_equal(p["coef"], one["coef"][j])
            assert np.array_equal(I[f, p["inlier_offset"]:p["inlier_offset"] + p["n_inliers"]], one["inliers"][j])
