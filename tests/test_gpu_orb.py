"""GPU parity: gfx950 ORB extractor (through the C ABI) vs the CPU oracle.

Bar: bit-exact for every stage -- pyramid levels, blurred levels, per-cell FAST
candidates (position, score, order), DistributeOctTree output (order
included), final keypoints (all cv::KeyPoint fields) and descriptors.
Reference: src/ORBextractor.cc (stage line numbers in the test names' docstrings).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import spslam_gpu
    ex = spslam_gpu.OrbExtractor(max_batch=4)
    yield ex
    ex.close()


@pytest.fixture(scope="module")
def oracle():
    import oracle_ctypes
    return oracle_ctypes.OrbOracle()


def _assert_kps_equal(a, b, what):
    assert len(a) == len(b), f"{what}: count {len(a)} vs {len(b)}"
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        bad = np.nonzero(a[f] != b[f])[0]
        assert bad.size == 0, f"{what}: field {f} differs at {bad[:10]} ({a[f][bad[:3]]} vs {b[f][bad[:3]]})"


def test_tables_match_oracle(gpu, oracle):
    """ORBextractor ctor tables, src/ORBextractor.cc:415-446."""
    t = gpu.tables()
    sc, isc, s2, is2 = oracle.scale_tables()
    assert np.array_equal(t["scale"], sc) and np.array_equal(t["inv_scale"], isc)
    assert np.array_equal(t["sigma2"], s2) and np.array_equal(t["inv_sigma2"], is2)
    assert np.array_equal(t["features"], oracle.features_per_level())


@pytest.mark.parametrize("fi", [0, 1, 2, 3])
def test_stages_bit_exact(gpu, oracle, synth_frames, fi):
    """Pyramid (:1107-1132), blur (:1085-1086), cell FAST (:789-829), octree (:834-847)."""
    g = synth_frames[fi][0]
    gpu(g)
    oracle.pyramid(g)
    for level in range(8):
        assert np.array_equal(gpu.debug_stage(0, level, 0), oracle.level_image(level)), f"pyramid L{level}"
        assert np.array_equal(gpu.debug_stage(0, level, 1), oracle.level_blurred(level)), f"blur L{level}"
        cg, co = gpu.debug_stage(0, level, 2), oracle.level_candidates(level)
        assert len(cg) == len(co), f"candidates L{level}: {len(cg)} vs {len(co)}"
        for f in ("x", "y", "response"):
            assert np.array_equal(cg[f], co[f]), f"candidates L{level} field {f}"
        kg, ko = gpu.debug_stage(0, level, 3), oracle.level_keypoints(level)
        assert len(kg) == len(ko), f"octree L{level}: {len(kg)} vs {len(ko)}"
        for f in ("x", "y", "response", "octave", "size"):
            assert np.array_equal(kg[f], ko[f]), f"octree L{level} field {f}"


@pytest.mark.parametrize("fi", [0, 1, 2, 3])
def test_extract_bit_exact(gpu, oracle, synth_frames, fi):
    """ORBextractor::operator(), src/ORBextractor.cc:1043-1105."""
    g = synth_frames[fi][0]
    kg, dg = gpu(g)
    ko, do = oracle.extract(g)
    _assert_kps_equal(kg, ko, f"frame {fi}")
    assert np.array_equal(dg, do), f"descriptors differ in {np.nonzero((dg != do).any(1))[0][:10]}"


def test_constant_image_has_no_keypoints(gpu, oracle):
    g = np.full((480, 640), 128, np.uint8)
    kg, dg = gpu(g)
    ko, _ = oracle.extract(g)
    assert len(kg) == len(ko) == 0


def test_noise_image(gpu, oracle):
    """Dense corners everywhere: stresses the octree final phase and cell capacity."""
    rng = np.random.default_rng(5)
    g = rng.integers(0, 256, (480, 640), dtype=np.uint8)
    kg, dg = gpu(g)
    ko, do = oracle.extract(g)
    _assert_kps_equal(kg, ko, "noise")
    assert np.array_equal(dg, do)


def test_low_contrast_uses_min_threshold(gpu, oracle, synth_frames):
    """Contrast squeezed so most cells find nothing at iniThFAST=20 (retry at 7, :812-816)."""
    g = synth_frames[0][0].astype(np.int32)
    g = (128 + (g - 128) // 6).astype(np.uint8)
    kg, dg = gpu(g)
    ko, do = oracle.extract(g)
    assert len(ko) > 100
    _assert_kps_equal(kg, ko, "low contrast")
    assert np.array_equal(dg, do)


def test_empty_image_is_noop(gpu):
    kps, desc = gpu(np.zeros((0, 0), np.uint8))
    assert len(kps) == 0 and len(desc) == 0


def test_batch_device_matches_single(gpu, synth_frames):
    torch = pytest.importorskip("torch")
    import spslam_gpu
    frames = np.stack([f[0] for f in synth_frames])
    dev = torch.from_numpy(frames).cuda()
    cap = gpu.max_kp
    kps = torch.zeros((4, cap, 7), dtype=torch.float32, device="cuda")
    desc = torch.zeros((4, cap, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(4, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    gpu.extract_batch_device(dev.data_ptr(), 4, 640 * 480, 640, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(),
                             cap, stream)
    torch.cuda.synchronize()
    kb = kps.cpu().numpy().view(spslam_gpu.KEYPOINT_DTYPE).reshape(4, cap)
    db, nb = desc.cpu().numpy(), cnt.cpu().numpy()
    for i in range(4):
        k1, d1 = gpu(frames[i])
        assert nb[i] == len(k1)
        _assert_kps_equal(kb[i, :nb[i]], k1, f"batch frame {i}")
        assert np.array_equal(db[i, :nb[i]], d1)


def test_hd_config_nf4000(synth_frames):
    """C5-style geometry: 1280x960, nFeatures=4000."""
    import oracle_ctypes
    import spslam_gpu
    import synth
    sc = synth.Scene(3, n_boxes=5)
    g, _, _ = sc.render(sc.pose(5), 1280, 960)
    ex = spslam_gpu.OrbExtractor(nfeatures=4000, width=1280, height=960)
    try:
        kg, dg = ex(g)
    finally:
        ex.close()
    ko, do = oracle_ctypes.OrbOracle(nfeatures=4000).extract(g, cap=20000)
    _assert_kps_equal(kg, ko, "1280x960")
    assert np.array_equal(dg, do)
