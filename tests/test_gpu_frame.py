"""GPU parity: RGB-D Frame per-keypoint steps (UndistortKeyPoints,
ComputeStereoFromRGBD, AssignFeaturesToGrid; src/Frame.cc:146-181) vs the
CPU oracle (oracle/frame_oracle.cpp).  Bar: bit-exact mvKeysUn, mvDepth,
mvuRight and identical mGrid lists, with and without lens distortion (TUM1
calibration has k1..k3 != 0, TUM3 has none)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TUM1 = dict(fx=517.306408, fy=516.469215, cx=318.643040, cy=255.313989,
            dist=(0.262383, -0.953104, -0.005358, 0.002628, 1.163314), bf=40.0)
TUM3 = dict(fx=535.4, fy=539.2, cx=320.1, cy=247.6, dist=(0, 0, 0, 0, 0), bf=40.0)


@pytest.fixture(scope="module")
def ex():
    import spslam_gpu
    e = spslam_gpu.OrbExtractor(max_batch=4)
    yield e
    e.close()


def _frames():
    import oracle_ctypes
    import oracle_planes
    import synth
    orb = oracle_ctypes.OrbOracle()
    for seq, fi in ((0, 5), (1, 30), (2, 11)):
        sc = synth.Scene(seq)
        g, d, _ = sc.render(sc.pose(fi), noise_seed=fi)
        kps, _ = orb.extract(g)
        yield kps, oracle_planes.depth_to_float(d)


@pytest.mark.parametrize("calib", ["tum1", "tum3"])
def test_frame_rgbd_bit_exact(ex, calib):
    import oracle_frame
    import spslam_frame
    cal = TUM1 if calib == "tum1" else TUM3
    fs = spslam_frame.FrameStage(ex, **cal)
    for kps, depth in _frames():
        kxy = np.stack([kps["x"], kps["y"]], 1)
        o = oracle_frame.frame_rgbd(kxy, depth, **cal)
        r = fs(kps, depth)
        assert np.array_equal(fs.bounds, o["bounds"])
        assert np.array_equal(r["keys_un"]["x"], o["un"][:, 0]) and np.array_equal(r["keys_un"]["y"], o["un"][:, 1])
        for f in ("size", "angle", "response", "octave", "class_id"):
            assert np.array_equal(r["keys_un"][f], kps[f]), f
        assert np.array_equal(r["depth"], o["depth"]) and np.array_equal(r["uright"], o["uright"])
        assert np.array_equal(r["grid_off"], o["grid_off"]) and np.array_equal(r["grid_idx"], o["grid_idx"])
        if calib == "tum1":
            assert not np.array_equal(r["keys_un"]["x"], kps["x"])  # distortion really applied
        assert (r["depth"] > 0).mean() > 0.9


def test_frame_rgbd_empty_and_batch(ex):
    import torch
    import spslam_frame
    import spslam_gpu
    fs = spslam_frame.FrameStage(ex, **TUM3)
    r = fs(np.zeros(0, spslam_gpu.KEYPOINT_DTYPE), np.ones((480, 640), np.float32))
    assert len(r["keys_un"]) == 0 and r["grid_off"][-1] == 0
    frames = list(_frames())
    B, cap = len(frames), max(len(k) for k, _ in frames) + 5
    kp = np.zeros((B, cap), spslam_gpu.KEYPOINT_DTYPE)
    cnt = np.array([len(k) for k, _ in frames] , np.int32)
    cnt[1] = 0  # a frame without keypoints: its plane counts are zeroed (Frame.cc:148-149)
    for f, (k, _) in enumerate(frames):
        kp[f, :len(k)] = k
    dk = torch.from_numpy(kp.view(np.uint8).copy()).cuda()
    dc = torch.from_numpy(cnt).cuda()
    dd = torch.from_numpy(np.stack([d for _, d in frames])).cuda()
    un = torch.zeros_like(dk)
    dep = torch.zeros(B * cap, dtype=torch.float32, device="cuda")
    ur = torch.zeros_like(dep)
    go = torch.zeros(B * (spslam_frame.N_CELLS + 1), dtype=torch.int32, device="cuda")
    gi = torch.zeros(B * cap, dtype=torch.int32, device="cuda")
    pc = torch.full((B,), 7, dtype=torch.int32, device="cuda")
    fs.batch_device(dk.data_ptr(), dc.data_ptr(), cap, dd.data_ptr(), B, 640 * 480, 640, un.data_ptr(),
                    dep.data_ptr(), ur.data_ptr(), go.data_ptr(), gi.data_ptr(), pc.data_ptr(), None)
    torch.cuda.synchronize()
    un = un.cpu().numpy().view(spslam_gpu.KEYPOINT_DTYPE).reshape(B, cap)
    go = go.cpu().numpy().reshape(B, -1)
    gi = gi.cpu().numpy().reshape(B, cap)
    assert list(pc.cpu().numpy()) == [7, 0, 7]
    for f, (k, d) in enumerate(frames):
        if cnt[f] == 0:
            assert go[f, -1] == 0
            continue
        r = fs(k, d)
        assert np.array_equal(un[f, :cnt[f]].view(np.uint8), r["keys_un"].view(np.uint8))
        assert np.array_equal(go[f], r["grid_off"]) and np.array_equal(gi[f, :go[f, -1]], r["grid_idx"])
