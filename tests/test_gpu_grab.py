"""GPU parity of GrabImageRGBD's image preparation (spslam_grab_rgbd*, src/Tracking.cc:208-229)
against oracle/oracle_grab.py: every channel count / order, u16 and f32 depth, the vector path
(width % 8 == 0) and the scalar path (odd width, padded strides), bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ex():
    import spslam_gpu
    e = spslam_gpu.OrbExtractor(max_batch=1)
    yield e
    e.close()


@pytest.mark.parametrize("channels,rgb", [(1, True), (3, True), (3, False), (4, True), (4, False)])
@pytest.mark.parametrize("w,h", [(640, 480), (333, 77)])
@pytest.mark.parametrize("u16", [True, False])
def test_grab_single(ex, channels, rgb, w, h, u16):
    import oracle_grab as OG
    import spslam_grab
    rng = np.random.default_rng(w * 7 + channels + 2 * int(rgb) + int(u16))
    shape = (h, w) if channels == 1 else (h, w, channels)
    color = rng.integers(0, 256, shape, dtype=np.uint8)
    if u16:
        depth = rng.integers(0, 65536, (h, w), dtype=np.uint16)
        factor = 5000.0
    else:
        depth = (rng.random((h, w)) * 8).astype(np.float32)
        factor = 1000.0
    g = spslam_grab.Grabber(ex, channels=channels, rgb=rgb, depth_u16=u16, depth_factor=factor)
    gray, z = g(color, depth)
    assert np.array_equal(gray, OG.cvt_gray(color, rgb=rgb))
    assert z.tobytes() == OG.convert_depth(depth, OG.depth_scale(factor)).tobytes()


def test_grab_float_depth_factor_one_is_a_copy(ex):
    import spslam_grab
    depth = np.array([[1.0, np.nan, 0.0, 3.25] * 2], np.float32)
    color = np.zeros((1, 8, 3), np.uint8)
    _, z = spslam_grab.Grabber(ex, depth_u16=False, depth_factor=1.0)(color, depth)
    assert z.tobytes() == depth.tobytes()


def test_grab_batch_device_matches_single(ex):
    import torch

    import oracle_grab as OG
    import spslam_grab
    rng = np.random.default_rng(5)
    B, h, w = 5, 96, 128
    color = rng.integers(0, 256, (B, h, w, 3), dtype=np.uint8)
    depth = rng.integers(0, 65536, (B, h, w), dtype=np.uint16)
    g = spslam_grab.Grabber(ex)
    d_c = torch.from_numpy(color).cuda()
    d_d = torch.from_numpy(depth.view(np.int16)).cuda()
    d_g = torch.zeros((B, h, w), dtype=torch.uint8, device="cuda")
    d_z = torch.zeros((B, h, w), dtype=torch.float32, device="cuda")
    g.batch_device(B, d_c.data_ptr(), h * w * 3, w * 3, d_d.data_ptr(), h * w, w, w, h, d_g.data_ptr(),
                   d_z.data_ptr())
    torch.cuda.synchronize()
    s = OG.depth_scale(5000.0)
    for f in range(B):
        assert np.array_equal(d_g[f].cpu().numpy(), OG.cvt_gray(color[f]))
        assert d_z[f].cpu().numpy().tobytes() == OG.convert_depth(depth[f], s).tobytes()


@pytest.mark.parametrize("w,h,dis", [(640, 480, 3), (333, 77, 4)])
def test_grab_fused_cloud(w, h, dis):
    """spslam_grab_fuse_cloud: the grab writes the plane stage's organized cloud (Frame.cc:857-874) in the same
    pass -- bit-identical to the oracle's, for the vector path (640x480, Cloud.Dis 3) and the scalar path (odd width,
    Cloud.Dis 4) -- and the next extraction over that depth uses it as it is (shown by changing the depth after the
    grab: the cloud stays the grab's), while an extraction over other depth makes its own; the plane results of a
    fused step equal the unfused ones."""
    import torch

    import oracle_grab as OG
    import oracle_planes
    import spslam_gpu
    import spslam_grab
    import spslam_planes
    import synth
    K = synth.TUM3
    B = 3
    ex = spslam_gpu.OrbExtractor(max_batch=B)  # (ORB geometry unused: the plane stage has its own size)
    try:
        pe = spslam_planes.PlaneExtractor(ex, K["fx"], K["fy"], K["cx"], K["cy"], w, h, cloud_dis=dis)
        g = spslam_grab.Grabber(ex)
        sc = synth.Scene(1, n_boxes=4)
        depth = np.stack([sc.render(sc.pose(5 * f), w, h, noise_seed=f)[1] for f in range(B)])
        color = np.random.default_rng(3).integers(0, 256, (B, h, w, 3), dtype=np.uint8)
        d_c = torch.from_numpy(color).cuda()
        d_d = torch.from_numpy(depth.view(np.int16)).cuda()
        z = np.stack([OG.convert_depth(depth[f], OG.depth_scale(5000.0)) for f in range(B)])

        def run(fuse, change_depth=False):
            g.fuse_cloud(fuse)
            d_g = torch.zeros((B, h, w), dtype=torch.uint8, device="cuda")
            d_z = torch.zeros((B, h, w), dtype=torch.float32, device="cuda")
            g.batch_device(B, d_c.data_ptr(), h * w * 3, w * 3, d_d.data_ptr(), h * w, w, w, h, d_g.data_ptr(),
                           d_z.data_ptr())
            torch.cuda.synchronize()
            if change_depth:
                d_z.mul_(2.0)
                torch.cuda.synchronize()
            out = [torch.zeros(n, dtype=torch.int32, device="cuda") for n in
                   (pe.planes_cap * B * spslam_planes.PLANE_DTYPE.itemsize // 4, B, pe.inlier_cap * B,
                    pe.contour_cap * B)]
            pe.extract_batch_device(d_z.data_ptr(), B, h * w, w, *[o.data_ptr() for o in out])
            torch.cuda.synchronize()
            assert d_z[0].cpu().numpy().tobytes() == (z[0] * (2 if change_depth else 1)).tobytes()
            return [pe.debug(f, 0) for f in range(B)], [o.cpu().numpy() for o in out]

        clouds, res = run(True)
        for f in range(B):
            po = oracle_planes.PlaneOracle()
            po.extract(z[f], K["fx"], K["fy"], K["cx"], K["cy"], cloud_dis=dis)
            assert np.array_equal(clouds[f], po.cloud(), equal_nan=True), f"frame {f}: fused cloud"
        clouds2, res2 = run(False)
        for f in range(B):
            assert np.array_equal(clouds2[f], clouds[f], equal_nan=True)
        for a, b in zip(res, res2):
            assert np.array_equal(a, b)
        # the tagged cloud is used as it is: the doubled depth does not reach the cloud
        stale, _ = run(True, change_depth=True)
        for f in range(B):
            assert np.array_equal(stale[f], clouds[f], equal_nan=True)
        # an extraction over other depth makes its own cloud (the tag names the grab's output only)
        _, _ = run(True)
        d_x = torch.from_numpy(2 * z).cuda()
        out = [torch.zeros(n, dtype=torch.int32, device="cuda") for n in
               (pe.planes_cap * B * spslam_planes.PLANE_DTYPE.itemsize // 4, B, pe.inlier_cap * B, pe.contour_cap * B)]
        pe.extract_batch_device(d_x.data_ptr(), B, h * w, w, *[o.data_ptr() for o in out])
        torch.cuda.synchronize()
        po = oracle_planes.PlaneOracle()
        po.extract(2 * z[0], K["fx"], K["fy"], K["cx"], K["cy"], cloud_dis=dis)
        assert np.array_equal(pe.debug(0, 0), po.cloud(), equal_nan=True)
    finally:
        ex.close()
