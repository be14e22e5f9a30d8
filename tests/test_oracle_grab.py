"""CPU checks of the GrabImageRGBD oracle (oracle/oracle_grab.py, src/Tracking.cc:208-229):
OpenCV's published 8U RGB2GRAY values and the convertTo scale."""
import numpy as np

import oracle_grab as OG


def test_cvtcolor_known_answers():
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [128, 128, 128]]], np.uint8)
    # OpenCV: pure red -> 76, green -> 150, blue -> 29 (RGB2GRAY); white stays 255, gray stays gray
    assert list(OG.cvt_gray(px, rgb=True)[0]) == [76, 150, 29, 255, 0, 128]
    # BGR order swaps the red and blue weights
    assert list(OG.cvt_gray(px, rgb=False)[0]) == [29, 150, 76, 255, 0, 128]
    # 4 channels: alpha ignored
    rgba = np.concatenate([px, np.full(px.shape[:2] + (1,), 7, np.uint8)], -1)
    assert np.array_equal(OG.cvt_gray(rgba, rgb=True), OG.cvt_gray(px, rgb=True))


def test_cvtcolor_matches_float_weights_within_one():
    rng = np.random.default_rng(0)
    c = rng.integers(0, 256, (64, 64, 3), dtype=np.uint8)
    want = 0.299 * c[..., 0] + 0.587 * c[..., 1] + 0.114 * c[..., 2]
    assert np.abs(OG.cvt_gray(c).astype(np.float64) - want).max() <= 0.51


def test_depth_conversion():
    s = OG.depth_scale(5000.0)
    assert s == np.float32(np.float32(1) / np.float32(5000))
    d = np.array([[0, 1, 5000, 65535]], np.uint16)
    z = OG.convert_depth(d, s)
    assert z.dtype == np.float32 and z[0, 2] == np.float32(5000) * s and z[0, 0] == 0
    f = np.array([[1.5, 2.25]], np.float32)
    assert np.array_equal(OG.convert_depth(f, OG.depth_scale(1.0)), f)
    assert OG.depth_scale(0.0) == 1.0
