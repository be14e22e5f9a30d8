"""CPU tests of the ORB oracle (oracle/orb_oracle.cpp) -- the parity checker.

The reference ships no tests or fixtures, so the oracle is
pinned by independent known-answer tests of each inherited routine, written
from the published algorithms (OpenCV FAST-9/16 + cornerScore, INTER_LINEAR
8U fixed point, bit-exact GaussianBlur, fastAtan2, glibc sinf/cosf), and by
the committed golden fixtures in tests/golden/ (regression pins).
"""
import math

import numpy as np
import pytest

import oracle_ctypes as O

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def corner_score_ref(img, y, x, threshold):
    """OpenCV cornerScore<16> scalar loop (features2d/fast_score.cpp), verbatim algorithm."""
    v = int(img[y, x])
    d = [v - int(img[y + dy, x + dx]) for dx, dy in CIRCLE]
    d = d + d[:9]
    a0 = threshold
    for k in range(0, 16, 2):
        a = min(d[k + 1], d[k + 2], d[k + 3])
        if a <= a0:
            continue
        a = min(a, d[k + 4], d[k + 5], d[k + 6], d[k + 7], d[k + 8])
        a0 = max(a0, min(a, d[k]))
        a0 = max(a0, min(a, d[k + 9]))
    b0 = -a0
    for k in range(0, 16, 2):
        b = max(d[k + 1], d[k + 2], d[k + 3], d[k + 4], d[k + 5])
        if b >= b0:
            continue
        b = max(b, d[k + 6], d[k + 7], d[k + 8])
        b0 = min(b0, max(b, d[k]))
        b0 = min(b0, max(b, d[k + 9]))
    return -b0 - 1


def is_corner_ref(img, y, x, t):
    v = int(img[y, x])
    s = [int(img[y + dy, x + dx]) for dx, dy in CIRCLE]
    for sign in (1, -1):
        run = 0
        for k in range(25):
            if sign * (s[k % 16] - v) > t:
                run += 1
                if run >= 9:
                    return True
            else:
                run = 0
    return False


def fast_ref(img, t):
    """OpenCV FAST_t<16> with nonmax suppression, pure Python (small images only)."""
    h, w = img.shape
    sc = np.zeros((h, w), np.int32)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            if is_corner_ref(img, y, x, t):
                sc[y, x] = corner_score_ref(img, y, x, t)
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            s = sc[y, x]
            if s and all(s > sc[y + dy, x + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dy or dx):
                out.append((x, y, s))
    return out


def test_fast_single_corner_kat():
    img = np.full((9, 9), 100, np.uint8)
    img[4, 4] = 200  # bright center, uniform ring: corner with score min(d)-1 = 99
    k = O.fast(img, 20)
    assert len(k) == 1 and (k[0]["x"], k[0]["y"], k[0]["response"]) == (4, 4, 99)


def test_fast_arc_length_kat():
    """8 contiguous darker pixels are not a corner, 9 are."""
    for n, expect in ((8, 0), (9, 1)):
        img = np.full((9, 9), 100, np.uint8)
        for k in range(n):
            dx, dy = CIRCLE[k]
            img[4 + dy, 4 + dx] = 10
        assert len(O.fast(img, 20)) == expect


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_fast_matches_opencv_algorithm(seed):
    rng = np.random.default_rng(seed)
    img = (rng.integers(0, 4, (24, 26)) * 60 + rng.integers(0, 20, (24, 26))).astype(np.uint8)
    for t in (7, 20):
        got = [(int(k["x"]), int(k["y"]), int(k["response"])) for k in O.fast(img, t)]
        assert got == fast_ref(img, t)


def test_fast_atan2_kat():
    for y, x in ((0.0, 1.0), (1.0, 0.0), (0.0, -1.0), (-1.0, 0.0), (1.0, 1.0), (-3.0, 4.0)):
        a = O.fast_atan2(y, x)
        ref = math.degrees(math.atan2(y, x)) % 360.0
        assert abs(a - ref) < 0.02, (y, x, a, ref)
    assert O.fast_atan2(0.0, 1.0) == 0.0 and O.fast_atan2(1.0, 0.0) == 90.0


def test_glibc_sincos_restatement_matches_libm():
    import ctypes
    import ctypes.util
    libm = ctypes.CDLL(ctypes.util.find_library("m"))
    libm.sinf.restype = libm.cosf.restype = ctypes.c_float
    libm.sinf.argtypes = libm.cosf.argtypes = [ctypes.c_float]
    xs = np.random.default_rng(0).uniform(0, 2 * math.pi, 20000).astype(np.float32)
    xs = np.concatenate([xs, np.float32([0, 1e-5, 0.7853982, 1.5707964, 3.1415927, 6.2831855])])
    for x in xs:
        assert O.sinf(float(x)) == libm.sinf(float(x)) and O.cosf(float(x)) == libm.cosf(float(x)), x


def test_gaussian_blur_kat():
    img = np.zeros((15, 15), np.uint8)
    img[7, 7] = 255
    out = O.gaussian_blur(img)
    k = np.array([18, 34, 48, 56, 48, 34, 18])
    ref = (np.outer(k, k) * 255 + (1 << 15)) >> 16
    assert np.array_equal(out[4:11, 4:11], ref.astype(np.uint8))
    assert np.array_equal(O.gaussian_blur(np.full((10, 12), 77, np.uint8)), np.full((10, 12), 77, np.uint8))


def resize_ref(src, dw, dh):
    """OpenCV INTER_LINEAR 8U (coefficients INTER_RESIZE_COEF_BITS=11), numpy restatement."""
    sh, sw = src.shape
    sx_ = 1.0 / (dw / sw)
    sy_ = 1.0 / (dh / sh)
    fx = np.float32((np.arange(dw) + 0.5) * sx_ - 0.5)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx).astype(np.float32)
    neg = sx < 0
    fx[neg], sx[neg] = 0, 0
    tail = sx + 1 >= sw
    clamp = sx >= sw - 1
    fx[clamp], sx[clamp] = 0, sw - 1
    a0 = np.rint((np.float32(1) - fx) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(fx * np.float32(2048)).astype(np.int64)
    fy = np.float32((np.arange(dh) + 0.5) * sy_ - 0.5)
    sy = np.floor(fy).astype(np.int64)
    fy = (fy - sy).astype(np.float32)
    b0 = np.rint((np.float32(1) - fy) * np.float32(2048)).astype(np.int64)
    b1 = np.rint(fy * np.float32(2048)).astype(np.int64)
    S = src.astype(np.int64)
    sx1 = np.minimum(sx + 1, sw - 1)

    def hrow(y):
        r = S[y, sx] * a0 + S[y, sx1] * a1
        return np.where(tail, S[y, sx] * 2048, r)

    out = np.zeros((dh, dw), np.uint8)
    for y in range(dh):
        r0, r1 = hrow(min(max(sy[y], 0), sh - 1)), hrow(min(max(sy[y] + 1, 0), sh - 1))
        out[y] = ((((b0[y] * (r0 >> 4)) >> 16) + ((b1[y] * (r1 >> 4)) >> 16) + 2) >> 2).astype(np.uint8)
    return out


@pytest.mark.parametrize("shape", [((480, 640), (400, 533)), ((61, 77), (51, 64))])
def test_resize_matches_numpy_restatement(shape):
    (sh, sw), (dh, dw) = shape
    src = np.random.default_rng(3).integers(0, 256, (sh, sw), dtype=np.uint8)
    assert np.array_equal(O.resize_linear(src, dw, dh), resize_ref(src, dw, dh))


def test_brief_constant_image_is_zero():
    img = np.full((64, 64), 90, np.uint8)
    for ang in (0.0, 33.3, 271.0):
        assert not O.descriptor(img, 32.0, 32.0, ang).any()


def test_tables_match_reference_geometry():
    orb = O.OrbOracle()
    assert list(orb.features_per_level()) == [217, 181, 151, 126, 105, 87, 73, 60]
    assert list(orb.umax()) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    sc = orb.scale_tables()[0]
    assert sc[0] == 1.0 and abs(sc[7] - 1.2 ** 7) < 1e-5


def test_extract_properties(synth_frames):
    orb = O.OrbOracle()
    g = synth_frames[0][0]
    kps, desc = orb.extract(g)
    assert 1000 <= len(kps) <= 1016 and desc.shape == (len(kps), 32)
    assert np.all(np.diff(kps["octave"]) >= 0)              # level order (:1076-1104)
    assert np.all(kps["x"] >= 0) and np.all(kps["x"] < 640) and np.all(kps["y"] < 480)
    assert np.all((kps["angle"] >= 0) & (kps["angle"] < 360))
    assert np.all(kps["class_id"] == -1)
    # per-level counts reach the quota (DistributeOctTree may overshoot by <= 3)
    q = orb.features_per_level()
    counts = np.bincount(kps["octave"], minlength=8)
    assert np.all(counts >= np.minimum(q, 1)) and np.all(counts <= q + 3)
    # empty image: no output
    k0, d0 = orb.extract(np.zeros((0, 0), np.uint8))
    assert len(k0) == 0


def test_golden_orb_fixture():
    """Regression pin: committed keypoints/descriptors of a synthetic frame."""
    import pathlib
    import synth
    p = pathlib.Path(__file__).parent / "golden" / "orb_seq0_f5.npz"
    ref = np.load(p)
    sc = synth.Scene(0)
    g, _, _ = sc.render(sc.pose(5), noise_seed=5)
    assert int(ref["gray_sum"]) == int(g.astype(np.int64).sum()), "synthetic renderer changed"
    kps, desc = O.OrbOracle().extract(g)
    assert np.array_equal(kps.view(np.uint8), ref["kps"].view(np.uint8))
    assert np.array_equal(desc, ref["desc"])
