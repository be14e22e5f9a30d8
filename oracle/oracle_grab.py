"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Tracking::GrabImageRGBD's image preparation (src/Tracking.cc:208-229) restated
in numpy (integer / single-rounding float work):

* cvtColor(RGB2GRAY / BGR2GRAY / RGBA2GRAY / BGRA2GRAY), OpenCV 3.4 8U path
  (imgproc color_rgb RGB2Gray<uchar>: coefficients R2Y = 4899, G2Y = 9617,
  B2Y = 1868 at yuv_shift = 14, Y = (b*cb + g*cg + r*cr + (1 << 13)) >> 14 --
  the scalar, lookup-table and universal-intrinsic versions all compute this);
  OpenCV's optional IPP path is not restated (DESIGN.md parity semantics);
* Mat::convertTo(CV_32F, alpha) for CV_16U / CV_32F sources: float(src) * (float)alpha
  + 0 in float (cvtScale / cvt_32f), one rounding.
"""
from __future__ import annotations

import numpy as np

R2Y, G2Y, B2Y, SHIFT = 4899, 9617, 1868, 14


def cvt_gray(color, rgb=True):
    c = np.asarray(color, np.uint8)
    if c.ndim == 2:
        return c.copy()
    c = c.astype(np.int64)
    r, b = (c[..., 0], c[..., 2]) if rgb else (c[..., 2], c[..., 0])
    return ((r * R2Y + c[..., 1] * G2Y + b * B2Y + (1 << (SHIFT - 1))) >> SHIFT).astype(np.uint8)


def depth_scale(depth_map_factor):
    """mDepthMapFactor as Tracking.cc:142-146 stores it (float reciprocal, 1 if ~0)."""
    f = np.float32(depth_map_factor)
    return np.float32(1.0) if abs(float(f)) < 1e-5 else np.float32(np.float32(1.0) / f)


def convert_depth(depth, scale):
    d = np.asarray(depth)
    s = np.float32(scale)
    if d.dtype == np.float32 and abs(float(s) - 1.0) <= 1e-5:
        return d.copy()
    return (d.astype(np.float32) * s).astype(np.float32)
