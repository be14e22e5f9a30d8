"""Diagnostic: per-phase time of plane_segment_kernel from its in-kernel stamps.

    python tools/seg_phases.py [--batch B]

Runs the bench pipeline's plane stage and prints, per phase, the mean and
max over frames of the s_memrealtime deltas (100 MHz ticks -> microseconds).
"""
import argparse
import ctypes
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sp-slam_amd"))
sys.path.insert(0, str(ROOT))

PHASES = ["A runs", "B union", "C flatten", "D labels+sizes", "E+F big+tags", "G covariance", "H models",
          "K refine", "L+M inliers", "N contours"]
ORDER = [15, 0, 1, 2, 3, 5, 6, 7, 8, 4, 9]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--config", default="c2")
    a = ap.parse_args()
    import torch
    import pipeline
    hp = pipeline.HotPath(a.batch, **pipeline.CONFIGS[a.config])
    for _ in range(3):
        hp.planes()
    torch.cuda.synchronize()
    lib = hp.ex.lib
    ts = np.zeros((a.batch, 16), np.int64)
    n = ctypes.c_int()
    for f in range(a.batch):
        lib.spslam_planes_debug(hp.ex.ctx, f, 4, ts[f].ctypes.data_as(ctypes.c_void_p), ctypes.byref(n))
    d = np.diff(ts[:, ORDER], axis=1) / 100.0  # us
    tot = (ts[:, 9] - ts[:, 15]) / 100.0
    for k, name in enumerate(PHASES):
        print(f"{name:18s} mean {d[:, k].mean():9.1f} us   max {d[:, k].max():9.1f} us")
    print(f"{'total':18s} mean {tot.mean():9.1f} us   max {tot.max():9.1f} us")
    k = ts[:, 10] > 0
    ref = (ts[:, 8] - ts[:, 7]) / 100.0
    print(f"fast-path frames {k.sum()} / {len(k)}: refine mean {ref[k].mean() if k.any() else 0:.1f} us, "
          f"max {ref[k].max() if k.any() else 0:.1f};  general-path refine mean "
          f"{ref[~k].mean() if (~k).any() else 0:.1f} us, max {ref[~k].max() if (~k).any() else 0:.1f}")
    nm = ts[:, 13]
    print("models per frame: narrow (<=14)", int((nm <= 14).sum()), " wide (15-30)", int(((nm > 14) & (nm <= 30)).sum()),
          " general (>30)", int((nm > 30).sum()), " max", int(nm.max()))
    print("total per frame (us) percentiles 50/90/99/100:", np.percentile(tot, [50, 90, 99, 100]).round(1).tolist())
    if k.any():
        print(f"refine: cand-bitmap {((ts[k, 10] - ts[k, 7]) / 100).mean():.1f} us, forward "
              f"{((ts[k, 11] - ts[k, 10]) / 100).mean():.1f} us, events {ts[k, 12].mean():.1f}")
    hp.close()


if __name__ == "__main__":
    main()
