"""Diagnostic: per-phase time of supp_lines_kernel (one workgroup per (frame, boundary)) from the clocks of
the SPSLAM_SUPP_PROF build (make variant VARIANT=suppprof VAR_FLAGS=-DSPSLAM_SUPP_PROF; loaded through
SPSLAM_GPU_LIB).

    SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_suppprof.so python tools/supp_phases.py [--config c2] [--batch B]
"""
import argparse
import ctypes
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sp-slam_amd"))
sys.path.insert(0, str(ROOT))

PHASES = ["load points", "sampler (wave 0)", "inlier counts", "decision (lane 0)", "optimize + select",
          "extract + border"]


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
    rows = []
    n = ctypes.c_int()
    buf = np.zeros((64, 8), np.int64)
    for f in range(a.batch):
        buf[:] = 0
        lib.spslam_planes_debug(hp.ex.ctx, f, 5, buf.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n))
        for r in buf:
            if r[7] > 0:
                rows.append(r.copy())
    R = np.array(rows, np.float64)
    us = R[:, :6] / 100.0
    tot = us.sum(1)
    print(f"boundaries with >= 50 points: {len(R)} ({len(R) / a.batch:.2f} per frame); points mean "
          f"{R[:, 7].mean():.0f} max {R[:, 7].max():.0f}; RANSAC rounds mean {R[:, 6].mean():.1f} max {R[:, 6].max():.0f}")
    for k, name in enumerate(PHASES):
        print(f"{name:20s} mean {us[:, k].mean():8.1f} us   max {us[:, k].max():8.1f} us   share {us[:, k].sum() / tot.sum():5.1%}")
    print(f"{'workgroup total':20s} mean {tot.mean():8.1f} us   max {tot.max():8.1f} us")
    print("workgroup total (us) percentiles 50/90/99/100:", np.percentile(tot, [50, 90, 99, 100]).round(1).tolist())
    big = R[:, 7] > 2048
    if big.any():
        print(f"boundaries beyond the LDS tile: {int(big.sum())}, mean total {tot[big].mean():.1f} us")
    hp.close()


if __name__ == "__main__":
    main()
