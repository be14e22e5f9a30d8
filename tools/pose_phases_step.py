#!/usr/bin/env python3
"""PoseOptimization phases inside the pipelined C2 step (diagnostic build, SPSLAM_GPU_LIB=libspslam_gpu_prof.so):
the phase ticks of every pose launch of `--steps` steps, per problem, next to tools/pose_phases.py's alone numbers.
    SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so python tools/pose_phases_step.py [--steps 20]"""
import argparse
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT / "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pipeline  # noqa: E402
import spslam_gpu as G  # noqa: E402
from pose_phases import PHASES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    hp = pipeline.HotPath(a.batch, pipelined=True, **pipeline.CONFIGS["c2"])
    read = G.load_library().spslam_pose_prof_read
    read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 24)()
    for _ in range(3):
        hp.step()
    torch.cuda.synchronize()
    read(buf, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        hp.step()
    e1.record()
    torch.cuda.synchronize()
    read(buf, 1)
    v = np.array(list(buf), dtype=np.float64)
    n = hp.B * a.steps * 2  # problems (two graphs per step)
    its, trials = v[11] / n, v[10] / n
    tot = (v[:10].sum() + v[16:20].sum()) / n * 0.01
    print(f"in-step: {e0.elapsed_time(e1) / a.steps:.3f} ms/step, thread-0 total {tot:.1f} us/problem, "
          f"{its:.1f} LM iterations, {trials:.1f} trials per problem")
    for k, name in enumerate(PHASES):
        print(f"   {name:18s} {v[k] / n * 0.01:8.1f} us")
    ev, st, bp, bl = (v[16:20] / n * 0.01).tolist()
    print(f"   pass A plane evaluations {ev:.1f} us, staging {st:.1f}; pass B point rounds {bp:.1f}, plane rounds {bl:.1f}")
    ca, wa, cb, wb = (v[12:16] / n * 0.01).tolist()
    print(f"   chain wave: pass A adding {ca:.1f} us, waiting {wa:.1f}; pass B adding {cb:.1f}, waiting {wb:.1f}")
    hp.close()


if __name__ == "__main__":
    main()
