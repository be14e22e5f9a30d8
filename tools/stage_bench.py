"""Diagnostic: each hot-path stage timed alone (one stream), per-kernel HIP-event times.

    python tools/stage_bench.py [--batch B] [--steps K] [--config c2|c5]
"""
import argparse
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sp-slam_amd"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--config", default="c2")
    a = ap.parse_args()
    import torch
    import pipeline
    hp = pipeline.HotPath(a.batch, **pipeline.CONFIGS[a.config])
    stages = {"grab": hp.grab, "orb": hp.orb, "planes": hp.planes, "tail": hp._tail}
    for name, fn in stages.items():
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        hp.ex.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps * 1e3
        times = {k: round(v[0] / a.steps, 3) for k, v in hp.ex.kernel_times().items() if v[1] > 0}
        hp.ex.set_timing(False)
        print(f"{name:7s} {dt:8.3f} ms/step  {a.batch / dt * 1e3:10.0f} frames/s  {times}", flush=True)
    hp.close()


if __name__ == "__main__":
    main()
