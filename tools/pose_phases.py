#!/usr/bin/env python3
"""Where does one PoseOptimization problem's time go?  Needs the diagnostic build (make prof), loaded with
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so.  Runs the benchmarked step once to build both graphs
(motion model, local map), then times the batched pose kernel alone on each and prints thread 0's
per-problem phase times (wall_clock64, 100 MHz) per LM iteration / trial.

    SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so python tools/pose_phases.py [--config c2]
"""
import argparse
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sp-slam_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pipeline  # noqa: E402
import spslam_gpu as G  # noqa: E402

PHASES = ["setup", "passA points", "passA planes", "reduceA+setup", "solve(t0)+bcast", "passB", "reduceB+decide",
          "stop test", "relabel", "outputs"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-prof", action="store_true", help="plain library (under rocprofv3 counters): launch times only")
    a = ap.parse_args()
    hp = pipeline.HotPath(a.batch, **pipeline.CONFIGS[a.config])
    lib = G.load_library()
    if a.no_prof:
        def read(buf, reset):
            return 0
    else:
        read = lib.spslam_pose_prof_read
        read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 24)()
    hp.step()
    torch.cuda.synchronize()
    for gi, g in enumerate(hp.graphs):
        P = g["P"].cpu().numpy().view(G.POSE_PROBLEM_DTYPE)
        res = torch.zeros_like(hp.d_res1)
        torch.cuda.synchronize()
        read(buf, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            G.pose_optimize_batch_device(hp.ex, hp.B, g["P"].data_ptr(), g["pts"].data_ptr(), g["pls"].data_ptr(),
                                         res.data_ptr(), g["pout"].data_ptr(), g["plout"].data_ptr(),
                                         stream=torch.cuda.current_stream().cuda_stream)
        e1.record()
        torch.cuda.synchronize()
        read(buf, 1)
        ms = e0.elapsed_time(e1) / a.reps
        v = np.array(list(buf), dtype=np.float64)
        n = hp.B * a.reps
        if a.no_prof:
            print(f"graph {gi}: {ms:.3f} ms/launch alone")
            continue
        its, trials = v[11] / n, v[10] / n
        tot = max((v[:10].sum() + v[16:20].sum()) / n * 0.01, 1e-9)
        print(f"graph {gi}: points {P['n_points'].mean():.0f} planes {P['n_planes'].mean():.1f}  "
              f"{ms:.3f} ms/launch alone, thread-0 total {tot:.1f} us/problem, "
              f"{its:.1f} LM iterations, {trials:.1f} trials per problem")
        for k, name in enumerate(PHASES):
            us = v[k] / n * 0.01
            per = f"{us / its:6.2f} us/it" if k in (1, 2, 3, 7) else (f"{us / trials:6.2f} us/trial" if k in (4, 5, 6) else "")
            print(f"   {name:18s} {us:8.1f} us  {100 * us / tot:5.1f} %  {per}")
        ev, st, bp, bl = (v[16:20] / n * 0.01).tolist()
        print(f"   (pass A plane evaluations {ev / its:.2f} us/it, staging {st / its:.2f}; pass B point rounds "
              f"{bp / trials:.2f} us/pass, plane rounds {bl / trials:.2f})")
        ca, wa, cb, wb = (v[12:16] / n * 0.01).tolist()
        print(f"   chain wave: pass A adding {ca:.1f} us ({ca / its:.2f}/it), waiting {wa:.1f} us; "
              f"pass B adding {cb:.1f} us ({cb / trials:.2f}/pass), waiting {wb:.1f} us")
    hp.close()


if __name__ == "__main__":
    main()
