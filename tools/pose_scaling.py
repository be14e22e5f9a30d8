#!/usr/bin/env python3
"""Where does PoseOptimization's time go?  Times the batched pose kernel on the benchmarked step's own
motion-model graphs (B = 256) with the point edges truncated to N and with / without plane edges, and
reports the mean LM iteration count (per-iteration cost = time / iterations)."""
import sys
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sp-slam_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pipeline  # noqa: E402
import spslam_gpu as G  # noqa: E402


def main():
    hp = pipeline.HotPath(256)
    hp.step()
    torch.cuda.synchronize()
    g = hp.graphs[0]
    P0 = g["P"].cpu().numpy().view(G.POSE_PROBLEM_DTYPE).copy()
    res = torch.zeros_like(hp.d_res1)
    print("mean edges", P0["n_points"].mean(), "planes", P0["n_planes"].mean())
    for planes in (True, False):
        for N in (4, 32, 128, 512, 100000):
            P = P0.copy()
            P["n_points"] = np.minimum(P["n_points"], N)
            if not planes:
                P["n_planes"] = 0
            d_P = torch.from_numpy(P.view(np.uint8).copy()).cuda()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for rep in range(4):
                if rep == 1:
                    e0.record()
                G.pose_optimize_batch_device(hp.ex, hp.B, d_P.data_ptr(), g["pts"].data_ptr(), g["pls"].data_ptr(),
                                             res.data_ptr(), g["pout"].data_ptr(), g["plout"].data_ptr(),
                                             stream=torch.cuda.current_stream().cuda_stream)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 3
            rr = res.cpu().numpy().view(G.POSE_RESULT_DTYPE)
            its = rr["lm_iterations"]
            pad = rr["pad"].astype(np.float64)
            if pad.any():  # phase timers (wall_clock64, 100 MHz) when the kernel is built with them
                print(f"   passA+reduce {10 * pad[:, 0].mean() / its.mean():7.2f} us/it   "
                      f"solve(t0) {10 * pad[:, 1].mean() / its.mean():7.2f} us/it")
            print(f"planes={planes} N={N:6d} points={P['n_points'].mean():7.1f} {ms:7.3f} ms/launch "
                  f"its={its.mean():5.1f} max {its.max()} -> {1e3 * ms / its.max():6.2f} us/iteration(max)",
                  flush=True)
    hp.close()


if __name__ == "__main__":
    main()
