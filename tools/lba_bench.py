"""Diagnostic: the C3 LocalMapping workload alone -- one batched LocalBundleAdjustment call over the step's
local maps (51 maps at B = 256; --config c3s: 12 keyframes / 1500 points, c3: the fr1/room-sized window of 35
keyframes / 4000 points), wall time and LM step count.
    python tools/lba_bench.py [--reps 5] [--order g2o|fast] [--config c3s|c3]"""
import argparse
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--order", default="g2o", choices=("g2o", "fast"))
    ap.add_argument("--config", default="c3s", choices=("c3s", "c3"))
    ap.add_argument("--team", type=int, nargs="*", default=[0], help="workgroups per problem (0 = auto); several: "
                    "interleaved")
    a = ap.parse_args()
    import numpy as np
    import torch
    import pipeline
    import spslam_lba as L
    hp = pipeline.HotPath(a.batch, lba_order=0 if a.order == "g2o" else 1, **pipeline.CONFIGS[a.config])
    for r in range(a.reps * len(a.team)):
        team = a.team[r % len(a.team)]
        hp.lba.set_team(team)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hp.local_ba()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res = hp.lba_out[5].cpu().numpy().view(L.LBA_RESULT_DTYPE)
        print(f"rep {r} ({a.order}, team {team}): {dt * 1e3:.2f} ms for {hp.n_lba} maps; iterations max {res['iterations'].max(0)} "
              f"trials max {res['trials'].max()} device us max {res['phase_us'][:, 0].max():.0f}; phases (us, slowest "
              f"map) {np.round(res['phase_us'][int(res['phase_us'][:, 0].argmax())], 0).tolist()} pad {res['pad'].max()}", flush=True)
    hp.close()


if __name__ == "__main__":
    main()
