"""Diagnostic: where a LocalBundleAdjustment window first differs from the oracle -- per team size, the state after
LM trial k (pbStopFlag raised by the device's stop-after hook) against the oracle's after the same trial.
    python tools/lba_wide_diag.py [--windows 130:2:3:900 66:2:3:900 27:2:4:1200:9] [--teams 1 8] [--trials 1 2 3 4 6]
(a trial count of 0: the full run, no stop flag)"""
import argparse
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT / "oracle"), str(ROOT / "tests"), str(ROOT)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", nargs="*", default=["130:2:3:900", "66:2:3:900"])
    ap.add_argument("--teams", type=int, nargs="*", default=[1, 8])
    ap.add_argument("--trials", type=int, nargs="*", default=[1, 2, 3, 4, 6])
    a = ap.parse_args()
    import numpy as np
    import oracle_lba
    import spslam_gpu
    import spslam_lba as L
    import test_gpu_lba_large as T
    ex = spslam_gpu.OrbExtractor(max_batch=1)
    lba = L.LocalBA(ex)
    for w in a.windows:
        f = [int(x) for x in w.split(":")]  # keyframes:fixed:step:points[:seed]
        P = T._window(f[0], f[1], f[2], n_points=f[3], **({"seed": f[4]} if len(f) > 4 else {}))
        full = oracle_lba.lba_optimize(*P[:6])
        print(f"window {w}: free {int((P[1]['fixed'] == 0).sum())}, oracle iterations "
              f"{list(full['result']['iterations'])} trials {int(full['result']['trials'])}", flush=True)
        for k in a.trials:
            o = oracle_lba.lba_optimize(*P[:6], stop_after=k if k > 0 else -1)
            for team in a.teams:
                lba.set_team(team)
                lba.debug_stop_after(k if k > 0 else -1)
                g = lba(*P[:6])
                lba.debug_stop_after(-1)
                dT = float(np.abs(g["Tcw"] - o["Tcw"]).max())
                dp = float(np.abs(g["points"] - o["points"]).max())
                nout = int((g["point_outlier"] != o["point_outlier"]).sum())
                print(f"  trial {k} team {team}: status {int(g['result']['status'])} iterations "
                      f"{list(g['result']['iterations'])} vs {list(o['result']['iterations'])}; max |dTcw| {dT:.3e} "
                      f"max |dpoint| {dp:.3e}; outlier flags differing {nout}", flush=True)
    lba.set_team(0)
    ex.close()


if __name__ == "__main__":
    main()
