"""One LocalBundleAdjustment call, the reference's pattern (LocalMapping::Run calls Optimizer::LocalBundleAdjustment
once per new keyframe, src/LocalMapping.cc:84-90): GPU latency of a single local map at several team sizes next to
the CPU oracle's one-core time for the same map, with the results compared bit for bit.

Maps: the C3 bench's (12 keyframes of which 2 fixed, 1500 points: pipeline.py _setup_lba) and an fr1/room-sized
window (25 local + 10 fixed keyframes, 4000 points).
    python tools/lba_single.py [--reps 7] [--teams 1 5 16] > gpurun_out/lba_single.json"""
import argparse
import json
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT / "oracle"), str(ROOT)]


def maps():
    import numpy as np
    import synth
    sc = synth.Scene(0, n_boxes=5)
    K = dict(synth.TUM3)
    out = {"c3_map_12kf_1500pt": synth.lba_problem(sc, list(range(0, 72, 6)), np.random.default_rng(131), n_fixed=2,
                                                    n_points=1500, K=K)}
    # fr1/room-like window: 35 keyframes along the trajectory, the last 10 fixed, 4000 points
    out["room_window_25local_10fixed_4000pt"] = synth.lba_problem(sc, list(range(0, 35 * 4, 4)),
                                                                 np.random.default_rng(977), n_fixed=10,
                                                                 n_points=4000, K=K)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--teams", type=int, nargs="*", default=[1, 5, 16])
    ap.add_argument("--cpu-reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import oracle_ctypes
    import oracle_lba
    import spslam_gpu
    import spslam_lba as L
    ex = spslam_gpu.OrbExtractor(max_batch=1)
    lba = L.LocalBA(ex)
    report = {"kind": "one LocalBundleAdjustment call per map (the reference's LocalMapping pattern), "
                      "spslam_lba_optimize (host buffers in and out, synchronous)", "maps": {}}
    for name, P in maps().items():
        prob = P[0]
        ent = {"keyframes": int(prob["n_kf"]), "fixed": int(P[1]["fixed"].sum()), "points": int(prob["n_points"]),
               "planes": int(prob["n_planes"]), "point_edges": int(prob["n_point_obs"]),
               "plane_edges": int(prob["n_plane_obs"]), "gpu": {}}
        # CPU oracle, one core (the host glibc's libm, as a current build of the reference runs; the result checked
        # below is the pinned correctly rounded one)
        ts = []
        with oracle_ctypes.libm(oracle_ctypes.LIBM_GLIBC):
            for _ in range(a.cpu_reps):
                t0 = time.perf_counter()
                oracle_lba.lba_optimize(*P[:6])
                ts.append(time.perf_counter() - t0)
        o = oracle_lba.lba_optimize(*P[:6])
        ent["cpu_1core_ms"] = 1e3 * statistics.median(ts)
        ent["cpu_iterations"] = [int(x) for x in o["result"]["iterations"]]
        for team in a.teams:
            lba.set_team(team)
            ts, dev_us = [], []
            r = None
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = lba(*P[:6])
                ts.append(time.perf_counter() - t0)
                dev_us.append(float(r["result"]["phase_us"][0]))
            same = (np.array_equal(r["Tcw"], o["Tcw"]) and np.array_equal(r["points"], o["points"]) and
                    np.array_equal(r["planes"], o["planes"]) and
                    np.array_equal(r["point_outlier"], o["point_outlier"]) and
                    list(r["result"]["iterations"]) == list(o["result"]["iterations"]))
            ent["gpu"][f"team{team}"] = {"call_ms_median": 1e3 * statistics.median(ts), "call_ms_min": 1e3 * min(ts),
                                         "device_us_median": statistics.median(dev_us), "bit_exact_vs_oracle": same,
                                         "phases_us": [round(float(x), 1) for x in r["result"]["phase_us"]]}
        best = min(v["call_ms_median"] for v in ent["gpu"].values())
        ent["speedup_vs_cpu_1core_best_team"] = ent["cpu_1core_ms"] / best
        report["maps"][name] = ent
        print(json.dumps({name: ent}), file=sys.stderr, flush=True)
    lba.set_team(0)
    ex.close()
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
