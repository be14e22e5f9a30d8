"""LBA wall time on one synthetic local map (12 keyframes, 1500 points + planes)."""
import sys, time
sys.path[:0] = ["sp-slam_amd", "oracle"]
import numpy as np, synth, spslam_gpu, spslam_lba
ex = spslam_gpu.OrbExtractor(max_batch=1)
lba = spslam_lba.LocalBA(ex)
rng = np.random.default_rng(1)
P = synth.lba_problem(synth.Scene(0), list(range(0, 72, 6)), rng, n_fixed=2, n_points=1500)
for _ in range(3):
    t = time.time(); r = lba(*P[:6]); dt = time.time() - t
print("wall ms", dt * 1e3, "iters", r["result"]["iterations"], "trials", r["result"]["trials"],
      "device us", float(r["result"]["phase_us"][0]))
ex.close()
