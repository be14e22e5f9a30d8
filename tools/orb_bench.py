#!/usr/bin/env python3
"""ORB extraction alone on the benchmarked batch (B frames of the C2 workload, no other stream active):
per-kind kernel times, to tune the ORB kernels in isolation.  SPSLAM_GPU_LIB selects a library variant."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sp-slam_amd"))

import torch  # noqa: E402

import pipeline  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    hp = pipeline.HotPath(B, **pipeline.CONFIGS["c2"])
    for _ in range(2):
        hp.orb()
    torch.cuda.synchronize()
    hp.ex.set_timing(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    with torch.cuda.stream(hp.main):
        e0.record()
        for _ in range(n):
            hp.orb()
        e1.record()
    torch.cuda.synchronize()
    t = hp.ex.kernel_times()
    print(f"B={B} orb total {e0.elapsed_time(e1) / n:.3f} ms/batch  " +
          "  ".join(f"{k} {v[0] / n:.3f}" for k, v in sorted(t.items()) if v[1]))
    hp.close()


if __name__ == "__main__" and len(sys.argv) <= 2:
    main()


def thresholds_experiment(B=256):
    """Same frames through extractors with FAST thresholds (ini, min) = (20, 7) and (250, 250): the second
    finds almost no corners, so its level_kernel time is the blur / resize / store part alone."""
    import spslam_gpu as G
    hp = pipeline.HotPath(B)
    torch.cuda.synchronize()
    for ini, mn in ((20, 7), (250, 250)):
        ex = G.OrbExtractor(max_batch=B, ini_th_fast=ini, min_th_fast=mn)
        for rep in range(3):
            if rep == 2:
                ex.set_timing(True)
            ex.extract_batch_device(hp.d_gray.data_ptr(), B, hp.W * hp.H, hp.W, hp.d_kps.data_ptr(),
                                    hp.d_desc.data_ptr(), hp.d_cnt.data_ptr(), hp.kp_cap, hp.stream)
        torch.cuda.synchronize()
        t = ex.kernel_times()
        print(f"th=({ini},{mn}) " + "  ".join(f"{k} {v[0]:.3f}" for k, v in sorted(t.items()) if v[1]), flush=True)
        ex.close()
    hp.close()


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "th":
    thresholds_experiment(int(sys.argv[1]))
