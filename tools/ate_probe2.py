"""Diagnostic: track n frames, then re-run the last frame's local-map PoseOptimization graph (GPU) through the
CPU oracle and compare flags / pose; dump the graph.   python tools/ate_probe2.py n slot"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT / "oracle"), str(ROOT)]


def main(n, slot):
    import oracle_ctypes
    import pipeline
    import sequence
    import spslam_gpu as G
    sp = sequence.SequencePath(2, n + 1, n_sequences=2, render_workers=16, **pipeline.CONFIGS["c2"])
    for _ in range(n):
        sp.step()
    sp.torch.cuda.synchronize()
    print("history", sp.history()[n, slot], flush=True)
    for k in (0, 1):
        P, pts, pls, po, plo = sp.graph(k)
        res = (sp.d_res1 if k == 0 else sp.d_res2).cpu().numpy().view(G.POSE_RESULT_DTYPE)[slot]
        r, opo, oplo = oracle_ctypes.pose_optimize(P[slot], pts[slot], pls[slot], cfg=sp.plane_cfg)
        g2, gpo, gplo = G.pose_optimize(sp.ex, P[slot], pts[slot], pls[slot], cfg=sp.plane_cfg)
        print(f"graph {k}: edges {len(pts[slot])} + {len(pls[slot])}; batch inliers {res['n_inliers']} its "
              f"{res['lm_iterations']}; single gpu {g2['n_inliers']} its {g2['lm_iterations']}; oracle "
              f"{r['n_inliers']} its {r['lm_iterations']}", flush=True)
        print("  flags batch==oracle", np.array_equal(po[slot], opo), np.array_equal(plo[slot], oplo),
              " single==oracle", np.array_equal(gpo, opo), " max|dT| batch-oracle",
              float(np.abs(res["Tcw"] - r["Tcw"]).max()), flush=True)
        d = np.nonzero(po[slot] != opo)[0]
        print("  differing point flags", d[:10], flush=True)
        np.savez(f"gpurun_out/probe_graph{k}_f{n}_s{slot}.npz", P=P[slot], pts=pts[slot], pls=pls[slot],
                 gpo=po[slot], gplo=plo[slot], gres=res)
    sp.close()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]))
