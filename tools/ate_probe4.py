"""Diagnostic: GPU tracked sequence and CPU oracle in lockstep; stop at the first frame where any stage differs
and print what differs.   python tools/ate_probe4.py n slot"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT / "oracle"), str(ROOT)]


def main(n, slot):
    import oracle_ctypes
    import oracle_grab
    import oracle_match as OM
    import oracle_planes
    import oracle_step
    import oracle_track as OT
    import pipeline
    import sequence
    import spslam_gpu as G
    sp = sequence.SequencePath(2, n + 1, n_sequences=2, render_workers=16, **pipeline.CONFIGS["c2"])
    cam, geo, inv_s2 = oracle_step.camera_inputs(sp)
    orb, po = oracle_ctypes.OrbOracle(), oracle_planes.PlaneOracle()
    frames, T0, P0, local_of = sp.oracle_inputs(slot)
    Tlw, V, P = T0, np.eye(4, dtype=np.float32), P0
    scale = oracle_grab.depth_scale(sp.depth_factor)
    cap = sp.kp_cap
    for t in range(1, n + 1):
        used = sp.d_pframes  # the set this batch reads (MOTION_PRIOR writes its Tcw during the step)
        sp.step()
        sp.torch.cuda.synchronize()
        cur_pf = used.cpu()
        rgb, d = frames[t - 1]
        pfr = np.zeros((), OM.PROJ_FRAME_DTYPE)
        pfr["Tcw"] = OT.mat4(V, Tlw).reshape(16)
        pfr["Tlw"] = Tlw.reshape(16)
        pfr["n_points"] = len(P)
        LP = local_of(t)
        lfr = np.zeros((), OM.LOCAL_FRAME_DTYPE)
        lfr["n_points"] = len(LP)
        fi = oracle_step.FrameInputs(oracle_grab.cvt_gray(rgb, rgb=True), oracle_grab.convert_depth(d, scale), cam,
                                     geo, inv_s2, (pfr, P), (lfr, LP), sp.assoc_map, sp.assoc_boundary,
                                     min_size=sp.min_size, pose_cfg=sp.plane_cfg, local_seen=True)
        o = oracle_step.run(fi, orb, po, supp_cap=sp.pe.supp_cap)
        gpf = cur_pf.numpy().view(OM.PROJ_FRAME_DTYPE)[slot]
        res = sp.results()
        nk = int(res["kp_counts"][slot])
        checks = {
            "prior Tcw": np.array_equal(gpf["Tcw"], pfr["Tcw"]),
            "match": np.array_equal(res["match"][slot, :nk], o["match"]),
            "local_match": np.array_equal(res["local_match"][slot, :nk], o["local_match"]),
        }
        g1, g2 = sp.graph(0), sp.graph(1)
        checks["graph1 pts"] = g1[1][slot].tobytes() == o["graph1"][1].tobytes()
        checks["graph1 pls"] = g1[2][slot].tobytes() == o["graph1"][2].tobytes()
        checks["pose1"] = np.array_equal(res["pose1"][slot]["Tcw"], o["pose1"][0]["Tcw"])
        checks["graph2 pts"] = g2[1][slot].tobytes() == o["graph2"][1].tobytes()
        checks["graph2 pls"] = g2[2][slot].tobytes() == o["graph2"][2].tobytes()
        checks["pose2"] = np.array_equal(res["pose2"][slot]["Tcw"], o["pose2"][0]["Tcw"])
        checks["flags2"] = np.array_equal(g2[3][slot], o["pose2"][1])
        T2 = np.asarray(o["pose2"][0]["Tcw"], np.float32).reshape(4, 4)
        Pn = OT.last_frame(P, o["match"], o["keep"], LP, o["local_match"], o["keys_un"], o["pose2"][1])
        nxt = sp.d_pframes.cpu().numpy().view(OM.PROJ_FRAME_DTYPE)[slot]
        gp = sp.d_ppoints.cpu().numpy().view(OM.PROJ_POINT_DTYPE)[slot * cap:slot * cap + int(nxt["n_points"])]
        checks["next points"] = gp.tobytes() == Pn.tobytes()
        V = OT.mat4(T2, OT.inverse_pose(Tlw))
        Tlw, P = T2, Pn
        bad = [k for k, v in checks.items() if not v]
        if bad or t % 25 == 0:
            print(f"frame {t}: differs {bad}", flush=True)
        if bad:
            if "graph2 pts" in bad:
                a, b = g2[1][slot], o["graph2"][1]
                print("  graph2 sizes", len(a), len(b))
                m = min(len(a), len(b))
                dd = [i for i in range(m) if a[i].tobytes() != b[i].tobytes()]
                print("  first differing edges", dd[:5], a[dd[0]] if dd else None, b[dd[0]] if dd else None)
            if "pose1" in bad or "pose2" in bad:
                print("  pose1 diff", np.abs(res["pose1"][slot]["Tcw"] - o["pose1"][0]["Tcw"]).max(),
                      "pose2 diff", np.abs(res["pose2"][slot]["Tcw"] - o["pose2"][0]["Tcw"]).max())
                print("  iters gpu", res["pose1"][slot]["lm_iterations"], res["pose2"][slot]["lm_iterations"],
                      "cpu", o["pose1"][0]["lm_iterations"], o["pose2"][0]["lm_iterations"])
            break
    sp.close()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]))
