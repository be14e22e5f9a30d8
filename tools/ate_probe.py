"""Diagnostic: tracked sequences on the GPU vs the CPU oracle, frame by frame (decision counts and pose
differences) up to the first frame where they differ.   python tools/ate_probe.py [frames] [sequences]"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT / "oracle"), str(ROOT)]


def main(n=300, S=2):
    import oracle_ctypes
    import oracle_grab
    import oracle_planes
    import oracle_sequence
    import oracle_step
    import pipeline
    import sequence
    sp = sequence.SequencePath(S, n + 1, n_sequences=S, render_workers=16, **pipeline.CONFIGS["c2"])
    for _ in range(n):
        sp.step()
    tr, hist = sp.trajectory(), sp.history()
    cam, geo, inv_s2 = oracle_step.camera_inputs(sp)
    orb, po = oracle_ctypes.OrbOracle(), oracle_planes.PlaneOracle()
    for slot in range(S):
        frames, T0, P0, local_of = sp.oracle_inputs(slot)
        ch = {}
        cpu = oracle_sequence.track(frames[:n], 1, T0, P0, local_of, cam, geo, inv_s2, sp.assoc_map,
                                    sp.assoc_boundary, orb, po, supp_cap=sp.pe.supp_cap, min_size=sp.min_size,
                                    pose_cfg=sp.plane_cfg, depth_scale=oracle_grab.depth_scale(sp.depth_factor),
                                    on_frame=lambda t, o, P: ch.__setitem__(t, (o["nmatches"], o["local_nmatches"],
                                                                                int(o["pose1"][0]["n_inliers"]),
                                                                                int(o["pose2"][0]["n_inliers"]))))
        first = None
        for t in range(1, n + 1):
            g = tuple(int(x) for x in hist[t, slot])
            d = np.abs(tr[t, slot] - cpu[t - 1]).max()
            if g != ch[t] and first is None:
                first = t
            if first is not None and t <= first + 3 or t % 50 == 0:
                print(f"slot {slot} frame {t}: gpu {g} cpu {ch[t]} max|dT| {d:.2e}", flush=True)
        print(f"slot {slot}: first decision difference at frame {first}", flush=True)
    sp.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
