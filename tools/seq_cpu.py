"""CPU-only tracked sequence (no GPU): the inputs sp-slam_amd/sequence.py builds for one slot, built with
the oracle ORB (bit-identical to the device's), run through oracle/oracle_sequence.track under a chosen
PoseOptimization mode.  Diagnostic for the summation-order / libm study."""
import argparse
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in (ROOT / "sp-slam_amd", ROOT / "oracle"):
    sys.path.insert(0, str(p))

import oracle_assoc  # noqa: E402
import oracle_ctypes  # noqa: E402
import oracle_frame  # noqa: E402
import oracle_grab  # noqa: E402
import oracle_planes  # noqa: E402
import oracle_sequence  # noqa: E402
import synth  # noqa: E402

SEQ_STRIDE = 53
CFG = {"c2": dict(K=synth.TUM3, min_size=500, chi=300.0, vp_chi=300.0),
       "c3": dict(K=synth.TUM3, min_size=500, chi=300.0, vp_chi=300.0, local_mapping=True),
       "c4": dict(K=synth.ICL, min_size=1000, chi=1000.0, vp_chi=200.0)}


def inputs(cfg, u=0, n_frames=300, seq_id=0, n_boxes=5, W=640, H=480, nfeatures=1000, cap=1200):
    c = CFG[cfg]
    K = c["K"]
    scene = synth.Scene(seq_id, n_boxes=n_boxes)
    frames = []
    for t in range(SEQ_STRIDE * u, SEQ_STRIDE * u + n_frames + 1):
        g, d, fid = scene.render(scene.pose(t), W, H, K=K, noise_seed=seq_id * 100003 + t)
        frames.append((synth.colorize(g, fid), d))
    orb = oracle_ctypes.OrbOracle(nfeatures=nfeatures)
    kf_t = list(range(0, n_frames + 1, synth.KEYFRAME_STEP))
    kfp, kfk, kfd = [], [], []
    for j, t in enumerate(kf_t):
        k, dsc = orb.extract(oracle_grab.cvt_gray(frames[t][0], rgb=True))
        kfp.append(synth.keyframe_points(scene, SEQ_STRIDE * u + t, k, dsc, frames[t][1], j * cap, K=K))
        kfk.append(k)
        kfd.append(dsc)
    has = np.zeros(len(kfk[0]), np.uint8)
    row = np.full(len(kfk[0]), -1, np.int32)
    ids = kfp[0]["id"].astype(np.int64)
    has[ids], row[ids] = 1, np.arange(len(ids), dtype=np.int32)
    ref = oracle_sequence.reference_keyframe((kfk[0], kfd[0], has, row), synth.shape_vocabulary_text())
    P0 = synth.as_last_frame_points(kfp[0], kfk[0], 0)
    T0 = np.linalg.inv(scene.pose(SEQ_STRIDE * u)).astype(np.float32)

    def local_of(t):
        j = (t - 1) // synth.KEYFRAME_STEP
        return np.concatenate(kfp[max(j - 1, 0):j + 1])
    scale = oracle_grab.depth_scale(K["depth_factor"])
    fx, fy, cx, cy, bf = K["fx"], K["fy"], K["cx"], K["cy"], K["bf"]
    depth0 = oracle_grab.convert_depth(frames[0][1], scale)
    b = oracle_frame.frame_rgbd(np.zeros((0, 2), np.float32), depth0, fx, fy, cx, cy, bf=bf,
                                dist=K.get("dist", (0,) * 5))["bounds"]
    ginv = [np.float32(64) / np.float32(b[1] - b[0]), np.float32(48) / np.float32(b[3] - b[2])]
    sc, _, _, inv_s2 = orb.scale_tables()
    geo = np.concatenate([[fx, fy, cx, cy, bf, *b, *ginv], sc]).astype(np.float32)
    mp, bxyz = synth.map_planes(scene, np.random.default_rng(seq_id * 31 + 7))
    m = np.zeros(len(mp["world"]), oracle_assoc.MAP_PLANE_DTYPE)
    for k, v in mp.items():
        m[k] = v
    import spslam_gpu as G  # PlaneConfig record only (no device call)
    pcfg = G.PlaneConfig(1.0, 100.0, 0.5, 0.5, c["chi"], c["vp_chi"])
    lm = None
    if c.get("local_mapping"):
        import oracle_local_map as LM
        lm = LM.KeyframeMap(kfp, cap, (fx, fy, cx, cy, bf), sc, inv_s2, m)
        LM.insert_initial_keyframe(lm, T0, kfk[0], frames[0][1], K["depth_factor"], bf)
    return dict(lm=lm, frames=frames[1:], T0=T0, P0=P0, local_of=local_of, cam=(fx, fy, cx, cy, bf), geo=geo,
                inv_s2=np.asarray(inv_s2, np.float32), map=m, boundary=bxyz, min_size=c["min_size"], pcfg=pcfg, ref=ref,
                scale=scale, scene=scene, u=u, nfeatures=nfeatures)


def run(inp, order, n_frames):
    import copy
    hist = {}

    def rec(t, o, P):
        hist[t] = (int(o["nmatches"]), int(o["local_nmatches"]), int(o["pose1"][0]["n_inliers"]),
                   int(o["pose2"][0]["n_inliers"]))
    poses = oracle_sequence.track(inp["frames"][:n_frames], 1, inp["T0"], inp["P0"], inp["local_of"], inp["cam"],
                                  inp["geo"], inp["inv_s2"], inp["map"], inp["boundary"],
                                  oracle_ctypes.OrbOracle(nfeatures=inp["nfeatures"]), oracle_planes.PlaneOracle(),
                                  supp_cap=32, min_size=inp["min_size"], pose_cfg=inp["pcfg"],
                                  depth_scale=inp["scale"], on_frame=rec, libm=order, ref_kf=inp["ref"],
                                  local_map=copy.deepcopy(inp["lm"]),
                                  on_lba=lambda t, r: print("LBA", t, r["result"], flush=True))
    return np.array(poses), hist


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--seq", type=int, default=0)
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--orders", default="0,1")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    t0 = time.time()
    inp = inputs(a.config, a.seq, a.frames)
    print(f"inputs {time.time() - t0:.1f}s", flush=True)
    orders = [int(x) for x in a.orders.split(",")]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(len(orders)) as ex:
        res = dict(zip(orders, ex.map(lambda o: run(inp, o, a.frames), orders)))
    import trajectory
    out = {}
    base = orders[0]
    for o in orders:
        P, h = res[o]
        cen = [trajectory.camera_center(T.reshape(16)) for T in P]
        cb = [trajectory.camera_center(T.reshape(16)) for T in res[base][0]]
        div = next((t for t in sorted(h) if h[t] != res[base][1][t]), None)
        out[o] = {"ate_vs_%d" % base: trajectory.ate_rmse(cen, cb),
                  "max_center_diff": float(np.linalg.norm(np.array(cen) - np.array(cb), axis=1).max()),
                  "first_decision_diff_frame": div}
        print(o, out[o], flush=True)
    if a.out:
        np.savez(a.out, **{f"poses{o}": res[o][0] for o in orders},
                 **{f"hist{o}": np.array([res[o][1][t] for t in sorted(res[o][1])]) for o in orders})
    print(f"total {time.time() - t0:.1f}s")
