"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle.

The reference ships no fixtures for this path, so these
pin the restatement against regressions; they are data (inputs are
reproducible from sp-slam_amd/synth.py; outputs are oracle results).
    python tools/make_golden.py            # every fixture
    python tools/make_golden.py lba        # only the named ones (orb, planes, supposed, pose, lba)
"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT / "oracle")]
import oracle_ctypes as O  # noqa: E402
import oracle_planes as OP  # noqa: E402
import oracle_supposed as OS  # noqa: E402
import oracle_lba as OL  # noqa: E402
import synth  # noqa: E402

out = ROOT / "tests" / "golden"
ONLY = set(sys.argv[1:])


def want(name):
    return not ONLY or name in ONLY


out.mkdir(parents=True, exist_ok=True)
sc = synth.Scene(0)
g, d, fid = sc.render(sc.pose(5), noise_seed=5)
orb = O.OrbOracle()
kps, desc = orb.extract(g)
want("orb") and np.savez_compressed(out / "orb_seq0_f5.npz", kps=kps, desc=desc, gray_sum=np.int64(g.astype(np.int64).sum()))
# planes
df = OP.depth_to_float(d)
po = OP.PlaneOracle()
K = synth.TUM3
res = po.extract(df, K["fx"], K["fy"], K["cx"], K["cy"])
want("planes") and np.savez_compressed(out / "planes_seq0_f5.npz", coef=np.array(res["coef"]), n_inliers=np.array([len(i) for i in res["inliers"]]),
                    inliers=np.concatenate(res["inliers"]) if res["inliers"] else np.zeros(0, np.int32),
                    n_contour=np.array([len(c) for c in res["contour"]]),
                    contours=np.concatenate(res["contour"]) if res["contour"] else np.zeros(0, np.int32),
                    depth_sum=np.int64(d.astype(np.int64).sum()))
# supposed planes (GeneratePlanesFromBoundries) on a box scene that produces some
sc2 = synth.Scene(2, n_boxes=6)
_, d2, _ = sc2.render(sc2.pose(20), noise_seed=20)
df2 = OP.depth_to_float(d2)
po2 = OP.PlaneOracle()
r2 = po2.extract(df2, K["fx"], K["fy"], K["cx"], K["cy"])
s2 = OS.generate(df2, po2.cloud(), r2["coef"], r2["contour"], K["fx"], K["fy"], K["cx"], K["cy"])
cands = s2["candidates"]
want("supposed") and np.savez_compressed(out / "supposed_seq2_f20.npz", coef=np.array(s2["coef"]).reshape(-1, 4),
                    line=np.array(s2["line"]).reshape(-1, 6), source=np.array(s2["source"], np.int32),
                    n_line=np.array([len(x) for x in s2["line_idx"]], np.int32),
                    line_idx=np.concatenate(s2["line_idx"]) if s2["line_idx"] else np.zeros(0, np.int32),
                    cand_info=np.array([[c["plane"], c["j"], c["n_inliers"], c["iterations"], c["flags"]]
                                        for c in cands], np.int32).reshape(-1, 5),
                    depth_sum=np.int64(d2.astype(np.int64).sum()))
# pose
invs2 = orb.scale_tables()[3]
rng = np.random.default_rng(11)
prob, pts, pls, Tgt = synth.pose_problem(sc, 5, kps, d, fid, invs2, rng)
r, pout, plout = O.pose_optimize(prob, pts, pls)
want("pose") and np.savez_compressed(out / "pose_seq0_f5.npz", prob=prob, pts=pts, pls=pls, Tcw=r["Tcw"], n_inliers=r["n_inliers"],
                    pout=pout, plout=plout, Tgt=Tgt)
# local bundle adjustment (inputs are synthetic and stored with the outputs)
lrng = np.random.default_rng(21)
LP = synth.lba_problem(synth.Scene(1, n_boxes=3), list(range(0, 48, 6)), lrng, n_fixed=2, n_points=400)
lr = OL.lba_optimize(*LP[:6])
want("lba") and np.savez_compressed(out / "lba_seq1.npz", prob=LP[0], kfs=LP[1], points=LP[2], point_obs=LP[3], planes=LP[4],
                    plane_obs=LP[5], Tcw=lr["Tcw"], pts_out=lr["points"], pls_out=lr["planes"],
                    point_outlier=lr["point_outlier"], plane_outlier=lr["plane_outlier"],
                    iterations=lr["result"]["iterations"])
print("wrote", sorted(p.name for p in out.iterdir()))
