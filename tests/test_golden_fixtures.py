"""Regression pins: the CPU oracle against the committed golden fixtures in
tests/golden/ (written by tools/make_golden.py).  The reference ships no
fixtures for this path, so these pin the restatement
against accidental change; the GPU tests compare the HIP path with the same
oracle."""
import pathlib

import numpy as np

import oracle_ctypes as O
import oracle_lba as OL
import oracle_planes as OP
import oracle_supposed as OS
import synth

GOLDEN = pathlib.Path(__file__).parent / "golden"
K = synth.TUM3


def test_golden_planes_fixture():
    ref = np.load(GOLDEN / "planes_seq0_f5.npz")
    sc = synth.Scene(0)
    _, d, _ = sc.render(sc.pose(5), noise_seed=5)
    assert int(ref["depth_sum"]) == int(d.astype(np.int64).sum()), "synthetic renderer changed"
    po = OP.PlaneOracle()
    r = po.extract(OP.depth_to_float(d), K["fx"], K["fy"], K["cx"], K["cy"])
    assert np.array_equal(np.array(r["coef"]), ref["coef"])
    assert np.array_equal(np.array([len(i) for i in r["inliers"]]), ref["n_inliers"])
    assert np.array_equal(np.concatenate(r["inliers"]), ref["inliers"])
    assert np.array_equal(np.array([len(c) for c in r["contour"]]), ref["n_contour"])
    assert np.array_equal(np.concatenate(r["contour"]), ref["contours"])
    # segmentAndRefine traces each boundary from the model's last inlier: real outer contours
    assert all(n > 100 for n in ref["n_contour"])


def test_golden_supposed_fixture():
    ref = np.load(GOLDEN / "supposed_seq2_f20.npz")
    sc = synth.Scene(2, n_boxes=6)
    _, d, _ = sc.render(sc.pose(20), noise_seed=20)
    assert int(ref["depth_sum"]) == int(d.astype(np.int64).sum()), "synthetic renderer changed"
    df = OP.depth_to_float(d)
    po = OP.PlaneOracle()
    r = po.extract(df, K["fx"], K["fy"], K["cx"], K["cy"])
    s = OS.generate(df, po.cloud(), r["coef"], r["contour"], K["fx"], K["fy"], K["cx"], K["cy"])
    assert len(ref["coef"]) >= 1
    assert np.array_equal(np.array(s["coef"]).reshape(-1, 4), ref["coef"])
    assert np.array_equal(np.array(s["line"]).reshape(-1, 6), ref["line"])
    assert np.array_equal(np.array(s["source"], np.int32), ref["source"])
    assert np.array_equal(np.concatenate(s["line_idx"]), ref["line_idx"])
    info = np.array([[c["plane"], c["j"], c["n_inliers"], c["iterations"], c["flags"]] for c in s["candidates"]])
    assert np.array_equal(info, ref["cand_info"])


def test_golden_pose_fixture():
    ref = np.load(GOLDEN / "pose_seq0_f5.npz")
    r, pout, plout = O.pose_optimize(ref["prob"], ref["pts"], ref["pls"])
    assert np.array_equal(r["Tcw"], ref["Tcw"])
    assert int(r["n_inliers"]) == int(ref["n_inliers"])
    assert np.array_equal(pout, ref["pout"]) and np.array_equal(plout, ref["plout"])


def test_golden_lba_fixture():
    ref = np.load(GOLDEN / "lba_seq1.npz")
    r = OL.lba_optimize(ref["prob"], ref["kfs"], ref["points"], ref["point_obs"], ref["planes"], ref["plane_obs"])
    assert np.array_equal(r["Tcw"], ref["Tcw"]) and np.array_equal(r["points"], ref["pts_out"])
    assert np.array_equal(r["planes"], ref["pls_out"])
    assert np.array_equal(r["point_outlier"], ref["point_outlier"])
    assert np.array_equal(r["plane_outlier"], ref["plane_outlier"])
    assert list(r["result"]["iterations"]) == list(ref["iterations"])
