"""GPU parity of tracked sequences (sp-slam_amd/sequence.py): every frame's
motion prior comes from the previous frame's optimised pose and velocity
(Tracking.cc:443-450, 958), its last-frame map points from the previous frame's
tracked matches (:456-505), and SearchLocalPoints skips the map points the
motion model already matched (mnLastFrameSeen).  The CPU oracle runs the same
loop (oracle/oracle_sequence.py); bar: every frame's local-map pose bit-identical
to the CPU's (PoseOptimization sums in g2o's order with the pinned, correctly
rounded libm on both), hence ATE against the CPU trajectory 0 (north star: <= 1e-4
m), every frame's decisions (matches, local matches, inliers of both
PoseOptimizations) identical, and the pipelined step bit-identical to the serial
one.  Frame 1 runs TrackReferenceKeyFrame (BoW against keyframe 0) on both sides.
C2 over 21 frames of two sequences; C4 (ICL.yaml parameters) over 90 frames,
past frame 70 where the previous kernel's tree-order sums and fdlibm-based libm
first changed an outlier decision."""
import pathlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B, T, U = 4, 23, 2


@pytest.fixture(scope="module")
def tracked():
    import pipeline
    import sequence
    out = {}
    try:
        for mode in (False, True, 3):  # serial, pipelined (lookahead 1), pipelined with lookahead 3
            sp = sequence.SequencePath(B, T, n_sequences=U, pipelined=bool(mode), lookahead=int(mode) or 1,
                                       **pipeline.CONFIGS["c2"])
            out[mode] = (None, sp)
            for _ in range(T - 2):
                sp.step()
            out[mode] = (sp.trajectory(), sp)
        yield out
    finally:
        for _, sp in out.values():
            sp.close()


def sequence_path(B, T, U, config, pipelined=True):
    import pipeline
    import sequence
    return sequence.SequencePath(B, T, n_sequences=U, pipelined=pipelined, **pipeline.CONFIGS[config])


def _oracle(sp, slot, n, on_frame=None, local_map=None, on_lba=None, refkf=False, perturb=None):
    import oracle_ctypes
    import oracle_grab
    import oracle_planes
    import oracle_seq_inputs as OSI
    import oracle_sequence
    import oracle_step
    import synth
    frames, T0, P0, local_of = OSI.inputs(sp, slot)
    cam, geo, inv_s2 = oracle_step.camera_inputs(sp)
    ref = oracle_sequence.reference_keyframe(OSI.reference_keyframe(sp, slot), synth.shape_vocabulary_text())
    return oracle_sequence.track(frames[:n], 1, T0, P0, local_of, cam, geo, inv_s2, sp.assoc_map, sp.assoc_boundary,
                                 oracle_ctypes.OrbOracle(nfeatures=sp.ex.params.nfeatures),
                                 oracle_planes.PlaneOracle(), supp_cap=sp.pe.supp_cap, min_size=sp.min_size,
                                 pose_cfg=sp.plane_cfg, depth_scale=oracle_grab.depth_scale(sp.depth_factor),
                                 on_frame=on_frame, ref_kf=ref, local_map=local_map, on_lba=on_lba,
                                 refkf_of=OSI.refkf_of(sp, slot, synth.shape_vocabulary_text()) if refkf else None,
                                 perturb=perturb, kf_id_stride=sp.kp_cap)


def test_pipelined_equals_serial(tracked):
    (ts, _), (tp, _), (t3, _) = tracked[False], tracked[True], tracked[3]
    assert ts.shape == tp.shape == t3.shape == (T - 1, B, 4, 4)
    assert ts.tobytes() == tp.tobytes()
    assert ts.tobytes() == t3.tobytes()  # three batches extracted ahead, on two extraction units side by side
    assert np.array_equal(tracked[False][1].history(), tracked[3][1].history())


def test_single_sequence_lookahead_equals_serial():
    """The reference's call pattern (B = 1): frames extracted two ahead of tracking on two extraction units
    (bench.py single_sequence) track bit-identically to the serial step."""
    import pipeline
    import sequence
    n, tr = 12, {}
    for look in (0, 2):
        sp = sequence.SequencePath(1, n + 4, n_sequences=1, pipelined=bool(look), lookahead=look or 1,
                                   **pipeline.CONFIGS["c2"])
        try:
            for _ in range(n):
                sp.step()
            tr[look] = (sp.trajectory(), sp.history())
        finally:
            sp.close()
    assert tr[0][0].tobytes() == tr[2][0].tobytes()
    assert np.array_equal(tr[0][1], tr[2][1])


def test_trajectory_matches_oracle(tracked):
    import trajectory
    from test_gpu_pose import pose_close
    tr, sp = tracked[False]
    n = T - 2
    for slot in range(U):
        cpu = _oracle(sp, slot, n)
        for k in range(n):
            ok, err = pose_close(tr[k + 1, slot].reshape(16), cpu[k].reshape(16))
            assert ok, (slot, k + 1, err)
            assert tr[k + 1, slot].tobytes() == cpu[k].tobytes(), (slot, k + 1)
        g = [trajectory.camera_center(tr[k + 1, slot].reshape(16)) for k in range(n)]
        c = [trajectory.camera_center(cpu[k].reshape(16)) for k in range(n)]
        assert trajectory.ate_rmse(g, c) <= 1e-4
        # and the tracking is real: within 2 cm of the synthetic ground truth
        gt = [np.linalg.inv(sp._true_pose(slot % U, k + 1))[:3, 3] for k in range(n)]
        assert trajectory.ate_rmse(g, gt) < 0.02
    # slots sharing a sequence track identically
    assert tr[:, 0].tobytes() == tr[:, U].tobytes()


def test_c4_long_sequence_matches_oracle():
    """ICL.yaml parameters (fy < 0, Plane.MinSize 1000, Chi 1000, VPChi 200), sequence 0, 90 tracked frames:
    identical decisions and bit-identical poses on every frame, ATE vs the CPU trajectory <= 1e-4 m."""
    import pipeline
    import sequence
    import trajectory
    n = 90
    sp = sequence.SequencePath(2, n + 2, n_sequences=1, pipelined=True, **pipeline.CONFIGS["c4"])
    try:
        for _ in range(n):
            sp.step()
        tr, hist = sp.trajectory(), sp.history()
        got = {}

        def rec(t, o, P):
            got[t] = (o["nmatches"], o["local_nmatches"], int(o["pose1"][0]["n_inliers"]),
                      int(o["pose2"][0]["n_inliers"]))
        cpu = _oracle(sp, 0, n, on_frame=rec)
        for t in range(1, n + 1):
            assert tuple(int(x) for x in hist[t, 0]) == tuple(int(x) for x in got[t]), t
            assert tr[t, 0].tobytes() == cpu[t - 1].tobytes(), t
        g = [trajectory.camera_center(tr[k + 1, 0].reshape(16)) for k in range(n)]
        c = [trajectory.camera_center(cpu[k].reshape(16)) for k in range(n)]
        assert trajectory.ate_rmse(g, c) <= 1e-4
    finally:
        sp.close()


def test_frame1_tracks_reference_keyframe(tracked):
    """Frame 1 (no velocity yet): SearchByBoW against keyframe 0 on the device equals the oracle's (matches per
    keypoint, count), and the frame's pose equals the oracle's TrackReferenceKeyFrame + TrackLocalMap pose."""
    import oracle_bow
    import oracle_sequence
    import synth
    tr, sp = tracked[False]
    V = oracle_sequence.vocabulary(synth.shape_vocabulary_text())
    hist = sp.history()
    for slot in range(U):
        import oracle_seq_inputs as OSI
        kps, desc, has, row = OSI.reference_keyframe(sp, slot)
        got = {}
        cpu = _oracle(sp, slot, 1, on_frame=lambda t, o, P: got.update(o=o))
        o = got["o"]
        fd = o["desc"]
        om, on = oracle_bow.search_by_bow(desc, kps["angle"], has, V.transform(desc), fd, o["kps"]["angle"],
                                          V.transform(fd), 0.7, True)
        assert np.array_equal(o["bow_match"], om) and on == o["nmatches"] > 50, slot
        assert int(hist[1, slot][0]) == on, slot  # the device's SearchByBoW count (d_nmatch)
        assert tr[1, slot].tobytes() == cpu[0].tobytes(), slot


def test_c3_local_mapping_in_the_loop():
    """C3 as a pipeline: the deterministic LocalMapping (sp-slam_amd/local_mapping.py) after every keyframe frame
    -- keyframe insertion from the tracked frame, LocalBundleAdjustment of the local window on the device, its
    result written back into the map the next frames track against (local-map points, last-frame points and
    pose, map planes).  The CPU oracle runs the same loop with the oracle's LocalBundleAdjustment.  Both sum in
    g2o's order, so the bar is bit equality over 160 frames (15 LocalBundleAdjustments, past frame
    80 where the round-3 tree-order LBA first changed a decision): every LocalBundleAdjustment's poses, points,
    LM iteration / trial / outlier counts, every frame's pose and decisions, hence ATE vs the CPU trajectory 0
    (up to the rounding of the Horn alignment itself, ~1e-16 m).
    The per-frame differences (all zero) are written to gpurun_out/c3_local_mapping_parity.json."""
    import json
    import trajectory
    from test_gpu_pose import pose_close
    n = 160
    sp = sequence_path(2, n + 2, 1, "c3")
    try:
        assert sp.local_mapping
        for _ in range(n):
            sp.step()
        tr, hist = sp.trajectory(), sp.history()
        got, lbas = {}, {}

        def rec(t, o, P):
            got[t] = (o["nmatches"], o["local_nmatches"], int(o["pose1"][0]["n_inliers"]),
                      int(o["pose2"][0]["n_inliers"]))
        import oracle_seq_inputs as OSI
        cpu = _oracle(sp, 0, n, on_frame=rec, local_map=OSI.local_map(sp, 0),
                      on_lba=lambda t, r: lbas.update({t: r}))
        runs = dict(sp.lm_runs)
        diag = {"lba": {}, "frame_pose_diff": []}
        assert sorted(runs) == sorted(lbas) == list(range(20, n + 1, 10))
        for t, r in lbas.items():
            g = runs[t][0]
            diag["lba"][t] = {"iterations": [int(x) for x in r["result"]["iterations"]],
                              "trials": int(r["result"]["trials"]), "keyframes": len(g["kfs"]),
                              "max_pose_diff": float(np.abs(g["Tcw"] - r["Tcw"]).max()),
                              "max_point_diff": float(np.abs(g["points"] - r["points"]).max())}
            assert g["kfs"] == r["kfs"], t
            assert list(g["result"]["iterations"]) == list(r["result"]["iterations"]), t
            assert int(g["result"]["trials"]) == int(r["result"]["trials"]), t
            assert int(g["result"]["n_point_outliers"]) == int(r["result"]["n_point_outliers"]), t
            assert np.array_equal(g["Tcw"], r["Tcw"]), (t, diag["lba"][t])
            assert np.array_equal(g["points"], r["points"]), (t, diag["lba"][t])
        for t in range(1, n + 1):
            assert tuple(int(x) for x in hist[t, 0]) == tuple(int(x) for x in got[t]), t
            diag["frame_pose_diff"].append([float(x) for x in pose_close(tr[t, 0].reshape(16), cpu[t - 1].reshape(16))[1]])
            assert tr[t, 0].tobytes() == cpu[t - 1].tobytes(), (t, diag["frame_pose_diff"][-1])
        g = [trajectory.camera_center(tr[k + 1, 0].reshape(16)) for k in range(n)]
        c = [trajectory.camera_center(cpu[k].reshape(16)) for k in range(n)]
        diag["ate_vs_cpu_m"] = trajectory.ate_rmse(g, c)
        (pathlib.Path(__file__).resolve().parents[1] / "gpurun_out").mkdir(exist_ok=True)
        (pathlib.Path(__file__).resolve().parents[1] / "gpurun_out" / "c3_local_mapping_parity.json").write_text(
            json.dumps(diag, indent=1))
        assert diag["ate_vs_cpu_m"] <= 1e-12, diag["ate_vs_cpu_m"]  # identical trajectories (Horn's SVD rounding)
    finally:
        sp.close()


def test_motion_model_failure_falls_back_to_reference_keyframe():
    """Tracking.cc:318-324: where TrackWithMotionModel fails, TrackReferenceKeyFrame (BoW against the reference
    keyframe, pose from the last frame) takes over inside the batched step.  The failure is forced by a wrong
    velocity (a 25 degree yaw and 0.3 m) at frame 6 of slot 0 and frame 9 of slot 3, so SearchByProjection finds
    almost nothing; the other slots and frames keep the motion model.  Bar: the device's per-frame decisions
    (motion model / reference keyframe), matches, inliers and poses identical to the CPU loop's."""
    import sequence
    import pipeline
    B, U, n = 4, 4, 12
    c, s_ = np.cos(np.radians(25.0)), np.sin(np.radians(25.0))
    V = np.array([[c, 0, s_, 0.3], [0, 1, 0, 0], [-s_, 0, c, 0], [0, 0, 0, 1]], np.float32)
    bad = {0: 6, 3: 9}
    sp = sequence.SequencePath(B, n + 2, n_sequences=U, pipelined=True, **pipeline.CONFIGS["c2"])
    try:
        assert sp.refkf_fallback
        for slot, t in bad.items():
            sp.perturb_velocity(t, slot, V)
        for _ in range(n):
            sp.step()
        tr, hist, fbh = sp.trajectory(), sp.history(), sp.fallback_history()
        rkh = sp.reference_keyframe_history()
        for slot in range(B):
            got = {}

            def rec(t, o, P):
                got[t] = (o["nmatches"], o["local_nmatches"], int(o["pose1"][0]["n_inliers"]),
                          int(o["pose2"][0]["n_inliers"]), o["fallback"], o["reference_keyframe"])
            cpu = _oracle(sp, slot, n, on_frame=rec, refkf=True,
                          perturb={bad[slot]: V} if slot in bad else None)
            for t in range(1, n + 1):
                want = 1 if bad.get(slot) == t else 0
                assert got[t][4] == want and int(fbh[t, slot]) == want, (slot, t, got[t][4], int(fbh[t, slot]))
                assert tuple(int(x) for x in hist[t, slot]) == tuple(int(x) for x in got[t][:4]), (slot, t)
                assert int(rkh[t, slot]) == got[t][5], (slot, t, int(rkh[t, slot]), got[t][5])
                assert tr[t, slot].tobytes() == cpu[t - 1].tobytes(), (slot, t)
    finally:
        sp.close()


def test_c1_low_texture_sequence_matches_oracle():
    """C1 proxy (BASELINE configs[0], TUM fr3 structure_notexture_far; Examples/RGB-D/TUM3.yaml): nearly untextured
    faces (synth._texture_low: most FAST cells are decided by the minThFAST retry, ORBextractor.cc:812-816, and
    ~200-300 keypoints per frame come from the structure's edges and a few stains) and a hand-held trajectory with
    jolts (synth._jolts).  Nothing is forced: on the jolts SearchByProjection finds few or wrong matches, the motion
    model fails by itself (nmatches < 10 or nmatchesMap < 5, Tracking.cc:977-1053) and TrackReferenceKeyFrame
    against the reference keyframe (UpdateLocalKeyFrames' pKFmax, :1459-1570) takes over (:318-324).  Two sequence
    offsets, 90 tracked frames each.  Bar, every frame: SearchByProjection / SearchLocalPoints matches, inliers of
    both PoseOptimizations, the motion model / reference keyframe / lost state and the reference keyframe identical
    to the CPU loop's, poses bit-identical (hence ATE vs the CPU trajectory 0)."""
    import json
    from concurrent.futures import ThreadPoolExecutor
    import pipeline
    import sequence
    import trajectory
    B, U, n = 2, 2, 90
    sp = sequence.SequencePath(B, n + 2, n_sequences=U, pipelined=True, render_workers=8, **pipeline.CONFIGS["c1"])
    try:
        assert sp.refkf_fallback and sp.texture == "low" and sp.motion == "shaky"
        for _ in range(n):
            sp.step()
        tr, hist, fbh, rkh = sp.trajectory(), sp.history(), sp.fallback_history(), sp.reference_keyframe_history()
        kp = sp.d_kf_cnt.cpu().numpy()
        got = [{} for _ in range(U)]

        def run(slot):
            def rec(t, o, P):
                got[slot][t] = (o["nmatches"], o["local_nmatches"], int(o["pose1"][0]["n_inliers"]),
                                int(o["pose2"][0]["n_inliers"]), o["fallback"], o["reference_keyframe"], len(o["kps"]))
            return _oracle(sp, slot, n, on_frame=rec, refkf=True)
        with ThreadPoolExecutor(U) as pool:
            cpus = list(pool.map(run, range(U)))
        diag = {"fallback_frames": [], "lost_frames": [], "mean_keypoints": [], "keyframe_keypoints": kp.tolist(),
                "ate_vs_cpu_m": [], "ate_vs_ground_truth_m": []}
        for slot in range(U):
            g = got[slot]
            for t in range(1, n + 1):
                assert int(fbh[t, slot]) == g[t][4], (slot, t, int(fbh[t, slot]), g[t][4])
                assert tuple(int(x) for x in hist[t, slot]) == tuple(int(x) for x in g[t][:4]), (slot, t)
                assert int(rkh[t, slot]) == g[t][5], (slot, t, int(rkh[t, slot]), g[t][5])
                assert tr[t, slot].tobytes() == cpus[slot][t - 1].tobytes(), (slot, t)
            diag["fallback_frames"].append([t for t in range(1, n + 1) if g[t][4] == 1])
            diag["lost_frames"].append([t for t in range(1, n + 1) if g[t][4] == 2])
            diag["mean_keypoints"].append(float(np.mean([g[t][6] for t in range(1, n + 1)])))
            gc = [trajectory.camera_center(tr[k + 1, slot].reshape(16)) for k in range(n)]
            cc = [trajectory.camera_center(cpus[slot][k].reshape(16)) for k in range(n)]
            gt = [np.linalg.inv(sp._true_pose(slot, k + 1))[:3, 3] for k in range(n)]
            diag["ate_vs_cpu_m"].append(trajectory.ate_rmse(gc, cc))
            diag["ate_vs_ground_truth_m"].append(trajectory.ate_rmse(gc, gt))
        out = pathlib.Path(__file__).resolve().parents[1] / "gpurun_out"
        out.mkdir(exist_ok=True)
        (out / "c1_sequence_parity.json").write_text(json.dumps(diag, indent=1))
        # the regime the proxy stands for: a low-texture scene and natural motion-model failures
        assert all(100 <= m <= 330 for m in diag["mean_keypoints"]), diag
        assert sum(len(f) for f in diag["fallback_frames"]) >= 3, diag
        assert max(diag["ate_vs_cpu_m"]) <= 1e-12, diag
    finally:
        sp.close()
