"""ORACLE -- TEST INFRASTRUCTURE ONLY.

CPU restatement of a tracked RGB-D sequence (the checker of
sp-slam_amd/sequence.py and bench.py's ATE): Tracking::Track frame after
frame (src/Tracking.cc:276-526) with the motion model --
  mCurrentFrame.SetPose(mVelocity * mLastFrame.mTcw)       :958
  TrackWithMotionModel + TrackLocalMap                     :950-1136 (oracle_step.run)
  mVelocity = mCurrentFrame.mTcw * LastTwc                 :443-450
  VO-match clean-up, outlier drop, mLastFrame = current    :456-505
against a map of keyframe points on a fixed keyframe schedule (the harness's
stand-in for LocalMapping; sp-slam_amd/sequence.py describes it), and, where the
motion model fails, TrackReferenceKeyFrame against the reference keyframe (:318-324): mpReferenceKF,
UpdateLocalKeyFrames' pKFmax after every tracked frame (:1459-1570, the keyframe that created the most of
the frame's map points, first maximum in keyframe order; not on a LOST frame) or the keyframe a keyframe
frame creates (CreateNewKeyFrame, :1258).  The first
tracked frame has no velocity yet and runs TrackReferenceKeyFrame (:791-882:
ComputeBoW, SearchByBoW against keyframe 0, the same graph / PoseOptimization /
discard) when the keyframe's BoW inputs are given."""
from __future__ import annotations

import numpy as np

import oracle_grab
import oracle_match as OM
import oracle_step
import oracle_track as OT


_VOCAB = {}
KEYFRAME_STEP = 10  # synth.KEYFRAME_STEP


def _local_mapping(lm, t, T2, P, o, pose_cfg, on_lba):
    """sp-slam_amd/sequence.py SequencePath._local_mapping for one sequence: the bookkeeping by
    oracle_local_map.KeyframeMap, LocalBundleAdjustment by the oracle."""
    import oracle_lba
    import oracle_local_map as OLM
    j = t // KEYFRAME_STEP
    _, _, pls = o["graph2"]
    _, _, plo2 = o["pose2"]
    kun = o["keys_un"]
    matched, keys, ur, octave, edges = OLM.keyframe_inputs(P, kun, o["frame"]["uright"], len(kun), pls, plo2)
    lm.insert_keyframe(j, T2, keys, ur, octave, matched, edges)
    if j < 2:
        return T2, P
    arrays, book = lm.lba_problem(j)
    cfg = None
    if pose_cfg is not None:
        cfg = np.array([pose_cfg.angle_info, pose_cfg.distance_info, pose_cfg.parallel_info, pose_cfg.vertical_info,
                        pose_cfg.chi, pose_cfg.vp_chi], np.float64)
    r = oracle_lba.lba_optimize(*arrays, **({} if cfg is None else {"cfg": cfg}))
    lm.apply(book, r["Tcw"], r["points"], r["planes"], r["point_outlier"], int(r["result"]["stopped"]))
    if on_lba:
        on_lba(t, dict(r, kfs=list(book["kfs"])))
    return lm.kfs[j]["Tcw"].copy(), lm.refresh_last_frame(P)


def vocabulary(text):
    """oracle_bow.Vocabulary of a vocabulary text, loaded once per process."""
    import hashlib
    import oracle_bow
    key = hashlib.sha1(text).hexdigest()
    if key not in _VOCAB:
        _VOCAB[key] = oracle_bow.Vocabulary(text)
    return _VOCAB[key]


def reference_keyframe(ref, vocab_text):
    """ref = (keypoints, descriptors, has_point, row) of the reference keyframe (sequence.py
    oracle_seq_inputs.reference_keyframe) -> FrameInputs.ref_kf."""
    kps, desc, has, row = ref
    V = vocabulary(vocab_text)
    return dict(vocab=V, desc=desc, angle=kps["angle"], has_point=has, fv=V.transform(desc), row=row)


def track(frames, first, T0, P0, local_of, cam, geometry, inv_sigma2, map_planes, boundary, orb, planes,
          supp_cap=None, min_size=500, pose_cfg=None, depth_scale=None, on_frame=None, libm=None, ref_kf=None,
          local_map=None, on_lba=None, refkf_of=None, perturb=None, kf_id_stride=None):
    """frames: [(rgb, depth_u16)] of frames first .. ; T0 / P0: the pose and last-frame points of frame
    first - 1; local_of(t): the local map points of frame t (whole; the seen ones are skipped).  Returns the
    local-map pose (float 4x4) of every frame.  local_map: an oracle_local_map.KeyframeMap (keyframe 0
    inserted) -- the deterministic LocalMapping after every keyframe frame, LocalBundleAdjustment by the CPU
    oracle (oracle/lba_oracle.cpp), the map it reads replaced by the SeqMap's (local points, map planes);
    on_lba(t, result) sees each LocalBundleAdjustment.  refkf_of(j): FrameInputs.refkf_fallback of keyframe j (the
    TrackWithMotionModel -> TrackReferenceKeyFrame switch against the reference keyframe; None: no fallback);
    kf_id_stride: map point id // kf_id_stride = the keyframe that created it (the reference-keyframe vote).  perturb: {t: 4x4 velocity} replacing
    frame t's motion-model velocity (a test hook).  ref_kf: FrameInputs.ref_kf of frame `first` (reference_keyframe;
    None keeps the motion model with a constant-position prior there).  libm: the elementary functions of PoseOptimization
    (oracle_ctypes.LIBM_*) for this call, on the calling thread; None keeps the current one."""
    if libm is not None:
        import oracle_ctypes
        with oracle_ctypes.libm(libm):
            return track(frames, first, T0, P0, local_of, cam, geometry, inv_sigma2, map_planes, boundary, orb,
                         planes, supp_cap, min_size, pose_cfg, depth_scale, on_frame, None, ref_kf, local_map, on_lba,
                         refkf_of, perturb, kf_id_stride)
    Tlw = np.asarray(T0, np.float32).reshape(4, 4)
    V = np.eye(4, dtype=np.float32)  # the first tracked frame starts at the last frame's pose (SetPose(mLastFrame.mTcw))
    P = P0
    ref_j = 0  # mpReferenceKF: keyframe 0 (StereoInitialization, :584)
    poses = []
    for k, (rgb, d) in enumerate(frames):
        t = first + k
        gray = oracle_grab.cvt_gray(rgb, rgb=True)
        depth = oracle_grab.convert_depth(d, depth_scale)
        pfr = np.zeros((), OM.PROJ_FRAME_DTYPE)
        if perturb and t in perturb:
            V = np.asarray(perturb[t], np.float32).reshape(4, 4)
        pfr["Tcw"] = OT.mat4(V, Tlw).reshape(16)
        pfr["Tlw"] = Tlw.reshape(16)
        pfr["n_points"] = len(P)
        LP = local_of(t) if local_map is None else local_map.local_points(t)
        if local_map is not None:
            map_planes = local_map.planes
        lfr = np.zeros((), OM.LOCAL_FRAME_DTYPE)
        lfr["n_points"] = len(LP)
        fi = oracle_step.FrameInputs(gray, depth, cam, geometry, inv_sigma2, (pfr, P), (lfr, LP), map_planes,
                                     boundary, min_size=min_size, pose_cfg=pose_cfg, local_seen=True,
                                     ref_kf=ref_kf if k == 0 else None,
                                     refkf_fallback=(lambda j=ref_j: refkf_of(j)) if refkf_of and not (k == 0 and ref_kf)
                                     else None)
        o = oracle_step.run(fi, orb, planes, supp_cap=supp_cap)
        if kf_id_stride and o["fallback"] != 2:  # UpdateLocalKeyFrames (TrackLocalMap runs unless LOST)
            ids = o["proj_points"]["id"][o["match"][o["keep"]]].astype(np.int64)
            if len(ids):
                ref_j = int(np.argmax(np.bincount(ids // kf_id_stride)))  # the first maximum
        if t % KEYFRAME_STEP == 0:
            ref_j = t // KEYFRAME_STEP  # CreateNewKeyFrame
        o["reference_keyframe"] = ref_j
        T2 = np.asarray(o["pose2"][0]["Tcw"], np.float32).reshape(4, 4)
        P = OT.last_frame(o["proj_points"], o["match"], o["keep"], LP, o["local_match"], o["keys_un"], o["pose2"][1])
        V = OT.mat4(T2, OT.inverse_pose(Tlw))
        Tlw = T2
        if local_map is not None and t % KEYFRAME_STEP == 0:
            Tlw, P = _local_mapping(local_map, t, T2, P, o, pose_cfg, on_lba)
        poses.append(T2.copy())
        if on_frame:
            on_frame(t, o, P)
    return poses
