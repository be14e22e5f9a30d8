"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Host copies of what a slot of a tracked sequence (sp-slam_amd/sequence.py SequencePath) tracks, in the form the
CPU oracle's loop takes them (oracle/oracle_sequence.track): the frames, the frame-0 pose and last-frame points, the
local map of every frame, the keyframes' BoW inputs and map points for TrackReferenceKeyFrame, and a fresh copy of
the deterministic LocalMapping's map.  Used by tests/test_gpu_sequence.py and bench.py's ATE leg (the checker); the
product package does not import it."""
from __future__ import annotations

import numpy as np

import oracle_sequence
import spslam_gpu as G
import synth


def inputs(sp, slot):
    """(frames 1 .. T-1, frame-0 pose, frame-0 last-frame points, local_of(t) = frame t's whole local map)."""
    u = slot % sp.U
    P0 = synth.as_last_frame_points(sp.kf_points[u, 0], sp.kf_kps[u, 0], 0)
    T0 = sp._true_pose(u, 0).astype(np.float32)
    allp = np.concatenate([sp.kf_points[u, j] for j in range(len(sp.kf_t))])
    base = sp.local_offsets[u, 0]

    def local_of(t):
        r = sp.local_table[t, slot]
        o = int(r["point_offset"]) - base
        return allp[o:o + int(r["n_points"])]
    return sp.seq_frames[u][1:], T0, P0, local_of


def reference_keyframe(sp, slot):
    """(keypoints, descriptors, has_point, row) of the slot's keyframe 0 -- frame 1's TrackReferenceKeyFrame
    reference -- for oracle_sequence.reference_keyframe."""
    u = slot % sp.U
    n = int(sp.d_kf0_cnt[u])
    kps = sp.d_kf0_kps[u, :n].cpu().numpy().view(G.KEYPOINT_DTYPE).reshape(n)
    return kps, sp.d_kf0_desc[u, :n].cpu().numpy(), sp.kf0_has[u, :n], sp.kf0_row[u, :n]


def refkf_of(sp, slot, vocab_text):
    """refkf_of(j) for oracle_sequence.track: keyframe j of the slot's sequence as
    oracle_step.FrameInputs.refkf_fallback -- BoW inputs, feature -> row map and its map points."""
    u, nkf, cap = slot % sp.U, len(sp.kf_t), sp.kp_cap
    cache = {}

    def of(j):
        q = u * nkf + j
        if q not in cache:
            n = int(sp.d_kf_cnt[q])
            kps = sp.d_kf_kps[q, :n].cpu().numpy().view(G.KEYPOINT_DTYPE).reshape(n)
            has = sp.d_kf_has[q, :n].cpu().numpy()
            row = sp.d_kf_row[q, :n].cpu().numpy()
            R = oracle_sequence.reference_keyframe((kps, sp.d_kf_desc[q, :n].cpu().numpy(), has, row), vocab_text)
            R["points"] = synth.as_last_frame_points(sp.kf_points[u, j], sp.kf_kps[u, j], j * cap)
            cache[q] = R
        return cache[q]
    return of


def local_map(sp, slot):
    """A fresh oracle_local_map.KeyframeMap of the slot's sequence as it stood before frame 1 (keyframe 0
    inserted) -- the checker's own LocalMapping bookkeeping (the GPU loop runs sp-slam_amd/local_mapping.py)."""
    import oracle_local_map as LM
    u = slot % sp.U
    tab = sp.ex.tables()
    m = LM.KeyframeMap([sp.kf_points[u, j] for j in range(len(sp.kf_t))], sp.kp_cap,
                  (sp.fx, sp.fy, sp.cx, sp.cy, sp.bf), tab["scale"], tab["inv_sigma2"], sp.assoc_map)
    LM.insert_initial_keyframe(m, sp._true_pose(u, 0).astype(np.float32), sp.kf_kps[u, 0], sp.seq_frames[u][0][1],
                               sp.depth_factor, sp.bf)
    return m
