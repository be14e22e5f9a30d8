"""Tracked RGB-D sequences on the GPU: the batched hot path run frame after frame,
each batch slot carrying its own tracking state (Tracking::Track, src/Tracking.cc:
276-526).

Batch k holds frame t = k + 1 of every slot's sequence.  Per batch the tracking tail
(one HIP stream, nothing returns to the host) is

  SPSLAM_TRACK_MOTION_PRIOR  mCurrentFrame.SetPose(mVelocity * mLastFrame.mTcw)  (:958)
  frame steps, SearchByProjection against the last frame's map points, association,
  PoseOptimization, outlier discard (+ mnLastFrameSeen stamps), SearchLocalPoints over
  the local map (seen points skipped on the device), association, PoseOptimization
                                                       (pipeline.HotPath, :950-1136)
  SPSLAM_TRACK_LAST_FRAME    mVelocity, VO-match clean-up, outlier drop,
                             mLastFrame = mCurrentFrame  (:443-505)

so frame t's prior, last-frame map points and matches all come from frame t-1's
tracked result.  The map is the harness's stand-in for LocalMapping: keyframes on a
fixed schedule (every synth.KEYFRAME_STEP frames) whose map points are their own
keypoints back-projected at the true pose (synth.keyframe_points); frame t's local map
is the points of the two latest keyframes before it; map planes are the scene faces.
Deviations from the reference, all shared with the CPU oracle
(oracle/oracle_sequence.py): keyframes are not chosen by NeedNewKeyFrame and do not
add the current frame's VO points; LocalBundleAdjustment does not move them;
mLastFrame's pose is not re-derived through its reference keyframe (UpdateLastFrame,
an identity up to float rounding with fixed keyframes); frame 0 is initialised at its
true pose with keyframe 0's points (StereoInitialization).  Frame 1 has no velocity
yet and runs TrackReferenceKeyFrame (:791-882) on the device: ComputeBoW of the
frame, SearchByBoW against keyframe 0 (ORBmatcher(0.7, true)), then the same graph,
PoseOptimization and outlier discard as the motion model, from SetPose(mLastFrame.mTcw).
The vocabulary is synth.shape_vocabulary_text() (ORBvoc.txt's k = 10, L = 6 shape;
the trained file is not vendored).

Sequence u of a rank is the scene's trajectory from frame `SEQ_STRIDE * u`; slot i
tracks sequence i % U (slots sharing a sequence carry identical, independent state).
"""
from __future__ import annotations

import time

import numpy as np

import pipeline
import spslam_gpu as G
import spslam_match as SM
import synth

SEQ_STRIDE = 53


def _render_job(args):
    scene_seq, n_boxes, first, n, w, h, K, noise_base, style = args
    sc = synth.Scene(scene_seq, n_boxes=n_boxes, **style)
    out = []
    for t in range(first, first + n):
        g, d, fid = sc.render(sc.pose(t), w, h, K=K, noise_seed=noise_base + t)
        out.append((synth.colorize(g, fid), d))
    return out


def render_sequences(seq_id, n_boxes, U, T, w, h, K, workers=0, texture="dots", motion="smooth"):
    """frames[u][t] = (rgb, depth u16) of sequence u (scene seq_id, trajectory from SEQ_STRIDE * u)."""
    style = dict(texture=texture, motion=motion)
    jobs = [(seq_id, n_boxes, SEQ_STRIDE * u, T, w, h, K, seq_id * 100003, style) for u in range(U)]
    if workers and workers > 1:
        import concurrent.futures as cf
        import multiprocessing as mp
        chunks = []
        for seq, nb, first, n, ww, hh, KK, nz, tx in jobs:  # split sequences into chunks of frames
            step = max(1, -(-n // max(1, workers // len(jobs))))
            chunks += [(seq, nb, f0, min(step, first + n - f0), ww, hh, KK, nz, tx)
                       for f0 in range(first, first + n, step)]
        with cf.ProcessPoolExecutor(workers, mp_context=mp.get_context("spawn")) as pool:
            parts = list(pool.map(_render_job, chunks))
        out, k = [], 0
        for seq, nb, first, n, *_ in jobs:
            frames = []
            while len(frames) < n:
                frames += parts[k]
                k += 1
            out.append(frames)
        return out
    return [_render_job(j) for j in jobs]


class SequencePath(pipeline.HotPath):
    """HotPath over T frames of U sequences (B slots, slot i -> sequence i % U)."""

    def __init__(self, B, n_frames, n_sequences=None, render_workers=0, local_mapping=None, refkf_fallback=None,
                 **kw):
        """local_mapping: run the deterministic LocalMapping (local_mapping.py: keyframe insertion and
        LocalBundleAdjustment written back into the map) after every keyframe frame; default: on when the
        config asks for LocalBundleAdjustment (C3's lba_every), off otherwise."""
        self.T = n_frames
        self.U = min(n_sequences or B, B)
        self.d_load_idx = None
        self.vel_perturb = {}
        self.render_workers = render_workers
        self.n_boxes = kw.get("n_boxes", 3)
        lba_every = kw.pop("lba_every", 0)  # the side-by-side synthetic local maps of the open-loop HotPath
        self.local_mapping = bool(lba_every) if local_mapping is None else bool(local_mapping)
        # TrackWithMotionModel -> TrackReferenceKeyFrame on the device (default: on without LocalMapping; the
        # LocalMapping harness moves the keyframes' points, which the reference keyframe sets do not follow)
        self.refkf_fallback = (not self.local_mapping) if refkf_fallback is None else bool(refkf_fallback)
        if self.refkf_fallback and self.local_mapping:
            raise ValueError("refkf_fallback with local_mapping is not supported")
        kw.pop("unique_frames", None)
        kw.pop("rotate_inputs", None)
        super().__init__(B, unique_frames=self.U, **kw)

    # ---- inputs: every frame of every sequence resident in HBM, loaded per batch
    def _setup_inputs(self, seq_id, unique_frames):
        torch, B, U, T = self.torch, self.B, self.U, self.T
        self.seq_id = seq_id
        self.seq_frames = render_sequences(seq_id, self.n_boxes, U, T, self.W, self.H, self.K, self.render_workers,
                                           texture=self.texture, motion=self.motion)
        rgb = np.stack([self.seq_frames[u][t][0] for t in range(T) for u in range(U)])
        dep = np.stack([self.seq_frames[u][t][1] for t in range(T) for u in range(U)]).view(np.int16)
        self.d_rgb_all = torch.from_numpy(rgb).cuda()         # [T * U] frames, frame t of sequence u at t*U + u
        self.d_depth_all = torch.from_numpy(dep).cuda()
        self.frames = [(SEQ_STRIDE * u, self.seq_frames[u][0][0], self.seq_frames[u][0][1], None) for u in range(U)]
        self.d_rgb = self.d_rgb_all[[U + i % U for i in range(B)]].clone()   # frame 1 (batch 0)
        self.d_depth_raw = self.d_depth_all[[U + i % U for i in range(B)]].clone()
        if B > U:
            self.d_load_idx = torch.tensor([[t * U + i % U for i in range(B)] for t in range(T)], dtype=torch.long,
                                           device="cuda")

    def _true_pose(self, u, t):
        return np.linalg.inv(self.scene.pose(SEQ_STRIDE * u + t))

    # ---- the map: keyframe points, the initial last frame, the per-batch local maps
    def _setup_match(self, seq_id):
        torch, B, U, T, cap = self.torch, self.B, self.U, self.T, self.kp_cap
        kf_t = list(range(0, T, synth.KEYFRAME_STEP))
        self.kf_t = kf_t
        # ORB of every keyframe frame, on the device (bit-exact with the oracle)
        idx = [t * U + u for u in range(U) for t in kf_t]
        n = len(idx)
        d_g = torch.zeros((n, self.H, self.W), dtype=torch.uint8, device="cuda")
        d_d = torch.zeros((n, self.H, self.W), dtype=torch.float32, device="cuda")
        rgb, dep = self.d_rgb_all[idx].contiguous(), self.d_depth_all[idx].contiguous()
        self.grabber.batch_device(n, rgb.data_ptr(), self.H * self.W * 3, self.W * 3, dep.data_ptr(), self.H * self.W,
                                  self.W, self.W, self.H, d_g.data_ptr(), d_d.data_ptr(), self.stream)
        d_k = torch.zeros((n, cap, 7), dtype=torch.float32, device="cuda")
        d_ds = torch.zeros((n, cap, 32), dtype=torch.uint8, device="cuda")
        d_n = torch.zeros(n, dtype=torch.int32, device="cuda")
        for c0 in range(0, n, B):  # the context's batch capacity
            m = min(B, n - c0)
            self.ex.extract_batch_device(d_g[c0].data_ptr(), m, self.W * self.H, self.W, d_k[c0].data_ptr(),
                                         d_ds[c0].data_ptr(), d_n[c0].data_ptr(), cap, self.stream)
        torch.cuda.synchronize()
        kps = d_k.cpu().numpy().view(G.KEYPOINT_DTYPE).reshape(n, cap)
        desc, cnt = d_ds.cpu().numpy(), d_n.cpu().numpy()
        kf0 = [u * len(kf_t) for u in range(U)]  # keyframe 0 of each sequence: TrackReferenceKeyFrame's reference
        self.d_kf0_kps, self.d_kf0_desc, self.d_kf0_cnt = d_k[kf0].clone(), d_ds[kf0].clone(), d_n[kf0].clone()
        self.d_kf_kps, self.d_kf_desc, self.d_kf_cnt = d_k, d_ds, d_n  # every keyframe (q = u * len(kf_t) + j)
        self.n_ids = len(kf_t) * cap                   # map point ids per sequence: keyframe index * cap + keypoint
        self.kf_points, self.kf_kps = {}, {}
        offs, pts = {}, []
        o = 0
        for u in range(U):
            for j, t in enumerate(kf_t):
                q = u * len(kf_t) + j
                sc_t = SEQ_STRIDE * u + t
                P = synth.keyframe_points(self.scene, sc_t, kps[q, :cnt[q]], desc[q, :cnt[q]],
                                          self.seq_frames[u][t][1], j * cap, K=self.Ks)
                self.kf_points[u, j], self.kf_kps[u, j] = P, kps[q, :cnt[q]].copy()
                offs[u, j] = o
                pts.append(P)
                o += len(P)
        self.d_lpoints = torch.from_numpy(np.concatenate(pts).view(np.uint8).copy()).cuda()
        # frame t's local map: the two latest keyframes before it (contiguous in the point array)
        lfr = np.zeros((T, B), SM.LOCAL_FRAME_DTYPE)
        for t in range(1, T):
            j = (t - 1) // synth.KEYFRAME_STEP
            for i in range(B):
                u = i % U
                a = max(j - 1, 0)
                lfr[t, i]["point_offset"] = offs[u, a]
                lfr[t, i]["n_points"] = sum(len(self.kf_points[u, q]) for q in range(a, j + 1))
                lfr[t, i]["seen_offset"] = i * self.n_ids
                lfr[t, i]["stamp"] = t
        self.local_table = lfr
        self.max_local_points = int(lfr["n_points"].max())
        self.local_offsets = offs
        self.d_local_table = torch.from_numpy(lfr.view(np.uint8).reshape(T, -1).copy()).cuda()
        self.d_lframes = self.d_local_table[1].clone()
        self.d_seen = torch.full((B * self.n_ids,), -1, dtype=torch.int32, device="cuda")
        # frame 0 (StereoInitialization): true pose, keyframe 0's points are its map points
        pf = np.zeros(B, SM.PROJ_FRAME_DTYPE)
        # the last-frame point sets (f * cap), then every keyframe's map points as TrackReferenceKeyFrame's point
        # set (keypoint order, the rows its BoW matches index)
        nkf = len(kf_t)
        kfsets = [synth.as_last_frame_points(self.kf_points[u, j], self.kf_kps[u, j], j * cap) for u in range(U)
                  for j in range(nkf)]
        self.kf_set_off = B * cap + np.concatenate([[0], np.cumsum([len(k) for k in kfsets])[:-1]]).astype(np.int64)
        self.kf_set_len = np.array([len(k) for k in kfsets], np.int64)
        pp = np.zeros(B * cap + int(self.kf_set_len.sum()), SM.PROJ_POINT_DTYPE)
        for q, k in enumerate(kfsets):
            pp[self.kf_set_off[q]:self.kf_set_off[q] + len(k)] = k
        for i in range(B):
            u = i % U
            P0 = synth.as_last_frame_points(self.kf_points[u, 0], self.kf_kps[u, 0], 0)
            pp[i * cap:i * cap + len(P0)] = P0
            T0 = self._true_pose(u, 0).astype(np.float32).reshape(16)
            pf[i]["Tcw"], pf[i]["Tlw"], pf[i]["point_offset"], pf[i]["n_points"] = T0, T0, i * cap, len(P0)
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()  # noqa
        self.proj_sets = [(dev(pf), dev(pp)), (dev(pf), dev(pp))]
        self.d_pframes, self.d_ppoints = self.proj_sets[0]
        self.max_points = cap
        self.d_velocity = torch.from_numpy(np.tile(np.eye(4, dtype=np.float32).reshape(16), B)).cuda()
        self.match_probs = [(pf[i], None) for i in range(U)]   # _setup_assoc reads the initial pose
        self.mean_proj_points = float(np.mean([int(pf[i]["n_points"]) for i in range(B)]))
        self.mean_local_points = float(lfr["n_points"][1:].mean())
        self.d_match = torch.zeros((B, cap), dtype=torch.int32, device="cuda")
        self.d_nmatch = torch.zeros(B, dtype=torch.int32, device="cuda")
        self.local_matcher = SM.LocalMatcher(self.ex)
        self._setup_reference_keyframe()
        self.matcher = SM.Matcher(self.ex)
        self.d_taken = torch.zeros((B, cap), dtype=torch.uint8, device="cuda")
        self.d_lmatch = torch.zeros((B, cap), dtype=torch.int32, device="cuda")
        self.d_nlmatch = torch.zeros(B, dtype=torch.int32, device="cuda")
        self.local_probs = []
        self.traj = torch.zeros((T, B, 16), dtype=torch.float32, device="cuda")
        # per frame: SearchByProjection matches, SearchLocalPoints matches, inliers of both PoseOptimizations
        self.hist = torch.zeros((T, 4, B), dtype=torch.int32, device="cuda")
        self.n_tracked = 0

    def _setup_reference_keyframe(self):
        """Keyframe 0's BoW side of SearchByBoW (KeyFrame::ComputeBoW at its creation) and the map of its
        features to the rows of the frame-0 point set (the map point each feature holds, -1 without one)."""
        import spslam_bow as SB
        torch, B, U, cap = self.torch, self.B, self.U, self.kp_cap
        self.vocab = SB.Vocabulary(self.ex, synth.shape_vocabulary_text())
        i32 = dict(dtype=torch.int32, device="cuda")
        has = np.zeros((U, cap), np.uint8)
        row = np.full((U, cap), -1, np.int32)
        for u in range(U):
            kpi = (self.kf_points[u, 0]["id"] - 0).astype(np.int64)  # keyframe 0's ids: id_base 0 + keypoint
            has[u, kpi] = 1
            row[u, kpi] = np.arange(len(kpi), dtype=np.int32)       # as_last_frame_points keeps keypoint order
        self.d_kf0_has = torch.from_numpy(has).cuda()
        self.d_kf0_row = torch.from_numpy(row).cuda()
        self.kf0_has, self.kf0_row = has, row

        def fv_buffers(n):
            return dict(words=torch.zeros((n, cap), **i32), values=torch.zeros((n, cap), dtype=torch.float64,
                                                                              device="cuda"),
                        n_bow=torch.zeros(n, **i32), nodes=torch.zeros((n, cap), **i32),
                        start=torch.zeros((n, cap + 1), **i32), features=torch.zeros((n, cap), **i32),
                        n_fv=torch.zeros(n, **i32))
        self.kf0_bow, self.fr_bow = fv_buffers(U), fv_buffers(B)
        self._bow_transform(U, self.d_kf0_desc, self.d_kf0_cnt, self.kf0_bow)
        self.kf0_side = SB.BowSide(self.d_kf0_desc.data_ptr(), self.d_kf0_kps.data_ptr(), self.d_kf0_has.data_ptr(),
                                   self.d_kf0_cnt.data_ptr(), self.kf0_bow["nodes"].data_ptr(),
                                   self.kf0_bow["start"].data_ptr(), self.kf0_bow["features"].data_ptr(),
                                   self.kf0_bow["n_fv"].data_ptr(), cap, 0)
        self.d_bow_pairs = torch.tensor([(i % U, i) for i in range(B)], **i32)
        self.d_bow_match = torch.zeros((B, cap), **i32)
        self.d_bow_n = torch.zeros(B, **i32)
        self.slot_u = torch.tensor([i % U for i in range(B)], dtype=torch.long, device="cuda")
        torch.cuda.synchronize()

    def _bow_transform(self, n, d_desc, d_cnt, out):
        self.vocab.transform_batch_device(n, d_desc.data_ptr(), d_cnt.data_ptr(), self.kp_cap, 4,
                                          out["words"].data_ptr(), out["values"].data_ptr(), out["n_bow"].data_ptr(),
                                          out["nodes"].data_ptr(), out["start"].data_ptr(),
                                          out["features"].data_ptr(), out["n_fv"].data_ptr(), stream=self.stream)

    def match(self):
        if self.n_tracked > 0:
            return super().match()  # TrackWithMotionModel's SearchByProjection
        # frame 1: TrackReferenceKeyFrame -- mCurrentFrame.ComputeBoW(); SearchByBoW(mpReferenceKF, mCurrentFrame)
        import spslam_bow as SB
        self._bow_transform(self.B, self.d_desc, self.d_cnt, self.fr_bow)
        fr = SB.BowSide(self.d_desc.data_ptr(), self.d_kps.data_ptr(), 0, self.d_cnt.data_ptr(),
                        self.fr_bow["nodes"].data_ptr(), self.fr_bow["start"].data_ptr(),
                        self.fr_bow["features"].data_ptr(), self.fr_bow["n_fv"].data_ptr(), self.kp_cap, 0)
        SB.search_by_bow_batch_device(self.ex, self.B, self.d_bow_pairs.data_ptr(), self.kf0_side, fr,
                                      self.d_bow_match.data_ptr(), self.d_bow_n.data_ptr(), nn_ratio=0.7,
                                      check_orientation=True, stream=self.stream)
        # mvpMapPoints = vpMapPointMatches: keyframe feature -> its map point's row in the frame-0 point set
        torch = self.torch
        with torch.cuda.stream(self.main):
            m = self.d_bow_match
            rows = torch.gather(self.d_kf0_row[self.slot_u], 1, m.clamp(min=0).long())
            self.d_match.copy_(torch.where(m >= 0, rows, torch.full_like(rows, -1)))
            self.d_nmatch.copy_(self.d_bow_n)

    def _setup_assoc(self, seq_id):
        super()._setup_assoc(seq_id)
        self.d_afr_first = self.d_afr1  # MOTION_PRIOR writes the first association's pose
        if self.local_mapping:
            # each sequence its own copy of the map planes (LocalBundleAdjustment moves them): slot i reads copy
            # i % U (association indices are absolute into the copies)
            import spslam_assoc as SA
            U, n = self.U, self.n_map
            self.d_map = self.torch.from_numpy(np.tile(self.assoc_map, U).view(np.uint8).copy()).cuda()
            for d in (self.d_afr1, self.d_afr2):
                fr = d.cpu().numpy().view(SA.ASSOC_FRAME_DTYPE).copy()
                fr["map_offset"] = [(i % U) * n for i in range(self.B)]
                d.copy_(self.torch.from_numpy(fr.view(np.uint8)))

    def _setup_track(self):
        super()._setup_track()
        if self.local_mapping:
            self._setup_local_mapping()
        if self.refkf_fallback:
            self._setup_refkf()

    def _setup_refkf(self):
        """TrackWithMotionModel -> TrackReferenceKeyFrame (Tracking.cc:318-324): every keyframe's BoW side and the
        rows of its map points (its point set in the projection buffer), each slot's reference keyframe
        (mpReferenceKF: keyframe 0 after StereoInitialization, then UpdateLocalKeyFrames' pKFmax or the keyframe just
        created, spslam_track_refkf_vote_batch_device after every frame), and the re-tracking's own buffers."""
        import spslam_bow as SB
        import spslam_track as ST
        torch, B, U, cap, T = self.torch, self.B, self.U, self.kp_cap, self.T
        nkf = len(self.kf_t)
        if nkf > 1024:
            raise ValueError(f"{nkf} keyframes per sequence: the reference-keyframe vote holds at most 1024")
        i32 = dict(dtype=torch.int32, device="cuda")
        u8 = dict(dtype=torch.uint8, device="cuda")
        has = np.zeros((U * nkf, cap), np.uint8)
        row = np.full((U * nkf, cap), -1, np.int32)
        for u in range(U):
            for j in range(nkf):
                kpi = (self.kf_points[u, j]["id"] - j * cap).astype(np.int64)
                has[u * nkf + j, kpi] = 1
                row[u * nkf + j, kpi] = np.arange(len(kpi), dtype=np.int32)
        self.d_kf_has, self.d_kf_row = torch.from_numpy(has).cuda(), torch.from_numpy(row).cuda()
        self.kf_bow = self._fv_buffers(U * nkf)
        self._bow_transform(U * nkf, self.d_kf_desc, self.d_kf_cnt, self.kf_bow)
        self.kf_side = SB.BowSide(self.d_kf_desc.data_ptr(), self.d_kf_kps.data_ptr(), self.d_kf_has.data_ptr(),
                                  self.d_kf_cnt.data_ptr(), self.kf_bow["nodes"].data_ptr(),
                                  self.kf_bow["start"].data_ptr(), self.kf_bow["features"].data_ptr(),
                                  self.kf_bow["n_fv"].data_ptr(), cap, 0)
        # keyframe q = u * nkf + j: its map points' (offset, count) in the projection buffer; per slot its sequence's
        # keyframe 0 (kf_base) and the current reference keyframe with its point set and SearchByBoW pair
        kf_sets = np.stack([self.kf_set_off, self.kf_set_len], 1).astype(np.int32)
        base = np.array([(i % U) * nkf for i in range(B)], np.int32)
        self.d_kf_sets = torch.from_numpy(kf_sets).cuda()
        self.d_kf_base = torch.from_numpy(base).cuda()
        self.d_refkf_q = torch.from_numpy(base.copy()).cuda()
        self.d_refkf_sets = torch.from_numpy(kf_sets[base].copy()).cuda()
        self.d_refkf_pairs = torch.from_numpy(np.stack([base, np.arange(B, dtype=np.int32)], 1)).cuda()
        self.refkf_hist = torch.zeros((T, B), **i32)  # [t][slot] the reference keyframe after frame t
        self.refkf_hist[0].copy_(self.d_refkf_q)
        P = self.pe.planes_cap + self.pe.supp_cap
        self.fb = dict(
            fallback=torch.zeros(B, **u8), apply=torch.zeros(B, **u8), counts=torch.zeros(B, **i32),
            frames=torch.zeros_like(self.d_pframes), assoc_frames=torch.zeros_like(self.d_afr1),
            match=torch.zeros((B, cap), **i32), taken=torch.zeros((B, cap), **u8), edge=torch.zeros((B, cap), **i32),
            res=torch.zeros_like(self.d_res1), assoc=torch.zeros((3, B * P), **i32), newp=torch.zeros(B, **i32),
            next=torch.zeros((3, B * P), **i32), lframes=torch.zeros_like(self.d_lframes),
            afr2=torch.zeros_like(self.d_afr2), bow_match=torch.zeros((B, cap), **i32), bow_n=torch.zeros(B, **i32),
            graph={k: torch.zeros_like(v) for k, v in self.graphs[0].items()})
        self.fb_hist = torch.zeros((T, B), dtype=torch.int8, device="cuda")  # 0 motion model, 1 reference kf, 2 lost
        self._track_mod = ST

    def _fv_buffers(self, n):
        torch, cap = self.torch, self.kp_cap
        i32 = dict(dtype=torch.int32, device="cuda")
        return dict(words=torch.zeros((n, cap), **i32), values=torch.zeros((n, cap), dtype=torch.float64,
                                                                          device="cuda"),
                    n_bow=torch.zeros(n, **i32), nodes=torch.zeros((n, cap), **i32),
                    start=torch.zeros((n, cap + 1), **i32), features=torch.zeros((n, cap), **i32),
                    n_fv=torch.zeros(n, **i32))

    def _after_motion_model(self):
        """TrackWithMotionModel's verdict and, for the frames it fails, TrackReferenceKeyFrame (_refkf_fallback); then
        the reference keyframe the next frame falls back to (_refkf_vote)."""
        if not self.refkf_fallback:
            return
        if self.n_tracked > 0:  # frame 1 already tracks the reference keyframe
            self._refkf_fallback()
        self._refkf_vote()

    def _refkf_vote(self):
        """mpReferenceKF after frame t (spslam_track_refkf_vote_batch_device): TrackLocalMap's UpdateLocalKeyFrames
        makes it pKFmax, the keyframe that created the most of the frame's map points after the discard
        (Tracking.cc:1459-1570; not on a LOST frame), and a keyframe frame's CreateNewKeyFrame makes it the new
        keyframe (:1258)."""
        ST, torch = self._track_mod, self.torch
        t = self.n_tracked + 1
        v = ST.RefkfVote(kf_base=self.d_kf_base.data_ptr(), kf_sets=self.d_kf_sets.data_ptr(), ids_per_kf=self.kp_cap,
                         n_kf=len(self.kf_t), new_kf=t // synth.KEYFRAME_STEP if t % synth.KEYFRAME_STEP == 0 else -1,
                         state=self.fb_hist[t].data_ptr(), refkf_index=self.d_refkf_q.data_ptr(),
                         refkf_sets=self.d_refkf_sets.data_ptr(), refkf_pairs=self.d_refkf_pairs.data_ptr())
        self.track.refkf_vote_device(self.B, self._track_batch(0), v, stream=self.stream)
        with torch.cuda.stream(self.main):
            self.refkf_hist[t].copy_(self.d_refkf_q)

    def _refkf_fallback(self):
        """TrackWithMotionModel's verdict and, for the frames it fails, TrackReferenceKeyFrame (Tracking.cc:318-324,
        791-882) on the device: ComputeBoW + SearchByBoW against the reference keyframe; where that finds >= 10
        matches, association, graph, PoseOptimization and discard from the last frame's pose over the keyframe's
        map points, moved over the motion model's outputs (spslam_track_refkf_batch_device,
        spslam_masked_frame_copy_device).  Frames where the motion model holds pass through every kernel as empty
        problems."""
        import spslam_bow as SB
        import spslam_planes as SP
        ST, torch, B, cap, fb = self._track_mod, self.torch, self.B, self.kp_cap, self.fb
        t = self.n_tracked + 1
        mm = self._track_batch(0)
        rk = ST.RefkfBatch(nmatches=self.d_nmatch.data_ptr(), fallback=fb["fallback"].data_ptr(),
                           refkf_counts=fb["counts"].data_ptr(), bow_nmatches=fb["bow_n"].data_ptr(),
                           bow_match=fb["bow_match"].data_ptr(), refkf_rows=self.d_kf_row.data_ptr(),
                           refkf_index=self.d_refkf_q.data_ptr(), rows_stride=cap,
                           refkf_sets=self.d_refkf_sets.data_ptr(), assoc_frames=self.d_afr1.data_ptr(),
                           apply=fb["apply"].data_ptr(), state=self.fb_hist[t].data_ptr(),
                           refkf_match=fb["match"].data_ptr(), refkf_frames=fb["frames"].data_ptr(),
                           refkf_assoc=fb["assoc_frames"].data_ptr())
        self.track.refkf_device(B, ST.REFKF_PREPARE, mm, rk, stream=self.stream)
        # mCurrentFrame.ComputeBoW(); SearchByBoW(mpReferenceKF, mCurrentFrame) -- on the failing frames only
        self._bow_transform(B, self.d_desc, fb["counts"], self.fr_bow)
        fr = SB.BowSide(self.d_desc.data_ptr(), self.d_kps.data_ptr(), 0, fb["counts"].data_ptr(),
                        self.fr_bow["nodes"].data_ptr(), self.fr_bow["start"].data_ptr(),
                        self.fr_bow["features"].data_ptr(), self.fr_bow["n_fv"].data_ptr(), cap, 0)
        SB.search_by_bow_batch_device(self.ex, B, self.d_refkf_pairs.data_ptr(), self.kf_side, fr,
                                      fb["bow_match"].data_ptr(), fb["bow_n"].data_ptr(), nn_ratio=0.7,
                                      check_orientation=True, stream=self.stream)
        self.track.refkf_device(B, ST.REFKF_SELECT, mm, rk, stream=self.stream)
        # the re-tracking starts from the motion model's surviving planes and its local-frame / next-association
        # records (the frames it is applied to)
        a, n = fb["assoc"], fb["next"]
        self.track.masked_copy_device(B, fb["apply"].data_ptr(),
                                      [(a[k], self.d_assoc[1][k]) for k in range(3)] +
                                      [(fb["lframes"], self.d_lframes), (fb["afr2"], self.d_afr2)], stream=self.stream)
        # mCurrentFrame.SetPose(mLastFrame.mTcw); AssociatePlanesByBoundary; PoseOptimization; discard
        self.assoc.batch_device(B, fb["assoc_frames"].data_ptr(), self.d_planes.data_ptr(), SP.PLANE_DTYPE.itemsize,
                                self.d_pcnt.data_ptr(), self.pe.planes_cap, self.d_supp.data_ptr(),
                                SP.SUPPOSED_DTYPE.itemsize, self.d_scnt.data_ptr(), self.pe.supp_cap,
                                self.d_map.data_ptr(), self.d_bound.data_ptr(), self.n_map, a[0].data_ptr(),
                                a[1].data_ptr(), a[2].data_ptr(), fb["newp"].data_ptr(), stream=self.stream)
        g = fb["graph"]
        b = self._track_batch(0)
        b.proj_frames, b.proj_match = fb["frames"].data_ptr(), fb["match"].data_ptr()
        b.local_frames, b.taken = fb["lframes"].data_ptr(), fb["taken"].data_ptr()
        b.assoc_match, b.assoc_parallel, b.assoc_vertical = a[0].data_ptr(), a[1].data_ptr(), a[2].data_ptr()
        b.assoc_frames_next, b.plane_outlier = fb["afr2"].data_ptr(), g["plout"].data_ptr()
        b.next_match, b.next_parallel, b.next_vertical = n[0].data_ptr(), n[1].data_ptr(), n[2].data_ptr()
        b.problems, b.points, b.planes = g["P"].data_ptr(), g["pts"].data_ptr(), g["pls"].data_ptr()
        b.edge_of_kp, b.results, b.point_outlier = fb["edge"].data_ptr(), fb["res"].data_ptr(), g["pout"].data_ptr()
        b.assoc_frames_first = 0
        self.track.batch_device(B, ST.MOTION_MODEL, b, stream=self.stream)
        G.pose_optimize_batch_device(self.ex, B, g["P"].data_ptr(), g["pts"].data_ptr(), g["pls"].data_ptr(),
                                     fb["res"].data_ptr(), g["pout"].data_ptr(), g["plout"].data_ptr(),
                                     cfg=self.plane_cfg, stream=self.stream)
        self.track.batch_device(B, ST.DISCARD, b, stream=self.stream)
        g0 = self.graphs[0]
        regions = [(self.d_pframes, fb["frames"]), (self.d_match, fb["match"]), (self.d_nmatch, fb["bow_n"]),
                   (self.d_taken, fb["taken"]), (self.d_edge, fb["edge"]), (self.d_res1, fb["res"]),
                   (self.d_newp[0], fb["newp"]), (self.d_afr2, fb["afr2"]), (self.d_lframes, fb["lframes"])]
        regions += [(g0[k], g[k]) for k in ("P", "pts", "pls", "pout", "plout")]
        regions += [(self.d_assoc[0][k], a[k]) for k in range(3)] + [(self.d_assoc[1][k], n[k]) for k in range(3)]
        self.track.masked_copy_device(B, fb["apply"].data_ptr(), regions, stream=self.stream)

    def _setup_local_mapping(self):
        """local_mapping.SeqMap per sequence, keyframe 0 inserted (StereoInitialization: its own points), and the
        LocalMapping context (the reference's LocalMapping thread has its own; here it runs synchronously)."""
        import local_mapping as LM
        import spslam_lba as L
        U, cap = self.U, self.kp_cap
        tab = self.ex.tables()
        cam = (self.fx, self.fy, self.cx, self.cy, self.bf)
        pc = self.plane_cfg
        self.lm_cfg = (pc.angle_info, pc.distance_info, pc.parallel_info, pc.vertical_info, pc.chi, pc.vp_chi)
        self.maps = []
        for u in range(U):
            m = LM.SeqMap([self.kf_points[u, j] for j in range(len(self.kf_t))], cap, cam, tab["scale"],
                          tab["inv_sigma2"], self.assoc_map)
            LM.insert_initial_keyframe(m, self._true_pose(u, 0).astype(np.float32), self.kf_kps[u, 0],
                                       self.seq_frames[u][0][1], self.depth_factor, self.bf)
            self.maps.append(m)
        self.lm_ba = L.LocalBA(self.ex, cfg=self.lm_cfg)
        self.lm_runs = []  # per LocalBundleAdjustment: (frame, results of slot 0..U-1)
        # wall time of the LocalMapping events (host bookkeeping + the synchronous device LocalBundleAdjustment)
        self.lm_time = {"total_s": 0.0, "lba_s": 0.0}

    def _local_mapping(self, t):
        """After keyframe frame t's tail: insert keyframe t / STEP into every sequence's map and, with more than
        two keyframes, run LocalBundleAdjustment for every slot (one problem each, on the device) and write the
        result back (local-map points, the last frame's points and pose, map planes)."""
        import local_mapping as LM
        import spslam_lba as L
        torch, B, U, cap = self.torch, self.B, self.U, self.kp_cap
        j = t // synth.KEYFRAME_STEP
        self.main.synchronize()
        t_lm0 = time.perf_counter()
        pf = self.d_pframes.cpu().numpy().view(SM.PROJ_FRAME_DTYPE)
        npp = B * cap * SM.PROJ_POINT_DTYPE.itemsize  # the last-frame sets (the keyframe sets follow)
        pp = self.d_ppoints[:npp].cpu().numpy().view(SM.PROJ_POINT_DTYPE).reshape(B, cap)
        traj = self.traj[t].cpu().numpy().reshape(B, 4, 4)
        cnt = self.d_cnt.cpu().numpy()
        kun = self.d_kun.cpu().numpy().view(G.KEYPOINT_DTYPE).reshape(B, cap)
        kur = self.d_kur.cpu().numpy()
        g1 = self.graphs[1]
        P2 = g1["P"].cpu().numpy().view(G.POSE_PROBLEM_DTYPE)
        pls = g1["pls"].cpu().numpy().view(G.PLANE_OBS_DTYPE)
        plout = g1["plout"].cpu().numpy()
        for u in range(U):  # slot u carries sequence u (slots u + k U are identical copies)
            n = int(pf[u]["n_points"])
            o, nl = int(P2[u]["plane_offset"]), int(P2[u]["n_planes"])
            ins = LM.frame_keyframe_inputs(pp[u, :n], kun[u], kur[u], int(cnt[u]), pls[o:o + nl], plout[o:o + nl])
            matched, keys, ur, octave, edges = ins
            self.maps[u].insert_keyframe(j, traj[u], keys, ur, octave, matched, edges)
        if j < 2:  # LocalMapping::Run: LocalBundleAdjustment once the map holds more than two keyframes
            return
        probs = [self.maps[u].lba_problem(j) for u in range(U)]
        hdr = np.zeros(B, L.LBA_PROBLEM_DTYPE)
        parts = [[] for _ in range(5)]
        nk = npt = npo = npl = nplo = 0
        for i in range(B):
            prob, kfs, pts, pobs, pls_, plobs = probs[i % U][0]
            hdr[i] = prob
            hdr[i]["kf_offset"], hdr[i]["point_offset"], hdr[i]["plane_offset"] = nk, npt, npl
            pts = pts.copy()
            pts["obs_offset"] += npo
            pls_ = pls_.copy()
            pls_["obs_offset"] += nplo
            for q, a in enumerate((kfs, pts, pobs, pls_, plobs)):
                parts[q].append(a)
            nk += len(kfs); npt += len(pts); npo += len(pobs); npl += len(pls_); nplo += len(plobs)
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()  # noqa: E731
        ins = [dev(hdr)] + [dev(np.concatenate(p)) if sum(len(x) for x in p) else
                            torch.zeros(64, dtype=torch.uint8, device="cuda") for p in parts]
        outs = [torch.zeros((max(nk, 1), 16), dtype=torch.float32, device="cuda"),
                torch.zeros((max(npt, 1), 3), dtype=torch.float32, device="cuda"),
                torch.zeros((max(npl, 1), 4), dtype=torch.float32, device="cuda"),
                torch.zeros(max(npo, 1), dtype=torch.uint8, device="cuda"),
                torch.zeros(max(nplo, 1), dtype=torch.uint8, device="cuda"),
                torch.zeros(B * L.LBA_RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")]
        t_ba0 = time.perf_counter()
        self.lm_ba.batch_device(B, hdr, *[x.data_ptr() for x in ins], *[x.data_ptr() for x in outs],
                                stream=self.stream)
        self.main.synchronize()
        self.lm_time["lba_s"] += time.perf_counter() - t_ba0
        kf_o, pt_o, pl_o, po_o = (x.cpu().numpy() for x in outs[:4])
        res = outs[5].cpu().numpy().view(L.LBA_RESULT_DTYPE)
        run = []
        lp = self.d_lpoints.view(-1, SM.LOCAL_POINT_DTYPE.itemsize)
        for u in range(U):
            (_, kfs, pts, pobs, pls_, _), book = probs[u]
            h = hdr[u]
            k0, p0, q0 = int(h["kf_offset"]), int(h["point_offset"]), int(h["plane_offset"])
            o0 = sum(len(x) for x in parts[2][:u])  # slot u's first point observation
            m = self.maps[u]
            m.apply(book, kf_o[k0:k0 + len(kfs)], pt_o[p0:p0 + len(pts)], pl_o[q0:q0 + len(pls_)],
                    po_o[o0:o0 + len(pobs)], int(res[u]["stopped"]))
            run.append(dict(result=res[u].copy(), Tcw=kf_o[k0:k0 + len(kfs)].copy(),
                            points=pt_o[p0:p0 + len(pts)].copy(), kfs=list(book["kfs"])))
            # write-back: the sequence's local-map point table, the map planes, and for every slot of the
            # sequence the last frame's map points and pose (UpdateLastFrame: Tlr = I for the keyframe's frame)
            a = self.local_offsets[u, 0]
            lp[a:a + len(m.table)].copy_(torch.from_numpy(m.table.view(np.uint8).reshape(len(m.table), -1)))
            self.d_map.view(-1, 32)[u * self.n_map:(u + 1) * self.n_map].copy_(
                torch.from_numpy(m.planes.view(np.uint8).reshape(self.n_map, 32)))
            n = int(pf[u]["n_points"])
            P = m.refresh_last_frame(pp[u, :n])
            Tl = m.kfs[j]["Tcw"].reshape(16)
            for i in range(u, B, U):
                pp[i, :n] = P
                pf[i]["Tlw"] = Tl
        self.d_ppoints[:npp].copy_(torch.from_numpy(pp.view(np.uint8).reshape(-1)))
        self.d_pframes.copy_(torch.from_numpy(pf.view(np.uint8).reshape(-1)))
        self.lm_runs.append((t, run))
        self.lm_time["total_s"] += time.perf_counter() - t_lm0
        torch.cuda.synchronize()

    # ---- per batch: frame t of every slot's sequence and its local map
    INPUT_BUFFERS = ("d_rgb", "d_depth_raw", "d_lframes")

    def _load(self, stream):
        k = self.n_loaded
        self.n_loaded += 1
        # a pipelined step extracts up to `lookahead` frames ahead of tracking: past the last rendered frame it
        # extracts that frame again (never tracked; _tail raises before tracking past the end)
        t = min(k + 1, self.T - 1)
        torch = self.torch
        with torch.cuda.stream(stream):
            if self.B <= self.U:  # slot i = sequence i: frame t of the slots is contiguous
                a, b = t * self.U, t * self.U + self.B
                self.d_rgb.copy_(self.d_rgb_all[a:b])
                self.d_depth_raw.copy_(self.d_depth_all[a:b])
            else:  # (rows built once in _setup_inputs: a host list -> device tensor per call costs ~1 ms)
                idx = self.d_load_idx[t]
                self.d_rgb.copy_(self.d_rgb_all.index_select(0, idx))
                self.d_depth_raw.copy_(self.d_depth_all.index_select(0, idx))
            self.d_lframes.copy_(self.d_local_table[t])

    def _setup_pipeline(self):
        self.rotate_inputs = True  # per-batch inputs are double-buffered with the extraction outputs
        super()._setup_pipeline()

    # ---- the tail with the sequence state
    def _tail(self):
        import spslam_track as ST
        if self.n_tracked + 1 >= self.T:
            raise RuntimeError(f"sequence exhausted: {self.T} frames rendered")
        for slot, V in self.vel_perturb.get(self.n_tracked + 1, []):
            with self.torch.cuda.stream(self.main):
                self.d_velocity[16 * slot:16 * slot + 16].copy_(self.torch.from_numpy(V).cuda(non_blocking=False))
        self.track.batch_device(self.B, ST.MOTION_PRIOR, self._track_batch(0), stream=self.stream)
        super()._tail()
        nxt = self.proj_sets[1] if self.d_pframes.data_ptr() == self.proj_sets[0][0].data_ptr() else self.proj_sets[0]
        b = self._track_batch(1)
        b.results = self.d_res2.data_ptr()
        b.point_outlier_local = self.graphs[1]["pout"].data_ptr()
        b.next_frames, b.next_points = nxt[0].data_ptr(), nxt[1].data_ptr()
        self.track.batch_device(self.B, ST.LAST_FRAME, b, stream=self.stream)
        with self.torch.cuda.stream(self.main):
            res = self.d_res2.view(self.B, G.POSE_RESULT_DTYPE.itemsize)[:, :64].contiguous()
            self.traj[self.n_tracked + 1].copy_(res.view(self.torch.float32).view(self.B, 16))
            h = self.hist[self.n_tracked + 1]
            h[0].copy_(self.d_nmatch)
            h[1].copy_(self.d_nlmatch)
            for r, d in ((2, self.d_res1), (3, self.d_res2)):  # n_inliers follows the 16 pose floats
                h[r].copy_(d.view(self.B, G.POSE_RESULT_DTYPE.itemsize)[:, 64:68].contiguous().view(self.torch.int32)
                           .view(self.B))
        self.n_tracked += 1
        self.d_pframes, self.d_ppoints = nxt
        if self.local_mapping and self.n_tracked % synth.KEYFRAME_STEP == 0:
            self._local_mapping(self.n_tracked)

    def history(self):
        """[t][slot] (nmatches, local nmatches, inliers of the motion-model and local-map PoseOptimization)."""
        self.torch.cuda.synchronize()
        return self.hist[:self.n_tracked + 1].cpu().numpy().transpose(0, 2, 1)

    def trajectory(self):
        """Local-map pose (float 4x4) of frames 1 .. n_tracked of every slot: [t][slot] 4x4 (frame 0 = truth)."""
        self.torch.cuda.synchronize()
        tr = self.traj[:self.n_tracked + 1].cpu().numpy().reshape(-1, self.B, 4, 4)
        for i in range(self.B):
            tr[0, i] = self._true_pose(i % self.U, 0).astype(np.float32)
        return tr

    def perturb_velocity(self, t, slot, V):
        """Test hook: frame t of slot `slot` predicts its pose from velocity V (4x4) instead of its predecessor's
        (a motion-model failure on demand); oracle_sequence.track(perturb={t: V}) is the CPU side."""
        self.vel_perturb.setdefault(t, []).append((slot, np.asarray(V, np.float32).reshape(16).copy()))

    def fallback_history(self):
        """[t][slot]: 0 the motion model held, 1 TrackReferenceKeyFrame took over, 2 both failed (lost)."""
        self.torch.cuda.synchronize()
        return self.fb_hist[:self.n_tracked + 1].cpu().numpy()

    def reference_keyframe_history(self):
        """[t][slot]: the reference keyframe (keyframe index in the slot's sequence) after frame t."""
        self.torch.cuda.synchronize()
        return self.refkf_hist[:self.n_tracked + 1].cpu().numpy() - self.d_kf_base.cpu().numpy()[None, :]
