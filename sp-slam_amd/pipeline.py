"""Batched per-frame tracking hot path on one GPU (the throughput step of bench.py).

One step = for each of B frames resident in HBM (gray u8 + depth f32), the
sequence Tracking::Track runs per RGB-D frame (src/Tracking.cc:233-1080):
  ORBextractor::operator()                      spslam_orb_extract_batch_device
  Frame::ComputePlanesFromOrganizedPointCloud   spslam_planes_extract_batch_device
  Frame::GeneratePlanesFromBoundries            spslam_planes_generate_from_boundaries_batch_device
  Frame::UndistortKeyPoints / ComputeStereoFromRGBD / AssignFeaturesToGrid
                                                spslam_frame_rgbd_batch_device
  TrackWithMotionModel:
    ORBmatcher::SearchByProjection(Cur, Last)   spslam_search_by_projection_batch_device
    Map::AssociatePlanesByBoundary              spslam_planes_associate_batch_device
    graph from the matches                      spslam_track_graph_batch_device (MOTION_MODEL)
    Optimizer::PoseOptimization                 spslam_pose_optimize_batch_device
    outlier discard                             spslam_track_graph_batch_device (DISCARD)
  TrackLocalMap:
    SearchLocalPoints                           spslam_search_local_points_batch_device
    Map::AssociatePlanesByBoundary              (at the optimized pose)
    graph                                       spslam_track_graph_batch_device (LOCAL_MAP)
    Optimizer::PoseOptimization                 spslam_pose_optimize_batch_device

The map the frames track against is synthesized once per sequence from the
scene (sp-slam_amd/synth.py): the last frame's map points (its keypoints
back-projected with the true depth and pose), a keyframe's local map points,
and the map planes with boundary clouds.  Every correspondence PoseOptimization
consumes is produced inside the step by the path's own matching and plane
association.  ORB and plane extraction run on two HIP streams (independent
inputs), joined before the frame steps; nothing returns to the host inside a
step.
"""
from __future__ import annotations


import os

import numpy as np

import spslam_frame
import spslam_grab
import spslam_gpu as G
import spslam_planes
import synth


# Parameter sets of the BASELINE.json configs (the YAML keys the path reads):
#   c2/c3  TUM-style 640x480 (Examples/RGB-D/TUM3.yaml intrinsics, TUM1.yaml plane keys)
#   c4     ICL-NUIM (Examples/RGB-D/ICL.yaml: fx 481.2, fy -480.0, Plane.MinSize 1000, Chi 1000, VPChi 200)
#   c5     1280x960, nFeatures 4000, dense-plane scene
# 640x480 scenes hold 5 boxes: about 6 extracted planes and 0.4 supposed planes per frame (GeneratePlanesFromBoundries
# accepts a boundary line only where a box edge is not an occlusion border; 3 boxes gave none on sequence 0)
CONFIGS = {
    # C1 proxy (TUM fr3 structure_notexture_far, Examples/RGB-D/TUM3.yaml): the C2 geometry with nearly untextured
    # faces (synth._texture_low) and a hand-held trajectory with jolts (the motion model fails on them)
    "c1": dict(width=640, height=480, nfeatures=1000, n_boxes=5, texture="low", motion="shaky"),
    "c2": dict(width=640, height=480, nfeatures=1000, n_boxes=5),
    # C3: LocalBundleAdjustment for every 5th frame over an fr1/room-sized window (25 local + 10 fixed keyframes,
    # 4000 points); c3s keeps rounds 1-5's smaller window (10 local + 2 fixed keyframes, 1500 points)
    "c3": dict(width=640, height=480, nfeatures=1000, n_boxes=5, lba_every=5, lba_kf=35, lba_fixed=10,
               lba_points=4000, lba_kf_step=4),
    "c3s": dict(width=640, height=480, nfeatures=1000, n_boxes=5, lba_every=5),
    "c4": dict(width=640, height=480, nfeatures=1000, n_boxes=5, K=synth.ICL, min_size=1000, chi=1000.0,
               vp_chi=200.0),
    "c5": dict(width=1280, height=960, nfeatures=4000, n_boxes=8),
}


def _ptr(t):
    return t.data_ptr() if t is not None else 0


class HotPath:
    def __init__(self, B, width=640, height=480, nfeatures=1000, n_boxes=3, seq_id=0, unique_frames=16,
                 device=0, K=synth.TUM3, lba_every=0, lba_unique=4, lba_points=1500, lba_kf=12, lba_fixed=2,
                 lba_kf_step=6,
                 pipelined=False, tail_priority=True, orb_priority=False, planes_priority=False, min_size=500, chi=300.0, vp_chi=300.0,
                 rotate_inputs=False, lba_order=0, native=False, lba_depth=0, lba_team=0, lookahead=1,
                 max_inflight=0, texture="dots", motion="smooth"):
        import torch
        self.torch = torch
        self.B, self.W, self.H = B, width, height
        self.nfeatures = nfeatures
        # pipelined: batches extracted ahead of the tracking tail (1: batch k+1 beside batch k's tail) and the
        # steps the host may run ahead of the device (0: unbounded)
        self.lookahead = max(1, int(lookahead))
        self.max_inflight = int(max_inflight)
        self.device = device
        self.lba_order = lba_order  # spslam_lba.G2O_ORDER (default) / FAST_ORDER
        s = width / 640.0
        self.K = K
        self.fx, self.fy, self.cx, self.cy = K["fx"] * s, K["fy"] * s, K["cx"] * s, K["cy"] * s
        self.Ks = dict(K, fx=self.fx, fy=self.fy, cx=self.cx, cy=self.cy)  # intrinsics at this resolution
        self.bf = K["bf"]
        self.min_size = min_size
        # Plane.AngleInfo / DistanceInfo / ParallelInfo / VerticalInfo / Chi / VPChi (Optimizer.cc:681-693)
        self.plane_cfg = G.PlaneConfig(1.0, 100.0, 0.5, 0.5, chi, vp_chi)
        self.texture, self.motion = texture, motion
        self.scene = synth.Scene(seq_id, n_boxes=n_boxes, texture=texture, motion=motion)
        self.ex = G.OrbExtractor(nfeatures=nfeatures, width=width, height=height, max_batch=B, device=device)
        self.pe = spslam_planes.PlaneExtractor(self.ex, self.fx, self.fy, self.cx, self.cy, width, height,
                                               min_size=min_size)
        self.fs = spslam_frame.FrameStage(self.ex, self.fx, self.fy, self.cx, self.cy, K.get("dist", (0,) * 5),
                                          K["bf"], width, height)
        # sequence state written by the tracking tail (sp-slam_amd/sequence.py); unused here
        self.d_seen = self.d_afr_first = self.d_velocity = None
        self._setup_inputs(seq_id, unique_frames)
        U = len(self.frames)
        dev = "cuda"
        self.depth_factor = K["depth_factor"]
        self.grabber = spslam_grab.Grabber(self.ex, channels=3, rgb=True, depth_u16=True,
                                           depth_factor=K["depth_factor"])
        self.d_gray = torch.zeros((B, height, width), dtype=torch.uint8, device=dev)
        self.d_depth = torch.zeros((B, height, width), dtype=torch.float32, device=dev)
        cap = self.ex.max_kp
        self.kp_cap = cap
        self.d_kps = torch.zeros((B, cap, 7), dtype=torch.float32, device=dev)
        self.d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
        self.d_cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        self.d_kun = torch.zeros_like(self.d_kps)
        self.d_kdepth = torch.zeros((B, cap), dtype=torch.float32, device=dev)
        self.d_kur = torch.zeros((B, cap), dtype=torch.float32, device=dev)
        self.d_grid_off = torch.zeros((B, spslam_frame.N_CELLS + 1), dtype=torch.int32, device=dev)
        self.d_grid_idx = torch.zeros((B, cap), dtype=torch.int32, device=dev)
        pe = self.pe
        self.d_planes = torch.zeros(B * pe.planes_cap * 8, dtype=torch.int32, device=dev)
        self.d_pcnt = torch.zeros(B, dtype=torch.int32, device=dev)
        self.d_inl = torch.zeros(B * pe.inlier_cap, dtype=torch.int32, device=dev)
        self.d_con = torch.zeros(B * pe.contour_cap, dtype=torch.int32, device=dev)
        self.d_supp = torch.zeros(B * pe.supp_cap * 16, dtype=torch.int32, device=dev)
        self.d_scnt = torch.zeros(B, dtype=torch.int32, device=dev)
        self.d_lines = torch.zeros(B * pe.line_cap, dtype=torch.int32, device=dev)
        self.d_patch = torch.zeros(B * pe.supp_cap * pe.patch_points * 3, dtype=torch.float32, device=dev)
        # --- streams: ORB on the main stream, plane extraction beside it (independent inputs);
        #     PoseOptimization joins both
        # (an explicit stream: torch's default is the legacy NULL stream, which a HIP call given
        # stream 0 would replace by the context's own non-blocking stream, outside these events)
        # the tracking tail is a chain of latency-bound one-workgroup-per-frame kernels: in pipelined mode its
        # stream gets the high priority so its workgroups dispatch ahead of the next batch's extraction
        self.main = torch.cuda.Stream(priority=-1 if pipelined and tail_priority else 0)
        self.side = torch.cuda.Stream()
        self.stream = self.main.cuda_stream
        self.side_stream = self.side.cuda_stream
        self.ev_fork = torch.cuda.Event()
        self.ev_join = torch.cuda.Event()
        # --- one grab + ORB pass for the map-point generators (they back-project the frames' own keypoints)
        self.grab()
        self.orb()
        torch.cuda.synchronize()
        cnts = self.d_cnt.cpu().numpy()
        # FAST cell candidates per frame (DistributeOctTree's input; bench roofline bytes of octree_kernel)
        nf = min(U, 4)
        self.mean_fast_candidates = sum(len(self.ex.debug_stage(f, l, 2, cap=1 << 16)) for f in range(nf)
                                        for l in range(self.ex.params.nlevels)) / nf
        self.inv_sigma2 = self.ex.tables()["inv_sigma2"]
        self.mean_keypoints = float(cnts.mean())
        self._setup_match(seq_id)
        self._setup_assoc(seq_id)
        self._setup_track()
        # --- LocalBundleAdjustment (C3): one local map per `lba_every` frames (a keyframe), run on the
        #     LocalMapping stream beside tracking like the reference's LocalMapping thread
        self.n_lba = B // lba_every if lba_every else 0
        self.lba_every = lba_every
        if self.n_lba:
            self._setup_lba(seq_id, lba_unique, lba_points, lba_depth, lba_team, lba_kf, lba_fixed, lba_kf_step)
        # rotate_inputs (tests): batch k's slot i takes the inputs of slot (i + k) % B -- images and the per-frame
        # tracking records together -- so consecutive batches differ and a stage reading the wrong buffer set shows
        self.rotate_inputs = rotate_inputs
        self.n_loaded = 0
        if rotate_inputs:
            self.base_inputs = {k: getattr(self, k).clone() for k in self.INPUT_BUFFERS}
        self.pipelined = pipelined
        self.orb_priority = orb_priority
        self.planes_priority = planes_priority
        if pipelined:
            self._setup_pipeline()
        # native: the library enqueues the whole step (spslam_step_run, csrc/spslam_step.cpp) on its own streams
        # and events over these same buffers; Python only makes the call
        self.native = None
        if native:
            self._setup_native()
        torch.cuda.synchronize()  # buffers were filled on the default stream

    def _setup_inputs(self, seq_id, unique_frames):
        """Unique synthetic frames: colour (R,G,B u8) + raw depth (u16, DepthMapFactor 5000), as GrabImageRGBD
        receives them; the step converts them on the device (spslam_grab_rgbd).  Slot i holds frame i % U."""
        torch, B, U = self.torch, self.B, min(unique_frames, self.B)
        self.frames = []
        for i in range(U):
            fi = 3 * i
            g, d, fid = self.scene.render(self.scene.pose(fi), self.W, self.H, K=self.K,
                                          noise_seed=seq_id * 1000 + fi)
            self.frames.append((fi, synth.colorize(g, fid), d, fid))
        self.d_rgb = torch.from_numpy(np.stack([self.frames[i % U][1] for i in range(B)])).cuda()
        self.d_depth_raw = torch.from_numpy(np.stack([self.frames[i % U][2] for i in range(B)]).view(np.int16)).cuda()

    def _setup_assoc(self, seq_id):
        """Map::AssociatePlanesByBoundary before each PoseOptimization (TrackWithMotionModel,
        TrackLocalMap): the frame's extracted + supposed planes against the sequence's map planes
        (the scene faces with boundary clouds).  The first call uses the motion-model pose, the
        second the pose after the first optimisation (written by the DISCARD graph stage)."""
        import spslam_assoc as SA
        torch, B = self.torch, self.B
        rng = np.random.default_rng(seq_id * 31 + 7)
        mp, bxyz = synth.map_planes(self.scene, rng)
        m = np.zeros(len(mp["world"]), SA.MAP_PLANE_DTYPE)
        for k, v in mp.items():
            m[k] = v
        fr = np.zeros(B, SA.ASSOC_FRAME_DTYPE)
        for i in range(B):  # the first association runs at the motion-model prediction (Tracking.cc:958, 979)
            fr[i]["Tcw"] = self.match_probs[i % len(self.match_probs)][0]["Tcw"]
        fr["map_offset"], fr["n_map"] = 0, len(m)
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()  # noqa
        self.assoc = SA.PlaneAssociator(self.ex)
        self.d_map, self.d_bound = dev(m), dev(bxyz)
        fr2 = fr.copy()
        fr2["carry"] = 1  # TrackLocalMap's association keeps what survived TrackWithMotionModel's discard
        self.d_afr1, self.d_afr2 = dev(fr), dev(fr2)
        self.n_map, self.n_boundary = len(m), len(bxyz)
        self.assoc_map, self.assoc_boundary = m, bxyz  # host copies (CPU baseline)
        P = self.pe.planes_cap + self.pe.supp_cap
        self.d_assoc = torch.zeros((2, 3, B * P), dtype=torch.int32, device="cuda")
        self.d_newp = torch.zeros((2, B), dtype=torch.int32, device="cuda")

    def _setup_match(self, seq_id):
        """ORBmatcher::SearchByProjection(CurrentFrame, LastFrame) of TrackWithMotionModel: every frame
        of the batch is matched against the map points of the frame rendered just before it (its ORB
        keypoints back-projected with the true depth, descriptors with a few flipped bits), from a
        motion-model pose prediction."""
        import spslam_match as SM
        torch, B, U = self.torch, self.B, len(self.frames)
        rng = np.random.default_rng(seq_id * 977 + 3)
        last = [self.scene.render(self.scene.pose(f[0] - 1), self.W, self.H, K=self.K,
                                  noise_seed=seq_id * 1000 + f[0] + 500) for f in self.frames]
        d_g = torch.from_numpy(np.stack([g for g, _, _ in last])).cuda()
        cap = self.kp_cap
        d_k = torch.zeros((U, cap, 7), dtype=torch.float32, device="cuda")
        d_d = torch.zeros((U, cap, 32), dtype=torch.uint8, device="cuda")
        d_n = torch.zeros(U, dtype=torch.int32, device="cuda")
        self.ex.extract_batch_device(d_g.data_ptr(), U, self.W * self.H, self.W, d_k.data_ptr(), d_d.data_ptr(),
                                     d_n.data_ptr(), cap, self.stream)
        torch.cuda.synchronize()
        kps = d_k.cpu().numpy().view(G.KEYPOINT_DTYPE).reshape(U, cap)
        desc, cnt = d_d.cpu().numpy(), d_n.cpu().numpy()
        Ks = self.Ks
        probs = [synth.proj_problem(self.scene, self.frames[i][0] - 1, self.frames[i][0], kps[i, :cnt[i]],
                                    desc[i, :cnt[i]], last[i][1], rng, K=Ks) for i in range(U)]
        offs = np.cumsum([0] + [len(p[1]) for p in probs])
        fr = np.zeros(B, SM.PROJ_FRAME_DTYPE)
        for i in range(B):
            fr[i] = probs[i % U][0]
            fr[i]["point_offset"] = offs[i % U]
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()  # noqa
        self.match_probs = probs
        self.matcher = SM.Matcher(self.ex)
        self.d_pframes, self.d_ppoints = dev(fr), dev(np.concatenate([p[1] for p in probs]))
        self.max_points = int(max(len(p[1]) for p in probs))
        self.mean_proj_points = float(np.mean([len(probs[i % U][1]) for i in range(B)]))
        self.d_match = torch.zeros((B, cap), dtype=torch.int32, device="cuda")
        self.d_nmatch = torch.zeros(B, dtype=torch.int32, device="cuda")
        # Tracking::SearchLocalPoints (TrackLocalMap): the local map = map points of the keyframe four
        # frames back (true depth, MapPoint normal / distance range), matched after the first pose
        # optimisation; keypoints holding a motion-model match are taken
        kf = [self.scene.render(self.scene.pose(f[0] - 4), self.W, self.H, K=self.K,
                                noise_seed=seq_id * 1000 + f[0] + 900) for f in self.frames]
        d_g = torch.from_numpy(np.stack([g for g, _, _ in kf])).cuda()
        self.ex.extract_batch_device(d_g.data_ptr(), U, self.W * self.H, self.W, d_k.data_ptr(), d_d.data_ptr(),
                                     d_n.data_ptr(), cap, self.stream)
        torch.cuda.synchronize()
        kps = d_k.cpu().numpy().view(G.KEYPOINT_DTYPE).reshape(U, cap)
        desc, cnt = d_d.cpu().numpy(), d_n.cpu().numpy()
        lprobs = [synth.local_problem(self.scene, self.frames[i][0] - 4, self.frames[i][0], kps[i, :cnt[i]],
                                      desc[i, :cnt[i]], kf[i][1], rng, K=Ks) for i in range(U)]
        loffs = np.cumsum([0] + [len(p[1]) for p in lprobs])
        lfr = np.zeros(B, SM.LOCAL_FRAME_DTYPE)
        for i in range(B):
            lfr[i] = lprobs[i % U][0]
            lfr[i]["point_offset"] = loffs[i % U]
        self.local_probs = lprobs
        self.local_matcher = SM.LocalMatcher(self.ex)
        self.d_lframes, self.d_lpoints = dev(lfr), dev(np.concatenate([p[1] for p in lprobs]))
        self.max_local_points = int(max(len(p[1]) for p in lprobs))
        self.mean_local_points = float(np.mean([len(lprobs[i % U][1]) for i in range(B)]))
        self.d_taken = torch.zeros((B, cap), dtype=torch.uint8, device="cuda")
        self.d_lmatch = torch.zeros((B, cap), dtype=torch.int32, device="cuda")
        self.d_nlmatch = torch.zeros(B, dtype=torch.int32, device="cuda")

    def match(self):
        self.matcher.batch_device(self.B, self.d_pframes.data_ptr(), self.d_ppoints.data_ptr(), self.max_points,
                                  self.d_kun.data_ptr(), self.d_desc.data_ptr(), self.d_kur.data_ptr(),
                                  self.d_grid_off.data_ptr(), self.d_grid_idx.data_ptr(), self.d_cnt.data_ptr(),
                                  self.kp_cap, self.d_match.data_ptr(), self.d_nmatch.data_ptr(), stream=self.stream)

    def search_local_points(self):
        # taken flags and the local frames' pose come from the DISCARD graph stage
        self.local_matcher.batch_device(self.B, self.d_lframes.data_ptr(), self.d_lpoints.data_ptr(),
                                        self.max_local_points, self.d_kun.data_ptr(), self.d_desc.data_ptr(),
                                        self.d_kur.data_ptr(), self.d_grid_off.data_ptr(),
                                        self.d_grid_idx.data_ptr(), self.d_cnt.data_ptr(), self.kp_cap,
                                        self.d_taken.data_ptr(), self.d_lmatch.data_ptr(), self.d_nlmatch.data_ptr(),
                                        stream=self.stream, d_seen=_ptr(self.d_seen))

    def associate(self, k):
        import spslam_planes as SP
        d_fr = self.d_afr1 if k == 0 else self.d_afr2
        o = self.d_assoc[k]
        self.assoc.batch_device(self.B, d_fr.data_ptr(), self.d_planes.data_ptr(), SP.PLANE_DTYPE.itemsize,
                                self.d_pcnt.data_ptr(), self.pe.planes_cap, self.d_supp.data_ptr(),
                                SP.SUPPOSED_DTYPE.itemsize, self.d_scnt.data_ptr(), self.pe.supp_cap,
                                self.d_map.data_ptr(), self.d_bound.data_ptr(), self.n_map, o[0].data_ptr(),
                                o[1].data_ptr(), o[2].data_ptr(), self.d_newp[k].data_ptr(), stream=self.stream)

    def _setup_track(self):
        """Device buffers of the two PoseOptimization graphs (spslam_track_graph_batch_device): point
        edges at f * cap, plane edges at f * 3 * (planes_cap + supp_cap), outlier flags alike."""
        import spslam_track as ST
        torch, B, cap = self.torch, self.B, self.kp_cap
        self.plane_edge_cap = 3 * (self.pe.planes_cap + self.pe.supp_cap)
        self.track = ST.TrackGraph(self.ex)
        u8 = dict(dtype=torch.uint8, device="cuda")
        self.graphs = []
        for _ in range(2):  # motion model, local map
            self.graphs.append(dict(
                P=torch.zeros(B * G.POSE_PROBLEM_DTYPE.itemsize, **u8),
                pts=torch.zeros(B * cap * G.POINT_OBS_DTYPE.itemsize, **u8),
                pls=torch.zeros(B * self.plane_edge_cap * G.PLANE_OBS_DTYPE.itemsize, **u8),
                pout=torch.zeros(B * cap, **u8), plout=torch.zeros(B * self.plane_edge_cap, **u8)))
        self.d_edge = torch.zeros((B, cap), dtype=torch.int32, device="cuda")
        self.d_res1 = torch.zeros(B * G.POSE_RESULT_DTYPE.itemsize, **u8)
        self.d_res2 = torch.zeros_like(self.d_res1)

    def _track_batch(self, k):
        """spslam_track_batch for graph k (0 = motion model, 1 = local map) on the current buffers."""
        import spslam_planes as SP
        import spslam_track as ST
        g = self.graphs[k]
        a = self.d_assoc[k]
        return ST.TrackBatch(
            keys_un=self.d_kun.data_ptr(), uright=self.d_kur.data_ptr(), kp_counts=self.d_cnt.data_ptr(),
            cap=self.kp_cap, proj_frames=self.d_pframes.data_ptr(), proj_points=self.d_ppoints.data_ptr(),
            proj_match=self.d_match.data_ptr(), local_frames=self.d_lframes.data_ptr(),
            local_points=self.d_lpoints.data_ptr(), local_match=self.d_lmatch.data_ptr(),
            taken=self.d_taken.data_ptr(), planes_a=self.d_planes.data_ptr(), planes_b=self.d_supp.data_ptr(),
            count_a=self.d_pcnt.data_ptr(), count_b=self.d_scnt.data_ptr(), stride_a=SP.PLANE_DTYPE.itemsize,
            stride_b=SP.SUPPOSED_DTYPE.itemsize, cap_a=self.pe.planes_cap, cap_b=self.pe.supp_cap,
            map=self.d_map.data_ptr(), assoc_match=a[0].data_ptr(), assoc_parallel=a[1].data_ptr(),
            assoc_vertical=a[2].data_ptr(), assoc_frames_next=self.d_afr2.data_ptr(),
            plane_outlier=self.graphs[0]["plout"].data_ptr(), next_match=self.d_assoc[1][0].data_ptr(),
            next_parallel=self.d_assoc[1][1].data_ptr(), next_vertical=self.d_assoc[1][2].data_ptr(),
            assoc_frames_first=_ptr(self.d_afr_first), seen=_ptr(self.d_seen), velocity=_ptr(self.d_velocity),
            problems=g["P"].data_ptr(), points=g["pts"].data_ptr(), planes=g["pls"].data_ptr(),
            edge_of_kp=self.d_edge.data_ptr(), results=self.d_res1.data_ptr(),
            point_outlier=self.graphs[0]["pout"].data_ptr(), fx=self.fx, fy=self.fy, cx=self.cx, cy=self.cy,
            bf=self.bf)

    # --- stages
    def grab(self, stream=None):
        """GrabImageRGBD's cvtColor + depth convertTo (src/Tracking.cc:214-229) into d_gray / d_depth."""
        s = self.stream if stream is None else stream
        self.grabber.batch_device(self.B, self.d_rgb.data_ptr(), self.H * self.W * 3, self.W * 3,
                                  self.d_depth_raw.data_ptr(), self.H * self.W, self.W, self.W, self.H,
                                  self.d_gray.data_ptr(), self.d_depth.data_ptr(), s)

    def orb(self, stream=None):
        s = self.stream if stream is None else stream
        self.ex.extract_batch_device(self.d_gray.data_ptr(), self.B, self.W * self.H, self.W, self.d_kps.data_ptr(),
                                     self.d_desc.data_ptr(), self.d_cnt.data_ptr(), self.kp_cap, s)

    def planes(self, stream=None):
        self.planes_extract(stream)
        self.planes_supposed(stream)

    def planes_extract(self, stream=None):
        """ComputePlanesFromOrganizedPointCloud for the batch."""
        s = self.stream if stream is None else stream
        self.pe.extract_batch_device(self.d_depth.data_ptr(), self.B, self.W * self.H, self.W,
                                     self.d_planes.data_ptr(), self.d_pcnt.data_ptr(), self.d_inl.data_ptr(),
                                     self.d_con.data_ptr(), s)

    def planes_supposed(self, stream=None):
        """GeneratePlanesFromBoundries for the batch (reads the extraction's organized clouds)."""
        s = self.stream if stream is None else stream
        self.pe.generate_batch_device(self.d_depth.data_ptr(), self.B, self.W * self.H, self.W,
                                      self.d_planes.data_ptr(), self.d_pcnt.data_ptr(), self.d_con.data_ptr(),
                                      self.d_supp.data_ptr(), self.d_scnt.data_ptr(), self.d_lines.data_ptr(),
                                      self.d_patch.data_ptr(), s)

    def frame(self):
        self.fs.batch_device(self.d_kps.data_ptr(), self.d_cnt.data_ptr(), self.kp_cap, self.d_depth.data_ptr(),
                             self.B, self.W * self.H, self.W, self.d_kun.data_ptr(), self.d_kdepth.data_ptr(),
                             self.d_kur.data_ptr(), self.d_grid_off.data_ptr(), self.d_grid_idx.data_ptr(),
                             self.d_pcnt.data_ptr(), self.d_scnt.data_ptr(), self.stream)

    def pose(self):
        """TrackWithMotionModel then TrackLocalMap (src/Tracking.cc:951-1068) from the matches on."""
        import spslam_track as ST
        g1, g2 = self.graphs
        self._join_planes()
        self.associate(0)
        self.track.batch_device(self.B, ST.MOTION_MODEL, self._track_batch(0), stream=self.stream)
        G.pose_optimize_batch_device(self.ex, self.B, g1["P"].data_ptr(), g1["pts"].data_ptr(),
                                     g1["pls"].data_ptr(), self.d_res1.data_ptr(), g1["pout"].data_ptr(),
                                     g1["plout"].data_ptr(), cfg=self.plane_cfg, stream=self.stream)
        self.track.batch_device(self.B, ST.DISCARD, self._track_batch(0), stream=self.stream)
        self._after_motion_model()
        self.search_local_points()
        self.associate(1)
        self.track.batch_device(self.B, ST.LOCAL_MAP, self._track_batch(1), stream=self.stream)
        G.pose_optimize_batch_device(self.ex, self.B, g2["P"].data_ptr(), g2["pts"].data_ptr(),
                                     g2["pls"].data_ptr(), self.d_res2.data_ptr(), g2["pout"].data_ptr(),
                                     g2["plout"].data_ptr(), cfg=self.plane_cfg, stream=self.stream)

    def _after_motion_model(self):
        """Hook after TrackWithMotionModel's discard (sequence.SequencePath: the TrackReferenceKeyFrame switch)."""

    def _join_planes(self):
        if getattr(self, "_planes_pending", False):
            self.main.wait_event(self.ev_join)
            self._planes_pending = False

    def graph(self, k):
        """Host copy of PoseOptimization graph k: (problems, [points per frame], [planes per frame],
        point outlier flags per frame, plane outlier flags per frame)."""
        g = self.graphs[k]
        P = g["P"].cpu().numpy().view(G.POSE_PROBLEM_DTYPE)
        pts = g["pts"].cpu().numpy().view(G.POINT_OBS_DTYPE)
        pls = g["pls"].cpu().numpy().view(G.PLANE_OBS_DTYPE)
        po, plo = g["pout"].cpu().numpy(), g["plout"].cpu().numpy()
        sl = lambda a, o, n: a[o:o + n]  # noqa: E731
        return (P, [sl(pts, p["point_offset"], p["n_points"]) for p in P],
                [sl(pls, p["plane_offset"], p["n_planes"]) for p in P],
                [sl(po, p["point_offset"], p["n_points"]).astype(bool) for p in P],
                [sl(plo, p["plane_offset"], p["n_planes"]).astype(bool) for p in P])

    def _setup_lba(self, seq_id, unique, n_points, depth=0, team=0, n_kf=12, n_fixed=2, kf_step=6):
        """LocalMapping beside tracking.  The step's local maps (one per `lba_every` frames) go to one batched
        LocalBundleAdjustment call on its own stream and context, like the reference's LocalMapping thread
        (LocalMapping.cc:48-124), which never blocks Tracking.  depth d: step k's call is joined at the end of step
        k + d (d = 0: the same step), so up to d + 1 calls are in flight, each on its own context (scratch) and
        output buffers; the join point is fixed, so the results do not depend on timing."""
        import concurrent.futures as cf
        import os
        import spslam_lba as L
        torch = self.torch
        probs = []
        for u in range(min(unique, self.n_lba)):  # keyframes every kf_step frames, the last n_fixed fixed cameras
            rng = np.random.default_rng(seq_id * 131 + u)
            f0 = 6 * u
            probs.append(synth.lba_problem(self.scene, list(range(f0, f0 + n_kf * kf_step, kf_step)), rng,
                                           n_fixed=n_fixed, n_points=n_points, K=self.Ks))
        self.lba_window = dict(keyframes=n_kf, fixed=n_fixed, points=n_points, keyframe_step=kf_step)
        hdr = np.zeros(self.n_lba, L.LBA_PROBLEM_DTYPE)
        kf, pt, po, pl, plo = [], [], [], [], []
        nk = npt = npo = npl = nplo = 0
        for i in range(self.n_lba):
            prob, kfs, pts, pobs, pls, plobs, _ = probs[i % len(probs)]
            hdr[i] = prob
            hdr[i]["kf_offset"], hdr[i]["point_offset"], hdr[i]["plane_offset"] = nk, npt, npl
            pts = pts.copy()
            pts["obs_offset"] += npo
            pls = pls.copy()
            pls["obs_offset"] += nplo
            kf.append(kfs); pt.append(pts); po.append(pobs); pl.append(pls); plo.append(plobs)
            nk += len(kfs); npt += len(pts); npo += len(pobs); npl += len(pls); nplo += len(plobs)
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()  # noqa: E731
        self.lba_problems = probs
        self.lba_hdr = hdr
        self.lba_in = [dev(hdr), dev(np.concatenate(kf)), dev(np.concatenate(pt)), dev(np.concatenate(po)),
                       dev(np.concatenate(pl)), dev(np.concatenate(plo))]
        pc = self.plane_cfg
        team = int(os.environ.get("SPSLAM_LBA_TEAM", team))  # workgroups per local map (0: fill the chip)
        self.lba_depth = int(os.environ.get("SPSLAM_LBA_DEPTH", depth))
        self.lba_slots = []
        for _ in range(self.lba_depth + 1):
            ex = G.OrbExtractor(max_batch=1, device=self.device)
            lba = L.LocalBA(ex, cfg=(pc.angle_info, pc.distance_info, pc.parallel_info, pc.vertical_info, pc.chi,
                                     pc.vp_chi))
            lba.set_order(self.lba_order)
            lba.set_team(team)
            out = [torch.zeros((nk, 16), dtype=torch.float32, device="cuda"),
                   torch.zeros((npt, 3), dtype=torch.float32, device="cuda"),
                   torch.zeros((max(npl, 1), 4), dtype=torch.float32, device="cuda"),
                   torch.zeros(npo, dtype=torch.uint8, device="cuda"),
                   torch.zeros(max(nplo, 1), dtype=torch.uint8, device="cuda"),
                   torch.zeros(self.n_lba * L.LBA_RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")]
            self.lba_slots.append(dict(ex=ex, lba=lba, out=out, stream=torch.cuda.Stream(), ev=torch.cuda.Event()))
        s0 = self.lba_slots[0]
        self.lba_ex, self.lba, self.lba_out, self.lba_stream, self.ev_lba = (s0["ex"], s0["lba"], s0["out"],
                                                                             s0["stream"], s0["ev"])
        self.lba_pool = cf.ThreadPoolExecutor(len(self.lba_slots), initializer=torch.cuda.set_device,
                                              initargs=(self.device,))
        self.lba_pending = []  # (job, slot) in launch order
        self.lba_launched = 0
        self.lba_edges = (npo + nplo) / self.n_lba
        self.lba_points = npt / self.n_lba

    def local_ba(self, slot=0):
        sl = self.lba_slots[slot]
        sl["lba"].batch_device(self.n_lba, self.lba_hdr, *[x.data_ptr() for x in self.lba_in],
                               *[x.data_ptr() for x in sl["out"]], stream=sl["stream"].cuda_stream)
        sl["ev"].record(sl["stream"])

    def set_timing(self, on):
        self.ex.set_timing(on)
        if self.n_lba:
            for sl in self.lba_slots:
                sl["ex"].set_timing(on)

    def kernel_times(self):
        """{kernel name: (total ms, launches)} over both contexts (tracking, LocalMapping)."""
        t = dict(self.ex.kernel_times())
        if self.n_lba:
            for sl in self.lba_slots:
                for k, (ms, n) in sl["ex"].kernel_times().items():
                    a = t.get(k, (0.0, 0))
                    t[k] = (a[0] + ms, a[1] + n)
        return t

    # Extraction outputs: the only buffers written by ORB / plane extraction and read by the tracking tail.
    EXTRACTION_BUFFERS = ("d_gray", "d_depth", "d_kps", "d_desc", "d_cnt", "d_planes", "d_pcnt", "d_inl", "d_con", "d_supp", "d_scnt",
                          "d_lines", "d_patch")
    # Per-batch inputs: the colour / depth frames and the per-frame tracking records (the map point and plane
    # arrays they index are shared).  Static in the bench; rotated per batch with rotate_inputs.
    INPUT_BUFFERS = ("d_rgb", "d_depth_raw", "d_pframes", "d_lframes", "d_afr1", "d_afr2")

    def batch_slots(self, k):
        """Source slot of each slot of batch k (identity unless rotate_inputs)."""
        return [(i + k) % self.B if self.rotate_inputs else i for i in range(self.B)]

    def _load(self, stream):
        """Per-batch inputs of the next batch into the bound buffers, on `stream` (rotate_inputs only)."""
        k = self.n_loaded
        self.n_loaded += 1
        if not self.rotate_inputs:
            return
        torch = self.torch
        perm = torch.tensor(self.batch_slots(k), dtype=torch.long, device="cuda")
        with torch.cuda.stream(stream):
            perm.record_stream(stream)
            for name in self.INPUT_BUFFERS:
                dst, src = getattr(self, name), self.base_inputs[name]
                dst.view(self.B, -1).copy_(src.view(self.B, -1).index_select(0, perm))

    def _setup_pipeline(self):
        """Software pipelining across steps: batch k+1's extraction (ORB and planes, two streams) runs beside
        batch k's tracking tail (frame steps, matching, association, graphs, PoseOptimization), which is
        latency-bound and leaves most CUs idle.  The extraction outputs are double-buffered; set j may be
        overwritten once the tail that read it has finished (ev_tail[j])."""
        torch = self.torch
        names = self.EXTRACTION_BUFFERS + (self.INPUT_BUFFERS if self.rotate_inputs else ())
        # lookahead L: batches k+1 .. k+L are extracted ahead of batch k's tail (L + 1 buffer sets).  At small B
        # the extraction's plane chain (one workgroup per frame) is longer than the tail, so with L >= 2 two
        # extractions run side by side, each on its own ORB / plane context (their scratch) and streams; batch m
        # is extracted on unit m % L.  Extraction is per-frame and independent of tracking: results are those of
        # the serial step for every L.
        L = self.lookahead
        self.sets = [{k: getattr(self, k) for k in names}] + [{k: getattr(self, k).clone() for k in names}
                                                              for _ in range(L)]
        self.ext_units = []
        for e in range(L):
            if e == 0:
                ex, pe, grabber = self.ex, self.pe, self.grabber
            else:
                ex = G.OrbExtractor(nfeatures=self.nfeatures, width=self.W, height=self.H, max_batch=self.B,
                                    device=self.device)
                pe = spslam_planes.PlaneExtractor(ex, self.fx, self.fy, self.cx, self.cy, self.W, self.H,
                                                  min_size=self.min_size)
                grabber = spslam_grab.Grabber(ex, channels=3, rgb=True, depth_u16=True,
                                              depth_factor=self.depth_factor)
            # ORB extraction is the longest extraction chain at large B; orb_priority lets its workgroups dispatch
            # ahead of the plane chain's (the tracking tail keeps its high priority)
            self.ext_units.append(dict(ex=ex, pe=pe, grabber=grabber,
                                       orb=torch.cuda.Stream(priority=-1 if self.orb_priority else 0),
                                       planes=torch.cuda.Stream(priority=-1 if self.planes_priority else 0)))
        self.ext_orb, self.ext_planes = self.ext_units[0]["orb"], self.ext_units[0]["planes"]
        n = L + 1
        self.ev_orb = [torch.cuda.Event() for _ in range(n)]
        self.ev_planes = [torch.cuda.Event() for _ in range(n)]
        self.ev_tail = [torch.cuda.Event() for _ in range(n)]
        self.ev_grab = [torch.cuda.Event() for _ in range(n)]
        self.n_extracted = 0
        self.max_inflight = int(os.environ.get("SPSLAM_MAX_INFLIGHT", self.max_inflight))
        self.ev_inflight = [torch.cuda.Event() for _ in range(max(1, self.max_inflight))]
        # The supposed planes run on the plane stream right after the extraction.  Two alternatives were
        # measured slower in round 2 and removed: opening the tracking tail with them (1.5 %,
        # profiles/r02/ab_supp_on_tail) and holding the next pyramid until they finish (5 %,
        # profiles/r02/ab_orb_after_supp).
        self.k = 0
        self.primed = False
        torch.cuda.synchronize()

    SET_NAMES = dict(d_gray="gray", d_depth="depth", d_kps="kps", d_desc="desc", d_cnt="counts", d_planes="planes",
                     d_pcnt="plane_counts", d_inl="inliers", d_con="contours", d_supp="supposed",
                     d_scnt="supposed_counts", d_lines="lines", d_patch="patch")

    def _setup_native(self):
        import spslam_match as SM
        import spslam_step as SS
        if self.n_lba or self.rotate_inputs or self.lookahead != 1:
            raise ValueError("native step: no LocalMapping beside it, static inputs and lookahead 1 (use the Python "
                             "step)")
        cfg = SS.StepConfig(n_frames=self.B, width=self.W, height=self.H, kp_cap=self.kp_cap,
                            pipelined=int(self.pipelined), tail_priority=int(self.main.priority < 0),
                            orb_priority=int(getattr(self, "orb_priority", False)),
                            planes_priority=int(getattr(self, "planes_priority", False)),
                            grab=self.grabber.params, match=SM.MatchParams(*SM.MOTION_MODEL),
                            local=SM.LocalParams(*SM.SEARCH_LOCAL), assoc=self.assoc.params, pose=self.plane_cfg,
                            fx=self.fx, fy=self.fy, cx=self.cx, cy=self.cy, bf=self.bf)
        sets = [{v: getattr(self, k).data_ptr() for k, v in self.SET_NAMES.items()}]
        if self.pipelined:
            sets = [{v: st[k].data_ptr() for k, v in self.SET_NAMES.items()} for st in self.sets]
        else:
            sets.append(dict(sets[0]))  # (the serial step uses set 0 only)
        t = SS.StepTail(keys_un=self.d_kun.data_ptr(), mv_depth=self.d_kdepth.data_ptr(), uright=self.d_kur.data_ptr(),
                        grid_off=self.d_grid_off.data_ptr(), grid_idx=self.d_grid_idx.data_ptr(),
                        match=self.d_match.data_ptr(), nmatches=self.d_nmatch.data_ptr(),
                        taken=self.d_taken.data_ptr(), local_match=self.d_lmatch.data_ptr(),
                        local_nmatches=self.d_nlmatch.data_ptr(), edge_of_kp=self.d_edge.data_ptr())
        for g in range(2):
            for a in range(3):
                t.assoc[g][a] = self.d_assoc[g][a].data_ptr()
            t.new_plane[g] = self.d_newp[g].data_ptr()
            gr = self.graphs[g]
            t.problems[g], t.points[g], t.planes[g] = gr["P"].data_ptr(), gr["pts"].data_ptr(), gr["pls"].data_ptr()
            t.point_outlier[g], t.plane_outlier[g] = gr["pout"].data_ptr(), gr["plout"].data_ptr()
        t.results[0], t.results[1] = self.d_res1.data_ptr(), self.d_res2.data_ptr()
        self.native = SS.Step(self.ex, cfg, sets, t)
        self.native_frames = SS.StepFrames(color=self.d_rgb.data_ptr(), color_frame_stride=self.H * self.W * 3,
                                           depth=self.d_depth_raw.data_ptr(), depth_frame_stride=self.H * self.W,
                                           color_stride=self.W * 3, depth_stride=self.W)
        self.native_tracking = SS.StepTracking(
            proj_frames=self.d_pframes.data_ptr(), proj_points=self.d_ppoints.data_ptr(),
            local_frames=self.d_lframes.data_ptr(), local_points=self.d_lpoints.data_ptr(),
            assoc_frames1=self.d_afr1.data_ptr(), assoc_frames2=self.d_afr2.data_ptr(), map=self.d_map.data_ptr(),
            boundary_xyz=self.d_bound.data_ptr(), max_proj_points=self.max_points,
            max_local_points=self.max_local_points, max_map=self.n_map)
        self.native_k = 0

    def _step_native(self):
        if self.pipelined and self.native_k == 0:
            self.native.prime(self.native_frames)
        self.native.run(self.native_frames, self.native_tracking)
        if self.pipelined:
            self._bind(self.native_k % 2)  # results() reads the set batch k's tail used
        self.native_k += 1

    def _bind(self, j):
        for k, v in self.sets[j].items():
            setattr(self, k, v)

    def _extract(self, j):
        """The next batch's extraction into buffer set j, on extraction unit (batch index) % lookahead."""
        m = self.n_extracted
        self.n_extracted += 1
        u = self.ext_units[m % self.lookahead]
        orb_s, planes_s = u["orb"], u["planes"]
        main_units = self.ex, self.pe, self.grabber
        self.ex, self.pe, self.grabber = u["ex"], u["pe"], u["grabber"]
        try:
            self._bind(j)
            orb_s.wait_event(self.ev_tail[j])
            self._load(orb_s)
            # the unit's organized cloud alternates between its two sets (double-buffered like the other outputs);
            # selected before the grab, which makes the cloud in the same pass (spslam_grab_fuse_cloud)
            self.pe.select_cloud_set((m // self.lookahead) % 2)
            self.grab(orb_s.cuda_stream)
            self.ev_grab[j].record(orb_s)
            planes_s.wait_event(self.ev_grab[j])
            self.planes(planes_s.cuda_stream)
            self.ev_planes[j].record(planes_s)
            self.orb(orb_s.cuda_stream)
            self.ev_orb[j].record(orb_s)
        finally:
            self.ex, self.pe, self.grabber = main_units

    def _tail(self):
        self.frame()
        self.match()
        self.pose()

    def step(self):
        if self.native is not None:
            return self._step_native()
        if self.pipelined:
            return self._step_pipelined()
        # planes of step k may start once step k-1 is done with the plane buffers and this step's depth exists
        self._load(self.main)
        self.grab()
        self.ev_fork.record(self.main)
        self.side.wait_event(self.ev_fork)
        self._lba_begin()
        self.planes(self.side_stream)
        self.orb()
        self.ev_join.record(self.side)
        # the tail's frame steps and SearchByProjection read no plane output: the join waits in pose(), before the
        # first association, so they run beside the plane chain (B = 1 latency)
        self._planes_pending = True
        self._tail()
        self._join_planes()
        self._lba_end()

    def _step_pipelined(self):
        """One extraction (batch k + lookahead) and one tracking tail (batch k) per step."""
        n = self.lookahead + 1
        if not self.primed:  # the first batches' extraction (warmup absorbs it)
            for i in range(self.lookahead):
                self._extract(i)
            self.primed = True
        j = self.k % n
        self.ev_fork.record(self.main)
        self._lba_begin()
        self._extract((self.k + self.lookahead) % n)
        self._bind(j)
        self.main.wait_event(self.ev_orb[j])
        self.main.wait_event(self.ev_planes[j])
        self._tail()
        self.ev_tail[j].record(self.main)
        self._lba_end()
        self._throttle()
        self.k += 1

    def _throttle(self):
        """Host-side bound on the steps in flight: wait for the tail of step k - max_inflight before returning
        from step k.  Unbounded, the host runs hundreds of steps ahead and every extraction stream fills with
        packets waiting on tail events; at B = 1 that costs ~20 % (profiles/r05/b1_inflight.txt)."""
        if not self.max_inflight:
            return
        ev = self.ev_inflight[self.k % self.max_inflight]
        if self.k >= self.max_inflight:
            ev.synchronize()
        ev.record(self.main)

    def _lba_begin(self):
        if self.n_lba:
            # LocalMapping: the keyframes of this step, beside tracking, on the next slot (its previous call was
            # joined lba_depth steps ago)
            slot = self.lba_launched % len(self.lba_slots)
            self.lba_launched += 1
            self.lba_slots[slot]["stream"].wait_event(self.ev_fork)
            self.lba_pending.append((self.lba_pool.submit(self.local_ba, slot), slot))

    def _lba_end(self):
        if self.n_lba:  # join the call launched lba_depth steps ago
            while len(self.lba_pending) > self.lba_depth:
                job, slot = self.lba_pending.pop(0)
                job.result()
                self.main.wait_event(self.lba_slots[slot]["ev"])

    def lba_drain(self):
        """Join every LocalBundleAdjustment call still in flight (the end of a run)."""
        if self.n_lba:
            while self.lba_pending:
                job, slot = self.lba_pending.pop(0)
                job.result()
                self.main.wait_event(self.lba_slots[slot]["ev"])

    def results(self):
        torch = self.torch
        torch.cuda.synchronize()
        return dict(
            kps=self.d_kps.cpu().numpy().view(G.KEYPOINT_DTYPE).reshape(self.B, self.kp_cap),
            kp_counts=self.d_cnt.cpu().numpy(),
            plane_counts=self.d_pcnt.cpu().numpy(),
            supposed_counts=self.d_scnt.cpu().numpy(),
            contour_points=self._plane_field("n_contour"),
            line_points=self._supposed_line_points(),
            pose1=self.d_res1.cpu().numpy().view(G.POSE_RESULT_DTYPE),
            pose2=self.d_res2.cpu().numpy().view(G.POSE_RESULT_DTYPE),
            assoc=self.d_assoc.cpu().numpy().reshape(2, 3, self.B, -1),
            match=self.d_match.cpu().numpy(), nmatches=self.d_nmatch.cpu().numpy(),
            local_match=self.d_lmatch.cpu().numpy(), local_nmatches=self.d_nlmatch.cpu().numpy(),
            new_plane=self.d_newp.cpu().numpy())

    def _plane_field(self, name):
        pl = self.d_planes.cpu().numpy().view(spslam_planes.PLANE_DTYPE).reshape(self.B, self.pe.planes_cap)
        cnt = self.d_pcnt.cpu().numpy()
        return np.array([pl[f, :cnt[f]][name].sum() for f in range(self.B)], np.float64)

    def _supposed_line_points(self):
        sp = self.d_supp.cpu().numpy().view(spslam_planes.SUPPOSED_DTYPE).reshape(self.B, self.pe.supp_cap)
        cnt = np.minimum(self.d_scnt.cpu().numpy(), self.pe.supp_cap)
        return np.array([sp[f, :cnt[f]]["n_line"].sum() for f in range(self.B)], np.float64)

    def close(self):
        if getattr(self, "native", None) is not None:
            self.native.close()
            self.native = None
        if self.n_lba:
            self.lba_drain()
            self.lba_pool.shutdown()
            for sl in self.lba_slots:
                sl["ex"].close()
        for u in getattr(self, "ext_units", [])[1:]:
            u["ex"].close()
        self.ex.close()
