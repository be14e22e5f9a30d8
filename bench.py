#!/usr/bin/env python3
"""Throughput bench of the MI355X tracking hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config c2|c5]

A "step" is one pass of the hot path -- ORB extraction, plane extraction,
supposed planes from plane boundaries, the RGB-D Frame keypoint steps
(undistortion, depth / right coordinate, 64x48 grid), SearchByProjection,
plane association, the motion-model PoseOptimization, SearchLocalPoints, the
second association and the local-map PoseOptimization -- over one batch of B
synthetic RGB-D frames already resident in HBM (sp-slam_amd/pipeline.py).
By default steps are software-pipelined: step k runs the extraction of batch
k+1 beside the tracking of batch k (double-buffered extraction outputs), so
each timed step still does exactly one extraction and one tracking pass of B
frames (--no-pipeline runs them back to back).  One process per GPU; for N > 1
launch through torch.distributed.run: every rank runs its own independent
sequence (the path shards with no data-path collective; one all-reduce takes
the max time).

Rank 0 prints ONE JSON line.  `value` = frames processed by all ranks / max
over ranks of the timed region.  `roofline` is computed for the kernel with
the largest share of the timed region, from HIP events recorded on its launch
stream during the timed steps; `cpu_baseline` is the CPU oracle (one core) on
a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
# Hardware queues per process: HIP's default (and the GPU box's environment) is 4.  The pipelined step keeps
# up to six streams busy at once (tracking, next-batch ORB and plane extraction, LocalMapping, each context's
# own stream); with 4 queues the tracking stream shares a queue with the ORB extraction stream and the two
# serialize (measured: 9.2 ms vs 11.8 ms per C2 step).  The runtime takes the value from the environment the
# process starts with, so when it is lower the bench re-runs itself as a child process with 8 queues (before
# anything here touches the GPU) and exits with the child's status.
HW_QUEUES = 8
sys.path.insert(0, str(ROOT / "sp-slam_amd"))

# HotPath parameters of each config: sp-slam_amd/pipeline.py CONFIGS (the YAML keys of the path)
WORKLOADS = {
    # BASELINE.json configs[0]: TUM fr3 structure_notexture_far, single sequence (the dataset is absent: a proxy)
    "c1": "C1 (synthetic proxy of TUM fr3 structure_notexture_far, Examples/RGB-D/TUM3.yaml): the C2 room and boxes "
          "with nearly untextured faces (~250 ORB keypoints per frame, most FAST cells decided by the minThFAST "
          "retry) and a hand-held trajectory with 9-14 degree jolts on which the motion model fails and "
          "TrackReferenceKeyFrame takes over; ORB + planes + supposed planes + 2x PoseOptimization; the "
          "single_sequence line is the config's own (one sequence, B = 1)",
    # BASELINE.json configs[1]: single MI355X, 640x480 synthetic RGB-D stream, ORB + planes + PoseOptimization
    "c2": "C2: synthetic 640x480 RGB-D stream; ORB (nFeatures=1000, 8 levels) + organized-cloud plane extraction + "
          "supposed planes + 2x PoseOptimization (point+plane+parallel+perpendicular edges), no LBA",
    # configs[2]: full pipeline incl. LocalBundleAdjustment (a keyframe every 5 frames, fr1/room-sized local maps)
    "c3": "C3 (synthetic proxy): C2 + LocalBundleAdjustment with plane/parallel/perpendicular edges for every 5th "
          "frame over an fr1/room-sized window (25 local + 10 fixed keyframes, 4000 points per local map)",
    "c3s": "C3 with rounds 1-5's smaller LocalBundleAdjustment window (10 local + 2 fixed keyframes, 1500 points per "
           "local map)",
    # configs[3]: independent ICL-NUIM living-room sequences, one per GPU
    "c4": "C4 (synthetic proxy): ICL-NUIM parameter set (Examples/RGB-D/ICL.yaml: fx 481.2, fy -480.0, cx 319.5, "
          "cy 239.5, Plane.MinSize 1000, Plane.Chi 1000, Plane.VPChi 200), one independent sequence per GPU rank; "
          "ORB + planes + supposed planes + 2x PoseOptimization",
    # configs[4]: 1280x960, nFeatures=4000, dense-plane scene
    "c5": "C5: synthetic 1280x960 RGB-D; ORB nFeatures=4000 + planes + supposed planes + 2x PoseOptimization",
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# PoseOptimization's serial floor: g2o sums every value edge by edge (sparse_optimizer.cpp:100-114,
# block_solver.hpp:529-545), so each edge pass is a chain of one dependent fp64 add per edge.  One chain row (LDS
# read + dependent v_add_f64, 28 values side by side on one wave) measured 13.3 cycles on gfx950
# (tools/pose_micro.hip, profiles/r03/pose_micro.txt); clock: the 2.4 GHz nominal.
CHAIN_CYCLES_PER_ROW = 13.3
CLOCK_HZ = 2.4e9


def pose_chain_floor(P1, P2, r1, r2):
    """Per launch, the ordered-sum chain floor of the PoseOptimization kernel (ms): each problem chains its
    n_points + n_planes rows once per LM iteration (the quadratic form) and once per trial pass (the trial
    chi2); the problems of a launch run side by side (one CU each), so a launch lasts at least as long as its
    longest chain.  Mean over the two graphs."""
    import numpy as np
    out = []
    for P, r in ((P1, r1), (P2, r2)):
        rows = (P["n_points"] + P["n_planes"]).astype(np.float64)
        passes = r["lm_iterations"].astype(np.float64) + r["trial_passes"].astype(np.float64)
        out.append(float((rows * passes).max()) * CHAIN_CYCLES_PER_ROW / CLOCK_HZ * 1e3)
    return float(np.mean(out))


def level_sizes(w, h, nlevels=8, scale=1.2):
    """ORB pyramid level sizes (src/ORBextractor.cc:1111-1112)."""
    import numpy as np
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(float(s[-1]) * float(np.float32(scale))))
    out = []
    for l in range(nlevels):
        inv = np.float32(1.0) / s[l]
        out.append((int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))))
    return out


def algorithmic_bytes(cfg, n_kp, n_pts, n_pls, n_con=0, n_brd=0, n_sup=0, lba_bytes=0, n_fpl=0, n_map=0, n_bnd=0,
                      n_proj=0, n_local=0, n_cand=0):
    """Compulsory HBM bytes per frame for each kernel kind (DESIGN.md "Roofline" table)."""
    lv = level_sizes(cfg["width"], cfg["height"])
    px = [w * h for w, h in lv]
    W, H = -(-cfg["width"] // 3), -(-cfg["height"] // 3)
    N = W * H
    IWH = (W + 1) * (H + 1)
    return {
        # GrabImageRGBD: RGB u8 x3 + depth u16 in, gray u8 + depth f32 out
        "grab_rgbd_kernel": cfg["width"] * cfg["height"] * (3 + 2 + 1 + 4),
        # level l-1 (or the input frame) read; level image (l >= 1), blur and FAST score map written
        "level_kernel": px[0] + sum(px[:-1]) + sum(px[1:]) + 2 * sum(px),
        "fast_cells_kernel": sum(px),                         # score maps read once
        # FAST survivors (4 B each) + per-cell counts in, retained level keypoints (8 B) out
        "octree_kernel": n_cand * 4 + 2 * sum(_cells(w, h) for w, h in lv) + n_kp * 8,
        # per keypoint: the 31x31 patch around it read from the level (IC_Angle) and from the blurred level
        # (rotated BRIEF), keypoint + descriptor out
        "desc_kernel": n_kp * (2 * 31 * 31 + 28 + 32),
        "pose_kernel": (n_pts * 32 + n_pls * 48 + 80) / 2,    # observations in + result out, per call
        "plane_cloud_kernel": 4 * N + 12 * N,                 # depth samples in, xyz out
        # depth samples in (their lines: 12 B per cell at Cloud.Dis 3, as the cloud's x / y / z), distance map
        # + 6 fp64 integral images out (one wavefront kernel)
        "plane_dist_integral_kernel": 12 * N + 4 * N + 48 * IWH,
        "plane_normal_kernel": 16 * N + 48 * IWH + 16 * N,    # xyz+dist, integral, normal+plane_d out
        "plane_segment_kernel": 28 * N + 4 * N,               # xyz+normal+plane_d in, labels out
        "supp_lines_kernel": n_con * (4 + 12 + 4) + n_brd * 1600,  # contour idx + xyz in, line idx out, border windows
        "supp_assemble_kernel": n_sup * (64 + 2601 * 12),     # appended planes + synthetic patches out
        "frame_rgbd_kernel": n_kp * (28 + 4 + 28 + 4 + 4 + 4) + 4 * 3073,  # kp in, depth gather, kp/depth/uR/idx out
        # two AssociatePlanesByBoundary calls: frame + plane coefficients + map records + boundary cloud in,
        # match / parallel / vertical out
        "plane_assoc_kernel": 2 * (80 + n_fpl * (16 + 12) + n_map * 32 + n_bnd * 12),
        # SearchByProjection: last-frame map points in, current keypoints + descriptors + uR + grid read,
        # match out
        "search_projection": n_proj * 64 + n_kp * (28 + 32 + 4 + 4 + 4) + 4 * 3073,
        # SearchLocalPoints: local map points in, the same current-frame reads, taken flags in, match out
        "search_local_points": n_local * 80 + n_kp * (28 + 32 + 4 + 4 + 1 + 4) + 4 * 3073,
        # the three graph stages: MOTION_MODEL (match + keypoint + uR in, edge index out), DISCARD (edge index,
        # outlier flag, match in, taken out), LOCAL_MAP (local match, edge index, keypoint, uR in); map point
        # gathers and point / plane edges out for both graphs, problem headers
        "track_graph_kernel": n_kp * (40 + 10 + 40) + n_pts * (12 + 32) + n_pls * 48 + 3 * 104,
        "lba_batch": lba_bytes,                               # whole LM schedule of the step's local maps (all phase kernels): records in + results out
    }


def _cells(w, h, cell=30):
    """ComputeKeyPointsOctTree's FAST cell grid of one level: (cols - 32) / 30 x (rows - 32) / 30
    (src/ORBextractor.cc:772-787)."""
    return max((w - 32) // cell, 1) * max((h - 32) // cell, 1)


def max_over_ranks(elapsed, dist=None, device="cpu"):
    """Timed-region length of the slowest rank (the whole job ends when it does)."""
    if dist is None:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def per_rank(frames, elapsed, dist=None, device="cpu"):
    """[(frames, elapsed s)] of every rank (one all-gather of two numbers; RCCL over xGMI on the GPU node)."""
    if dist is None:
        return [(frames, elapsed)]
    import torch
    t = torch.tensor([float(frames), elapsed], dtype=torch.float64, device=device)
    got = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(got, t)
    return [(int(g[0].item()), float(g[1].item())) for g in got]


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n, argv):
    """`bench.py --gpus N` started without a launcher: start N rank processes of this script (one per GPU,
    LOCAL_RANK = GPU index) with the torch.distributed environment torch.distributed.run would give them, before
    anything here touches the GPU, and return the first non-zero exit status (0 if all succeed)."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("GPU_MAX_HW_QUEUES", str(HW_QUEUES))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc), 0)


def dist_check(args, rank, world):
    """CPU rehearsal of the multi-rank path (gloo): the same spawn, rendezvous, shard assignment and max / gather
    aggregation as a GPU run, each rank timing the CPU oracle's ORB on its own shard's first frame."""
    import numpy as np
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_ctypes
    import synth
    dist.init_process_group("gloo")
    try:
        shard = shard_of(rank)
        sc = synth.Scene(shard["seq_id"])
        g, _, _ = sc.render(sc.pose(0), noise_seed=shard["seq_id"] * 1000)
        t0 = time.perf_counter()
        kps, _ = oracle_ctypes.OrbOracle().extract(g)
        elapsed = time.perf_counter() - t0
        ranks = per_rank(1, elapsed, dist)
        elapsed = max_over_ranks(elapsed, dist)
        import torch
        chk = torch.tensor([float(len(kps)), float(g.astype(np.int64).sum())], dtype=torch.float64)
        got = [torch.zeros_like(chk) for _ in range(world)]
        dist.all_gather(got, chk)
        if rank == 0:
            print(json.dumps({"dist_check": True, "n_gpus": world, "value": sum(f for f, _ in ranks) / elapsed,
                              "max_elapsed_s": elapsed, "per_rank": [{"rank": r, "frames": f, "elapsed_s": e}
                                                                     for r, (f, e) in enumerate(ranks)],
                              "shards": [shard_of(r)["seq_id"] for r in range(world)],
                              "keypoints": [int(x[0].item()) for x in got],
                              "image_sums": [int(x[1].item()) for x in got]}), flush=True)
    finally:
        dist.destroy_process_group()


def shard_of(rank):
    """Rank r tracks its own synthetic sequence: frames are independent units, no data-path collective."""
    return dict(seq_id=rank)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _build_provenance():
    """The timed library: its sha256 and the build_info.json the Makefile wrote beside it (git commit)."""
    sys.path.insert(0, str(ROOT / "tools"))
    import build_info
    lib = ROOT / "sp-slam_amd" / "libspslam_gpu.so"
    bi = ROOT / "sp-slam_amd" / "build_info.json"
    out = json.loads(bi.read_text()) if bi.exists() else {}
    out["lib_sha256_loaded"] = build_info.lib_sha256(lib)
    out["lib_sha256"] = out["lib_sha256_loaded"]
    return out


def _cgroup_cpus():
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), None when unlimited or unreadable."""
    try:
        q, p = pathlib.Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else max(1, -(-int(q) // int(p)))
    except (OSError, ValueError):
        return None


def cpu_baseline(hp, timed=300, warmup=10, all_core_frames=40):
    """CPU restatement (oracle) of the same per-frame work, timed in C++ (oracle/step_oracle.cpp: the whole chain
    of oracle_step.run with no Python between stages): one core, `warmup` untimed then `timed` frames; then every
    core of this process's CPU set, one independent frame stream per thread.  Also returns the oracle's local-map
    pose of each distinct frame (the CPU reference of the ATE)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_step
    import oracle_step_cpp
    U = len(hp.frames)
    inputs = [oracle_step.from_hotpath(hp, i) for i in range(U)]
    lba = None
    if hp.n_lba:  # LocalMapping: one local BA per keyframe
        lba = ([p[:6] for p in hp.lba_problems], hp.lba_every, hp.plane_cfg)
    nf = hp.ex.params.nfeatures
    import oracle_ctypes
    # timed with the host glibc's double sin / cos / atan2 / pow (what a current build of the reference runs);
    # the CPU reference poses of the ATE come from an untimed pass with the pinned, correctly rounded libm
    el, _ = oracle_step_cpp.bench(inputs, nf, max(warmup, U), timed, 1, supp_cap=hp.pe.supp_cap, lba=lba,
                                  libm=oracle_ctypes.LIBM_GLIBC)
    _, outs = oracle_step_cpp.bench(inputs, nf, U, 0, 1, supp_cap=hp.pe.supp_cap, libm=oracle_ctypes.LIBM_CR)
    poses = {i: outs[i]["Tcw2"].reshape(16).copy() for i in range(U)}
    one = timed / el[0]
    # every core this process may use: its CPU set (sched_getaffinity), capped by the cgroup CPU quota when one
    # is set (a GPU box grants one job a share of the machine; nproc / os.cpu_count() report the whole machine)
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = _cgroup_cpus()
    share = int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit() else None
    threads = max(1, min(x for x in (affinity, quota, share) if x))
    el_all, _ = oracle_step_cpp.bench(inputs, nf, warmup, all_core_frames, threads, supp_cap=hp.pe.supp_cap, lba=lba,
                                      libm=oracle_ctypes.LIBM_GLIBC)
    allc = threads * all_core_frames / el_all.max()
    lba_s = f" + LocalBundleAdjustment every {hp.lba_every} frames" if hp.n_lba else ""
    return dict(value=one, unit="frames/s", cores=1, kind="port",
                sample=f"{timed} frames after {max(warmup, U)} warm-up ({U} distinct) of the same synthetic "
                       f"{hp.W}x{hp.H} workload (grab + ORB + planes + supposed planes + frame steps + "
                       f"SearchByProjection + 2x (plane association + graph + PoseOptimization) + SearchLocalPoints"
                       f"{lba_s}), {el[0]:.1f}s on one core, oracle/liboracle.so C++ -O3 x86-64-v3 "
                       f"(oracle/step_oracle.cpp, no Python between stages), host glibc libm",
                all_cores=dict(value=allc, unit="frames/s", threads=threads, affinity_cpus=affinity,
                               cgroup_cpu_quota=quota, omp_num_threads=share,
                               threads_rule="min(sched_getaffinity, cgroup cpu.max, OMP_NUM_THREADS): the CPU share "
                                            "granted to this job (the GPU box sets OMP_NUM_THREADS to it)",
                               frames_per_thread=all_core_frames,
                               warmup_per_thread=warmup, nproc=os.cpu_count(), cpu_model=_cpu_model(),
                               seconds=float(el_all.max()))), poses


def ate_report(hp, res, cpu_poses=None):
    """ATE (TUM evaluate_ate: Horn alignment + RMSE of camera centres, sp-slam_amd/trajectory.py) of the
    step's local-map poses over the distinct frames: against the CPU reference's poses on the same
    inputs, and against the synthetic ground truth."""
    import numpy as np
    import trajectory
    U = len(hp.frames)
    gpu = [trajectory.camera_center(res["pose2"][i]["Tcw"]) for i in range(U)]
    gt = [hp.scene.pose(hp.frames[i][0])[:3, 3] for i in range(U)]
    out = {"frames": U, "vs_ground_truth_m": trajectory.ate_rmse(gpu, gt), "vs_cpu_ref_m": None,
           "max_center_diff_vs_cpu_ref_m": None}
    if cpu_poses is not None:
        cpu = [trajectory.camera_center(cpu_poses[i]) for i in range(U)]
        out["vs_cpu_ref_m"] = trajectory.ate_rmse(gpu, cpu)
        d = np.linalg.norm(np.array(gpu, np.float64) - np.array(cpu, np.float64), axis=1)
        out["max_center_diff_vs_cpu_ref_m"] = float(d.max())
    return out


def closed_loop(cfg, device, B, steps, warmup, n_seq=16):
    """Closed-loop throughput beside the open-loop headline: sp-slam_amd/sequence.py's tracked sequences at B
    slots (B / n_seq slots per rendered sequence, each slot its own independent tracking state), one tracked
    frame per slot per step -- every frame's prior, last-frame points and matches from its predecessor's
    result, frame 1 by TrackReferenceKeyFrame (BoW).  Same pipelined step structure as the headline."""
    import torch
    import sequence
    sp = sequence.SequencePath(B, warmup + steps + 2, n_sequences=n_seq, device=device,
                               render_workers=min(16, os.cpu_count() or 1), pipelined=True, **cfg)
    try:
        for _ in range(warmup):
            sp.step()
        torch.cuda.synchronize()
        if sp.local_mapping:
            sp.lm_time = {"total_s": 0.0, "lba_s": 0.0}  # the timed steps' events only
        t0 = time.perf_counter()
        for _ in range(steps):
            sp.step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        h = sp.history()
        out = {"value": B * steps / el, "unit": "frames/s", "slots": B, "sequences": n_seq, "steps": steps,
               "warmup": warmup, "ms_per_step": el * 1e3 / steps,
               "mean_matches": float(h[warmup + 1:, :, 0].mean()),
               "mean_inliers_local_map": float(h[warmup + 1:, :, 3].mean()),
               "local_bundle_adjustments": len(getattr(sp, "lm_runs", [])),
               "kind": "tracked sequences (sp-slam_amd/sequence.py): motion model from the previous frame, "
                       "TrackReferenceKeyFrame at frame 1" +
                       (" and where the motion model fails" if sp.refkf_fallback else "") +
                       (", deterministic LocalMapping with LocalBundleAdjustment every 10 frames"
                        if sp.local_mapping else "")}
        if sp.refkf_fallback:
            out["reference_keyframe_frames"] = int((sp.fallback_history()[warmup + 1:] == 1).sum())
        if sp.local_mapping:
            # the LocalMapping events are synchronous and mostly host bookkeeping (local_mapping.py, caller side):
            # their wall time, the device LocalBundleAdjustment inside it, and the step without them
            lt = sp.lm_time
            out["local_mapping_wall_s"] = lt["total_s"]
            out["local_mapping_device_lba_s"] = lt["lba_s"]
            rest = max(el - lt["total_s"], 1e-9)
            out["ms_per_step_without_local_mapping"] = rest * 1e3 / steps
        return out
    finally:
        sp.close()


def single_sequence(cfg, device, n_frames=120, warmup=5, lookahead=None, modes=(True, False)):
    """The reference's own call pattern (Examples/RGB-D/SPSLAM.cc:90-136 -> System::TrackRGBD per frame): ONE
    tracked sequence, one frame at a time (B = 1, sp-slam_amd/sequence.py; every frame's prior and last-frame
    points from its predecessor).  frames_per_s: frames k+1 .. k+L's grab / ORB / planes overlapped with frame k's
    tracking tail (the pipelined step, L = SINGLE_LOOKAHEAD frames read ahead as SPSLAM.cc's loop over the image list
    allows; two extraction units side by side), the host waiting for frame k-1's tail before it returns from frame
    k (SINGLE_INFLIGHT).  latency_ms_*: the serial step (grab ->
    extraction -> tracking tail) with the host waiting for each frame's pose -- image on the device to pose on the
    device, the per-frame latency a TrackRGBD caller sees (the 64-byte pose read-back excluded)."""
    import numpy as np
    import torch
    import sequence
    look = SINGLE_LOOKAHEAD if lookahead is None else lookahead
    out = {"kind": "one sequence, B = 1 (sequence.SequencePath), frames device-resident", "frames": n_frames,
           "lookahead": look, "max_inflight": SINGLE_INFLIGHT}
    for pipelined in modes:
        sp = sequence.SequencePath(1, n_frames + warmup + 2, n_sequences=1, device=device, pipelined=pipelined,
                                   lookahead=look if pipelined else 1, max_inflight=SINGLE_INFLIGHT,
                                   render_workers=min(16, os.cpu_count() or 1), **cfg)
        try:
            for _ in range(warmup):
                sp.step()
            torch.cuda.synchronize()
            lat = []
            t0 = time.perf_counter()
            for _ in range(n_frames):
                ts = time.perf_counter()
                sp.step()
                if not pipelined:
                    torch.cuda.synchronize()
                    lat.append(time.perf_counter() - ts)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        finally:
            sp.close()
        if pipelined:
            out["frames_per_s"] = n_frames / el
        else:
            out["serial_frames_per_s"] = n_frames / el
            out["latency_ms_p50"] = float(np.percentile(lat, 50) * 1e3)
            out["latency_ms_p99"] = float(np.percentile(lat, 99) * 1e3)
            out["latency_ms_max"] = float(max(lat) * 1e3)
    return out


def single_sequence_line(config, device, n_frames):
    """single_sequence() in processes of their own on the same GPU (one for the pipelined rate, one for the serial
    latency), with HIP's default of 4 hardware queues: the reference's call pattern is one tracking process per
    sequence, and a B = 1 step's few streams run best on 4 queues (pipelined 710 frames/s against 594 with the 8
    this process opened for the C2 step, and ~430-475 run after the C2 step inside this process; serial p50 3.40
    ms alone against 3.58 after a pipelined run in the same process: profiles/r06/ab_single_sequence_queues.txt)."""
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env.update(GPU_MAX_HW_QUEUES=str(SINGLE_HW_QUEUES), SPSLAM_BENCH_CHILD="1")
    if "HIP_VISIBLE_DEVICES" not in env and "CUDA_VISIBLE_DEVICES" not in env:
        env["HIP_VISIBLE_DEVICES"] = str(device)
    out = {}
    for mode in ("pipelined", "serial"):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--config", config, "--single-sequence-child",
                            mode, "--single-sequence-frames", str(n_frames)], env=env, capture_output=True, text=True,
                           timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"single_sequence {mode} child failed ({r.returncode}): {r.stderr[-2000:]}")
        out.update(json.loads(r.stdout.strip().splitlines()[-1]))
    out["process"] = f"one process per mode, GPU_MAX_HW_QUEUES={SINGLE_HW_QUEUES}"
    return out


def ate_sequences(cfg, device, n_frames=300, n_seq=2):
    """ATE of tracked sequences (sp-slam_amd/sequence.py): n_seq sequences of n_frames tracked frames each on
    the GPU, every frame's prior and last-frame points from its predecessor's result, against the CPU oracle
    running the same loop (oracle/oracle_sequence.py) and against the synthetic ground truth.  TUM
    evaluate_ate (Horn alignment, RMSE of camera centres, sp-slam_amd/trajectory.py) per sequence."""
    import numpy as np
    import sequence
    import trajectory
    t0 = time.perf_counter()
    workers = min(16, os.cpu_count() or 1)
    sp = sequence.SequencePath(n_seq, n_frames + 1, n_sequences=n_seq, device=device, render_workers=workers, **cfg)
    try:
        for _ in range(n_frames):
            sp.step()
        tr = sp.trajectory()
        hist = sp.history()
        t_gpu = time.perf_counter() - t0
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle_ctypes
        import oracle_grab
        import oracle_planes
        import oracle_seq_inputs as OSI
        import oracle_sequence
        import oracle_step
        cam, geo, inv_s2 = oracle_step.camera_inputs(sp)
        out = {"kind": "tracked sequences (motion model from the previous frame; sp-slam_amd/sequence.py)" +
                       (" with the deterministic LocalMapping (local_mapping.py: keyframes every 10 frames, "
                        "LocalBundleAdjustment written back into the map)" if sp.local_mapping else ""),
               "sequences": n_seq, "frames": n_frames,
               "cpu_ref": "CPU oracle (oracle/oracle_sequence.py): PoseOptimization summed in g2o's edge order with "
                          "Eigen's per-edge arithmetic and correctly rounded sin/cos/atan2/pow (the pinned libm, "
                          "DESIGN.md 3.3); glibc_libm_cpu_ref: the same loop with the host glibc's double routines; "
                          "fma_contracted_cpu_ref: the same loop with the pose / LBA restatement compiled with GCC's "
                          "FP contraction (a -march=native g2o build, Thirdparty/g2o/CMakeLists.txt:57)",
               "vs_cpu_ref_m": [], "max_center_diff_vs_cpu_ref_m": [],
               "max_rotation_diff_vs_cpu_ref": [], "vs_ground_truth_m": [], "cpu_ref_vs_ground_truth_m": [],
               "ate_difference_vs_cpu_ref_m": [], "identical_decisions_until_frame": [],
               "glibc_libm_cpu_ref": {"vs_gpu_m": [], "vs_cpu_ref_m": [], "vs_ground_truth_m": [],
                                      "identical_decisions_until_frame": []},
               "fma_contracted_cpu_ref": {"vs_gpu_m": [], "vs_cpu_ref_m": [], "vs_ground_truth_m": [],
                                          "identical_decisions_until_frame": []}}
        t1 = time.perf_counter()

        import synth
        vocab_text = synth.shape_vocabulary_text()
        oracle_sequence.vocabulary(vocab_text)  # loaded once, before the threads

        def run_oracle(slot, order):
            if order == "fma":  # the pinned libm, contracted g2o arithmetic
                with oracle_ctypes.g2o_fma(True):
                    return run_oracle(slot, oracle_ctypes.LIBM_CR)
            frames, T0, P0, local_of = OSI.inputs(sp, slot)
            ch = {}

            def rec(t, o, P):
                ch[t] = (o["nmatches"], o["local_nmatches"], int(o["pose1"][0]["n_inliers"]),
                         int(o["pose2"][0]["n_inliers"]))
            orb, po = oracle_ctypes.OrbOracle(nfeatures=sp.ex.params.nfeatures), oracle_planes.PlaneOracle()
            ref = oracle_sequence.reference_keyframe(OSI.reference_keyframe(sp, slot), vocab_text)
            cpu = oracle_sequence.track(frames[:n_frames], 1, T0, P0, local_of, cam, geo, inv_s2, sp.assoc_map,
                                        sp.assoc_boundary, orb, po, supp_cap=sp.pe.supp_cap, min_size=sp.min_size,
                                        pose_cfg=sp.plane_cfg, depth_scale=oracle_grab.depth_scale(sp.depth_factor),
                                        on_frame=rec, libm=order, ref_kf=ref,
                                        local_map=OSI.local_map(sp, slot) if sp.local_mapping else None,
                                        refkf_of=OSI.refkf_of(sp, slot, vocab_text) if sp.refkf_fallback else None,
                                        kf_id_stride=sp.kp_cap)
            same = [tuple(int(x) for x in hist[t, slot]) == ch[t] for t in range(1, n_frames + 1)]
            return cpu, next((t for t, ok in enumerate(same, 1) if not ok), None)

        from concurrent.futures import ThreadPoolExecutor
        jobs = [(slot, order) for slot in range(n_seq)
                for order in (oracle_ctypes.LIBM_CR, oracle_ctypes.LIBM_GLIBC, "fma")]
        with ThreadPoolExecutor(len(jobs)) as pool:
            done = dict(zip(jobs, pool.map(lambda j: run_oracle(*j), jobs)))
        for slot in range(n_seq):
            cpu, div = done[(slot, oracle_ctypes.LIBM_CR)]
            cpu_g, div_g = done[(slot, oracle_ctypes.LIBM_GLIBC)]
            cpu_f, div_f = done[(slot, "fma")]
            out["identical_decisions_until_frame"].append(div)
            g = [trajectory.camera_center(tr[k + 1, slot].reshape(16)) for k in range(n_frames)]
            c = [trajectory.camera_center(cpu[k].reshape(16)) for k in range(n_frames)]
            cg = [trajectory.camera_center(cpu_g[k].reshape(16)) for k in range(n_frames)]
            cf = [trajectory.camera_center(cpu_f[k].reshape(16)) for k in range(n_frames)]
            gt = [np.linalg.inv(sp._true_pose(slot, k + 1))[:3, 3] for k in range(n_frames)]
            out["vs_cpu_ref_m"].append(trajectory.ate_rmse(g, c))
            out["max_center_diff_vs_cpu_ref_m"].append(float(np.linalg.norm(np.array(g) - np.array(c), axis=1).max()))
            out["max_rotation_diff_vs_cpu_ref"].append(float(max(
                np.abs(tr[k + 1, slot][:3, :3] - cpu[k][:3, :3]).max() for k in range(n_frames))))
            out["vs_ground_truth_m"].append(trajectory.ate_rmse(g, gt))
            out["cpu_ref_vs_ground_truth_m"].append(trajectory.ate_rmse(c, gt))
            out["ate_difference_vs_cpu_ref_m"].append(abs(out["vs_ground_truth_m"][-1] - out["cpu_ref_vs_ground_truth_m"][-1]))
            go = out["glibc_libm_cpu_ref"]
            go["vs_gpu_m"].append(trajectory.ate_rmse(g, cg))
            go["vs_cpu_ref_m"].append(trajectory.ate_rmse(c, cg))
            go["vs_ground_truth_m"].append(trajectory.ate_rmse(cg, gt))
            go["identical_decisions_until_frame"].append(div_g)
            fo = out["fma_contracted_cpu_ref"]
            fo["vs_gpu_m"].append(trajectory.ate_rmse(g, cf))
            fo["vs_cpu_ref_m"].append(trajectory.ate_rmse(c, cf))
            fo["vs_ground_truth_m"].append(trajectory.ate_rmse(cf, gt))
            fo["identical_decisions_until_frame"].append(div_f)
        out["cpu_frames_per_s"] = len(jobs) * n_frames / (time.perf_counter() - t1)  # len(jobs) threads
        out["wall_s"] = {"gpu_incl_render": t_gpu, "cpu": time.perf_counter() - t1}
        return out
    finally:
        sp.close()


def _ensure_hw_queues(want=None):
    want = want or HW_QUEUES
    try:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        cur = 4
    if cur >= want or os.environ.get("SPSLAM_BENCH_CHILD"):
        return
    import subprocess
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(want), SPSLAM_BENCH_CHILD="1")
    sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))


LBA_DEPTH, LBA_TEAM = 3, 1  # C3 defaults: 4 calls in flight, one CU per map (profiles/r06/ab_c3_depth.txt; r05/ab_c3_*)
# single_sequence: frames extracted ahead of tracking, and the host at most one step ahead of the device
# (profiles/r05/b1_lookahead.txt, b1_inflight.txt)
SINGLE_LOOKAHEAD, SINGLE_INFLIGHT, SINGLE_HW_QUEUES = 2, 1, 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="frames per step per GPU")
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--unique-frames", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=0,
                    help="timed one-core CPU baseline frames (default 300; 100 above 640x480)")
    ap.add_argument("--no-tail-priority", action="store_true", help="tracking stream at normal priority")
    ap.add_argument("--orb-priority", action="store_true", default=True,
                    help="next batch's ORB stream at high priority (default: the ORB chain is the C2 step's critical path, "
                         "profiles/r06/ab_stream_priority.txt)")
    ap.add_argument("--no-orb-priority", dest="orb_priority", action="store_false")
    ap.add_argument("--planes-priority", action="store_true",
                    help="next batch's plane stream at high priority (round 3's default; with the round-5 plane "
                         "wavefront 1.5 %% slower, profiles/r05/ab_octree_planes_pose.txt)")
    ap.add_argument("--no-planes-priority", action="store_true", help=argparse.SUPPRESS)  # (the default now)
    ap.add_argument("--lba-order", default="g2o", choices=("g2o", "fast"),
                    help="LocalBundleAdjustment summation order (C3): g2o = the reference's arithmetic, bit-exact "
                         "to the oracle (default); fast = the phase kernels (tree / matrix-core order)")
    ap.add_argument("--lba-depth", type=int, default=None,
                    help="C3: step k's LocalBundleAdjustment call is joined at the end of step k + d (LocalMapping "
                         "does not block Tracking, LocalMapping.cc:48-124); default %d" % 2)
    ap.add_argument("--lba-team", type=int, default=None,
                    help="C3: workgroups per local map (0: as many as fill the chip); default 1 (the least CU time per map: with two calls in flight the LBA overlaps tracking instead of crowding it)")
    ap.add_argument("--lookahead", type=int, default=1,
                    help="batches extracted ahead of the tracking tail (the Python step; the native step runs 1)")
    ap.add_argument("--python-step", action="store_true",
                    help="drive the step's stages from Python over torch streams (pipeline.py) instead of the "
                         "library's whole-step entry spslam_step_run (the default without LocalMapping)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run each step's extraction and tracking back to back (no cross-step overlap)")
    ap.add_argument("--ate-frames", type=int, default=300,
                    help="frames per tracked sequence of the ATE check (0 = skip)")
    ap.add_argument("--single-sequence-frames", type=int, default=120,
                    help="frames of the single-sequence (B = 1) line (0 = skip)")
    ap.add_argument("--single-sequence-child", choices=("pipelined", "serial"), help=argparse.SUPPRESS)  # (single_sequence_line)
    ap.add_argument("--closed-loop-steps", type=int, default=20,
                    help="timed steps of the closed-loop line (tracked sequences at --batch slots; 0 = skip)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="multi-rank rehearsal on a one-GPU box: every rank on GPU 0, collectives over gloo (the "
                         "per-rank HotPath and the aggregation run as in an N-GPU job; the value is not a scaling "
                         "number)")
    ap.add_argument("--dist-check", action="store_true",
                    help="CPU rehearsal of the multi-rank launch (gloo, no GPU): spawn, rendezvous, aggregation")
    args = ap.parse_args()
    if args.single_sequence_child:  # (single_sequence_line: one process, one GPU, no ranks)
        import pipeline
        print(json.dumps(single_sequence(pipeline.CONFIGS[args.config], 0, n_frames=args.single_sequence_frames,
                                         modes=(args.single_sequence_child == "pipelined",))))
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))  # one process per GPU (no launcher was used)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.dist_check:
        return dist_check(args, rank, world)
    # C3: every in-flight LocalBundleAdjustment call has its own context stream; with 8 hardware queues they alias
    # the tracking streams' queues and serialise (profiles/r05/ab_c3_hwq*.txt), so C3 runs with 16
    _ensure_hw_queues(16 if args.config in ("c3", "c3s") else None)
    import pipeline
    cfg = pipeline.CONFIGS[args.config]
    import torch
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    coll_dev = "cpu" if args.rehearse_one_gpu else "cuda"

    hp = pipeline.HotPath(args.batch, unique_frames=args.unique_frames, device=local,
                          pipelined=not args.no_pipeline, tail_priority=not args.no_tail_priority,
                          orb_priority=args.orb_priority, planes_priority=args.planes_priority,
                          lba_order=0 if args.lba_order == "g2o" else 1,
                          native=not args.python_step and not cfg.get("lba_every"), **cfg,
                          lba_depth=LBA_DEPTH if args.lba_depth is None else args.lba_depth,
                          lba_team=LBA_TEAM if args.lba_team is None else args.lba_team,
                          lookahead=args.lookahead, **shard_of(rank))
    for _ in range(args.warmup):
        hp.step()
    torch.cuda.synchronize()
    hp.set_timing(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hp.step()
    # C3: the LocalBundleAdjustment calls of the timed steps still in flight (a pool thread launches each call, so one
    # not yet enqueued would escape the synchronize) finish inside the timed region
    hp.lba_drain()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    times = {k: v for k, v in hp.kernel_times().items() if v[1] > 0}
    res = hp.results()
    ranks = per_rank(args.batch * args.steps, elapsed, dist, coll_dev)
    elapsed = max_over_ranks(elapsed, dist, coll_dev)

    frames = sum(f for f, _ in ranks)
    value = frames / elapsed
    total_kernel_ms = sum(v[0] for v in times.values())
    dom, (dom_ms, dom_n) = max(times.items(), key=lambda kv: kv[1][0])
    P1, P2 = hp.graph(0)[0], hp.graph(1)[0]
    n_pts = float((P1["n_points"].sum() + P2["n_points"].sum()) / args.batch)
    n_pls = float((P1["n_planes"].sum() + P2["n_planes"].sum()) / args.batch)
    n_con = float(res["contour_points"].mean())
    n_sup = float(res["supposed_counts"].mean())
    n_brd = float(res["line_points"].mean())
    lba_bytes = 0
    if hp.n_lba:  # per frame: the keyframe's local map in (records) and its results out
        lba_bytes = (hp.lba_points * (24 + 12) + hp.lba_edges * (20 + 1) +
                     hp.lba_window["keyframes"] * (96 + 64)) * hp.n_lba / args.batch
    n_fpl = float(res["plane_counts"].mean()) + n_sup
    alg = algorithmic_bytes(cfg, hp.mean_keypoints, n_pts, n_pls, n_con, n_brd, n_sup, lba_bytes, n_fpl, hp.n_map,
                            hp.n_boundary, hp.mean_proj_points, hp.mean_local_points, hp.mean_fast_candidates)
    launches_per_step = dom_n / args.steps
    avg_launch_s = dom_ms / 1e3 / max(dom_n, 1)
    bytes_per_launch = alg[dom] * args.batch * (2 if dom == "pose_kernel" else 1) / launches_per_step
    achieved = bytes_per_launch / avg_launch_s / 1e9
    # every kernel kind: algorithmic bytes of a step / its event time in a step, as a fraction of HBM peak
    by_kernel = {}
    for k, (ms, _) in sorted(times.items()):
        if k in alg and ms > 0:
            gbs = alg[k] * args.batch * (2 if k == "pose_kernel" else 1) / (ms / 1e3 / args.steps) / 1e9
            by_kernel[k] = {"achieved_gbs": gbs, "frac": gbs / HBM_PEAK_GBS}
    # HBM traffic cannot be counted inside this process (the PMC passes need rocprofv3 around it): it is read
    # from the committed summary of such a run and reported with where and when it was measured
    # (provenance: the library hash at PMC time against the library this process loaded; a mismatch marks the
    # committed traffic stale and it is not reported)
    traffic, traffic_src = None, None
    pmc = ROOT / "profiles" / f"pmc_{args.config}_b{args.batch}.json"
    build = _build_provenance()
    if pmc.exists():
        try:
            pj = json.loads(pmc.read_text())
            prov = pj.get("provenance", {})
            fresh = prov.get("lib_sha256") == build.get("lib_sha256")
            traffic = pj.get(dom) if fresh else None
            traffic_src = {"file": str(pmc.relative_to(ROOT)), **prov, "matches_timed_library": fresh}
        except Exception:
            traffic = None
    result = {
        "metric": "RGB-D frames/sec (track+planes+poseOpt) at 640x480; ATE vs CPU ref",
        "value": value,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8+f32+f64",
        "data": "synthetic (in-repo textured-room RGB-D renderer sp-slam_amd/synth.py; map points / map planes "
                "synthesized from the scene, every correspondence from the step's own matching + association)",
        "per_rank": [{"rank": r, "frames": f, "elapsed_s": e} for r, (f, e) in enumerate(ranks)],
        "config": {"workload": WORKLOADS[args.config], "name": args.config, "frames_per_step_per_gpu": args.batch,
                   "parallelism": f"shard{world}" + ("-rehearsal-on-gpu0-gloo" if args.rehearse_one_gpu else ""),
                   "mean_keypoints": hp.mean_keypoints,
                   **({"lba_window": hp.lba_window} if hp.n_lba else {}),
                   "pipelined": hp.pipelined,
                   "step": "spslam_step_run (library streams and events)" if hp.native is not None
                           else "pipeline.py over torch streams",
                   "mean_planes": float(res["plane_counts"].mean()),
                   "mean_supposed_planes": n_sup,
                   "pose_edges_per_frame": n_pts + n_pls},
        "kernels_ms_per_step": {k: v[0] / max(args.steps, 1) for k, v in sorted(times.items())},
        "roofline_by_kernel": by_kernel,
        "roofline": {"kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "bytes_per_launch": bytes_per_launch, "avg_launch_ms": avg_launch_s * 1e3,
                     "share_of_kernel_time": dom_ms / max(total_kernel_ms, 1e-9)},
        "cpu_baseline": None,
        "build": build,
    }
    if dom == "pose_kernel":
        # the bound that limits it: not HBM (a few MB per launch) but its ordered fp64 chains and the fp64 issue
        # of the plane-edge evaluations; achieved / frac stay the HBM reading of the contract
        result["roofline"]["bound"] = "fp64-issue/latency"
        floor = pose_chain_floor(P1, P2, res["pose1"], res["pose2"])
        result["roofline"]["latency_model"] = {
            "model": "ordered fp64 sums (g2o edge order): per problem (LM iterations + trial passes) x edges chain "
                     f"rows at {CHAIN_CYCLES_PER_ROW} cycles, longest problem of the launch, {CLOCK_HZ / 1e9} GHz",
            "chain_floor_ms_per_launch": floor, "avg_launch_ms": avg_launch_s * 1e3,
            "frac": floor / max(avg_launch_s * 1e3, 1e-9),
            "mean_lm_iterations": float((res["pose1"]["lm_iterations"].mean() + res["pose2"]["lm_iterations"].mean()) / 2),
            "mean_trial_passes": float((res["pose1"]["trial_passes"].mean() + res["pose2"]["trial_passes"].mean()) / 2)}
    elif dom == "level_kernel":
        # the pyramid's 8 launches stream 3.8 MB per frame, but inside the pipelined step their spans include the
        # wait for CUs held by the plane and tracking streams: the small levels' launches last ~345 us each in
        # the step against ~15 us alone
        result["roofline"]["note"] = ("event spans inside the pipelined step (three streams share the CUs); the "
                                      "small levels' launches mostly wait for CUs")
    elif dom == "lba_batch":
        # one workgroup per LocalBundleAdjustment problem walking g2o's ordered fp64 chains (buildSystem in edge
        # order, the Schur complement in landmark order, the up-looking LDLT): latency-bound, 16 MB per launch
        result["roofline"]["bound"] = "fp64-issue/latency"
        result["roofline"]["note"] = ("ordered fp64 chains per problem (DESIGN.md section 3.9); the launch ends with "
                                      "its slowest problem, phases in tools/lba_bench.py --order g2o")
    # validity of the timed results: no PoseOptimization gave up on a bounded device wait (lm_iterations = -1),
    # every LocalBundleAdjustment of the step finished (status 0)
    checks = {"pose_wait_give_ups": int((res["pose1"]["lm_iterations"] < 0).sum() + (res["pose2"]["lm_iterations"] < 0).sum())}
    if hp.n_lba:
        import spslam_lba
        lr = [sl["out"][-1].cpu().numpy().view(spslam_lba.LBA_RESULT_DTYPE) for sl in hp.lba_slots]
        checks["lba_failed"] = int(sum((r["status"] != 0).sum() for r in lr))
        checks["lba_order"] = "g2o" if hp.lba_order == spslam_lba.G2O_ORDER else "fast"
        checks["lba_in_flight"] = hp.lba_depth + 1
        checks["lba_team"] = hp.lba_slots[0]["lba"].team
    cpu_poses = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"], cpu_poses = cpu_baseline(hp, timed=args.cpu_frames or (300 if hp.W * hp.H <= 640 * 480 else 100))
    if rank == 0:
        result["open_loop_pose_agreement"] = ate_report(hp, res, cpu_poses)
    hp.close()
    if rank == 0 and args.closed_loop_steps > 0:
        result["closed_loop"] = closed_loop(cfg, local, args.batch, args.closed_loop_steps, args.warmup)
    if rank == 0 and args.single_sequence_frames > 0:
        result["single_sequence"] = single_sequence_line(args.config, local, args.single_sequence_frames)
        if result["cpu_baseline"]:  # one core, the same per-frame work (the oracle step, open loop)
            result["single_sequence"]["cpu_1core_frames_per_s"] = result["cpu_baseline"]["value"]
    if rank == 0 and args.ate_frames > 0:
        result["ate"] = ate_sequences(cfg, local, n_frames=args.ate_frames)
    if rank == 0:
        # the north-star bar: every tracked trajectory within 1e-4 m of the CPU reference's (trajectory vs
        # trajectory, not the difference of the two ATEs to ground truth) and no invalid result in the timed run
        ok = checks["pose_wait_give_ups"] == 0 and checks.get("lba_failed", 0) == 0
        if "ate" in result:
            v = result["ate"]["vs_cpu_ref_m"]
            checks["ate_vs_cpu_ref_m_max"] = max(v) if v else None
            checks["decisions_diverge_at"] = result["ate"]["identical_decisions_until_frame"]
            ok = ok and all(x <= 1e-4 for x in v)
        result["parity_ok"] = bool(ok)
        result["parity_checks"] = checks
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
