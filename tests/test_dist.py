"""World-size-2 gloo run of bench.py's multi-GPU logic on CPU.

The hot path shards by frame sequence (one synthetic sequence per rank, no
data-path collective); the only collective is the max over ranks of the timed
region.  Here each rank renders its shard's first frame, runs the CPU oracle
of the ORB stage on it, and the ranks exchange results to check the shards are
distinct and the timing reduction is the max.
"""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle_ctypes
        import synth
        shard = bench.shard_of(rank)
        sc = synth.Scene(shard["seq_id"])
        g, _, _ = sc.render(sc.pose(0), noise_seed=shard["seq_id"] * 1000)
        kps, _ = oracle_ctypes.OrbOracle().extract(g)
        elapsed = bench.max_over_ranks(1.0 + rank, dist)
        t = torch.tensor([float(len(kps)), float(g.astype(np.int64).sum())], dtype=torch.float64)
        got = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(got, t)
        out[rank] = (elapsed, [x.tolist() for x in got])
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo():
    import torch.multiprocessing as mp
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    assert sorted(out.keys()) == [0, 1]
    for r in range(world):
        elapsed, got = out[r]
        assert elapsed == 2.0                          # max over ranks
        assert got[0][1] != got[1][1]                  # distinct shards
        assert all(1000 <= g[0] <= 1016 for g in got)  # each shard ran the full ORB quota


def test_single_rank_helpers():
    import bench
    assert bench.max_over_ranks(3.5) == 3.5
    assert bench.shard_of(0) != bench.shard_of(1)
    pytest.importorskip("torch")


def _bench_json(out):
    import json
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_spawns_ranks_itself():
    """`python bench.py --gpus 2` with no launcher starts its own two rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set before any GPU work) and rank 0 reports both ranks' frames and the max elapsed.
    --dist-check runs that exact spawn + rendezvous + aggregation path over gloo on the CPU."""
    import os
    import pathlib
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--dist-check"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = _bench_json(p.stdout)
    assert r["n_gpus"] == 2 and [x["rank"] for x in r["per_rank"]] == [0, 1]
    assert r["max_elapsed_s"] == max(x["elapsed_s"] for x in r["per_rank"])
    assert r["shards"] == [0, 1] and r["image_sums"][0] != r["image_sums"][1]
    assert all(1000 <= k <= 1016 for k in r["keypoints"])


def test_bench_rejects_launcher_mismatch():
    """Launched as 2 ranks by torch.distributed.run but asked for --gpus 4: refuse instead of reporting a
    wrong n_gpus."""
    import os
    import pathlib
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    env = dict(os.environ, RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    p = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "4", "--dist-check"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "--gpus 4" in p.stderr
