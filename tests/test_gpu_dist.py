"""The N-rank benchmark path with the GPU work in it (verdict r02: the per-rank HotPath and the aggregation
never ran with world > 1): bench.py --gpus 2 --rehearse-one-gpu spawns two ranks that each build and time
their own HotPath (their own sequence, shard_of) on GPU 0, then aggregate over gloo exactly as an 8-GPU job
aggregates over RCCL.  Checks the JSON line's contract: world size, one entry per rank, value = all frames /
the slowest rank's time."""
import json
import os
import pathlib
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("config", ["c2", "c4"])
def test_two_ranks_on_one_gpu(config):
    cmd = [sys.executable, str(ROOT / "bench.py"), "--config", config, "--gpus", "2", "--rehearse-one-gpu", "--steps",
           "3", "--warmup", "1", "--batch", "16", "--no-cpu-baseline", "--ate-frames", "0", "--closed-loop-steps", "0"]
    if config != "c2":
        cmd += ["--single-sequence-frames", "0"]
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and len(out["per_rank"]) == 2
    assert [p["frames"] for p in out["per_rank"]] == [16 * 3, 16 * 3]
    slowest = max(p["elapsed_s"] for p in out["per_rank"])
    assert abs(out["value"] - 2 * 16 * 3 / slowest) <= 1e-6 * out["value"]
    assert out["config"]["parallelism"].startswith("shard2")
