"""bench.py's N-rank paths with the real engine (not a sleep): two ranks share
cuda:0 over gloo (`--dist-backend gloo --share-device`), once walker-sharded and
once as a 2-rung replica-exchange ladder (BASELINE config 5's exchange step).
The RCCL runs differ only by the backend string (bench.py main)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
W, STEPS = 256, 12


def _bench(extra, timeout=240):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo", "--share-device",
           "--walkers", str(W), "--steps", str(STEPS), "--warmup", "2", "--no-cpu-baseline",
           "--no-sub-records"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]   # rank 0 prints the one line
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_two_ranks_sharded():
    out = _bench([])
    assert out["n_gpus"] == 2 and out["config"]["global_walkers"] == 2 * W
    assert out["config"]["dist_backend"] == "gloo" and out["config"]["shared_device"]
    assert sum(out["config"]["outcomes"].values()) == 2 * W * STEPS   # summed over ranks
    assert out["value"] > 0 and out["roofline"]["kernel_ms_per_launch"] > 0
    assert "walker-sharded x2" in out["config"]["parallelism"]
    d = out["dist"]   # what torch.distributed reported (the RCCL run: backend "nccl")
    assert d["backend"] == "gloo" and d["world_size"] == 2 and len(d["per_rank_ms_per_step"]) == 2
    assert d["max_ms_per_step"] == max(d["per_rank_ms_per_step"])
    assert abs(d["max_ms_per_step"] - out["ms_per_step"]) <= 1e-9 * out["ms_per_step"]


@pytest.mark.gpu
def test_bench_two_ranks_replica_exchange():
    out = _bench(["--replica-interval", "4"])
    assert out["n_gpus"] == 2
    assert sum(out["config"]["outcomes"].values()) == 2 * W * STEPS
    ex = out["exchange"]
    # 12 steps every 4: rounds 0, 1, 2; the pair (0, 1) swaps on even rounds only
    assert ex["rounds_per_rank"] == 3
    assert ex["attempted"] == 2 * 2 * W            # two even rounds, counted on both ranks
    assert 0 <= ex["accepted"] <= ex["attempted"] and ex["accepted"] % 2 == 0
    assert ex["temperatures"] == [0.5, 0.75]
    assert "replica exchange x2 (gloo" in out["config"]["parallelism"]
