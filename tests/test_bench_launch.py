"""bench.py's rank launch (CPU, gloo): `--gpus N` without an outer launcher starts
torch.distributed.run itself, the JSON line reports all N ranks, and more GPUs
than are visible is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, timeout=240):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_bench_spawns_ranks_gloo():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["dry_run"] and out["steps"] == 3
    # max over ranks: rank 1 sleeps twice as long as rank 0 (2 x 3 ms)
    assert out["ms_per_step"] >= 1.9, out
    # what ran: the backend and world size torch.distributed reported, per-rank
    # step times and the max the value is computed from (the driver's SCALE
    # record reads the same fields with backend "nccl" = RCCL)
    d = out["dist"]
    assert d["backend"] == "gloo" and d["library"] == "gloo" and d["world_size"] == 2, d
    assert len(d["per_rank_ms_per_step"]) == 2
    # (each rank's clock runs from barrier to barrier, so it includes the wait
    # for the slowest rank: rank 1 sleeps 6 ms, every rank's time is >= that)
    assert min(d["per_rank_ms_per_step"]) >= 1.9, d
    assert d["max_ms_per_step"] == max(d["per_rank_ms_per_step"]) == out["ms_per_step"], d


def test_bench_refuses_more_gpus_than_visible():
    r = _run(["--gpus", "4096", "--steps", "1"])
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "visible" in r.stderr
