"""BASELINE configs[4] at its own size with the engine: an 8-rung replica
ladder (T_r = 0.5 * 1.5^r) x 4096 walkers per rung, one bench.py rank per
rung, all 8 ranks sharing cuda:0 over gloo (`--share-device`): the RCCL run
on a node differs only by the backend string (bench.py main).  Each rank
writes a swap audit (bench.py --replica-audit) that this test checks:

* the ladder and the alternating neighbour pairing with idle ends
  (replica.partner);
* configuration conservation: per round and walker slot, a pair's two
  configurations either stay or trade places, idle rungs keep theirs;
* both ranks of a pair see the same swaps, so the summed accept count is even;
* sampled final walkers' stored scores equal the oracle's MFE score of their
  final sequences (exact integer energies);
* counters cover W x steps per rank.
"""
import glob
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from addapt_amd import replica, workloads

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
WORLD, W, STEPS, INTERVAL = 8, 4096, 200, 100


@pytest.mark.gpu
def test_config5_ladder_8_rungs_4096_walkers(oracle, tmp_path):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    audit = str(tmp_path / "audit")
    cmd = [sys.executable, BENCH, "--gpus", str(WORLD), "--dist-backend", "gloo", "--share-device",
           "--replica-interval", str(INTERVAL), "--walkers", str(W), "--steps", str(STEPS),
           "--warmup", "2", "--no-cpu-baseline", "--no-sub-records", "--replica-audit", audit]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=220, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == WORLD and out["config"]["global_walkers"] == WORLD * W
    ex = out["exchange"]
    temps = [0.5 * 1.5 ** k for k in range(WORLD)]
    assert ex["temperatures"] == pytest.approx(temps, rel=0, abs=0)
    assert ex["rounds_per_rank"] == STEPS // INTERVAL
    assert sum(out["config"]["outcomes"].values()) == WORLD * W * STEPS
    assert "replica exchange x8 (gloo" in out["config"]["parallelism"]

    files = sorted(glob.glob(os.path.join(audit, "rank*.npz")))
    assert len(files) == WORLD
    A = {int(os.path.basename(f)[4:-4]): np.load(f) for f in files}
    rounds = STEPS // INTERVAL
    swapped_total = 0
    for rank in range(WORLD):
        a = A[rank]
        assert float(a["temperature"][0]) == temps[rank]
        assert list(a["round"]) == list(range(rounds))
        assert [int(p) for p in a["partner"]] == [
            -1 if replica.partner(rank, WORLD, k) is None else replica.partner(rank, WORLD, k)
            for k in range(rounds)]
        assert int(a["counters"].sum()) == W * STEPS
    for k in range(rounds):
        for rank in range(WORLD):
            p = int(A[rank]["partner"][k])
            b, f = A[rank]["before"][k], A[rank]["after"][k]
            if p < 0:                           # idle end of the ladder this round
                assert np.array_equal(b, f), (k, rank)
                assert rank in (0, WORLD - 1) and k % 2 == 1
                continue
            assert int(A[p]["partner"][k]) == rank
            if rank > p:
                continue
            pb, pf = A[p]["before"][k], A[p]["after"][k]
            stay = (f == b) & (pf == pb)
            trade = (f == pb) & (pf == b)
            assert np.all(stay | trade), (k, rank, p)
            swapped_total += int((trade & ~stay).sum())
    assert ex["accepted"] == 2 * swapped_total
    assert ex["accepted"] % 2 == 0 and ex["accepted"] > 0
    assert ex["attempted"] == sum(W * sum(1 for k in range(rounds) if int(A[r]["partner"][k]) >= 0)
                                  for r in range(WORLD))

    # sampled final walkers: stored scores equal the oracle's (MFE, exact dcal/mol)
    a0 = A[0]
    active = str(a0["active"][0])
    terms = workloads.config_objective(len(str(a0["template"][0])), bppm=False)
    m = oracle.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, oracle.theo_bonus())
    sf = oracle.ScoreFunction(terms, aptamer=m, mode=str(a0["fold"][0]))
    for rank in (0, 3, WORLD - 1):
        a = A[rank]
        for s, sc in zip(a["sample_seqs"], a["sample_scores"]):
            ref, _ = sf.score(str(s), [active])
            assert abs(float(sc) - ref) <= 1e-12 * max(1.0, abs(ref)), (rank, str(s), float(sc), ref)
