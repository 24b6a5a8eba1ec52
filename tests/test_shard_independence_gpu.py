"""A walker's trajectory does not depend on the GPU count (addapt_amd/shard.py;
the reference parallelises by seed, data/20160705_production_run_favor_wt/
production_run.sh:5-8): bench.py walker-sharded over G ranks (gloo, every rank
on cuda:0) against one rank holding all G*W walkers -- every global walker id's
final sequence, score and counters bit for bit.  And config 4's 8-way shard
(N = 150, pf + bppm, 4096 walkers per rank) rehearsed on one GPU: counters
and sampled walkers against the oracle."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _bench(args, timeout=600):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, BENCH, "--no-cpu-baseline", "--no-sub-records"] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]


def _load(d, world):
    out = {}
    for r in range(world):
        z = np.load(os.path.join(d, "rank%d.npz" % r))
        for k, g in enumerate(z["gids"]):
            out[int(g)] = (str(z["seqs"][k]), z["scores"][k].tobytes(), tuple(int(x) for x in z["counters"][k]))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("fold", ["mfe", "pf"])
def test_sharded_equals_single_rank(tmp_path, fold):
    W, steps = 256, 12
    common = ["--steps", str(steps), "--warmup", "2", "--fold", fold]
    _bench(["--gpus", "2", "--dist-backend", "gloo", "--share-device", "--walkers", str(W),
            "--dump-walkers", str(tmp_path / "g2")] + common)
    _bench(["--gpus", "1", "--walkers", str(2 * W), "--dump-walkers", str(tmp_path / "g1")] + common)
    two, one = _load(tmp_path / "g2", 2), _load(tmp_path / "g1", 1)
    assert sorted(two) == sorted(one) == list(range(2 * W))
    diff = [g for g in one if one[g] != two[g]]
    assert not diff, (len(diff), diff[:5])
    moved = sum(1 for g in one if one[g][2][0] + one[g][2][1] + one[g][2][3] > 0)
    assert moved > W   # the walkers did move


@pytest.mark.gpu
def test_config4_eight_way_shard_rehearsal(tmp_path):
    """BASELINE configs[3]: 32768 walkers, 150 nt, pf + bppm, sharded 8 ways --
    here 8 ranks sharing cuda:0 over gloo, 4096 walkers each."""
    from addapt_amd import workloads
    from oracle import oracle as O
    from parity_bounds import score_bound

    W, steps = 4096, 4
    _bench(["--gpus", "8", "--dist-backend", "gloo", "--share-device", "--walkers", str(W), "--length", "150",
            "--bppm", "--steps", str(steps), "--warmup", "1", "--dump-walkers", str(tmp_path)], timeout=900)
    got = _load(tmp_path, 8)
    assert sorted(got) == list(range(8 * W))
    z0 = np.load(os.path.join(tmp_path, "rank0.npz"))
    tmpl, active = str(z0["template"][0]), str(z0["active"][0])
    assert "pf_ring_kernel" in str(z0["kernels"][0]) and "outside_ring_kernel" in str(z0["kernels"][1])
    for g in got:
        assert sum(got[g][2]) == steps + 1   # warmup + timed steps, each counted once
    terms = workloads.config_objective(150, bppm=True)
    motif = O.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, O.theo_bonus())
    sf = O.ScoreFunction(terms, aptamer=motif)
    for g in (0, W - 1, 3 * W + 17, 8 * W - 1):   # a walker of ranks 0, 3, 7
        seq, sc, _ = got[g]
        ref, tv = sf.score(seq, [active])
        score = np.frombuffer(sc, dtype=np.float64)[0]
        assert abs(score - ref) <= score_bound(tv, terms), (g, score, ref)
