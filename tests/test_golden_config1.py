"""The config-1 golden trajectory (tests/golden/config1_rhf6_seed0.json, made
by tests/golden/gen_config1.py) is the oracle's: its first steps replay
exactly, and its per-step records are consistent."""
import json
import os

from addapt_amd import workloads

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_golden_prefix_replays(oracle):
    with open(os.path.join(ROOT, "tests", "golden", "config1_rhf6_seed0.json")) as f:
        g = json.load(f)
    assert g["steps"] == 10000 and len(g["pos"]) == len(g["base"]) == len(g["outcome"]) == 10000
    assert sum(g["counters"]) == 10000
    motif = oracle.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, oracle.theo_bonus())
    sf = oracle.ScoreFunction(workloads.default_objective(), aptamer=motif)
    th = oracle.thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300)
    n = 120
    r = oracle.mc_run(sf, workloads.RHF6_SEQ, [workloads.RHF6_ACTIVE], th, 0, n)
    assert r["pos"] == g["pos"][:n]
    assert r["base"] == g["base"][:n]
    assert "".join(str(o) for o in r["outcome"]) == g["outcome"][:n]
    # unchanged proposals carry no Metropolis margin, every other step does
    assert all((m is None) == (o == "2") for m, o in zip(g["margin"], g["outcome"]))
