#!/usr/bin/env python3
"""Golden trajectory of BASELINE config 1 (apps/addapt.cc:58-103): the addapt
CLI run on the reference's rhf(6) device (test_scoring.cc:57-58), default
objective (apo: not active, holo: active, THEO aptamer 0.32 uM), thermostat
"5 to 0 in 300 steps", seed 0, 10 000 steps -- restated by the oracle's
MonteCarlo::apply (oracle/mc.c, FP64 partition functions).

Per step: the mutated position and base of the move, the outcome and the
Metropolis margin log(crit) - log(u) (crit = exp(diff / T), sampling.cc:76-89),
so a GPU test can tell a real divergence from a near tie that the FP32 fold
may legitimately decide the other way.  Writes config1_rhf6_seed0.json here.

    python tests/golden/gen_config1.py [steps]      (~3 min for 10 000 steps)
"""
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from addapt_amd import workloads  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    motif = O.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, O.theo_bonus())
    sf = O.ScoreFunction(workloads.default_objective(), aptamer=motif)
    th = O.thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300)
    r = O.mc_run(sf, workloads.RHF6_SEQ, [workloads.RHF6_ACTIVE], th, 0, steps)
    assert r["rc"] == 0, r["rc"]
    margin = []
    for s in range(steps):
        if r["outcome"][s] == 2:          # ACCEPT_UNCHANGED: no Metropolis draw
            margin.append(None)
            continue
        diff = r["proposed_score"][s] - r["current_score"][s]
        T, u = r["temperature"][s], r["random_threshold"][s]
        if T == 0.0 or not math.isfinite(diff):
            margin.append(None if diff == 0.0 or not math.isfinite(diff) else
                          (math.inf if diff > 0 else -math.inf))
            continue
        margin.append(round(diff / T - math.log(u), 6))
    out = {
        "source": "tests/golden/gen_config1.py (oracle/mc.c orc_mc_run, FP64)",
        "device": workloads.RHF6_SEQ, "active": workloads.RHF6_ACTIVE,
        "thermostat": "5 to 0 in 300 steps", "seed": 0, "steps": steps,
        "pos": r["pos"], "base": r["base"], "outcome": "".join(str(o) for o in r["outcome"]),
        "margin": margin, "final_seq": r["seq"], "final_score": r["score"],
        "counters": r["counters"],
    }
    with open(os.path.join(HERE, "config1_rhf6_seed0.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote %d steps, counters %s" % (steps, r["counters"]))


if __name__ == "__main__":
    main()
