"""The unpaired part of the multiloop table qm as a column recursion.

pf_cells.hip / pf_ring.hip (M and Q roles) compute the unpaired part of
qm(i, j) (oracle/fold.c orc_pf_energy's fML recursion, ViennaRNA's
vrna_exp_E_ml_fast unpaired-prefix term) not as the sum

    U(i, j) = sum_{t = 0 .. min(T, up_i)} pw^t qm1(i + t, j),   T = j - i - 4

but as U(i, j) = qm1(i, j) + [up_i >= 1] pw U(i + 1, j), which holds because
the hard-constraint arrays give up_i = up_{i+1} + 1 whenever up_i >= 1
(adx_api.cpp, the unpaired-run lengths).  This checks the identity in float64
on random constraint masks and tables (CPU, no GPU)."""
import numpy as np
import pytest


def run_lengths(unp):
    """up[i] = number of consecutive positions i, i+1, ... that may stay unpaired."""
    n = len(unp)
    up = np.zeros(n + 1, dtype=np.int64)
    for i in range(n - 1, -1, -1):
        up[i] = up[i + 1] + 1 if unp[i] else 0
    return up[:n]


@pytest.mark.parametrize("seed", range(6))
def test_unpaired_part_recursion_equals_the_sum(seed):
    rng = np.random.default_rng(seed)
    N = 60
    unp = rng.random(N + 2) > (0.0 if seed == 0 else 0.25)   # seed 0: unconstrained
    up = run_lengths(unp)
    pw = float(rng.uniform(0.5, 1.5))
    qm1 = rng.random((N + 2, N + 2))
    for j in range(5, N + 1):
        U = {}
        for i in range(j - 4, 0, -1):        # span s = j - i from 4 upwards (i downwards)
            T = j - i - 4
            direct = sum(pw ** t * qm1[i + t, j] for t in range(0, min(T, up[i]) + 1))
            rec = qm1[i, j] + (pw * U[i + 1] if (T >= 1 and up[i] >= 1) else 0.0)
            U[i] = rec
            assert rec == pytest.approx(direct, rel=1e-12, abs=1e-300)
