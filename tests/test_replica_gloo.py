"""Replica-exchange rounds (addapt_amd/replica.py) across 2 and 3 CPU ranks
(gloo): both ranks of a pair take the same decisions, configurations are
conserved, and the acceptance rule is the detailed-balance one."""
import math
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from addapt_amd import replica


def _rendezvous():
    d = tempfile.mkdtemp(prefix="adx_gloo_")
    return os.path.join(d, "rdzv")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, N, rounds, q):
    # file rendezvous: no port to race for when tests run in parallel
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(1000 + rank)
        seqs = torch.randint(1, 5, (W, N), dtype=torch.uint8, generator=g)
        seqs[:, 0] = rank        # tag: which rung the configuration started on
        scores = -torch.rand(W, dtype=torch.float64, generator=g) * 5.0 - rank
        start = (seqs.clone(), scores.clone())
        temps = replica.ladder_temperatures(world)
        stats = []
        for r in range(rounds):
            a, b = replica.exchange_round(dist, r, rank, world, temps, seqs, scores, seed=7)
            stats.append((a, 0 if b is None else int(b)))
        # numpy copies travel by value (torch tensors go through shared memory that
        # can vanish when this process exits before the parent reads the queue)
        q.put((rank, (start[0].numpy().copy(), start[1].numpy().copy()),
               (seqs.numpy().copy(), scores.numpy().copy()), stats))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_rounds_conserve_configurations(world):
    W, N, rounds = 64, 12, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, N, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=180)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every (sequence, score) configuration survives exactly once per slot
    for w in range(W):
        before = sorted((bytes(res[r][1][0][w].tolist()), float(res[r][1][1][w])) for r in range(world))
        after = sorted((bytes(res[r][2][0][w].tolist()), float(res[r][2][1][w])) for r in range(world))
        assert before == after
    acc = sum(s[1] for r in range(world) for s in res[r][3])
    assert acc > 0


def test_swap_rule():
    t_lo, t_hi = 0.5, 0.75
    # the higher-scoring configuration always moves down to the colder rung
    assert replica.swap_accept(1, 0, 0, [-5.0], [-1.0], t_lo, t_hi).all()
    # and the reverse move is accepted with probability exp((S_hi - S_lo)(1/T_lo - 1/T_hi))
    n = 20000
    s_lo, s_hi = np.full(n, -1.0), np.full(n, -2.0)
    frac = replica.swap_accept(3, 1, 0, s_lo, s_hi, t_lo, t_hi).mean()
    assert abs(frac - math.exp(-1.0 * (1 / t_lo - 1 / t_hi))) < 0.02
    # same key -> same decisions on both ranks of the pair
    a = replica.swap_accept(9, 4, 2, s_lo[:50], s_hi[:50], t_lo, t_hi)
    b = replica.swap_accept(9, 4, 2, s_lo[:50], s_hi[:50], t_lo, t_hi)
    assert (a == b).all()
    assert not replica.swap_accept(0, 0, 0, [float("nan")], [0.0], t_lo, t_hi).any()


def test_pairing():
    assert [replica.partner(r, 4, 0) for r in range(4)] == [1, 0, 3, 2]
    assert [replica.partner(r, 4, 1) for r in range(4)] == [None, 2, 1, None]
    assert replica.ladder_temperatures(3) == [0.5, 0.75, 1.125]


class _HostEngine:
    """CPU stand-in for native.Engine's replica-exchange surface (export /
    import through raw pointers, set_temperature, run_steps): lets
    replica.run itself execute over gloo ranks without a GPU."""

    def __init__(self, rank, W, N):
        g = torch.Generator().manual_seed(500 + rank)
        self.W, self.N = W, N
        self.seqs = torch.randint(1, 5, (W, N), dtype=torch.uint8, generator=g)
        self.seqs[:, 0] = rank   # the rung the configuration started on
        self.scores = -torch.rand(W, dtype=torch.float64, generator=g) * 4.0 - 0.5 * rank
        self.temps, self.steps = [], 0

    def set_temperature(self, t):
        self.temps.append(t)

    def run_steps(self, k):
        self.steps += k

    def export_walkers(self, seqs_ptr, scores_ptr, on_stream=None):
        import ctypes

        ctypes.memmove(seqs_ptr, self.seqs.data_ptr(), self.W * self.N)
        ctypes.memmove(scores_ptr, self.scores.data_ptr(), self.W * 8)

    def import_walkers(self, seqs_ptr, scores_ptr, after_stream=None):
        import ctypes

        ctypes.memmove(self.seqs.data_ptr(), seqs_ptr, self.W * self.N)
        ctypes.memmove(self.scores.data_ptr(), scores_ptr, self.W * 8)


def _ladder_worker(rank, world, port, W, N, steps, interval, q):
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        eng = _HostEngine(rank, W, N)
        start = (eng.seqs.numpy().copy(), eng.scores.numpy().copy())
        temps = replica.ladder_temperatures(world)
        rounds = []

        def observe(rnd, _p, s0, c0, s1, c1):
            rounds.append((rnd, int((c0 != c1).sum())))

        stats = replica.run(eng, dist, rank, world, steps, interval, temps, seed=11, device="cpu",
                            observe=observe)
        q.put((rank, start, (eng.seqs.numpy().copy(), eng.scores.numpy().copy()), stats, rounds,
               eng.temps, eng.steps))
    finally:
        dist.destroy_process_group()


def test_ladder_world8_replica_run():
    """config 5's 8-rung ladder (gloo, world size 8) through replica.run: the
    pairing alternates by round parity, the unpaired ends (rank 0 on odd rounds,
    rank 7 on odd rounds) never change, every configuration survives exactly
    once per walker slot, and both ranks of a pair count the same swaps."""
    world, W, N, steps, interval = 8, 48, 10, 20, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous()
    procs = [ctx.Process(target=_ladder_worker, args=(r, world, port, W, N, steps, interval, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=240)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    temps = replica.ladder_temperatures(world)
    for r in range(world):
        _, start, end, stats, rounds, set_t, nsteps = res[r]
        assert set_t == [temps[r]] and nsteps == steps
        assert stats["rounds"] == steps // interval == 5
        for rnd, changed in rounds:
            if replica.partner(r, world, rnd) is None:
                assert changed == 0, (r, rnd)   # unpaired end: untouched
        # attempted: W per round in which this rank had a partner
        paired = sum(1 for rnd in range(stats["rounds"]) if replica.partner(r, world, rnd) is not None)
        assert stats["attempted"] == W * paired
    for rnd in range(5):   # partners agree on the number of swaps
        for r in range(world):
            p = replica.partner(r, world, rnd)
            if p is not None:
                assert p != r and replica.partner(p, world, rnd) == r
                assert abs(p - r) == 1 and (min(p, r) - rnd) % 2 == 0
    assert [replica.partner(0, world, k) for k in range(2)] == [1, None]
    assert [replica.partner(7, world, k) for k in range(2)] == [6, None]
    for w in range(W):
        before = sorted((bytes(res[r][1][0][w].tolist()), float(res[r][1][1][w])) for r in range(world))
        after = sorted((bytes(res[r][2][0][w].tolist()), float(res[r][2][1][w])) for r in range(world))
        assert before == after
    acc = [res[r][3]["accepted"] for r in range(world)]
    assert sum(acc) > 0
    # configurations moved more than one rung over the 5 rounds for some slot
    moved = max(abs(int(res[r][2][0][w, 0]) - r) for r in range(world) for w in range(W))
    assert moved >= 2
