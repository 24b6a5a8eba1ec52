"""Multi-process (gloo, world size 2, CPU) check of the walker sharding used
by bench.py --gpus N: disjoint walker ids covering [0, G*W), per-walker
initial sequences independent of G, max-over-ranks timing and counter sums."""
import os
import socket
import tempfile

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from addapt_amd import shard, workloads


def _rendezvous():
    d = tempfile.mkdtemp(prefix="adx_gloo_")
    return os.path.join(d, "rdzv")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, q):
    # file rendezvous: no port to race for when tests run in parallel
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        ids = shard.walker_ids(rank, world, W)
        tmpl, active = workloads.synthetic(60)
        seqs = workloads.walker_sequences(tmpl, [active], W, seed_base=1000 + ids[0])
        t = shard.max_over_ranks(1.5 + rank, dist)
        c = shard.sum_over_ranks([rank + 1, 2, 3, 4 * rank], dist)
        q.put((rank, ids, seqs, t, c))
    finally:
        dist.destroy_process_group()


def test_sharding_two_ranks():
    world, W = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    all_ids = res[0][1] + res[1][1]
    assert sorted(all_ids) == list(range(world * W))
    # same global walker -> same initial sequence as a single-process run of G*W walkers
    tmpl, active = workloads.synthetic(60)
    single = workloads.walker_sequences(tmpl, [active], world * W, seed_base=1000)
    assert res[0][2] + res[1][2] == single
    for r in range(world):
        assert res[r][3] == pytest.approx(2.5)
        assert res[r][4] == [3, 4, 6, 4]


def test_walker_ids_bounds():
    assert shard.walker_ids(1, 4, 5) == [5, 6, 7, 8, 9]
    with pytest.raises(ValueError):
        shard.walker_ids(4, 4, 5)
