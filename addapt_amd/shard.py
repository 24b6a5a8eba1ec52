"""Walker sharding across the GPUs of one node.

Walkers are independent (the reference parallelises by running one process
per seed), so rank r of a world of size G owns the global walker ids
[r*W, (r+1)*W): its template copies are re-randomised from mt19937(1000+gid)
and its MC streams are seeded with gid, so a walker's trajectory does not
depend on G.  There is no collective on the data path; the only collectives
are the barrier / max-over-ranks around the timed region and an optional
final reduction of the outcome counters.
"""


def walker_ids(rank, world, walkers_per_rank):
    if not (0 <= rank < world):
        raise ValueError("rank %d outside world %d" % (rank, world))
    return list(range(rank * walkers_per_rank, (rank + 1) * walkers_per_rank))


def max_over_ranks(value, dist=None, device=None):
    """Max of a float over all ranks (the timed region's wall clock)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, dist=None, device=None):
    """Element-wise sum of an int64 vector (outcome counters) over all ranks."""
    vals = [int(v) for v in values]
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return vals
    import torch

    t = torch.tensor(vals, dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]


def gather_over_ranks(value, dist=None, device=None):
    """A float from every rank, in rank order (per-rank step times)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [float(value)]
    import torch

    t = torch.zeros(dist.get_world_size(), dtype=torch.float64, device=device)
    t[dist.get_rank()] = float(value)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.tolist()]


def dist_record(dist, per_rank_ms, max_ms):
    """What the multi-rank timing ran on: the collective backend torch.distributed
    reports (on ROCm "nccl" is RCCL), the world size it reports, each rank's
    ms per step and the max over ranks the value is computed from."""
    on = dist is not None and dist.is_initialized()
    backend = dist.get_backend() if on else None
    return {"backend": backend,
            "library": ("RCCL" if backend == "nccl" else backend) if on else None,
            "world_size": dist.get_world_size() if on else 1,
            "per_rank_ms_per_step": [float(x) for x in per_rank_ms],
            "max_ms_per_step": float(max_ms)}
