"""Replica exchange across the GPUs of one node (BASELINE config 5).

One temperature rung per rank, T_r = t0 * ratio**r (SURVEY: 0.5 * 1.5**k,
k = 0..7), W walkers per rung with a fixed thermostat.  Every `interval` MC
steps, neighbouring rungs (r, r+1) with r even on even rounds and r odd on
odd rounds propose to swap the configuration (sequence, score) of walker
slot w.  For the sampled distribution pi_T(x) ~ exp(S(x) / T) (the score is
maximised, sampling.cc:77), a swap of x on rung lo and y on rung hi is
accepted with probability

    min(1, exp((S(y) - S(x)) * (1/T_lo - 1/T_hi))).

Both ranks of a pair draw the same uniforms (a generator keyed by the run
seed, the round and the pair), so the decision needs no extra message; the
one exchange per round is the pair's full configuration arrays, W*(N + 8)
bytes each way, sent point to point over RCCL (xGMI) from device buffers the
engine exports (adx_walkers_export / adx_walkers_import).  RNG streams,
counters and thermostat state stay with the walker slot.
"""
import math

import numpy as np


def ladder_temperatures(n, t0=0.5, ratio=1.5):
    return [t0 * ratio ** k for k in range(n)]


def partner(rank, world, round_idx):
    """Neighbour of `rank` in this round, or None (unpaired end of the ladder)."""
    if (rank - round_idx) % 2 == 0:
        p = rank + 1
    else:
        p = rank - 1
    return p if 0 <= p < world else None


def swap_accept(seed, round_idx, lo_rank, s_lo, s_hi, t_lo, t_hi):
    """Boolean mask over walker slots: swap slot w between rungs lo and hi."""
    s_lo = np.asarray(s_lo, dtype=np.float64)
    s_hi = np.asarray(s_hi, dtype=np.float64)
    rng = np.random.Generator(np.random.PCG64([int(seed), int(round_idx), int(lo_rank)]))
    u = rng.random(s_lo.shape[0])
    with np.errstate(invalid="ignore", over="ignore"):
        a = (s_hi - s_lo) * (1.0 / t_lo - 1.0 / t_hi)
        acc = (a >= 0) | (np.log(u) < a)
    return acc & np.isfinite(s_lo) & np.isfinite(s_hi)


def exchange_round(dist, round_idx, rank, world, temps, seqs, scores, seed=0):
    """One exchange round on this rank.  seqs (uint8 [W, N]) and scores
    (float64 [W]) are torch tensors on the communication device (CUDA for
    RCCL, CPU for gloo), updated in place.  Returns (attempted, accepted)."""
    import torch

    p = partner(rank, world, round_idx)
    if p is None:
        return 0, 0
    # RCCL moves the device buffers directly; gloo (CPU tests) needs host copies
    host = dist.get_backend() == "gloo" and seqs.is_cuda
    snd_seqs, snd_scores = (seqs.cpu(), scores.cpu()) if host else (seqs, scores)
    other_seqs = torch.empty_like(snd_seqs)
    other_scores = torch.empty_like(snd_scores)
    ops = [dist.P2POp(dist.isend, snd_seqs, p), dist.P2POp(dist.isend, snd_scores, p),
           dist.P2POp(dist.irecv, other_seqs, p), dist.P2POp(dist.irecv, other_scores, p)]
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    if host:
        other_seqs, other_scores = other_seqs.to(seqs.device), other_scores.to(seqs.device)
    lo, hi = min(rank, p), max(rank, p)
    mine = scores.cpu().numpy()
    theirs = other_scores.cpu().numpy()
    s_lo, s_hi = (mine, theirs) if rank == lo else (theirs, mine)
    acc = swap_accept(seed, round_idx, lo, s_lo, s_hi, temps[lo], temps[hi])
    if acc.any():
        idx = torch.from_numpy(np.nonzero(acc)[0]).to(seqs.device)
        seqs[idx] = other_seqs[idx]
        scores[idx] = other_scores[idx]
    return int(acc.size), int(acc.sum())


def run(engine, dist, rank, world, steps, interval, temps, seed=0, device="cuda"):
    """Advance `engine` (a native.Engine of this rank, fixed thermostat) by
    `steps` MC steps with an exchange every `interval` steps."""
    import torch

    engine.set_temperature(temps[rank])
    W, N = engine.W, engine.N
    seqs = torch.empty((W, N), dtype=torch.uint8, device=device)
    scores = torch.empty((W,), dtype=torch.float64, device=device)
    done, rnd, att, acc = 0, 0, 0, 0
    while done < steps:
        k = min(interval, steps - done)
        engine.run_steps(k)
        done += k
        if done < steps or k == interval:
            engine.export_walkers(seqs.data_ptr(), scores.data_ptr())
            a, b = exchange_round(dist, rnd, rank, world, temps, seqs, scores, seed)
            if seqs.is_cuda:
                torch.cuda.synchronize()   # the engine copies on its own stream
            engine.import_walkers(seqs.data_ptr(), scores.data_ptr())
            att += a
            acc += b
            rnd += 1
    return {"rounds": rnd, "attempted": att, "accepted": acc}
