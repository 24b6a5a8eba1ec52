"""Replica exchange across the GPUs of one node (BASELINE config 5).

One temperature rung per rank, T_r = t0 * ratio**r (SURVEY: 0.5 * 1.5**k,
k = 0..7), W walkers per rung with a fixed thermostat.  Every `interval` MC
steps, neighbouring rungs (r, r+1) with r even on even rounds and r odd on
odd rounds propose to swap the configuration (sequence, score) of walker
slot w.  For the sampled distribution pi_T(x) ~ exp(S(x) / T) (the score is
maximised, sampling.cc:77), a swap of x on rung lo and y on rung hi is
accepted with probability

    min(1, exp((S(y) - S(x)) * (1/T_lo - 1/T_hi))).

Both ranks of a pair draw the same uniforms (a generator on the device keyed
by the run seed, the round and the pair), so the decision needs no extra
message; the one exchange per round is the pair's configurations packed into
a single W*(N + 8)-byte buffer each way, sent point to point over RCCL (xGMI)
from device buffers the engine exports (adx_walkers_export /
adx_walkers_import), and the accept mask and the swap are computed on the
device.  RNG streams, counters and thermostat state stay with the walker
slot.
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


def digests(seqs, scores):
    """64-bit digest per walker slot of its configuration (sequence codes and
    the score's bit pattern), host numpy in, uint64 [W] out: a swap audit
    compares these across the ranks of a pair."""
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    sb = np.ascontiguousarray(scores, dtype=np.float64).view(np.uint8).reshape(-1, 8)
    rows = np.concatenate([seqs, sb], axis=1).astype(np.uint64)
    h = np.full(rows.shape[0], 0xCBF29CE484222325, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for c in range(rows.shape[1]):   # FNV-1a over the row's bytes
            h = (h ^ rows[:, c]) * np.uint64(0x100000001B3)
    return h


def _key(seed, round_idx, lo_rank):
    """63-bit generator key shared by both ranks of a pair."""
    k = 0x9E3779B97F4A7C15
    for x in (int(seed), int(round_idx), int(lo_rank)):
        k = ((k ^ (x & 0xFFFFFFFFFFFFFFFF)) * 0xBF58476D1CE4E5B9 + 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return k >> 1


def swap_mask(seed, round_idx, lo_rank, s_lo, s_hi, t_lo, t_hi):
    """Boolean mask over walker slots (a tensor on the scores' device): swap slot
    w between rungs lo and hi.  The uniforms come from a generator on that
    device keyed by (seed, round, lower rank), so both ranks of a pair -- on the
    same kind of device -- take the same decisions without a message and
    without a host round trip."""
    import torch

    g = torch.Generator(device=s_lo.device)
    g.manual_seed(_key(seed, round_idx, lo_rank))
    u = torch.rand(s_lo.shape, generator=g, device=s_lo.device, dtype=torch.float64)
    a = (s_hi - s_lo) * (1.0 / t_lo - 1.0 / t_hi)
    acc = (a >= 0) | (torch.log(u) < a)          # NaN a (inf - inf) compares false
    return acc & torch.isfinite(s_lo) & torch.isfinite(s_hi)


def swap_accept(seed, round_idx, lo_rank, s_lo, s_hi, t_lo, t_hi):
    """swap_mask on host arrays (CPU generator), as a numpy bool array."""
    import torch

    m = swap_mask(seed, round_idx, lo_rank, torch.as_tensor(np.asarray(s_lo, dtype=np.float64)),
                  torch.as_tensor(np.asarray(s_hi, dtype=np.float64)), t_lo, t_hi)
    return m.numpy()


def exchange_round(dist, round_idx, rank, world, temps, seqs, scores, seed=0):
    """One exchange round on this rank.  seqs (uint8 [W, N]) and scores
    (float64 [W]) are torch tensors on the communication device (CUDA for
    RCCL, CPU for gloo), updated in place.  The pair's configurations travel
    as ONE packed [W, N + 8] byte buffer each way (one send + one receive,
    device to device over RCCL/xGMI); the decision and the swap stay on the
    device.  Returns (attempted, accepted): attempted a host int (W or 0),
    accepted a 0-d tensor on the walkers' device (summed by the caller at the
    end of the run, so a round needs no host read-back)."""
    import torch

    p = partner(rank, world, round_idx)
    if p is None:
        return 0, None
    W, N = seqs.shape
    packed = torch.cat([seqs, scores.view(torch.uint8).reshape(W, 8)], dim=1).contiguous()
    # gloo (CPU tests) moves host tensors only
    host = dist.get_backend() == "gloo" and packed.is_cuda
    snd = packed.cpu() if host else packed
    rcv = torch.empty_like(snd)
    ops = [dist.P2POp(dist.isend, snd, p), dist.P2POp(dist.irecv, rcv, p)]
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    if host:
        rcv = rcv.to(seqs.device)
    other_seqs = rcv[:, :N]
    other_scores = rcv[:, N:].contiguous().view(torch.float64).reshape(W)
    lo, hi = min(rank, p), max(rank, p)
    s_lo, s_hi = (scores, other_scores) if rank == lo else (other_scores, scores)
    # both ranks of the pair draw on the same kind of device: the CPU generator
    # under gloo, the device generator under RCCL
    dev_scores = s_lo if not host else s_lo.cpu()
    acc = swap_mask(seed, round_idx, lo, dev_scores, s_hi if not host else s_hi.cpu(),
                    temps[lo], temps[hi]).to(seqs.device)
    seqs.copy_(torch.where(acc[:, None], other_seqs, seqs))
    scores.copy_(torch.where(acc, other_scores, scores))
    return int(acc.numel()), acc.sum()


def run(engine, dist, rank, world, steps, interval, temps, seed=0, device="cuda", observe=None):
    """Advance `engine` (a native.Engine of this rank, fixed thermostat) by
    `steps` MC steps with an exchange every `interval` steps.  `observe`
    (tests, audits): called per round with host copies (round, partner, seqs,
    scores before, seqs, scores after the exchange).

    Per round the host does no read-back and no synchronisation of its own:
    the accept count stays a device tensor (summed once after the last round),
    and export and import are ordered against the exchange's device work on
    torch's current stream by stream waits (adx_walkers_export_on /
    adx_walkers_import_after; the null stream, handle 0, is a stream too)."""
    import torch

    engine.set_temperature(temps[rank])
    W, N = engine.W, engine.N
    seqs = torch.empty((W, N), dtype=torch.uint8, device=device)
    scores = torch.empty((W,), dtype=torch.float64, device=device)
    done, rnd, att = 0, 0, 0
    acc = torch.zeros((), dtype=torch.int64, device=device)
    while done < steps:
        k = min(interval, steps - done)
        engine.run_steps(k)
        done += k
        if done < steps or k == interval:
            stream = torch.cuda.current_stream(seqs.device).cuda_stream if seqs.is_cuda else None
            engine.export_walkers(seqs.data_ptr(), scores.data_ptr(), on_stream=stream)
            before = (seqs.cpu().numpy().copy(), scores.cpu().numpy().copy()) if observe else None
            a, b = exchange_round(dist, rnd, rank, world, temps, seqs, scores, seed)
            if observe:
                observe(rnd, partner(rank, world, rnd), before[0], before[1],
                        seqs.cpu().numpy().copy(), scores.cpu().numpy().copy())
            engine.import_walkers(seqs.data_ptr(), scores.data_ptr(), after_stream=stream)
            att += a
            if b is not None:
                acc += b
            rnd += 1
    return {"rounds": rnd, "attempted": att, "accepted": int(acc)}
