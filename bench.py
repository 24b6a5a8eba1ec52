#!/usr/bin/env python3
"""Benchmark: MC steps/s (fold + score + accept), 100-nt sgRNA, 4096 walkers per GPU.

A "step" is one MonteCarlo::apply iteration (sampling.cc:55-99) for every
walker of the batch: thermostat, mutation move, and -- when the sequence
changed -- the default objective's 4 folds (apo/holo x unconstrained/"active",
scoring.cc:145-146, 58, 65) and the Metropolis test.  ACCEPT_UNCHANGED steps
count, as in the reference counters.

--fold mfe (default): BASELINE.json configs[1], the configuration the metric is
quoted on -- "4096 independent walkers, 100-nt, MFE-fold score only": the 4
folds are minimum free energies (ADX_FOLD_MFE).
--fold pf: the same objective over McCaskill partition functions (vrna_pf, the
reference's own scoring path; config 3 without the bppm term).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--walkers 4096] [--length 100] [--fold mfe|pf]

N > 1: one rank per GPU.  Under torch.distributed.run (WORLD_SIZE set) each
process is one rank; a plain `python bench.py --gpus N` starts that launcher
itself as a child process before anything touches the GPU (N larger than the
visible GPU count is refused with exit status 2).  Walkers are sharded (weak
scaling, global walker id = rank * W + w), no collective on the data path; a
barrier + max-over-ranks brackets the timed region.  `--dry-run` replaces the
engine by a host sleep over gloo (CPU-only test of the launch path).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MC steps/sec (fold+score+accept), 100-nt sgRNA, 4096 walkers, 1/8 GPU"
HBM_PEAK_GBPS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300,
                    help="timed steps (default: one annealing cycle of the 5 -> 0 in 300 schedule)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--walkers", type=int, default=4096)
    ap.add_argument("--length", type=int, default=100)
    ap.add_argument("--fold", choices=("mfe", "pf"), default="mfe",
                    help="mfe = BASELINE configs[1] (default); pf = partition-function objective")
    ap.add_argument("--bppm", action="store_true",
                    help="configs 3/4: add apo/holo base-pair probability terms (outside pass; --fold pf)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="approximate budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--replica-interval", type=int, default=0,
                    help="BASELINE config 5: one temperature rung per rank (0.5*1.5^r), RCCL swap of "
                         "walker configurations between neighbouring rungs every K steps (N > 1 only)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (tools/pmc_traffic.py) of this workload, fills roofline.traffic "
                         "(default profiles/traffic_latest_<fold>.json)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo ranks, a host sleep per step (tests the --gpus N launch path)")
    return ap.parse_args()


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(a):
    """`bench.py --gpus N` without a launcher: start torch.distributed.run as a
    child (nothing here has touched the GPU: device_count() does not initialise
    it) and return its exit status."""
    import subprocess

    if not a.dry_run:
        import torch

        visible = torch.cuda.device_count()
        if a.gpus > visible:
            print("bench.py: --gpus %d but %d GPU(s) visible" % (a.gpus, visible), file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def host_cores():
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota
    (a GPU box shares its host; nproc shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"usable": min(n, quota) if quota else n, "nproc": os.cpu_count(), "affinity": n,
            "cgroup_quota": quota, "cpu_model": model}


def cpu_baseline(tmpl, active, walker_seqs, budget_s, fold, terms):
    """Oracle MC (the C++-equivalent CPU restatement, 'port') on the host cores."""
    from oracle import oracle as O
    from addapt_amd import workloads

    hc = host_cores()
    threads = hc["usable"]
    motif = O.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, O.theo_bonus())
    sf = O.ScoreFunction(terms, aptamer=motif, mode=fold)
    th = O.thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300)
    # probe: 1 walker x 4 steps on one thread to size the sample
    t_probe, _ = O.mc_run_batch(sf, walker_seqs[:1], [active], th, [0], 4, 1)
    per_step = max(t_probe / 4.0, 1e-4)
    steps = 8
    walkers = max(threads, int(budget_s * threads / (per_step * steps)))
    walkers = min(walkers, len(walker_seqs))
    walkers = max(threads, (walkers // threads) * threads)
    seqs = walker_seqs[:walkers]
    t, counters = O.mc_run_batch(sf, seqs, [active], th, list(range(walkers)), steps, threads)
    total = walkers * steps
    return {"value": total / t, "unit": "MC steps/s", "cores": threads, "kind": "port",
            "sample": "%d walkers x %d steps of the same workload (oracle/ C restatement of "
                      "MonteCarlo::apply + %s, 1 walker per OpenMP thread), %.1f s"
                      % (walkers, steps, "ViennaRNA-style pf, FP64" if fold == "pf"
                         else "integer-dcal MFE", t),
            "per_core": total / t / threads,
            "nproc": hc["nproc"], "cgroup_quota": hc["cgroup_quota"], "cpu_model": hc["cpu_model"],
            "reference_2016_per_core": 14.4}


def pf_kernel_label(bppm, length=100):
    """The PF kernels of one step's score window (kernels.hip launch_score_m / launch_steps):
    pf_cells_kernel up to N = 100 (pf_cells.hip PX_NMAX), outside_cells_kernel up to
    N = 112 (outside_cells.hip OX_NMAX), the general kernels beyond (their LDS)."""
    inside = ("score_kernel<SumProd> (lanes = terms)"
              if os.environ.get("ADX_PF_KERNEL") == "rows" or length > 100
              else "pf_cells_kernel (lanes = cells)")
    if bppm:
        return inside + " + %s + combine_kernel (one event window per step)" % outside_kernel(length)
    return inside + " + combine_kernel"


def outside_kernel(length):
    return "outside_cells_kernel" if length <= 112 else "bppm_kernel<512, GOUT>"


def mfe_kernel_label():
    """The MFE fold kernel the engine launches (kernels.hip mfe_kernel_choice)."""
    k = os.environ.get("ADX_MFE_KERNEL", "cells")
    return {"rows": "score_kernel<MinPlus16> (lanes = terms)"}.get(
        k, "mfe_cells_kernel (lanes = cells, 2 folds per cell)") + " + FP32 MinPlus fallback launch"


def dry_run(a, rank, world):
    """CPU-only rehearsal of the rank launch: gloo barrier, a sleep per step, max over ranks."""
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    from addapt_amd import shard

    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.001 * a.steps * (1 + rank))
    if world > 1:
        dist.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist if world > 1 else None)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": a.walkers * a.steps * world / elapsed,
                          "unit": "MC steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": elapsed / a.steps * 1e3, "dry_run": True,
                          "ranks": shard.walker_ids(rank, world, a.walkers)[:1]}))
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (a.gpus, world), file=sys.stderr)
        sys.exit(2)
    if a.dry_run:
        return dry_run(a, rank, world)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_

        torch.cuda.set_device(local_rank)
        dist_.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = dist_

    from addapt_amd import native, roofline, shard, workloads

    if a.bppm:
        a.fold = "pf"
    tmpl, active = workloads.synthetic(a.length)
    terms = workloads.config_objective(a.length, bppm=a.bppm)
    apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
    replica_mode = a.replica_interval > 0 and world > 1
    if replica_mode:
        from addapt_amd import replica

        temps = replica.ladder_temperatures(world)
        th = native.make_thermostat("fixed", t=temps[rank])
    else:
        th = native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300)
    eng = native.Engine(tmpl, [active], terms, aptamer=apt, thermostat=th, device=local_rank,
                        fold_mode=a.fold)
    W = a.walkers
    gids = shard.walker_ids(rank, world, W)
    seqs = workloads.walker_sequences(tmpl, [active], W, seed_base=1000 + gids[0])
    eng.walkers_init(gids, seqs)

    def barrier():
        if dist is not None:
            import torch

            dist.barrier()
            torch.cuda.synchronize()

    if a.warmup > 0:
        eng.run_steps(a.warmup)
    _, _, c0 = eng.download()
    barrier()
    t0 = time.perf_counter()
    if replica_mode:
        rx = replica.run(eng, dist, rank, world, a.steps, a.replica_interval, temps, seed=0,
                         device="cuda")
    else:
        eng.run_steps(a.steps)
    barrier()
    t1 = time.perf_counter()
    kernel_ms = eng.last_kernel_ms()            # whole timed run_steps (3 kernels per step)
    score_ms, launches = eng.last_score_kernel_ms()   # the step's score window, per launch
    inside_ms, outside_ms = eng.last_kernel_split_ms()   # the same window split per kernel
    _, _, c1 = eng.download()
    elapsed = shard.max_over_ranks(t1 - t0, dist, device="cuda" if dist is not None else None)
    steps_total = W * a.steps * world
    value = steps_total / elapsed

    # algorithmic FLOPs of the launch: scored steps x sum over the PF variants
    dc = c1 - c0
    scored = int(dc[:, 0].sum() + dc[:, 1].sum() + dc[:, 3].sum())
    outcomes = shard.sum_over_ranks(dc.sum(axis=0), dist, device="cuda" if dist is not None else None)
    sample = [tmpl] + seqs[:7]
    work = roofline.pf_flops if a.fold == "pf" else roofline.mfe_ops
    f_free = sum(work(s, None) for s in sample) / len(sample)
    f_act = sum(work(s, active) for s in sample) / len(sample)
    flop_inside = 2 * f_free + 2 * f_act           # apo/holo x free/active
    flop_per_scored = flop_inside
    f_out = 0.0
    if a.bppm:   # outside passes of the apo and holo unconstrained folds (on the stored inside tables)
        f_out = 2 * sum(roofline.outside_flops(s, None) for s in sample) / len(sample)
        flop_per_scored += f_out
    scored_pl = scored / max(1, a.steps)                             # scored walkers per launch
    launch_flops = scored_pl * flop_per_scored                      # per score window (one per step)
    # the dominant kernel's own time: the outside pass with --bppm, else the window
    # (inside folds + the score combine)
    kern_ms, kern_flops = (outside_ms, scored_pl * f_out) if a.bppm else (score_ms, launch_flops)
    achieved_tflops = kern_flops / (kern_ms * 1e-3) / 1e12 if kern_ms > 0 else None
    # incremental-fold state written per scored walker (kernels.hip Inc): 2 fold
    # groups x value arrays (MFE: one packed apo/holo array; PF: two) x
    # (3 cell tables + q5) x 4 B
    cells = (a.length - 4) * (a.length - 3) // 2
    state_bytes = 2 * (1 if a.fold == "mfe" else 2) * (3 * cells + a.length + 2) * 4
    traffic, traffic_src = None, None
    if a.traffic_json is None:
        # the PMC summary of this exact workload (fold, pair terms, length), else null
        a.traffic_json = os.path.join(ROOT, "profiles", "traffic_latest_%s%s%s.json" % (
            a.fold, "_bppm" if a.bppm else "", "" if a.length == 100 else "_n%d" % a.length))
    if a.traffic_json and os.path.exists(a.traffic_json):
        with open(a.traffic_json) as f:
            tj = json.load(f)
        traffic = tj.get("bytes_per_launch")
        if a.bppm:   # the dominant kernel's own bytes (the summary holds every kernel of the window)
            own = [k["bytes"] for name, k in tj.get("kernels", {}).items() if outside_kernel(a.length).split("<")[0] in name]
            traffic = own[0] if own else None
        traffic_src = os.path.relpath(a.traffic_json, ROOT)
    peak, peak_note = roofline.valu_peak(a.fold)
    roof = {
        "bound": "valu",
        "achieved": achieved_tflops,
        "peak": peak,
        "unit": "TFLOP/s" if a.fold == "pf" else "Top/s",
        "frac": (achieved_tflops / peak) if achieved_tflops else None,
        "traffic": traffic,
        "compute_unit": peak_note,
        "kernel": (outside_kernel(a.length) + " (events around its launch; the window also holds "
                   + pf_kernel_label(False, a.length) + ")") if a.bppm
                  else mfe_kernel_label() if a.fold == "mfe" else pf_kernel_label(False, a.length),
        "traffic_source": traffic_src,
        "kernel_ms_per_launch": kern_ms,
        "window_ms_per_launch": score_ms,
        "inside_ms_per_launch": inside_ms,
        "outside_ms_per_launch": outside_ms if a.bppm else None,
        "inside_frac": ((scored_pl * flop_inside / (inside_ms * 1e-3) / 1e12) / peak
                        if a.bppm and inside_ms > 0 else None),
        "launches": launches,
        "all_kernels_ms_per_step": kernel_ms / a.steps,
        "flop_per_scored_step": flop_per_scored,
        "flop_per_launch": launch_flops,
        "scored_walkers_per_launch": scored / max(1, a.steps),
        # HBM bytes of one launch by design: each scored walker reads its proposal
        # (N B), writes its score (8 B), and writes its fold tables for the next
        # incremental refold (read back for the unchanged cells, <= the same again)
        "algorithmic_bytes_per_launch": (scored / max(1, a.steps)) * (a.length + 8 + 2 * state_bytes),
        "state_bytes_per_scored_walker": state_bytes,
        "hbm_peak_GBps": HBM_PEAK_GBPS,
    }
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "MC steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        # MFE: integer dcal/mol, apo|holo as two int16 halves of one 32-bit word
        # (v_pk_add_i16 / v_pk_min_i16); PF: fp32 Boltzmann factors
        "dtype": "i16x2" if a.fold == "mfe" else "fp32",
        "data": "synthetic",
        "config": {
            "workload": "%s: default objective (apo: not active, holo: active; THEO aptamer "
                        "0.32 uM)%s, 4 %s%s per scored step, synthetic %d-nt sgRNA template "
                        "(SURVEY.md 8d), %d walkers per GPU, annealing 5 to 0 in 300 steps"
                        % ("BASELINE configs[1] (MFE-fold score only)" if a.fold == "mfe"
                           else ("BASELINE config 3/4 (pf + bppm score)" if a.bppm
                                 else "partition-function score (config 3 without bppm)"),
                           " + apo 'not pair(0,N-1)' / holo 'pair(0,N-1)'" if a.bppm else "",
                           "minimum-free-energy folds" if a.fold == "mfe" else "McCaskill inside PFs",
                           " + 2 inside/outside (bppm) passes" if a.bppm else "",
                           a.length, W),
            "fold": a.fold,
            "bppm": a.bppm,
            "walkers_per_gpu": W,
            "global_walkers": W * world,
            "length": a.length,
            "parallelism": ("replica exchange x%d (RCCL neighbour swap every %d steps)"
                            % (world, a.replica_interval)) if replica_mode
            else "walker-sharded x%d (no data-path collective)" % world,
            "outcomes": {k: int(v) for k, v in zip(native.OUTCOMES, outcomes)},
        },
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(tmpl, active, seqs, a.cpu_seconds, a.fold, terms)
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
