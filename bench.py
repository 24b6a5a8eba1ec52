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

The default (MFE) line also carries `sub_records` measured in the same run:
"pf" (the reference's own vrna_pf scoring path), "config3" (pf + bppm, N = 100)
and "config4" (pf + bppm, N = 150, one GPU's shard), each with value,
ms_per_step, the roofline of its dominant kernel (named from the engine's own
dispatch, adx_last_kernel_names) and, for pf / config3, a CPU baseline.

N > 1: one rank per GPU.  Under torch.distributed.run (WORLD_SIZE set) each
process is one rank; a plain `python bench.py --gpus N` starts that launcher
itself as a child process before anything touches the GPU (N larger than the
visible GPU count, read from the kfd topology, is refused with exit status 2).
Walkers are sharded (weak scaling, global walker id = rank * W + w), no
collective on the data path; a barrier + max-over-ranks brackets the timed
region.  `--dist-backend gloo --share-device` rehearses the N-rank paths
(sharding, replica exchange) on one GPU; `--dry-run` replaces the engine by a
host sleep over gloo (CPU-only test of the launch path).
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
    ap.add_argument("--replica-audit", default=None, metavar="DIR",
                    help="replica exchange: each rank writes DIR/rank<r>.npz with per-round configuration "
                         "digests before/after the swap and sampled final walkers (tests; off the timed path "
                         "only in the sense that it adds host copies per round)")
    ap.add_argument("--dump-walkers", default=None, metavar="DIR",
                    help="each rank writes DIR/rank<r>.npz with its global walker ids and final sequences, "
                         "scores and counters (after the timed region; tests of G-independence)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (tools/pmc_traffic.py) of this workload, fills roofline.traffic "
                         "(default profiles/traffic_latest_<fold>.json)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo ranks, a host sleep per step (tests the --gpus N launch path)")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="N > 1: nccl (= RCCL, one GPU per rank) or gloo (rehearsal on host tensors)")
    ap.add_argument("--share-device", action="store_true",
                    help="N > 1 rehearsal on one GPU: every rank runs its engine on device 0 "
                         "(use with --dist-backend gloo)")
    ap.add_argument("--no-sub-records", action="store_true",
                    help="skip the PF / config 3 / config 4 sub-records of the default (MFE) run")
    ap.add_argument("--sub-steps-c4", type=int, default=60,
                    help="timed steps of the config-4 sub-record (N = 150)")
    return ap.parse_args()


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(a):
    """`bench.py --gpus N` without a launcher: start torch.distributed.run as a
    child and return its exit status.  Nothing here touches the GPU: the
    visible GPUs are counted from the kfd topology (gpu_count); each rank
    checks its own device again after the launch."""
    import subprocess

    if not a.dry_run and not a.share_device:
        visible = gpu_count()
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
    mine = time.perf_counter() - t0
    d = dist if world > 1 else None
    elapsed = shard.max_over_ranks(mine, d)
    per_rank = shard.gather_over_ranks(mine / max(1, a.steps) * 1e3, d)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": a.walkers * a.steps * world / elapsed,
                          "unit": "MC steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": elapsed / a.steps * 1e3, "dry_run": True,
                          "dist": shard.dist_record(d, per_rank, elapsed / max(1, a.steps) * 1e3),
                          "ranks": shard.walker_ids(rank, world, a.walkers)[:1]}))
    if world > 1:
        dist.destroy_process_group()


def _traffic(a_traffic_json, fold, bppm, length, kernel_name):
    """PMC bytes per launch of the dominant kernel from the summary of this exact
    workload (tools/pmc_traffic.py), or (None, None)."""
    path = a_traffic_json or os.path.join(ROOT, "profiles", "traffic_latest_%s%s%s.json" % (
        fold, "_bppm" if bppm else "", "" if length == 100 else "_n%d" % length))
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        tj = json.load(f)
    traffic = tj.get("bytes_per_launch")
    if bppm:   # that kernel's own bytes (the summary holds every kernel of the window)
        key = kernel_name.split("<")[0].split(" ")[0]
        own = [k["bytes"] for name, k in tj.get("kernels", {}).items() if key and key in name]
        traffic = own[0] if own else None
    return traffic, os.path.relpath(path, ROOT)


def executed_inside_work(eng, cur_seqs, tmpl, active, fold, sample=32):
    """Work the incremental inside refolds actually execute per scored step.

    One traced step after the timed region (its state is not reused): for up
    to `sample` scored proposals, the proposal's sequence is the walker's
    current one with the move applied, the refolded band is the hull of the
    positions whose base changed (kernels.hip step_tail_kernel -> chg), and the
    band's terms are counted per cell (roofline.cell_terms / band_terms) for
    the 4 folds (apo / holo x unconstrained / active).  Returns (mean executed
    work per scored step, mean full-fold work of the same proposals, proposals
    sampled)."""
    from addapt_amd import roofline

    tr = eng.run_steps(1, trace=True)
    W = len(cur_seqs)
    partner = {}
    stk = []
    for i, c in enumerate(active):
        if c == "(":
            stk.append(i)
        elif c == ")":
            a = stk.pop()
            partner[a], partner[i] = i, a
    comp = {"A": "U", "U": "A", "G": "C", "C": "G"}
    ex_sum = full_sum = 0.0
    n = 0
    mul = 3 if fold == "pf" else 2
    for w in range(W):
        if n >= sample:
            break
        if int(tr["outcome"][0, w]) == 2:   # ACCEPT_UNCHANGED: not scored
            continue
        cur = cur_seqs[w].upper()
        p, b = int(tr["position"][0, w]), tr["base"][w]
        prop = list(cur)
        prop[p] = b
        if p in partner:
            prop[partner[p]] = comp[b]
        changed = [k for k in range(len(cur)) if prop[k] != cur[k]]
        if not changed:
            continue
        lo, hi = min(changed) + 1, max(changed) + 1
        ps = "".join(prop)
        for cst in (None, active):
            cnt = roofline.cell_terms(ps, cst)
            ei, em = roofline.band_terms(cnt, lo, hi)
            fi, fm = roofline.band_terms(cnt, None, None)
            ex_sum += 2 * (mul * ei + 2 * em)     # apo and holo share the cell work
            full_sum += 2 * (mul * fi + 2 * fm)
        n += 1
    return (ex_sum / n if n else None), (full_sum / n if n else None), n


def measure(a, fold, bppm, length, steps, warmup, rank, world, gids_rank, dist, dev, local_rank,
            traffic_json=None, cpu=False, cpu_seconds=15.0, dump=None):
    """Run one workload (W walkers of this rank) and return its record: value
    (all ranks), ms_per_step, roofline of the dominant kernel, outcomes."""
    from addapt_amd import native, roofline, shard, workloads

    tmpl, active = workloads.synthetic(length)
    terms = workloads.config_objective(length, bppm=bppm)
    apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
    replica_mode = a.replica_interval > 0 and world > 1
    if replica_mode:
        from addapt_amd import replica

        temps = replica.ladder_temperatures(world)
        th = native.make_thermostat("fixed", t=temps[rank])
    else:
        th = native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300)
    eng = native.Engine(tmpl, [active], terms, aptamer=apt, thermostat=th, device=local_rank, fold_mode=fold)
    W = a.walkers
    seqs = workloads.walker_sequences(tmpl, [active], W, seed_base=1000 + gids_rank[0])
    eng.walkers_init(gids_rank, seqs)

    def barrier():
        if dist is not None:
            import torch

            dist.barrier()
            torch.cuda.synchronize()

    if warmup > 0:
        eng.run_steps(warmup)
    _, _, c0 = eng.download()
    barrier()
    t0 = time.perf_counter()
    rx = None
    audit = None
    if replica_mode:
        observe = None
        if a.replica_audit:
            audit = {"round": [], "partner": [], "before": [], "after": [], "moved": []}

            def observe(rnd, p, s0, c0, s1, c1):
                audit["round"].append(rnd)
                audit["partner"].append(-1 if p is None else p)
                d0, d1 = replica.digests(s0, c0), replica.digests(s1, c1)
                audit["before"].append(d0)
                audit["after"].append(d1)
                audit["moved"].append(int((d0 != d1).sum()))
        rx = replica.run(eng, dist, rank, world, steps, a.replica_interval, temps, seed=0, device="cuda",
                         observe=observe)
    else:
        eng.run_steps(steps)
    barrier()
    t1 = time.perf_counter()
    kernel_ms = eng.last_kernel_ms()            # whole timed run_steps (3 kernels per step)
    score_ms, launches = eng.last_score_kernel_ms()   # the step's score window, per launch
    inside_ms, outside_ms = eng.last_kernel_split_ms()   # the same window split per kernel
    inside_name, outside_name = eng.last_kernel_names()  # what the engine launched
    fin_seqs, fin_scores, c1 = eng.download()
    elapsed = shard.max_over_ranks(t1 - t0, dist, device=dev)
    per_rank_ms = shard.gather_over_ranks((t1 - t0) / max(1, steps) * 1e3, dist, device=dev)
    if dump:
        import numpy as np

        os.makedirs(dump, exist_ok=True)
        np.savez(os.path.join(dump, "rank%d.npz" % rank), gids=np.array(gids_rank), seqs=np.array(fin_seqs),
                 scores=fin_scores, counters=c1, template=np.array([tmpl]), active=np.array([active]),
                 fold=np.array([fold]), bppm=np.array([bppm]), length=np.array([length]),
                 kernels=np.array([eng.last_kernel_names()[0], eng.last_kernel_names()[1]]))
    # executed (incremental) vs algorithmic inside work, from one traced step
    # after the timed region (rank 0 reports it)
    ex_inside, full_inside, ex_n = executed_inside_work(eng, fin_seqs, tmpl, active, fold) \
        if rank == 0 and not replica_mode else (None, None, 0)
    if audit is not None:
        import numpy as np

        os.makedirs(a.replica_audit, exist_ok=True)
        pick = sorted(set(range(0, W, max(1, W // 8))) | {W - 1})
        np.savez(os.path.join(a.replica_audit, "rank%d.npz" % rank),
                 round=np.array(audit["round"]), partner=np.array(audit["partner"]),
                 before=np.array(audit["before"], dtype=np.uint64),
                 after=np.array(audit["after"], dtype=np.uint64), moved=np.array(audit["moved"]),
                 temperature=np.array([temps[rank]]), accepted=np.array([rx["accepted"]]),
                 attempted=np.array([rx["attempted"]]), sample_slots=np.array(pick),
                 sample_seqs=np.array([fin_seqs[w] for w in pick]),
                 sample_scores=fin_scores[pick], counters=c1 - c0, template=np.array([tmpl]),
                 active=np.array([active]), fold=np.array([fold]))
    value = W * steps * world / elapsed

    # algorithmic work of the launch: scored steps x the folds' (+ outside passes') terms
    dc = c1 - c0
    scored = int(dc[:, 0].sum() + dc[:, 1].sum() + dc[:, 3].sum())
    outcomes = shard.sum_over_ranks(dc.sum(axis=0), dist, device=dev)
    sample = [tmpl] + seqs[:7]
    work = roofline.pf_flops if fold == "pf" else roofline.mfe_ops
    f_free = sum(work(x, None) for x in sample) / len(sample)
    f_act = sum(work(x, active) for x in sample) / len(sample)
    flop_inside = 2 * f_free + 2 * f_act           # apo/holo x free/active
    flop_per_scored = flop_inside
    f_out = 0.0
    if bppm:   # outside passes of the apo and holo unconstrained folds (on the stored inside tables)
        f_out = 2 * sum(roofline.outside_flops(x, None) for x in sample) / len(sample)
        flop_per_scored += f_out
    scored_pl = scored / max(1, steps)                             # scored walkers per launch
    launch_flops = scored_pl * flop_per_scored                     # per score window (one per step)
    # the dominant kernel by measured time: with pair terms the longer of the
    # inside folds and the outside pass, else the window (inside folds + the
    # score combine)
    outside_dominant = bppm and outside_ms >= inside_ms
    if not bppm:
        kern_ms, kern_flops, kern_name = score_ms, launch_flops, inside_name
    elif outside_dominant:
        kern_ms, kern_flops, kern_name = outside_ms, scored_pl * f_out, outside_name
    else:
        kern_ms, kern_flops, kern_name = inside_ms, scored_pl * flop_inside, inside_name
    achieved = kern_flops / (kern_ms * 1e-3) / 1e12 if kern_ms > 0 else None
    # executed work: the inside refolds recompute only the band of cells that
    # contain a changed position; the outside pass is a full pass.  Scaled from
    # the sampled proposals' executed / full ratio onto this run's algorithmic count.
    ex_ratio = (ex_inside / full_inside) if ex_inside and full_inside else None
    if ex_ratio is None:
        exec_flops = None
    elif outside_dominant:
        exec_flops = kern_flops
    else:
        exec_flops = scored_pl * flop_inside * ex_ratio
    exec_achieved = exec_flops / (kern_ms * 1e-3) / 1e12 if exec_flops and kern_ms > 0 else None
    # incremental-fold state written per scored walker (kernels.hip Inc): 2 fold
    # groups x value arrays (MFE: one packed apo/holo array; PF: two) x
    # (3 cell tables + q5) x 4 B
    cells = (length - 4) * (length - 3) // 2
    state_bytes = 2 * (1 if fold == "mfe" else 2) * (3 * cells + length + 2) * 4
    if fold == "mfe":   # round 6: MFE slots also keep each cell's inner-pair code (1 B)
        state_bytes += 2 * ((cells + 15) // 16) * 16
    traffic, traffic_src = _traffic(traffic_json, fold, bppm, length, kern_name)
    peak, peak_note = roofline.valu_peak(fold)
    roof = {
        "bound": "valu",
        "achieved": achieved,
        "peak": peak,
        "unit": "TFLOP/s" if fold == "pf" else "Top/s",
        "frac": (achieved / peak) if achieved else None,
        "traffic": traffic,
        "compute_unit": peak_note,
        "kernel": (kern_name + " (events around its launch; the window also holds " +
                   (inside_name if outside_dominant else outside_name) + ")") if bppm else inside_name,
        "executed_flop_per_launch": exec_flops,
        "executed_achieved": exec_achieved,
        "executed_frac": (exec_achieved / peak) if exec_achieved else None,
        "executed_note": ("inside refolds recompute the cells containing a changed position: "
                          "%.3f of the full folds' terms over %d sampled proposals (one traced step "
                          "after the timed region, roofline.band_terms)%s"
                          % (ex_ratio, ex_n, "; the priced kernel is the full outside pass"
                             if outside_dominant else "")) if ex_ratio else None,
        "inside_executed_ratio": ex_ratio,
        "inside_kernel": inside_name,
        "outside_kernel": outside_name or None,
        "traffic_source": traffic_src,
        "kernel_ms_per_launch": kern_ms,
        "window_ms_per_launch": score_ms,
        # since round 5 the per-variant score combine runs in step_tail_kernel,
        # after the window's end event: the window is the step's fold launches
        # (order_kernel, inside / outside folds, the MFE FP32-fallback scan) only
        "window_note": "score window = order_kernel + fold launches (+ MFE fallback scan); "
                       "excludes step_tail_kernel (accept, score combine, next proposal) since round 5",
        "inside_ms_per_launch": inside_ms,
        "outside_ms_per_launch": outside_ms if bppm else None,
        "inside_frac": ((scored_pl * flop_inside / (inside_ms * 1e-3) / 1e12) / peak
                        if bppm and inside_ms > 0 else None),
        "outside_frac": ((scored_pl * f_out / (outside_ms * 1e-3) / 1e12) / peak
                         if bppm and outside_ms > 0 else None),
        "launches": launches,
        "all_kernels_ms_per_step": kernel_ms / steps,
        "flop_per_scored_step": flop_per_scored,
        "flop_per_launch": launch_flops,
        "scored_walkers_per_launch": scored_pl,
        # HBM bytes of one launch by design: each scored walker reads its proposal
        # (N B), writes its score (8 B), and writes its fold tables for the next
        # incremental refold (read back for the unchanged cells, <= the same again)
        "algorithmic_bytes_per_launch": scored_pl * (length + 8 + 2 * state_bytes),
        "state_bytes_per_scored_walker": state_bytes,
        # the priced kernel's own compulsory bytes, comparable with `traffic` (its PMC
        # bytes): the inside folds' as above; the outside pass reads the stored inside
        # tables of the apo / holo unconstrained folds (3 cell tables + q5, FP32)
        "priced_kernel_algorithmic_bytes_per_launch": (
            scored_pl * 2 * (3 * cells + length + 2) * 4 if outside_dominant
            else scored_pl * (length + 8 + 2 * state_bytes)),
        "traffic_over_algorithmic": None,
        "hbm_peak_GBps": HBM_PEAK_GBPS,
    }
    if traffic and roof["priced_kernel_algorithmic_bytes_per_launch"]:
        roof["traffic_over_algorithmic"] = traffic / roof["priced_kernel_algorithmic_bytes_per_launch"]
    rec = {
        "value": value,
        "unit": "MC steps/s",
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "dist": shard.dist_record(dist, per_rank_ms, elapsed / steps * 1e3),
        "dtype": "i16x2" if fold == "mfe" else "fp32",
        "workload": "%s: default objective (apo: not active, holo: active; THEO aptamer "
                    "0.32 uM)%s, 4 %s%s per scored step, synthetic %d-nt sgRNA template "
                    "(SURVEY.md 8d), %d walkers per GPU, %s"
                    % ("BASELINE configs[1] (MFE-fold score only)" if fold == "mfe"
                       else ("BASELINE config %d (pf + bppm score)" % (3 if length == 100 else 4)) if bppm
                       else "partition-function score (config 3 without bppm)",
                       " + apo 'not pair(0,N-1)' / holo 'pair(0,N-1)'" if bppm else "",
                       "minimum-free-energy folds" if fold == "mfe" else "McCaskill inside PFs",
                       " + 2 inside/outside (bppm) passes" if bppm else "",
                       length, W,
                       "replica ladder T_r = 0.5*1.5^r" if replica_mode else "annealing 5 to 0 in 300 steps"),
        "fold": fold,
        "bppm": bppm,
        "length": length,
        "outcomes": {k: int(v) for k, v in zip(native.OUTCOMES, outcomes)},
        "roofline": roof,
    }
    if rx is not None:
        att = shard.sum_over_ranks([rx["attempted"], rx["accepted"], rx["rounds"]], dist, device=dev)
        rec["exchange"] = {"rounds_per_rank": rx["rounds"], "attempted": att[0], "accepted": att[1],
                           "interval": a.replica_interval, "temperatures": temps}
    if cpu and rank == 0 and world == 1:
        rec["cpu_baseline"] = cpu_baseline(tmpl, active, seqs, cpu_seconds, fold, terms)
    del eng
    return rec


def gpu_count():
    """Visible GPUs without touching HIP (the launcher starts before any GPU call):
    the kfd topology's GPU nodes, narrowed by *_VISIBLE_DEVICES."""
    n = 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for d in os.listdir(base):
            try:
                with open(os.path.join(base, d, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
                if int(props.get("simd_count", "0")) > 0:
                    n += 1
            except (OSError, ValueError):
                pass
    except OSError:
        n = 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids)) if n else len(ids)
    return n


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
    dev = None
    device = 0 if a.share_device else local_rank
    if world > 1:
        import torch
        import torch.distributed as dist_

        if not a.share_device and local_rank >= torch.cuda.device_count():
            print("bench.py: rank %d has no GPU (%d visible)" % (local_rank, torch.cuda.device_count()),
                  file=sys.stderr)
            sys.exit(2)
        torch.cuda.set_device(device)
        if a.dist_backend == "nccl":
            dist_.init_process_group("nccl", device_id=torch.device("cuda", device))
            dev = "cuda"
        else:   # rehearsal: gloo on host tensors (ranks may share one GPU)
            dist_.init_process_group("gloo")
        dist = dist_

    from addapt_amd import shard

    if a.bppm:
        a.fold = "pf"
    W = a.walkers
    gids = shard.walker_ids(rank, world, W)
    rec = measure(a, a.fold, a.bppm, a.length, a.steps, a.warmup, rank, world, gids, dist, dev, device,
                  traffic_json=a.traffic_json, cpu=not a.no_cpu_baseline, cpu_seconds=a.cpu_seconds,
                  dump=a.dump_walkers)
    out = {
        "metric": METRIC,
        "value": rec["value"],
        "unit": "MC steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": rec["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        # MFE: integer dcal/mol, apo|holo as two int16 halves of one 32-bit word
        # (v_pk_add_i16 / v_pk_min_i16); PF: fp32 Boltzmann factors
        "dtype": rec["dtype"],
        "data": "synthetic",
        "config": {
            "workload": rec["workload"],
            "fold": a.fold,
            "bppm": a.bppm,
            "walkers_per_gpu": W,
            "global_walkers": W * world,
            "length": a.length,
            "parallelism": ("replica exchange x%d (%s neighbour swap every %d steps)"
                            % (world, "RCCL" if a.dist_backend == "nccl" else "gloo", a.replica_interval))
            if a.replica_interval > 0 and world > 1
            else "walker-sharded x%d (no data-path collective)" % world,
            "dist_backend": a.dist_backend if world > 1 else None,
            "shared_device": bool(a.share_device and world > 1),
            "outcomes": rec["outcomes"],
        },
        "roofline": rec["roofline"],
        # the collective backend torch.distributed ran ("nccl" = RCCL on ROCm), the
        # world size it reported, each rank's ms per step and their max (the value's clock)
        "dist": rec["dist"],
    }
    if "exchange" in rec:
        out["exchange"] = rec["exchange"]
    if "cpu_baseline" in rec:
        out["cpu_baseline"] = rec["cpu_baseline"]
    # the reference's own scoring path (vrna_pf, scoring.cc:53-71) measured in the
    # same run: PF, config 3 (pf + bppm, N = 100) and config 4's per-GPU shard
    # (pf + bppm, N = 150), each with its dominant kernel's roofline
    if not a.no_sub_records and a.fold == "mfe" and not a.bppm and a.replica_interval == 0:
        subs = {}
        for name, fold, bppm, length, steps, cpu in (
                ("pf", "pf", False, 100, a.steps, True),
                ("config3", "pf", True, 100, a.steps, True),
                ("config4", "pf", True, 150, min(a.steps, a.sub_steps_c4), False)):
            r = measure(a, fold, bppm, length, steps, min(a.warmup, 5), rank, world, gids, dist, dev, device,
                        cpu=cpu and not a.no_cpu_baseline, cpu_seconds=a.cpu_seconds * 2.0 / 3.0)
            subs[name] = {k: r[k] for k in ("value", "unit", "steps", "ms_per_step", "dtype", "workload",
                                            "outcomes", "roofline") if k in r}
            if "cpu_baseline" in r:
                subs[name]["cpu_baseline"] = r["cpu_baseline"]
        out["sub_records"] = subs
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
