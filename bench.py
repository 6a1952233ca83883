#!/usr/bin/env python3
"""Placement-candidate throughput of the MI355X engine (BASELINE.json metric).

One step = one scheduling round of one policy over a synthetic round resident in HBM: reset
the host availability to the round's snapshot (one D2D copy), then
pvt_place (a2 ordering, fused score/top-K passes, merges, sequential commit walk).
Candidates per step = T x H, the round's logical task x host space.

Default workload (N=1): BASELINE config 5 shape on one GPU — 1M hosts x 10k ready tasks,
20 zones, cost_aware best-fit (every candidate fit-masked and scored). For N > 1 every rank runs
its own independent scenario (seed + rank), as in the scenario-batch config: weak scaling, no
collective on the data path; only the final timing max is reduced.

Run:  python bench.py [--gpus N --steps K --warmup W --mode ca_bf --hosts H --tasks T]
      torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]

import numpy as np  # noqa: E402

MODES = {"ca_ff": 0, "ca_bf": 1, "opp": 2, "vbp_ff": 3, "vbp_bf": 4}
POLICY = {"ca_ff": "cost_aware first-fit (sort_tasks, sort_hosts)", "ca_bf": "cost_aware best-fit",
          "opp": "opportunistic", "vbp_ff": "vbp first-fit decreasing", "vbp_bf": "vbp best-fit"}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--mode", default="ca_bf", choices=sorted(MODES))
    p.add_argument("--hosts", type=int, default=1_000_000)
    p.add_argument("--tasks", type=int, default=10_000)
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--window", type=int, default=0)
    p.add_argument("--pipeline", type=int, default=1,
                   help="1: score window k+1 while window k is walked (default); 0: sequential")
    p.add_argument("--shard", default="scenarios", choices=["scenarios", "hosts"],
                   help="N > 1: independent scenario per rank (weak scaling, config 4) or one "
                        "round with its host dimension split over the ranks (strong, config 5)")
    p.add_argument("--batch", type=int, default=0,
                   help="> 0: scenario-batch workload (BASELINE config 4): this many independent "
                        "scenarios per GPU (seeds seed + rank*batch + s) of --hosts x --tasks, all "
                        "placed by ONE pvt_place_batch launch per step (resident kernel)")
    p.add_argument("--cpu-baseline-seconds", type=float, default=10.0,
                   help="target CPU time of the oracle baseline sample (0 = skip)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="rocprofv3 PMC traffic summary (tools/pmc_traffic.py); absent = null")
    return p.parse_args()


def _time_oracle(r, budget_s, threads):
    """Candidates/s of the C restatement on the first n tasks of ``r``, n sized so the timed
    sample takes about ``budget_s`` seconds; returns (rate, n, seconds)."""
    from oracle import oracle
    from pivot_place.synthetic import subset_tasks
    n = min(r.n_tasks, 4 * max(threads, 1))
    while True:
        sub = subset_tasks(r, n)
        t = time.perf_counter()
        oracle.place(sub, threads=threads)
        dt = max(time.perf_counter() - t, 1e-6)
        if dt >= 0.5 * budget_s or n >= r.n_tasks:
            return float(n) * r.n_hosts / dt, n, dt
        n = int(min(r.n_tasks, max(n + 1, n * 1.2 * budget_s / dt)))


def cpu_baseline(r, budget_s):
    """The CPU restatement (oracle/) timed on this host beside the GPU: all the cores this job
    may use (OMP_NUM_THREADS, else os.cpu_count(); OpenMP host scans, oracle_place_mt) as the
    reported value, and 1 thread (scalar) alongside."""
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    v_all, n_all, dt_all = _time_oracle(r, budget_s, threads)
    v_one, n_one, dt_one = _time_oracle(r, budget_s / 3.0, 0)
    return {"value": v_all, "unit": "candidates/s", "cores": threads, "kind": "port",
            "value_1thread": v_one,
            "sample": "oracle/pivot_oracle.c (C restatement, -O2; OpenMP host scans over %d threads) "
                      "on the first %d tasks x %d hosts of the same round (%.1f s); 1 thread: first "
                      "%d tasks (%.1f s)" % (threads, n_all, r.n_hosts, dt_all, n_one, dt_one)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from pivot_place import _abi, synthetic
    from pivot_place.engine import DeviceRound, PlacementEngine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    mode = MODES[args.mode]
    H, T = args.hosts, args.tasks
    log("[rank %d] building synthetic round: %s, H=%d T=%d" % (rank, args.mode, H, T))
    hosts_sharded = args.shard == "hosts" and not args.batch
    B = max(args.batch, 0)
    eng = PlacementEngine(local, window=args.window)
    eng.set_pipeline(bool(args.pipeline))
    if B:
        from pivot_place.engine import DeviceBatch
        rounds = [synthetic.make_round(mode, H, T, seed=args.seed + rank * B + s) for s in range(B)]
        r = rounds[0]
        dr = DeviceBatch(rounds, eng.device)
        run = eng.run_batch
    else:
        r = synthetic.make_round(mode, H, T, seed=args.seed + (0 if hosts_sharded else rank))
        dr = DeviceRound(r, eng.device)
        run = eng.run
    if hosts_sharded:
        from pivot_place.sharded import HostShardedPlacer, torch_exchange
        placer = HostShardedPlacer(eng, rank, world, torch_exchange() if world > 1 else None)
        run = placer.run
    torch.cuda.synchronize()

    for i in range(args.warmup):
        dr.reset()
        run(dr)
    torch.cuda.synchronize()
    stats = eng.last_stats()
    placed = int(((dr.placement_of(0) if B else dr.placement[:T]) >= 0).sum().item())
    log("[rank %d] warmup done: %d/%d placed, windows=%d refills=%d"
        % (rank, placed, T, stats["windows"], stats["refills"]))

    eng.reset_kstats()
    eng.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        dr.reset()
        run(dr)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_profiling(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=eng.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    cand_per_step = float(T) * H * (1 if hosts_sharded else world) * (B if B else 1)
    value = cand_per_step / (elapsed / args.steps)

    ks = {name: eng.kstats(k) for name, k in (("score", _abi.PVT_K_SCORE), ("merge", _abi.PVT_K_MERGE),
                                               ("commit", _abi.PVT_K_COMMIT), ("other", _abi.PVT_K_OTHER))}
    score = ks["score"]
    avg_ms = score["ms"] / max(score["launches"], 1)
    bytes_per_launch = score["bytes"] / max(score["launches"], 1)
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("mode") == args.mode and tj.get("hosts") == H and tj.get("tasks") == T:
                # PMC bytes per candidate of the probe's launches (tools/pmc_traffic.py), scaled to
                # this run's average candidates per score launch
                per_cand = tj.get("hbm_bytes_per_candidate")
                cand_per_launch = score["candidates"] / max(score["launches"], 1)
                traffic = (per_cand * cand_per_launch if per_cand is not None
                           else tj.get("hbm_bytes_per_launch"))
        except (OSError, ValueError):
            traffic = None

    if rank == 0:
        out = {
            "metric": "task x host placement candidates scored/sec (HBM GB/s % peak) at 1/2/4/8 MI355X",
            "value": value,
            "unit": "candidates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if hosts_sharded else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8(d): trace demand rows, 20 locality.yml zones, seeded)",
            "config": {
                "workload": "synthetic %d hosts x %d ready tasks per round, 20 zones, %s, %s"
                            % (H, T, POLICY[args.mode],
                               "%d independent scenarios per GPU, one resident launch per step" % B
                               if B else
                               "host dimension split over the GPUs" if hosts_sharded
                               else "one independent scenario per GPU"),
                "scenarios_per_gpu": B if B else 1,
                "hosts": H, "tasks_per_round": T, "zones": 20, "policy": args.mode,
                "parallelism": ("host-sharded x%d (per-window candidate all-gather)" % world
                                if hosts_sharded else
                                "scenario-sharded x%d (no data-path collective)" % world),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": ("resident (registers-held hosts, full rescan per task)" if B
                           else "score (fused fit-mask + score + top-K)"),
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "avg_launch_ms": avg_ms,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "bytes_per_candidate": _abi.BYTES_PER_CANDIDATE[mode],
                "note": ("achieved = candidates per launch x bytes per candidate (SURVEY.md "
                         "section 8(d)) / average launch time; a host row read once serves the "
                         "tasks of a wave from registers/L1/L2, so the scan is not HBM-bound "
                         "(frac > 1); traffic = DRAM bytes per launch from rocprofv3 PMC "
                         "(tools/pmc_traffic.py)"),
            },
            "kernels_ms_per_step": {k: v["ms"] / args.steps for k, v in ks.items()},
            "windows_per_step": stats["windows"], "refills_per_step": stats["refills"],
        }
        if world == 1 and args.cpu_baseline_seconds > 0:
            log("[rank 0] cpu baseline (oracle, all cores and 1 thread) ...")
            out["cpu_baseline"] = cpu_baseline(r, args.cpu_baseline_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
