#!/usr/bin/env python3
"""Placement-candidate throughput of the MI355X engine (BASELINE.json metric).

One step = one scheduling round of one policy over a synthetic round resident in HBM: reset
the host availability to the round's snapshot (one D2D copy), then
pvt_place (a2 ordering, candidate lists, sequential commit walk in the reference's order).
Candidates per step = T x H, the round's logical task x host space.

Default workload (N=1): BASELINE config 5 shape on one GPU -- 1M hosts x 10k ready tasks,
20 zones, cost_aware best-fit. For N > 1 every rank runs its own independent scenario (seed +
rank), as in the scenario-batch config: weak scaling, no collective on the data path; only the
final timing max is reduced. `--shard hosts` splits one round's host dimension instead.

Parity: after the timed steps, rank 0 compares the round it placed (placement, processing
order, final availability, RNG state) with the CPU restatement (oracle/, itself pinned to the
reference's golden runs) on the same inputs and prints `"parity": true/false`. The default run
also times the other four policies at the config-5 size and all five at the config-3 size
(`extra`), each with its own parity check.

Run:  python bench.py [--gpus N --steps K --warmup W --mode ca_bf --hosts H --tasks T]
With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts N rank processes
itself (before anything touches the GPU); under torchrun WORLD_SIZE must equal N.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]

import numpy as np  # noqa: E402

MODES = {"ca_ff": 0, "ca_bf": 1, "opp": 2, "vbp_ff": 3, "vbp_bf": 4}
POLICY = {"ca_ff": "cost_aware first-fit (sort_tasks, sort_hosts)", "ca_bf": "cost_aware best-fit",
          "opp": "opportunistic", "vbp_ff": "vbp first-fit decreasing", "vbp_bf": "vbp best-fit"}
METRIC = "task x host placement candidates scored/sec (HBM GB/s % peak) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
DEFAULT_H, DEFAULT_T, DEFAULT_SEED = 1_000_000, 10_000, 20261015


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--mode", default="ca_bf", choices=sorted(MODES))
    p.add_argument("--hosts", type=int, default=DEFAULT_H)
    p.add_argument("--tasks", type=int, default=DEFAULT_T)
    p.add_argument("--seed", type=int, default=DEFAULT_SEED)
    p.add_argument("--window", type=int, default=0)
    p.add_argument("--pipeline", type=int, default=1,
                   help="1: score window k+1 while window k is walked (default); 0: sequential")
    p.add_argument("--epochs", type=int, default=1,
                   help="cost_aware best-fit: 1 walks groups side by side in speculative epochs "
                        "(default), 0: one group after the other")
    p.add_argument("--shard", default="scenarios", choices=["scenarios", "hosts"],
                   help="N > 1: independent scenario per rank (weak scaling, config 4) or one "
                        "round with its host dimension split over the ranks (strong, config 5)")
    p.add_argument("--batch", type=int, default=0,
                   help="> 0: scenario-batch workload (BASELINE config 4): this many independent "
                        "scenarios per GPU (seeds seed + rank*batch + s) of --hosts x --tasks, all "
                        "placed by ONE pvt_place_batch launch per step (resident kernel)")
    p.add_argument("--cpu-baseline-seconds", type=float, default=10.0,
                   help="target CPU time of the oracle baseline sample (0 = skip)")
    p.add_argument("--parity", type=int, default=1, help="1: check the placed round against the oracle")
    p.add_argument("--extra", type=int, default=-1,
                   help="1: also time (and parity-check) the other policies at config 5 and all "
                        "policies at config 3; -1 (default): only for the default workload at N=1")
    p.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r02c_score_pmc.json"),
                   help="rocprofv3 PMC summary of the score kernel of this binary "
                        "(tools/pmc_profile.py); absent or another config = counters null")
    return p.parse_args()


# ---------------------------------------------------------------------------- launcher
def spawn_ranks(n):
    """--gpus N without WORLD_SIZE: start N rank processes of this script (one per GPU) before
    anything touches the GPU, and exit with the worst return code. Rank 0 prints the line."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


# ---------------------------------------------------------------------------- CPU baseline
def oracle_threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)


def _time_oracle(r, budget_s, threads):
    """Candidates/s of the C restatement on the first n tasks of ``r``, n sized so the timed
    sample takes about ``budget_s`` seconds; returns (rate, n, seconds, result of the last run)."""
    from oracle import oracle
    from pivot_place.synthetic import subset_tasks
    n = min(r.n_tasks, 4 * max(threads, 1))
    while True:
        sub = r if n >= r.n_tasks else subset_tasks(r, n)
        t = time.perf_counter()
        res = oracle.place(sub, threads=threads)
        dt = max(time.perf_counter() - t, 1e-6)
        if dt >= 0.5 * budget_s or n >= r.n_tasks:
            return float(n) * r.n_hosts / dt, n, dt, res
        n = int(min(r.n_tasks, max(n + 1, n * 1.2 * budget_s / dt)))


def cpu_baseline(r, budget_s):
    """The CPU restatement (oracle/) timed on this host beside the GPU: all the cores this job
    may use (OMP_NUM_THREADS, else min(16, os.cpu_count()); OpenMP host scans) as the reported
    value, 1 thread alongside. Returns (baseline dict, full-round oracle result or None)."""
    threads = oracle_threads()
    v_all, n_all, dt_all, res_all = _time_oracle(r, budget_s, threads)
    v_one, n_one, dt_one, _ = _time_oracle(r, budget_s / 3.0, 0)
    out = {"value": v_all, "unit": "candidates/s", "cores": threads, "kind": "port",
           "value_1thread": v_one,
           "sample": "oracle/pivot_oracle.c (C restatement, -O2; a naive full T x H scan with "
                     "OpenMP host scans over %d threads -- not the engine's algorithm) on the first "
                     "%d tasks x %d hosts of the same round (%.1f s); 1 thread: first %d tasks "
                     "(%.1f s)" % (threads, n_all, r.n_hosts, dt_all, n_one, dt_one)}
    return out, (res_all if n_all >= r.n_tasks else None)


# ---------------------------------------------------------------------------- parity
def same_result(got, ref):
    ok = (np.array_equal(got.placement, ref.placement) and np.array_equal(got.order, ref.order)
          and np.array_equal(got.avail, ref.avail))
    if ref.mt_state is not None:
        ok = ok and np.array_equal(got.mt_state, ref.mt_state)
    return bool(ok)


def check_parity(got, r, ref=None):
    from oracle import oracle
    if ref is None:
        ref = oracle.place(r, threads=oracle_threads())
    return same_result(got, ref)


# ---------------------------------------------------------------------------- extra workloads
def time_round(eng, r, steps, warmup):
    """ms per step of pvt_place on a resident round (reset + place), and the placed result."""
    import torch
    from pivot_place.engine import DeviceRound
    dr = DeviceRound(r, eng.device)
    for _ in range(warmup):
        dr.reset()
        eng.run(dr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        dr.reset()
        eng.run(dr)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    return ms, dr.result()


def extra_workloads(eng, args, skip_mode):
    """Config 5 (1M x 10k) for the other policies and config 3 (100k x 1k) for all five, each
    timed on the same engine and checked against the oracle."""
    from pivot_place import synthetic
    out = {}
    steps, warm = max(1, min(args.steps, 5)), 1
    for tag, H, T, modes in (("c5", DEFAULT_H, DEFAULT_T, [m for m in MODES if m != skip_mode]),
                             ("c3", 100_000, 1000, list(MODES))):
        for m in modes:
            r = synthetic.make_round(MODES[m], H, T, seed=args.seed)
            ms, got = time_round(eng, r, steps, warm)
            ok = check_parity(got, r) if args.parity else None
            out["%s_%s" % (tag, m)] = {"value": float(T) * H / (ms * 1e-3), "ms_per_step": ms,
                                       "hosts": H, "tasks": T, "steps": steps, "parity": ok}
            log("[rank 0] extra %s %s: %.3e cand/s, %.2f ms, parity %s"
                % (tag, m, float(T) * H / (ms * 1e-3), ms, ok))
    return out


# ---------------------------------------------------------------------------- roofline
def roofline(args, ks, mode, B):
    """The score (candidate evaluation) kernel's roofline. `achieved` is the kernel's measured
    per-launch work from the rocprofv3 PMC profile of this binary and config (VALU busy cycles,
    LDS-array cycles, DRAM bytes; tools/pmc_profile.py -> profiles/) divided by the launch time
    measured live here with HIP events on the launch's stream. The bound is the resource with
    the highest utilisation. The SURVEY §8(d) figure (36 B per candidate) is kept as
    `hbm_equivalent_*`: bytes a per-task streaming scan would move, not bytes moved."""
    from pivot_place import _abi
    score = ks["score"]
    launches = max(score["launches"], 1)
    avg_ms = score["ms"] / launches
    cand = score["candidates"] / launches
    hbm_eq = score["bytes"] / launches / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    out = {"kernel": ("resident (registers-held hosts, full rescan per task)" if B
                      else "score (fused fit-mask + score + top-K)"),
           "avg_launch_ms": avg_ms, "candidates_per_launch": cand,
           "hbm_equivalent_GBs": hbm_eq,
           "hbm_equivalent_bytes_per_candidate": _abi.BYTES_PER_CANDIDATE[mode],
           "bound": None, "achieved": None, "peak": None, "unit": None, "frac": None,
           "traffic": None}
    pmc = None
    if os.path.exists(args.pmc_json):
        try:
            with open(args.pmc_json) as f:
                allp = json.load(f)
            key = "%s_%d_%d" % (args.mode, args.hosts, args.tasks)
            pmc = allp.get("configs", {}).get(key)
        except (OSError, ValueError):
            pmc = None
    if pmc is None or avg_ms <= 0:
        out["note"] = "no PMC profile of this config (tools/pmc_profile.py)"
        return out
    # per-launch work scaled to this run's candidates per launch (windows may differ)
    scale = cand / max(pmc["candidates_per_launch"], 1.0)
    t = avg_ms * 1e-3
    res = {
        "valu": (pmc["valu_busy_cycles_per_launch"] * scale / t, pmc["valu_peak_cycles_per_s"],
                 "SIMD-cycles/s"),
        "lds": (pmc["lds_busy_cycles_per_launch"] * scale / t, pmc["lds_peak_cycles_per_s"],
                "CU-LDS-cycles/s"),
        "hbm": (pmc["hbm_bytes_per_launch"] * scale / t / 1e9, HBM_PEAK_GBS, "GB/s"),
    }
    bound = max(res, key=lambda k: res[k][0] / res[k][1])
    a, p, u = res[bound]
    out.update({"bound": bound, "achieved": a, "peak": p, "unit": u, "frac": a / p,
                "traffic": pmc["hbm_bytes_per_launch"] * scale,
                "utilisation": {k: v[0] / v[1] for k, v in res.items()},
                "pmc_source": os.path.relpath(args.pmc_json, ROOT),
                "pmc_kernel": pmc.get("kernel"),
                "prefilter_survivor_frac": pmc.get("prefilter_survivor_frac")})
    return out


# Roofline of the sequential frontier walk. Each task reads the capacities the previous commit
# wrote, so the chain runs on ONE wave, and what bounds it is that wave's instruction issue: a
# wave issues at most one instruction per 4 cycles (MI355X_MICROARCH.md, 'vector-instruction
# ISSUE cost, one wave': v_add_f32 4 cycles, s_nop 4). `achieved` = the walk's instructions per
# second on its longest chain (instructions per task from the rocprofv3 PMC profile of this
# binary: SQ_INSTS_VALU + SALU + LDS + SMEM + VMEM over the chain tasks), `peak` = 2.4 GHz / 4.
# The latency floor (one dependent LDS round trip per task, ~50 cycles) is kept beside it.
ISSUE_CYCLES = 4
LDS_DEP_CYCLES = 50
SHADER_HZ = 2.4e9
WALK_PMC = os.path.join(ROOT, "profiles", "r02p", "pmc_r02p_zwalk.json")


def walk_roofline(ks, ep, steps, T):
    """The dominant kernel when no candidate lists are scored (cost_aware best-fit epochs whose
    chains the zero-cost frontier walk proves, pvt_zwalk.hip): the chain walks run side by side,
    so the round waits for the longest."""
    c = ks["commit"]
    ms = c["ms"] / max(steps, 1)
    longest = ep.get("longest_chain_tasks", 0)
    sequential = longest <= 0 and ep.get("frontier_chains", 0) > 0
    if sequential:
        # first-fit rounds (keyed / ordered frontier walks): the walks run one after another,
        # every task of the round on one of them
        longest = T
    out = {"kernel": "zwalk (zero-cost frontier walk: one wave per epoch chain, window in LDS)",
           "bound": "issue", "unit": "instructions/s (one wave)", "traffic": None,
           "walk_ms_per_step": ms, "longest_chain_tasks": longest,
           "peak_basis": "one instruction per %d cycles of one wave at %.1f GHz"
                         % (ISSUE_CYCLES, SHADER_HZ / 1e9)}
    if ms <= 0 or longest <= 0:
        out.update({"achieved": None, "peak": None, "frac": None})
        return out
    tasks_per_s = longest / (ms * 1e-3)
    ipt = None
    if sequential:
        out["kernel"] = "zwalk (keyed / ordered frontier walks in sequence, window in LDS)"
        out["note"] = "the walk's PMC profile is of the default line's launch; no instruction count here"
    try:
        if sequential:
            raise KeyError("no PMC profile of this mode")
        with open(WALK_PMC) as f:
            pmc = json.load(f)
        cnt = pmc["counters_per_launch"]
        ipt = sum(cnt.get(k, 0.0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                            "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
                                            "SQ_INSTS_VMEM_WR")) / max(T, 1)
        out["pmc_source"] = os.path.relpath(WALK_PMC, ROOT)
        out["instructions_per_task"] = ipt
        out["issue_active_frac_pmc"] = cnt["SQ_ACTIVE_INST_ANY"] / cnt["SQ_WAVE_CYCLES"]
        out["wait_frac_pmc"] = cnt["SQ_WAIT_ANY"] / cnt["SQ_WAVE_CYCLES"]
        traffic = 2.0 * cnt.get("FETCH_SIZE", 0.0) * 1024 + cnt.get("WRITE_SIZE", 0.0) * 1024
        out["traffic"] = traffic if traffic > 0 else None
    except (OSError, ValueError, KeyError):
        out.setdefault("note", "no PMC profile of the walk (tools/pmc_profile.py --kernel zwalk_kernel)")
    out["cycles_per_task"] = SHADER_HZ / tasks_per_s
    out["latency_floor"] = {"peak_tasks_per_s": SHADER_HZ / LDS_DEP_CYCLES,
                            "achieved_tasks_per_s": tasks_per_s,
                            "frac": tasks_per_s / (SHADER_HZ / LDS_DEP_CYCLES)}
    if ipt is None:
        out.update({"achieved": None, "peak": None, "frac": None})
        return out
    achieved = ipt * tasks_per_s
    peak = SHADER_HZ / ISSUE_CYCLES
    out.update({"achieved": achieved, "peak": peak, "frac": achieved / peak})
    return out


# ---------------------------------------------------------------------------- main
def main():
    args = parse()
    wenv = os.environ.get("WORLD_SIZE")
    if wenv is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(wenv or "1")
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d (launch N ranks, or omit WORLD_SIZE and "
                 "let bench.py start them)" % (args.gpus, world))
    import torch
    import torch.distributed as dist
    from pivot_place import _abi, synthetic
    from pivot_place.engine import DeviceRound, PlacementEngine

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
    eng.set_epochs(bool(args.epochs))
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
    ep = eng.epoch_stats()
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

    if rank == 0:
        out = {
            "metric": METRIC,
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
            "roofline": (walk_roofline(ks, ep, args.steps, T)
                         if not B and ks["score"]["launches"] == 0 and ks["commit"]["launches"] > 0
                         else roofline(args, ks, mode, B)),
            "kernels_ms_per_step": {k: v["ms"] / args.steps for k, v in ks.items()},
            "walk_us_per_task": (ks["commit"]["ms"] * 1e3 / args.steps / max(T * (B or 1), 1)
                                 if not B else None),
            "windows_per_step": stats["windows"], "refills_per_step": stats["refills"],
            "epochs_per_step": ep["epochs"], "segments_per_step": ep["segments"],
            "rejected_segments_per_step": ep["rejected"],
            "frontier_chains_per_step": ep.get("frontier_chains"),
            "list_chains_per_step": ep.get("list_chains"),
        }
        ref = None
        if world == 1 and args.cpu_baseline_seconds > 0:
            log("[rank 0] cpu baseline (oracle, all cores and 1 thread) ...")
            out["cpu_baseline"], ref = cpu_baseline(r, args.cpu_baseline_seconds)
        if args.parity:
            log("[rank 0] parity against the oracle ...")
            if B:
                from oracle import oracle
                got = dr.results()
                out["parity"] = all(same_result(g, oracle.place(x)) for g, x in zip(got, rounds))
            else:
                out["parity"] = check_parity(dr.result(), r, ref)
        default = (not B and not hosts_sharded and world == 1 and H == DEFAULT_H
                   and T == DEFAULT_T and args.window == 0 and args.pipeline == 1 and args.epochs == 1)
        if args.extra == 1 or (args.extra < 0 and default):
            out["extra"] = extra_workloads(eng, args, args.mode)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
