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
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]
LIB = os.path.join(ROOT, "pivot-scheduling_amd", "pivot_place", "libpivot_place.so")

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
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
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
    p.add_argument("--extra-cpu-seconds", type=float, default=3.0,
                   help="target CPU time of each extra line's oracle baseline sample")
    p.add_argument("--parity", type=int, default=1, help="1: check the placed round against the oracle")
    p.add_argument("--extra", type=int, default=-1,
                   help="1: also time (and parity-check) the other policies at config 5 and all "
                        "policies at config 3; -1 (default): only for the default workload at N=1")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="N > 1: torch.distributed backend (nccl = RCCL over xGMI; gloo: ranks may "
                        "share a GPU, e.g. to rehearse the multi-rank path on one card)")
    p.add_argument("--c4-batch", type=int, default=512,
                   help="N > 1: also run BASELINE config 4 as written -- this many independent "
                        "1000-host x 1000-task scenarios per rank (512 x 8 = 4096 at N = 8), one "
                        "pvt_place_batch launch per step, barrier + MAX-over-ranks timing, parity "
                        "of every rank's scenarios against the oracle (0 = off)")
    p.add_argument("--replay", type=int, default=-1,
                   help="1: also time BASELINE configs 1 and 2 -- every schedule() round of the "
                        "recorded reference simulations through the drop-in policy classes; -1 "
                        "(default): with the default workload's extras")
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


def _paired_oracle(r, budget_s, threads):
    """The C restatement on ONE task prefix at two thread counts: the first n tasks, n sized so
    one thread takes about budget_s / 3 seconds, then the same n tasks on ``threads`` threads
    (repeated to at least a second). A prefix is not a uniform sample of a round (first-fit
    tasks early in a round exit on the first hosts), so both rates must come from the same one.
    Returns (rate all threads, rate 1 thread, n, seconds all, seconds 1, full-round result or
    None)."""
    from oracle import oracle
    from pivot_place.synthetic import subset_tasks
    v_one, n, dt_one, res = _time_oracle(r, budget_s / 3.0, 0)
    sub = r if n >= r.n_tasks else subset_tasks(r, n)
    reps, t = 0, time.perf_counter()
    while True:
        res = oracle.place(sub, threads=threads)
        reps += 1
        dt_all = max(time.perf_counter() - t, 1e-6)
        if dt_all >= 1.0 or dt_all * (reps + 1) / reps > budget_s:
            break
    v_all = float(reps) * n * r.n_hosts / dt_all
    return v_all, v_one, n, dt_all / reps, dt_one, (res if n >= r.n_tasks else None)


def best_cpu(v_all, threads, v_one):
    """(value, cores) of a CPU baseline: the faster of the all-cores and the one-thread run of
    the same sample. The restatement's OpenMP host scans have no early exit, so on first-fit
    rounds (whose tasks stop at the first hosts) one thread beats all of them."""
    return (v_one, 1) if v_one > v_all else (v_all, threads)


def cpu_baseline(r, budget_s):
    """The CPU restatement (oracle/) timed on this host beside the GPU: all the cores this job
    may use (OMP_NUM_THREADS, else min(16, os.cpu_count()); OpenMP host scans) as the reported
    value, 1 thread alongside, both on the same first tasks of the round. Returns (baseline
    dict, full-round oracle result or None)."""
    threads = oracle_threads()
    v_all, v_one, n, dt_all, dt_one, res = _paired_oracle(r, budget_s, threads)
    value, cores = best_cpu(v_all, threads, v_one)
    out = {"value": value, "unit": "candidates/s", "cores": cores, "kind": "port",
           "value_1thread": v_one, "value_all_cores": v_all, "tasks": n,
           "sample": "oracle/pivot_oracle.c (naive T x H scan, not the engine's algorithm; "
                     "OpenMP host scans): the first %d tasks x %d hosts of the same round on "
                     "%d threads (%.2f s) and on 1 thread (%.1f s); value = the faster"
                     % (n, r.n_hosts, threads, dt_all, dt_one)}
    return out, res


# ---------------------------------------------------------------------------- the step
def step_reset(eng, dr, full):
    """The reset of one timed step (every place that prices a step -- main, time_round,
    tools/walk_probe.py for PMC profiles -- takes it from here). A single round restores only
    the hosts the previous step placed on (pvt_restore_hosts: a round changes no other
    capacity); a scenario batch or a host-sharded round copies the whole snapshot back
    (``full``)."""
    return dr.reset if full else (lambda: eng.restore(dr))


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
KCLASSES = (("score", 0), ("merge", 1), ("commit", 2), ("other", 3))
KCLASS_NAMES = tuple(n for n, _ in KCLASSES)


# the kernels of the path that can dominate a step, timed one by one (pvt_get_kernel_kstats)
WALK_KERNELS = ("zwalk_kernel", "commit_kernel", "lwalk_kernel", "opp_commit_kernel")
PAR_KERNELS = ("score_kernel", "band_score_kernel", "opp_count_kernel", "perm_scan_kernel",
               "ordered_kernel", "resident_kernel", "merge_kernel", "merge_small_kernel",
               "merge_pkg_kernel", "merge_path_kernel")


def kstats_all(eng):
    return {name: eng.kstats(k) for name, k in KCLASSES}


def kernel_times(eng):
    out = {}
    for name in WALK_KERNELS + PAR_KERNELS:
        k = eng.kernel_kstats(name)
        if k["launches"]:
            out[name] = k
    return out


def time_round(eng, r, steps, warmup, batch=None):
    """ms per step of pvt_place on a resident round (reset + place) -- or of pvt_place_batch on
    a resident batch -- the placed result(s) and the kernel-class times of the timed steps."""
    import torch
    from pivot_place.engine import DeviceBatch, DeviceRound
    dr = DeviceBatch(batch, eng.device) if batch else DeviceRound(r, eng.device)
    run = eng.run_batch if batch else eng.run
    reset = step_reset(eng, dr, bool(batch))
    for _ in range(warmup):
        reset()
        run(dr)
    torch.cuda.synchronize()
    dom, share, kms = dominant_kernel(eng, lambda: (reset(), run(dr)))
    eng.reset_kstats()
    eng.set_profiling(2, kernel=dom)
    t0 = time.perf_counter()
    for _ in range(steps):
        reset()
        run(dr)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    eng.set_profiling(False)
    ks = kstats_all(eng)
    ks["kernels"] = kernel_times(eng)
    ks["dominant_share"] = share
    ks["kernels_untimed_ms_per_step"] = kms
    return ms, (dr.results() if batch else dr.result()), ks


def loaded_round(seed):
    """Config 5 with every host holding at most 1 cpu free: a host takes one or two tasks, so the
    longest zero-cost chains need more than the frontier walk's 1024-host window and fall back to
    candidate lists (the list-walk cliff of the default line's engine)."""
    from pivot_place import synthetic
    r = synthetic.make_round(MODES["ca_bf"], DEFAULT_H, DEFAULT_T, seed=seed)
    r.avail[0] = np.minimum(r.avail[0], 1.0)
    return r


def extra_workloads(eng, args, skip_mode):
    """Config 5 (1M x 10k) for the other policies, a loaded config-5 cost_aware best-fit round,
    config 3 (100k x 1k) and config 4 at its per-GPU size (512 scenarios x 1000 hosts x 1000
    tasks, one pvt_place_batch launch) for all five; each timed on the same engine, with its
    kernel-class times, and checked against the oracle."""
    from oracle import oracle
    from pivot_place import synthetic
    out = {}
    steps, warm = max(1, min(args.steps, 5)), 1
    jobs = [("c5_%s" % m, MODES[m], DEFAULT_H, DEFAULT_T, None) for m in MODES if m != skip_mode]
    jobs.append(("c5_ca_bf_loaded", MODES["ca_bf"], DEFAULT_H, DEFAULT_T, "loaded"))
    jobs += [("c3_%s" % m, MODES[m], 100_000, 1000, None) for m in MODES]
    jobs += [("c4_%s" % m, MODES[m], 1000, 1000, "batch") for m in MODES]
    threads = oracle_threads()
    for tag, mode, H, T, kind in jobs:
        if kind == "batch":
            B = 512
            rounds = [synthetic.make_round(mode, H, T, seed=args.seed + s) for s in range(B)]
            ms, got, ks = time_round(eng, None, steps, warm, batch=rounds)
            ep = eng.epoch_stats()
            cand = float(B) * T * H
            cpu, refs = batch_cpu_baseline(rounds, threads)
            ok = all(same_result(g, x) for g, x in zip(got, refs)) if args.parity else None
        else:
            B = 0
            r = loaded_round(args.seed) if kind == "loaded" else synthetic.make_round(mode, H, T, seed=args.seed)
            ms, got, ks = time_round(eng, r, steps, warm)
            ep = eng.epoch_stats()
            cand = float(T) * H
            cpu, ref = round_cpu_baseline(r, threads, args.extra_cpu_seconds)
            ok = check_parity(got, r, ref) if args.parity else None
        e = {"value": cand / (ms * 1e-3), "ms_per_step": ms, "hosts": H, "tasks": T, "steps": steps,
             "parity": ok, "kernels_ms_per_step": {k: v["ms"] / steps for k, v in ks.items()
                                                   if k in KCLASS_NAMES},
             "kernel_ms_per_step": {k: v["ms"] / steps for k, v in ks["kernels"].items()}}
        if B:
            e["scenarios"] = B
        if mode == MODES["ca_bf"] and not B:
            e["frontier_chains_per_step"] = ep["frontier_chains"]
            e["list_chains_per_step"] = ep["list_chains"]
        variant = "_b%d" % B if B else ("_loaded" if kind == "loaded" else "")
        e["roofline"] = dominant_roofline(mode, H, T, ks, ep, steps, variant=variant,
                                          rounds_per_step=B or 1, warm=warm)
        e.update(step_hbm(mode, H, T, ms, variant))
        e["cpu_baseline"] = cpu
        out[tag] = e
        log("[rank 0] extra %s: %.3e cand/s, %.2f ms, parity %s, roofline %s frac %s, cpu %.3e"
            % (tag, e["value"], ms, ok, e["roofline"].get("kernel"), e["roofline"].get("frac"),
               cpu["value"]))
    return out


def round_cpu_baseline(r, threads, budget_s):
    """CPU baseline of one extra round: the C restatement on all the job's cores and on 1
    thread, both on the same first tasks of the round (the whole round when one thread takes it
    within the budget -- that run is then the parity reference)."""
    v_all, v_one, n, dt_all, dt_one, res = _paired_oracle(r, budget_s, threads)
    value, cores = best_cpu(v_all, threads, v_one)
    out = {"value": value, "unit": "candidates/s", "cores": cores, "kind": "port",
           "value_1thread": v_one, "value_all_cores": v_all, "tasks": n,
           "sample": "oracle/pivot_oracle.c (naive T x H scan, OpenMP host scans) on %s x %d "
                     "hosts: %d threads %.3f s, 1 thread %.2f s; value = the faster"
                     % ("all %d tasks" % n if n >= r.n_tasks else "the first %d tasks" % n,
                        r.n_hosts, threads, dt_all, dt_one)}
    return out, res


def batch_cpu_baseline(rounds, threads):
    """CPU baseline of a scenario batch (config 4): every scenario through the C restatement,
    one scenario per thread on all the job's cores (ctypes releases the GIL), the whole batch;
    then the first scenarios on 1 thread. Returns (baseline, the per-scenario results)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle
    cand = float(sum(r.n_tasks * r.n_hosts for r in rounds))
    t = time.perf_counter()
    with ThreadPoolExecutor(max_workers=max(threads, 1)) as ex:
        refs = list(ex.map(lambda x: oracle.place(x, threads=0), rounds))
    dt_all = max(time.perf_counter() - t, 1e-6)
    n1 = max(1, len(rounds) // 16)
    t = time.perf_counter()
    for x in rounds[:n1]:
        oracle.place(x, threads=0)
    dt_one = max(time.perf_counter() - t, 1e-6)
    c1 = float(sum(r.n_tasks * r.n_hosts for r in rounds[:n1]))
    value, cores = best_cpu(cand / dt_all, threads, c1 / dt_one)
    out = {"value": value, "unit": "candidates/s", "cores": cores, "kind": "port",
           "value_1thread": c1 / dt_one, "value_all_cores": cand / dt_all,
           "sample": "oracle/pivot_oracle.c on all %d scenarios, one scenario per thread over %d "
                     "threads (%.2f s); 1 thread: the first %d scenarios (%.2f s)"
                     % (len(rounds), threads, dt_all, n1, dt_one)}
    return out, refs


def scenario_batch_line(eng, args, rank, world, gloo, B, H=1000, T=1000):
    """BASELINE config 4 as written, on every rank of an N-GPU job: B independent scenarios per
    rank (seeds seed + rank * B + s; H hosts x T tasks each), placed by ONE pvt_place_batch launch
    per step (resident kernel), timed between barriers with the MAX over ranks, no collective on
    the data path (reference fan-out: alibaba/sim.py:187-195, runner.py:13-52). Parity: every rank
    checks its own scenarios against the oracle; the flags are reduced with a MIN. Returns the
    line on rank 0 (None elsewhere)."""
    import torch
    import torch.distributed as dist
    from oracle import oracle
    from pivot_place import synthetic
    mode = MODES[args.mode]
    steps, warm = max(1, min(args.steps, 5)), 1
    rounds = [synthetic.make_round(mode, H, T, seed=args.seed + rank * B + s) for s in range(B)]
    if world > 1:
        dist.barrier()
    ms, got, ks = time_round(eng, None, steps, warm, batch=rounds)   # (this rank's own clock)
    if world > 1:
        dist.barrier()
    ok = all(same_result(g, oracle.place(x)) for g, x in zip(got, rounds)) if args.parity else True
    if world > 1:
        dev = "cpu" if gloo else eng.device
        t = torch.tensor([ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        f = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = bool(f.item())
    if rank != 0:
        return None
    cand = float(B) * world * T * H
    return {"workload": "BASELINE config 4: %d independent scenarios (%d per GPU) x %d hosts x %d "
                        "tasks, %s, one pvt_place_batch launch per GPU per step, scenario-sharded "
                        "(no data-path collective)" % (B * world, B, H, T, POLICY[args.mode]),
            "value": cand / (ms * 1e-3), "unit": "candidates/s", "ms_per_step": ms,
            "n_gpus": world, "scenarios": B * world, "scenarios_per_gpu": B, "hosts": H,
            "tasks": T, "steps": steps, "scaling": "weak", "timing": "max over ranks of each "
            "rank's timed steps, between barriers", "parity": (ok if args.parity else None),
            "parity_scope": "every rank's scenarios vs the oracle (MIN-reduced)",
            "kernels_ms_per_step": {k: v["ms"] / steps for k, v in ks.items() if k in KCLASS_NAMES},
            "kernel_ms_per_step": {k: v["ms"] / steps for k, v in ks["kernels"].items()},
            "roofline": dominant_roofline(mode, H, T, ks, eng.epoch_stats(), steps,
                                          variant="_b%d" % B, rounds_per_step=B, warm=warm)}


# ---------------------------------------------------------------------------- roofline
# PMC profiles (tools/pmc_profile.py, collected into profiles/pmc_index.json by
# tools/pmc_index.py) are used only for the binary they were collected on: each entry carries the
# sha256 of libpivot_place.so, and an entry of another binary leaves the roofline's counters null.
PMC_INDEX = os.path.join(ROOT, "profiles", "pmc_index.json")
SIMDS, CUS = 1024, 256
SHADER_HZ = 2.4e9
ISSUE_CYCLES = 4          # one wave issues at most one instruction per 4 cycles
# Waves per workgroup of the one-workgroup-per-walk kernels (pvt_zwalk.hip ZW_THREADS, pvt_lwalk.hip,
# pvt_walk.hip WALK_THREADS, pvt_opp.hip OPP_NW). Their PMC instruction counts cover every wave,
# so the issue peak is that of min(waves, 4 SIMDs) waves of one CU.
WALK_WAVES = {"zwalk_kernel": 4, "lwalk_kernel": 1, "commit_kernel": 8, "opp_commit_kernel": 16}
LDS_DEP_CYCLES = 50       # one dependent LDS round trip (MI355X_MICROARCH.md constants table)
INSTS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
         "SQ_INSTS_VMEM_WR")
_SHA = []


def lib_sha256():
    if not _SHA:
        with open(LIB, "rb") as f:
            _SHA.append(hashlib.sha256(f.read()).hexdigest())
    return _SHA[0]


def pmc_entry(mode, H, T, kernel, variant=""):
    """(PMC entry, note): the counter profile of ``kernel`` on this config (variant "_b512": a
    512-scenario batch of H x T rounds; "_loaded": the loaded config-5 round), if it was
    collected on THIS binary."""
    name = [k for k, v in MODES.items() if v == mode][0]
    key = "%s_%d_%d%s:%s" % (name, H, T, variant, kernel)
    try:
        with open(PMC_INDEX) as f:
            e = json.load(f).get("entries", {}).get(key)
    except (OSError, ValueError):
        return None, "no PMC index (tools/pmc_index.py)"
    if e is None:
        return None, "no PMC profile of %s for this config (tools/pmc_profile.py)" % key
    if e.get("lib_sha256") != lib_sha256():
        return None, ("the PMC profile of %s was collected on another build (lib sha256 %s..., "
                      "this %s...): counters not used" % (key, str(e.get("lib_sha256"))[:12],
                                                           lib_sha256()[:12]))
    return e, None


def score_roofline(mode, H, T, k, kernel, variant=""):
    """A parallel pass (streaming score, band score, count pass, merge or the resident kernel):
    its PMC per-launch work (VALU busy cycles, LDS-array cycles, DRAM bytes) over the launch time
    measured here with HIP events on the launch's stream (``k``: that kernel's own timing); the
    bound is the most utilised resource. The SURVEY §8(d) 36 / 32 B per logical candidate is
    kept as hbm_equivalent_*: what a per-task streaming scan would move, not what moves."""
    from pivot_place import _abi
    launches = max(k["launches"], 1)
    avg_ms = k["ms"] / launches
    out = {"kernel": kernel, "avg_launch_ms": avg_ms, "launches": k["launches"],
           "candidates_per_launch": k["candidates"] / launches,
           "hbm_equivalent_GBs": (k["bytes"] / launches / (avg_ms * 1e-3) / 1e9) if avg_ms > 0 else 0.0,
           "hbm_equivalent_bytes_per_candidate": _abi.BYTES_PER_CANDIDATE[mode],
           "bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None}
    pmc, note = pmc_entry(mode, H, T, kernel, variant)
    if pmc is None or avg_ms <= 0:
        out["note"] = note or "no launch timed"
        return out
    t = avg_ms * 1e-3
    res = {"valu": (pmc["valu_busy_cycles_per_launch"] / t, SIMDS * SHADER_HZ, "SIMD-cycles/s"),
           "lds": (pmc["lds_busy_cycles_per_launch"] / t, CUS * SHADER_HZ, "CU-LDS-cycles/s"),
           "hbm": (pmc["hbm_bytes_per_launch"] / t / 1e9, HBM_PEAK_GBS, "GB/s")}
    bound = max(res, key=lambda x: res[x][0] / res[x][1])
    a, p, u = res[bound]
    out.update({"bound": bound, "achieved": a, "peak": p, "unit": u, "frac": a / p,
                "traffic": pmc["hbm_bytes_per_launch"],
                "utilisation": {x: v[0] / v[1] for x, v in res.items()},
                "pmc_source": pmc.get("source"), "pmc_lib_sha256": pmc.get("lib_sha256"),
                "pmc_profiled_launch_ms": pmc.get("profiled_duration_ms")})
    return out


def walk_roofline(mode, H, T, c, ep, steps, kernel="zwalk_kernel", variant="", rounds_per_step=1,
                  warm=0):
    """A sequential walk (the frontier walk, the list commit walk, the opportunistic walk): each
    task reads the capacities the previous commit wrote, so the chain is one wave's dependent
    instruction stream, bounded by issue: at most one instruction per 4 cycles per wave
    (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost, one wave'), for the min(waves, 4)
    waves of the walk's workgroup (the helper waves' instructions are counted too). achieved =
    instructions per task (PMC, every wave of the kernel, over the round's tasks) x tasks per
    second on the critical path (the longest frontier chain, or every task for the
    one-workgroup walks); peak = min(waves, 4) x 2.4 GHz / 4. The latency floor (one dependent
    LDS round trip per task) is beside it. ``c``: the walk kernel's own HIP-event timing."""
    ms = c["ms"] / max(steps, 1)
    # epoch chains (cost_aware best-fit) run side by side: the longest chain per epoch is the
    # critical path (engine counter of the last round, summed over its epochs)
    # (cost_aware first-fit's zero-key epochs walk their chains side by side as well)
    longest = (ep.get("longest_chain_tasks", 0)
               if kernel in ("zwalk_kernel", "commit_kernel") and mode in (MODES["ca_bf"], MODES["ca_ff"])
               else 0)
    if longest <= 0:
        longest = T                      # every task of the round on one walk after another
    issue_waves = min(4, WALK_WAVES.get(kernel, 1))
    out = {"kernel": kernel, "bound": "issue", "unit": "instructions/s (one workgroup)",
           "traffic": None, "walk_ms_per_step": ms, "critical_path_tasks": longest,
           "peak_basis": "one instruction per %d cycles per wave at %.1f GHz, %d wave(s) of %d "
                         "in the workgroup issuing (one per SIMD)"
                         % (ISSUE_CYCLES, SHADER_HZ / 1e9, issue_waves, WALK_WAVES.get(kernel, 1)),
           "achieved": None, "peak": None, "frac": None}
    if ms <= 0:
        return out
    tasks_per_s = longest / (ms * 1e-3)
    out["cycles_per_task"] = SHADER_HZ / tasks_per_s
    out["latency_floor"] = {"peak_tasks_per_s": SHADER_HZ / LDS_DEP_CYCLES,
                            "achieved_tasks_per_s": tasks_per_s,
                            "frac": tasks_per_s / (SHADER_HZ / LDS_DEP_CYCLES)}
    pmc, note = pmc_entry(mode, H, T, kernel, variant)
    if pmc is None:
        out["note"] = note
        return out
    cnt = pmc["counters_per_launch"]
    launches = float(pmc.get("launches_per_round", 1.0))
    ipt = sum(cnt.get(k, 0.0) for k in INSTS) * launches / max(T, 1)
    out.update({"instructions_per_task": ipt, "pmc_source": pmc.get("source"),
                "pmc_lib_sha256": pmc.get("lib_sha256"),
                "issue_active_frac_pmc": cnt["SQ_ACTIVE_INST_ANY"] / cnt["SQ_WAVE_CYCLES"],
                "wait_frac_pmc": cnt["SQ_WAIT_ANY"] / cnt["SQ_WAVE_CYCLES"],
                "waves_per_launch": cnt.get("SQ_WAVES")})
    traffic = 2.0 * cnt.get("FETCH_SIZE", 0.0) * 1024 + cnt.get("WRITE_SIZE", 0.0) * 1024
    out["traffic"] = traffic if traffic > 0 else None
    achieved = ipt * tasks_per_s
    peak = SHADER_HZ / ISSUE_CYCLES * issue_waves
    # (frac_one_wave: against a single wave's issue, as if the helper waves' instructions were
    # the walker's -- above 1 when the helpers do much of the work, as in the opportunistic walk)
    out.update({"achieved": achieved, "peak": peak, "frac": achieved / peak,
                "frac_one_wave": achieved / (SHADER_HZ / ISSUE_CYCLES)})
    if WALK_WAVES.get(kernel, 1) > 4:
        # A walker with helper waves that spin while it walks (opportunistic, scout list walk):
        # the instruction count includes the spin loops, so instructions / peak would overstate
        # the useful issue. frac is then the PMC issue-active fraction of the wave cycles.
        out.update({"frac_instructions": out["frac"], "frac": out["issue_active_frac_pmc"],
                    "achieved": out["issue_active_frac_pmc"] * peak,
                    "frac_basis": "SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (PMC issue-active "
                                  "fraction; instruction counts include the helpers' spin waits)"})
    return out


def dominant_kernel(eng, step, n=2):
    """(name, share of the timed kernels' device time, {name: ms per step}) of the kernel that
    takes the most device time over n untimed steps with every named kernel timed. The timed
    steps then record events around that kernel only (each event pair idles the stream a few
    microseconds: timing every named kernel cost 0.33 ms of a 2.74 ms vbp best-fit step)."""
    eng.reset_kstats()
    eng.set_profiling(2)
    for _ in range(n):
        step()
    import torch
    torch.cuda.synchronize()
    eng.set_profiling(False)
    kt = kernel_times(eng)
    eng.reset_kstats()
    if not kt:
        return None, None, {}
    name = max(kt, key=lambda k: kt[k]["ms"])
    share = kt[name]["ms"] / max(sum(v["ms"] for v in kt.values()), 1e-12)
    return name, share, {k: v["ms"] / n for k, v in kt.items()}


def dominant_roofline(mode, H, T, ks, ep, steps, variant="", rounds_per_step=1, warm=0):
    """The roofline of the kernel that takes the most device time in the timed steps (HIP events
    per kernel), with the PMC profile of that kernel on this config and this binary."""
    kt = ks.get("kernels") or {}
    if not kt:
        return {"kernel": None, "bound": None, "achieved": None, "peak": None, "frac": None,
                "traffic": None, "note": "no kernel of the path was timed"}
    kernel = max(kt, key=lambda n: kt[n]["ms"])
    share = kt[kernel]["ms"] / max(sum(v["ms"] for v in kt.values()), 1e-12)
    if ks.get("dominant_share") is not None:      # (the timed steps timed this kernel only)
        share = ks["dominant_share"]
    if kernel in WALK_KERNELS:
        out = walk_roofline(mode, H, T, kt[kernel], ep, steps, kernel, variant, rounds_per_step, warm)
    else:
        out = score_roofline(mode, H, T, kt[kernel], kernel, variant)
    out["dominant_share_of_timed_kernels"] = share
    return out


def step_hbm(mode, H, T, ms_per_step, variant=""):
    """The metric's HBM half as a measured figure: the HBM bytes of one whole step -- every
    dispatch of the round, from rocprofv3 FETCH_SIZE / WRITE_SIZE passes of THIS binary
    (tools/pmc_step.py, indexed as "<config>:step") -- over the step time measured here. Per GPU.
    Returns {} when no profile of this binary covers the config."""
    pmc, note = pmc_entry(mode, H, T, "step", variant)
    if pmc is None or ms_per_step <= 0:
        return {"hbm_GBs_measured": None, "hbm_note": note}
    b = pmc["hbm_bytes_per_step"]
    gbs = b / (ms_per_step * 1e-3) / 1e9
    return {"hbm_GBs_measured": gbs, "hbm_frac_measured": gbs / HBM_PEAK_GBS,
            "hbm_bytes_per_step": b, "hbm_pmc_source": pmc.get("source")}


# ---------------------------------------------------------------------------- the printed line
# The driver parses a bounded stdout tail: round 4's 33 KB line (every extra's full roofline and
# CPU-baseline dicts) was not parsed at all. The line keeps the contract's fields and a cut of each
# extra; the full dicts go to FULL_OUT, whose path the line names.
LINE_MAX = 8000
FULL_OUT = os.path.join(ROOT, "gpurun_out", "bench_full.json")
ROOF_TOP = ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "pmc_source",
            "cycles_per_task", "critical_path_tasks", "issue_active_frac_pmc", "frac_basis",
            "dominant_share_of_timed_kernels", "note")
ROOF_EXTRA = ("kernel", "bound", "achieved", "peak", "frac", "traffic", "pmc_source")
EXTRA_KEYS = ("value", "ms_per_step", "ms_per_round", "parity", "n_gpus", "scenarios",
              "engine_seconds", "max_rounds_per_launch", "hbm_GBs_measured", "error")
CPU_KEYS = ("value", "value_1thread", "tasks", "cores", "engine_seconds")
TOP_DROP = ("extra", "kernels_ms_per_step", "kernel_ms_per_step")


def _sig(x, n=4):
    """Floats to n significant digits (non-finite -> null: the line must be strict JSON)."""
    if isinstance(x, bool) or not isinstance(x, float):
        if isinstance(x, dict):
            return {k: _sig(v, n) for k, v in x.items()}
        if isinstance(x, (list, tuple)):
            return [_sig(v, n) for v in x]
        return x
    if x != x or x in (float("inf"), float("-inf")):
        return None
    return float("%.*g" % (n, x))


def _dumps(x):
    """Compact strict JSON with floats in their shortest %g form (3.512e+13, not
    35120000000000.0): _sig has already rounded them."""
    if isinstance(x, dict):
        return "{" + ",".join(json.dumps(str(k)) + ":" + _dumps(v) for k, v in x.items()) + "}"
    if isinstance(x, (list, tuple)):
        return "[" + ",".join(_dumps(v) for v in x) + "]"
    if isinstance(x, float) and not isinstance(x, bool):
        if x != x or x in (float("inf"), float("-inf")):
            return "null"
        r = repr(x)
        g = "%.17g" % x
        g = min((("%.*g" % (n, x)) for n in range(1, 18) if float("%.*g" % (n, x)) == x),
                key=len, default=g)
        return g if len(g) < len(r) else r
    return json.dumps(x)


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def short_source(path, name=None, kernel=None):
    """profiles/<tag>/pmc_<tag>_<stem>.json -> "<tag>:<stem>", or just "<tag>" when the stem is
    "<extra name>_<kernel>" (tools/pmc_all.sh's naming; PMC_SOURCE_FORM in the line)."""
    if not isinstance(path, str):
        return path
    d, f = os.path.split(path)
    tag = os.path.basename(d)
    pre = "pmc_%s_" % tag
    if f.startswith(pre) and f.endswith(".json"):
        stem = f[len(pre):-5]
        return tag if stem == "%s_%s" % (name, kernel) else "%s:%s" % (tag, stem)
    return path


PMC_SOURCE_FORM = ("extra roofline pmc_source: '<tag>' = profiles/<tag>/pmc_<tag>_<extra>_<kernel>"
                   ".json, '<tag>:<stem>' = profiles/<tag>/pmc_<tag>_<stem>.json")


def compact_extra(e, level=0, name=None):
    """One extra line cut to what the judge reads: value, time, parity, roofline, CPU baseline,
    measured step HBM GB/s. level 1 drops the PMC source paths, level 2 keeps only fractions."""
    c = _pick(e, EXTRA_KEYS)
    if "hbm_GBs_measured" in c:
        c["hbm_GBs"] = c.pop("hbm_GBs_measured")
    rl = e.get("roofline")
    if isinstance(rl, dict):
        keys = ROOF_EXTRA if level == 0 else ROOF_EXTRA[:-1] if level == 1 else ("kernel", "frac")
        c["roofline"] = _pick(rl, keys)
        if "pmc_source" in c["roofline"]:
            c["roofline"]["pmc_source"] = short_source(c["roofline"]["pmc_source"], name,
                                                       c["roofline"].get("kernel"))
    cb = e.get("cpu_baseline")
    if isinstance(cb, dict):
        c["cpu_baseline"] = _pick(cb, CPU_KEYS if level < 2 else ("value",))
    if isinstance(c.get("roofline"), dict):
        c["roofline"] = {k: v for k, v in c["roofline"].items() if v is not None}
    return _sig(c, 3)


def compact_line(out, full_path=None):
    """The one JSON line bench.py prints: every top-level field of ``out`` (the roofline cut to
    ROOF_TOP) and each extra cut by compact_extra, at most LINE_MAX bytes."""
    top = {k: v for k, v in out.items() if k not in TOP_DROP}
    if isinstance(top.get("roofline"), dict):
        top["roofline"] = _pick(top["roofline"], ROOF_TOP)
    for k, v in list(top.items()):
        if k not in ("value", "ms_per_step"):
            top[k] = _sig(v, 6)
    extra = out.get("extra") or {}
    if full_path:
        top["full_results"] = full_path
    if extra:
        top["pmc_source_form"] = PMC_SOURCE_FORM
    for level in (0, 1, 2, 3):
        line = dict(top)
        if extra and level < 3:
            line["extra"] = {k: compact_extra(v, level, k) for k, v in extra.items()}
        elif extra:
            line["extra"] = {k: _sig(_pick(v, ("value", "parity")), 4) for k, v in extra.items()}
        s = _dumps(line)
        if len(s) <= LINE_MAX:
            return s
    return s


def write_full(out, path=FULL_OUT):
    """The full result (every extra's kernel times, roofline and CPU-baseline dicts) as a file;
    returns its path relative to the repository root (None if it cannot be written)."""
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(_sig(out, 10), f, indent=1)
        return os.path.relpath(path, ROOT)
    except OSError:
        return None


# ---------------------------------------------------------------------------- configs 1 and 2
# BASELINE configs 1 and 2 run the reference's own simulator (alibaba/sim.py), which needs the
# reference sources and SimPy: the box has neither. tests/golden/sim_*.json.gz hold every
# schedule() round of those simulations (tests/golden/make_golden_sim.py, recorded in the build
# container): the snapshot, the ready queue with its predecessor placements, and the reference's
# placements. They are replayed here through the drop-in policy classes (pivot_place.policies)
# exactly as the reference's round loop calls them (scheduler/__init__.py:100-103): per round
# _update_resource_info() and schedule(ready tasks), timed end to end -- grouping, anchors (a3 on
# the GPU), marshalling, H2D, kernels, D2H and applying the results. Beside it the same replay
# with the C restatement behind the engine contract, on 1 thread and on all the job's cores.
REPLAYS = ("sim_c1_cost_aware", "sim_c2a1000_cost_aware", "sim_c2a1000_opportunistic",
           "sim_c2a1000_vbp_ff")


_REPLAY_CACHE = {}


class _OracleEngine:
    """The C restatement behind PlacementEngine's place() / anchor() contract (CPU baseline)."""

    def __init__(self, threads):
        self.threads = threads

    def place(self, r):
        from oracle import oracle
        return oracle.place(r, threads=self.threads)

    def anchor(self, off, lst, zone, inst_host=None):
        from oracle import oracle
        mode, az, rc = oracle.anchor(off, lst, zone, len(zone), inst_host)
        if rc != 0:
            raise RuntimeError("oracle anchor rc %d" % rc)
        return mode, az


def _replay(name, engine):
    """One pass over a recorded simulation's rounds: (seconds spent in the rounds, candidates,
    rounds, placements equal to the reference's in every round)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import fakes
    import golden_io
    from pivot_place import policies
    classes = {"cost_aware": policies.CostAwareGlobalScheduler,
               "opportunistic": policies.OpportunisticGlobalScheduler,
               "vbp_ff": policies.FirstFitGlobalScheduler, "vbp_bf": policies.BestFitGlobalScheduler}
    tr, cases = _REPLAY_CACHE.get(name) or _REPLAY_CACHE.setdefault(name, golden_io.sim_rounds(name))
    cluster, _ = fakes.build(cases[0])               # one cluster, its hosts set per round
    cls = classes[tr["policy"]]
    sched = cls(None, cluster, seed=tr["seed"], **tr["kwargs"])
    sched.engine = engine
    hidx = {h.id: i for i, h in enumerate(cluster.hosts)}
    cand, ok, secs = 0.0, True, 0.0
    for case in cases:
        fakes.refresh(cluster, case)                 # (the simulation's state this round)
        tasks = fakes.build_tasks(case, cluster)
        t0 = time.perf_counter()
        sched._update_resource_info()
        sched.schedule(list(tasks))
        secs += time.perf_counter() - t0
        cand += float(len(tasks)) * len(cluster.hosts)
        got = [-1 if t.placement is None else hidx[t.placement] for t in tasks]
        ok = ok and got == case["runs"][0]["placement"]
    return secs, cand, len(cases), ok, tr


def round_trip_floor_ms(eng, reps=200):
    """The least time one drop-in round can take on this engine: a pvt_place of a 1-host x
    1-task round from host arrays (H2D, one launch, D2H, one synchronisation), median of reps."""
    from pivot_place import synthetic
    r = synthetic.make_round(MODES["vbp_ff"], 1, 1, seed=1)
    for _ in range(20):
        eng.place(r)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        eng.place(r)
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e3


LOCKSTEP = ("sim_c2_cost_aware", "sim_c2_opportunistic", "sim_c2_vbp_ff",
            "sim_c2a1000_cost_aware", "sim_c2a1000_opportunistic", "sim_c2a1000_vbp_ff")


class _BatchOracleEngine(_OracleEngine):
    """The C restatement behind the batched engine contract (LockstepDriver)."""

    def place_batch(self, rounds):
        from oracle import oracle
        return [oracle.place(r, threads=self.threads) for r in rounds]


def lockstep_workload(eng):
    """BASELINE config 2 as a sweep through the lock-step driver (pivot_place.lockstep, §8(f)
    rank 2): the recorded reference simulations at 1000 hosts (two app counts x the three
    schedulers) run side by side, each in its own thread behind the drop-in policy classes;
    whenever every live simulation waits on the engine, their rounds go to one pvt_place_batch
    per policy mode and their anchors to one pvt_anchor. Every round is compared with the
    reference's. The same driver over the C restatement is timed beside it (1 thread)."""
    from pivot_place.lockstep import LockstepDriver

    def run(engine):
        driver = LockstepDriver(engine)
        t = time.perf_counter()
        out = driver.run([lambda e, n=n: _replay(n, e) for n in LOCKSTEP])
        return time.perf_counter() - t, out, driver.stats

    secs, out, st = run(eng)              # (the replay lines before it warmed the tables up)
    csecs, cout, cst = run(_BatchOracleEngine(0))
    rounds = sum(o[2] for o in out)
    cand = sum(o[1] for o in out)
    ok = all(o[3] for o in out)
    return {"workload": "config 2 sweep: %d recorded reference simulations (1000 hosts; %s) run "
                        "side by side through the lock-step driver, drop-in policy classes, every "
                        "waiting round of every policy in one pvt_place_host_batch per tick "
                        "(cost_aware groupings and anchor draws included)"
                        % (len(LOCKSTEP), ", ".join(n[4:] for n in LOCKSTEP)),
            "simulations": len(LOCKSTEP), "rounds": rounds, "candidates": cand,
            "value": cand / secs, "unit": "candidates/s", "seconds": secs,
            "ms_per_round": secs * 1e3 / rounds, "parity": bool(ok),
            "ticks": st["batches"], "place_calls": st["place_calls"],
            "place_launches": st["place_launches"], "anchor_calls": st["anchor_calls"],
            "anchor_launches": st["anchor_launches"],
            "max_rounds_per_launch": st["max_rounds_per_launch"],
            "engine_seconds": st["serve_s"], "engine_ms_per_round": st["serve_s"] * 1e3 / rounds,
            "note": "wall time of the whole lock-step run: the recorded rounds are rebuilt from "
                    "their fixtures in every simulation thread (Python, under one interpreter "
                    "lock) and only the engine calls are batched; engine_seconds is the time the "
                    "driver spent serving the batched calls",
            "cpu_baseline": {"value": cand / csecs, "unit": "candidates/s", "cores": 1,
                             "kind": "port", "seconds": csecs, "engine_seconds": cst["serve_s"],
                             "parity": bool(all(o[3] for o in cout)),
                             "sample": "the same lock-step run with the C restatement behind the "
                                       "batched engine contract (1 thread)"}}


def replay_workloads(eng):
    out = {}
    threads = oracle_threads()
    floor = round_trip_floor_ms(eng)
    for name in REPLAYS:
        try:
            _replay(name, eng)                               # warm-up (tables, scratch)
            secs, cand, nr, ok, tr = _replay(name, eng)
            c1, _, _, ok1, _ = _replay(name, _OracleEngine(0))
            ca, _, _, oka, _ = _replay(name, _OracleEngine(threads))
        except Exception as e:                               # (a missing fixture is reported)
            out["replay_" + name] = {"error": "%s: %s" % (type(e).__name__, e)}
            continue
        cfg = "c1" if name.startswith("sim_c1") else "c2"
        out["%s_replay_%s" % (cfg, name[4:].split("_", 1)[1])] = {
            "workload": "%s: every schedule() round of the recorded reference simulation (%d "
                        "hosts, %d apps, %s %s), through the drop-in policy class"
                        % (name, tr["n_hosts"], tr["n_apps"], tr["policy"], tr["kwargs"]),
            "rounds": nr, "candidates": cand, "value": cand / secs, "unit": "candidates/s",
            "seconds": secs, "ms_per_round": secs * 1e3 / nr, "parity": bool(ok),
            "cpu_1thread": {"seconds": c1, "value": cand / c1, "parity": bool(ok1)},
            "cpu_all": {"seconds": ca, "value": cand / ca, "cores": threads, "parity": bool(oka)},
            "cpu_baseline": {"value": max(cand / ca, cand / c1), "unit": "candidates/s",
                             "cores": threads if ca <= c1 else 1,
                             "kind": "port", "value_1thread": cand / c1, "value_all_cores": cand / ca,
                             "sample": "the same %d recorded rounds through the same drop-in "
                                       "policy class with the C restatement behind the engine "
                                       "contract (%d threads and 1 thread; value = the faster)"
                                       % (nr, threads)},
            "roofline": {"kernel": None, "bound": "round trip", "unit": "rounds/s",
                         "achieved": nr / secs, "peak": 1e3 / floor, "frac": floor / (secs * 1e3 / nr),
                         "traffic": None, "floor_ms_per_round": floor,
                         "peak_basis": "one synchronous pvt_place of a 1-host x 1-task round from "
                                       "host arrays on this engine (H2D, one launch, D2H, one "
                                       "synchronisation; median of 200): a round of these sizes "
                                       "(~1e5 candidates) is bound by the round trip and the host "
                                       "work around it, not by a kernel"},
            "reference_sim_wall_s": tr["e2e"].get("reference_wall_s"),
            "note": "times the whole drop-in round (Python grouping / marshalling included); "
                    "reference_sim_wall_s is the reference's whole simulation in the build "
                    "container (SimPy events included), for scale only"}
        log("[rank 0] replay %s: %d rounds, %.3f s (%.2f ms/round) vs CPU 1T %.3f s, %d T %.3f s, "
            "parity %s" % (name, nr, secs, secs * 1e3 / nr, c1, threads, ca, ok))
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
    dev = local
    gloo = world > 1 and args.dist_backend == "gloo"
    if world > 1:
        # (gloo: ranks may share the card -- a rehearsal of the multi-rank path on one GPU)
        dev = local % max(torch.cuda.device_count(), 1) if gloo else local
        torch.cuda.set_device(dev)
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    mode = MODES[args.mode]
    H, T = args.hosts, args.tasks
    log("[rank %d] building synthetic round: %s, H=%d T=%d" % (rank, args.mode, H, T))
    hosts_sharded = args.shard == "hosts" and not args.batch
    B = max(args.batch, 0)
    eng = PlacementEngine(dev, window=args.window)
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
    # each step places the same snapshot: a single round's reset restores the hosts the last
    # step placed on (pvt_restore_hosts, the only capacities a round changes; the parity check
    # below is on the last timed step, so an incomplete reset would show there)
    reset = step_reset(eng, dr, bool(B or hosts_sharded))

    for i in range(args.warmup):
        reset()
        run(dr)
    torch.cuda.synchronize()
    stats = eng.last_stats()
    ep = eng.epoch_stats()
    placed = int(((dr.placement_of(0) if B else dr.placement[:T]) >= 0).sum().item())
    log("[rank %d] warmup done: %d/%d placed, windows=%d refills=%d"
        % (rank, placed, T, stats["windows"], stats["refills"]))

    # events around the dominant kernel only (dominant_kernel: found over two untimed steps with
    # every named kernel timed); BENCH_PROF=0: no events at all, for A/B of their cost (the
    # roofline then has no kernel time), BENCH_PROF=1: every launch
    prof = int(os.environ.get("BENCH_PROF", "2"))
    dom, dom_share, dom_kms = dominant_kernel(eng, lambda: (reset(), run(dr))) if prof == 2 else (None, None, {})
    eng.reset_kstats()
    eng.set_profiling(prof, kernel=dom)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        reset()
        run(dr)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_profiling(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if gloo else eng.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    cand_per_step = float(T) * H * (1 if hosts_sharded else world) * (B if B else 1)
    value = cand_per_step / (elapsed / args.steps)
    ks = kstats_all(eng)
    ks["kernels"] = kernel_times(eng)
    ks["dominant_share"] = dom_share

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
                "parallelism": ("host-sharded x%d (per-step all-gather of window candidates / "
                                "candidate lists)" % world if hosts_sharded else
                                "scenario-sharded x%d (no data-path collective)" % world),
                "dist_backend": (("gloo" if gloo else "nccl") if world > 1 else None),
            },
            "roofline": dominant_roofline(mode, H, T, ks, ep, args.steps,
                                          variant=("_b%d" % B) if B else "",
                                          rounds_per_step=B or 1, warm=args.warmup),
            "kernels_ms_per_step": {k: v["ms"] / args.steps for k, v in ks.items() if k in KCLASS_NAMES},
            "kernel_ms_per_step": {k: v["ms"] / args.steps for k, v in ks["kernels"].items()},
            "walk_us_per_task": (ks["commit"]["ms"] * 1e3 / args.steps / max(T * (B or 1), 1)
                                 if not B and ks["commit"]["ms"] > 0 else None),
            "windows_per_step": stats["windows"], "refills_per_step": stats["refills"],
            "epochs_per_step": ep["epochs"], "segments_per_step": ep["segments"],
            "rejected_segments_per_step": ep["rejected"],
            "frontier_chains_per_step": ep.get("frontier_chains"),
            "list_chains_per_step": ep.get("list_chains"),
        }
        out.update(step_hbm(mode, H, T, ms_per_step, ("_b%d" % B) if B else ""))
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
        if args.replay == 1 or (args.replay < 0 and default and args.extra != 0):
            out.setdefault("extra", {}).update(replay_workloads(eng))
            try:
                out["extra"]["c2_lockstep"] = lockstep_workload(eng)
            except Exception as e:                       # (a missing fixture is reported)
                out["extra"]["c2_lockstep"] = {"error": "%s: %s" % (type(e).__name__, e)}
            log("[rank 0] lockstep: %s" % {k: v for k, v in out["extra"]["c2_lockstep"].items()
                                           if k not in ("workload", "cpu_baseline")})
    if world > 1 and args.c4_batch > 0 and not B:
        # (every rank: the barriers and the MAX / MIN reductions are collective)
        c4 = scenario_batch_line(eng, args, rank, world, gloo, args.c4_batch)
        if rank == 0:
            out.setdefault("extra", {})["c4_scenarios_%s_x%d" % (args.mode, world)] = c4
            log("[rank 0] config 4 x%d: %.3e cand/s, %.2f ms, parity %s"
                % (world, c4["value"], c4["ms_per_step"], c4["parity"]))
    if rank == 0:
        print(compact_line(out, write_full(out)), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
