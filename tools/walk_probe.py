#!/usr/bin/env python3
"""Whole-round probe for PMC counter runs and hang diagnosis: pvt_place on one synthetic round,
`--reps` times, with the window pipeline on or off, printing a line per rep (so a run that
stalls shows where). Exits non-zero if the engine reports an error (e.g. a hand-off timeout).

    python tools/walk_probe.py --mode ca_bf --hosts 100000 --tasks 2000 --pipeline 0 --reps 2
    python tools/walk_probe.py --mode ca_bf --hosts 1000 --tasks 1000 --batch 512 --reps 2
    python tools/walk_probe.py --mode ca_bf --hosts 1000000 --tasks 10000 --loaded 1 --reps 2

--batch B: the config-4 shape, B scenarios (seeds seed + s) in one pvt_place_batch per rep.
--loaded 1: bench.py's loaded config-5 round (every host capped at 1 free cpu).
--marker 1: a marker kernel before every rep (tools/pmc_step.py: HBM bytes of a whole step).
The shapes and the per-step reset are exactly those of bench.py's lines (bench.step_reset: a
single round restores the hosts the previous rep placed on, a batch copies its snapshot back),
so a PMC profile of the probe prices the launches bench.py times
(tests/test_gpu_restore.py::test_walk_probe_step_is_bench_step).
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]

MODES = {"ca_ff": 0, "ca_bf": 1, "opp": 2, "vbp_ff": 3, "vbp_bf": 4}


def probe_step(eng, dr, run, batched):
    """One rep: bench.py's step (its reset, then the placement)."""
    from bench import step_reset
    reset = step_reset(eng, dr, batched)

    def step():
        reset()
        run(dr)
    return step


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="ca_bf", choices=sorted(MODES))
    p.add_argument("--hosts", type=int, default=100_000)
    p.add_argument("--tasks", type=int, default=2000)
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--pipeline", type=int, default=1)
    p.add_argument("--window", type=int, default=0)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--batch", type=int, default=0)
    p.add_argument("--loaded", type=int, default=0)
    p.add_argument("--marker", type=int, default=0,
                   help="1: a one-element bitwise_not_ kernel before every rep (tools/pmc_step.py "
                        "splits the dispatch list at these markers)")
    a = p.parse_args()
    import numpy as np
    import torch
    from pivot_place import _abi, synthetic
    from pivot_place.engine import DeviceRound, PlacementEngine
    from pivot_place.engine import DeviceBatch
    eng = PlacementEngine(0, window=a.window)
    eng.set_pipeline(bool(a.pipeline))
    if a.batch:
        rounds = [synthetic.make_round(MODES[a.mode], a.hosts, a.tasks, seed=a.seed + s)
                  for s in range(a.batch)]
        dr, run = DeviceBatch(rounds, eng.device), eng.run_batch
    else:
        r = synthetic.make_round(MODES[a.mode], a.hosts, a.tasks, seed=a.seed)
        if a.loaded:
            r.avail[0] = np.minimum(r.avail[0], 1.0)
        if a.hosts > _abi.PVT_RESIDENT_MAX_HOSTS or a.tasks > _abi.PVT_RESIDENT_MAX_TASKS:
            eng.set_resident(0)
        dr, run = DeviceRound(r, eng.device), eng.run
    eng.reset_kstats()
    eng.set_profiling(True)
    mark = torch.zeros(1, dtype=torch.int64, device=eng.device) if a.marker else None
    step = probe_step(eng, dr, run, bool(a.batch))
    for rep in range(a.reps):
        if mark is not None:
            mark.bitwise_not_()
        t = time.perf_counter()
        step()
        torch.cuda.synchronize()
        st = eng.last_stats()
        print("walk probe rep %d: mode %s H=%d T=%d batch=%d loaded=%d pipeline=%d  %.2f ms  "
              "windows=%d refills=%d" % (rep, a.mode, a.hosts, a.tasks, a.batch, a.loaded,
                                         a.pipeline, (time.perf_counter() - t) * 1e3,
                                         st["windows"], st["refills"]), flush=True)
    eng.set_profiling(False)
    k = eng.kstats(_abi.PVT_K_COMMIT)
    print("commit launches=%d avg %.3f ms" % (k["launches"], k["ms"] / max(k["launches"], 1)),
          flush=True)
    for name in ("resident_kernel", "zwalk_kernel", "lwalk_kernel", "opp_commit_kernel"):
        k = eng.kernel_kstats(name)
        if k["launches"]:
            print("%s launches=%d avg %.4f ms" % (name, k["launches"], k["ms"] / k["launches"]),
                  flush=True)


if __name__ == "__main__":
    main()
