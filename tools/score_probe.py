#!/usr/bin/env python3
"""Score-pass probe for PMC counter runs: launches only the hot kernel (no commit walk).

Runs the first window of a synthetic round through the sharded entry points with world = 1
(pvt_shard_begin + pvt_shard_score: order, score_kernel, merge, pack), `--reps` times. The
score kernel is the same one pvt_place launches; its window here is the full 1024 tasks x H
hosts. Used by tools/pmc_traffic.py, because counter collection serialises dispatches and the
commit walk (a single 160 KiB-LDS workgroup with intra-workgroup spin hand-offs) does not run
to completion under it.

    python tools/score_probe.py --mode ca_bf --hosts 1000000 --tasks 10000 --reps 3
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]

MODES = {"ca_ff": 0, "ca_bf": 1, "vbp_ff": 3, "vbp_bf": 4}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="ca_bf", choices=sorted(MODES))
    p.add_argument("--hosts", type=int, default=1_000_000)
    p.add_argument("--tasks", type=int, default=10_000)
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--diag", action="store_true",
                   help="load the PVT_DIAG build (make -C pivot-scheduling_amd diag) and print the "
                        "score pass's candidate counters (prefilter survivors) as JSON")
    a = p.parse_args()
    import torch
    from pivot_place import _abi, synthetic
    from pivot_place.engine import DeviceRound, PlacementEngine
    r = synthetic.make_round(MODES[a.mode], a.hosts, a.tasks, seed=a.seed)
    lib = (os.path.join(ROOT, "pivot-scheduling_amd", "diag", "libpivot_place_diag.so")
           if a.diag else None)
    eng = PlacementEngine(0, lib_path=lib)
    dr = DeviceRound(r, eng.device)
    eng.reset_kstats()
    eng.set_profiling(True)
    nt = nb = 0
    t = time.perf_counter()
    for _ in range(a.reps):
        mx = eng.shard_begin(dr, 0, a.hosts, 1)
        send = torch.empty(max(mx, 1), dtype=torch.uint8, device=eng.device)
        nt, nb = eng.shard_score(send)
        torch.cuda.synchronize()
    dt = time.perf_counter() - t
    eng.set_profiling(False)
    k = eng.kstats(_abi.PVT_K_SCORE)
    print("score probe: mode %s H=%d window=%d tasks reps=%d  score launches=%d avg %.3f ms  (%.2f s)"
          % (a.mode, a.hosts, nt, a.reps, k["launches"], k["ms"] / max(k["launches"], 1), dt),
          flush=True)
    if a.diag:
        import ctypes
        import json
        f = eng.lib.pvt_debug_score_counts
        f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_int]
        buf = (ctypes.c_uint64 * 8)()
        assert f(eng.ctx, buf, 8, 1) == 0
        c = [int(buf[i]) for i in range(5)]
        print("DIAG " + json.dumps({
            "mode": a.mode, "hosts": a.hosts, "window_tasks": nt, "reps": a.reps,
            "candidates_streamed": c[0], "prefilter_survivors": c[1], "exact_survivors": c[2],
            "list_merges": c[3], "wave_host_blocks": c[4],
            "logical_candidates": nt * a.hosts * a.reps,
            "prefilter_survivor_frac": c[1] / max(c[0], 1),
            "streamed_frac_of_logical": c[0] / max(nt * a.hosts * a.reps, 1)}), flush=True)


if __name__ == "__main__":
    main()
