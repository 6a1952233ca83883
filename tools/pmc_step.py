#!/usr/bin/env python3
"""HBM bytes of one whole bench step, from rocprofv3 counters (run on the GPU box; every pass is
a child `rocprofv3 --pmc ... -- python tools/walk_probe.py --marker 1 ...` under a hard limit).

The step's traffic is the sum over EVERY kernel dispatch of one round (bench.py's reset --
pvt_restore_hosts of the hosts the previous rep placed on for a single round, the snapshot copy
for a batch --, ordering, epochs, walks, validation, apply), not just the dominant kernel's:
    hbm_bytes_per_step = sum over the step's dispatches of (2 x FETCH_SIZE + WRITE_SIZE) KiB
(FETCH_SIZE doubled, WRITE_SIZE as read: MI355X_MICROARCH.md §HBM; FETCH_SIZE and WRITE_SIZE
need 3 + 2 TCC slots, so they are two passes.) walk_probe.py --marker 1 launches a one-element
`bitwise_not_` before every rep, so the dispatches between two markers are exactly one rep
(reset + pvt_place); the first rep is dropped (warm-up), the others are averaged.

    python tools/pmc_step.py --tag r05a_c5_ca_bf -- --mode ca_bf --hosts 1000000 --tasks 10000
Writes gpurun_out/pmc_<tag>_step.json (kernel "step", with the library's sha256) for
tools/pmc_index.py, which files it under "<mode>_<hosts>_<tasks>[variant]:step".
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pmc_profile import lib_sha256  # noqa: E402

MARKER = "bitwise_not"
PASSES = (("fetch", ["FETCH_SIZE"]), ("write", ["WRITE_SIZE", "GRBM_GUI_ACTIVE"]))


def dispatches(path):
    """[(dispatch id, kernel name, {counter: value summed over rows}, ns)] in dispatch order."""
    rows = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            d = int(row["Dispatch_Id"])
            e = rows.setdefault(d, [row.get("Kernel_Name", ""), {}, 0.0])
            c = row["Counter_Name"]
            e[1][c] = e[1].get(c, 0.0) + float(row["Counter_Value"])
            try:
                e[2] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
            except (KeyError, ValueError):
                pass
    return [(d,) + tuple(rows[d]) for d in sorted(rows)]


def steps_between_markers(ds):
    """Split the dispatch list at the marker kernels: one list of dispatches per rep."""
    reps, cur = [], None
    for d in ds:
        if MARKER in d[1]:
            if cur is not None:
                reps.append(cur)
            cur = []
        elif cur is not None:
            cur.append(d)
    if cur:
        reps.append(cur)
    return reps


def per_step(ds, counter):
    reps = steps_between_markers(ds)
    if len(reps) < 2:
        raise RuntimeError("fewer than two marked reps (%d markers found)" % len(reps))
    timed = reps[1:]
    total = [sum(d[2].get(counter, 0.0) for d in rep) for rep in timed]
    kernels = {}
    for rep in timed:
        for d in rep:
            base = d[1].split("(")[0].split("<")[0].split("::")[-1].split(" ")[-1]
            kernels[base] = kernels.get(base, 0.0) + d[2].get(counter, 0.0) / len(timed)
    return (sum(total) / len(total), len(timed[0]), kernels,
            sum(sum(d[3] for d in rep) for rep in timed) / len(timed))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--secs", type=int, default=150)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("probe_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    pargs = [x for x in a.probe_args if x != "--"]
    probe = [os.path.join(ROOT, "tools", "walk_probe.py")] + pargs + [
        "--reps", str(a.reps), "--marker", "1"]
    res = {}
    for name, counters in PASSES:
        out_dir = os.path.join(ROOT, "gpurun_out", "pmcstep_%s_%s" % (a.tag, name))
        cmd = ["timeout", "-s", "KILL", str(a.secs), "rocprofv3", "--pmc"] + counters + [
            "--output-format", "csv", "-d", out_dir, "-o", "pmc", "--", sys.executable] + probe
        print("pass %s: %s" % (name, " ".join(counters)), flush=True)
        subprocess.run(cmd, check=True, env=dict(os.environ, TMPDIR="/tmp"), timeout=a.secs + 30)
        files = glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            raise RuntimeError("no counter_collection.csv under %s" % out_dir)
        ds = dispatches(files[0])
        for c in counters:
            res[c] = per_step(ds, c)
    fetch, n_disp, fetch_k, ns = res["FETCH_SIZE"]
    write, _, write_k, _ = res["WRITE_SIZE"]
    step_bytes = (2.0 * fetch + write) * 1024.0
    by_kernel = {k: (2.0 * fetch_k.get(k, 0.0) + write_k.get(k, 0.0)) * 1024.0
                 for k in set(fetch_k) | set(write_k)}
    out = {"kernel": "step", "probe": ["tools/walk_probe.py"] + pargs + ["--reps", str(a.reps)],
           "lib_sha256": lib_sha256(),
           "counters_per_launch": {"FETCH_SIZE": fetch, "WRITE_SIZE": write,
                                   "dispatches_sq": float(a.reps), "dispatches_per_step": n_disp},
           "hbm_bytes_per_step": step_bytes,
           "hbm_bytes_per_step_by_kernel": dict(sorted(by_kernel.items(), key=lambda x: -x[1])),
           "profiled_kernel_ms_per_step": ns * 1e-6,
           "basis": "sum over every dispatch of a rep (between walk_probe markers, first rep "
                    "dropped) of 2 x FETCH_SIZE + WRITE_SIZE KiB"}
    path = os.path.join(ROOT, "gpurun_out", "pmc_%s_step.json" % a.tag)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
