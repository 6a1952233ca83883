#!/usr/bin/env python3
"""HBM traffic of the score kernel from rocprofv3 PMC counters (run on the GPU box).

Two separate passes (FETCH_SIZE and WRITE_SIZE cannot share one: TCC slots), each as
`rocprofv3 --pmc <counter> -- python tools/score_probe.py ...` started as a child process under
a hard time limit (this script never touches the GPU itself). The probe launches only the score
pass (first window, 1024 tasks x H hosts); the commit walk does not run under counter
collection (tools/score_probe.py). Per MI355X_MICROARCH.md §HBM, FETCH_SIZE on gfx950 reports half
the bytes of a wide coalesced streaming read, so the read side is doubled; WRITE_SIZE is taken
as is. Counters are summed per dispatch of `score_kernel` / `opp_count_kernel` and averaged.
Writes gpurun_out/traffic.json (copy it to profiles/traffic.json), which bench.py reports as roofline.traffic when its config
matches.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOT = ("score_kernel", "opp_count_kernel", "ordered_kernel")


def run_pass(counter, out_dir, bench_args):
    cmd = ["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc", counter, "--output-format", "csv",
           "-d", out_dir, "-o", "pmc", "--", sys.executable,
           os.path.join(ROOT, "tools", "score_probe.py")] + bench_args
    env = dict(os.environ, TMPDIR="/tmp")
    subprocess.run(cmd, check=True, env=env, timeout=120)
    files = glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise RuntimeError("no counter_collection.csv under %s" % out_dir)
    per_dispatch = {}
    names = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if not any(h in name for h in HOT):
                continue
            if row.get("Counter_Name") != counter:
                continue
            d = row.get("Dispatch_Id")
            per_dispatch[d] = per_dispatch.get(d, 0.0) + float(row["Counter_Value"])
            names[d] = name
    return per_dispatch, names


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "ca_bf"
    hosts = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    tasks = int(sys.argv[3]) if len(sys.argv) > 3 else 10_000
    bench_args = ["--mode", mode, "--hosts", str(hosts), "--tasks", str(tasks), "--reps", "3"]
    base = os.path.join(ROOT, "gpurun_out", "pmc")
    fetch, names = run_pass("FETCH_SIZE", base + "_fetch", bench_args)
    write, _ = run_pass("WRITE_SIZE", base + "_write", bench_args)
    n = len(fetch)
    if n == 0:
        raise RuntimeError("no hot-kernel dispatches found")
    fetch_kb = sum(fetch.values()) / n
    write_kb = sum(write.values()) / max(len(write), 1)
    out = {
        "mode": mode, "hosts": hosts, "tasks": tasks,
        "kernel": sorted(set(names.values()))[0],
        "dispatches": n,
        "fetch_size_kb_per_launch_raw": fetch_kb,
        "write_size_kb_per_launch": write_kb,
        "read_correction": 2.0,
        "hbm_bytes_per_launch": (2.0 * fetch_kb + write_kb) * 1024.0,
        "candidates_per_launch": float(min(tasks, 1024)) * hosts,
        "hbm_bytes_per_candidate": (2.0 * fetch_kb + write_kb) * 1024.0 / (float(min(tasks, 1024)) * hosts),
        "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 reports half of a wide "
                "streaming read); the kernel's 8-B-per-lane loads are not separately calibrated. "
                "The host table (36 MB at 1M hosts) is resident in the 256 MiB Infinity Cache, "
                "whose hits these counters include.",
    }
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
