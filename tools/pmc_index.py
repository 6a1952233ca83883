#!/usr/bin/env python3
"""Collect tools/pmc_profile.py outputs into the index bench.py reads (profiles/pmc_index.json):

    python tools/pmc_index.py [--dest profiles/r06a] profiles/pmc_index.json ca_bf:1000000:10000:gpurun_out/pmc_r03_zwalk.json ...

--dest DIR: the tracked directory the profiles are copied to (gpurun_out/ is scratch); each
entry's "source" then names DIR/<file> instead of the scratch path it was read from.

Each argument after the output is mode:hosts:tasks:pmc_json. The entry key is
"<mode>_<hosts>_<tasks>:<kernel>" (kernel = the short __global__ name the profile matched); the
entry keeps the profile (with the sha256 of the library it was collected on: bench.py ignores an
entry of another build) plus launches_per_round = dispatches / the probe's --reps."""
import json
import os
import sys

KERNELS = ("zwalk_kernel", "opp_commit_kernel", "opp_count_kernel", "band_score_kernel",
           "score_kernel", "commit_kernel", "resident_kernel", "merge_kernel")


def short(name):
    base = name.split("(")[0].split("<")[0].split("::")[-1].split(" ")[-1]
    for k in KERNELS:
        if base == k:
            return k
    return base


def main():
    argv = sys.argv[1:]
    dest = None
    if argv[:1] == ["--dest"]:
        dest, argv = argv[1], argv[2:]
    out_path = argv[0]
    idx = {"entries": {}}
    if os.path.exists(out_path):
        with open(out_path) as f:
            idx = json.load(f)
        idx.setdefault("entries", {})
    for spec in argv[1:]:
        mode, hosts, tasks, path = spec.split(":", 3)
        with open(path) as f:
            p = json.load(f)
        probe = p.get("probe", [])
        reps = int(probe[probe.index("--reps") + 1]) if "--reps" in probe else 1
        disp = p["counters_per_launch"].get("dispatches_sq", reps)
        p["launches_per_round"] = disp / float(max(reps, 1))
        p["source"] = (os.path.join(dest, os.path.basename(path)) if dest
                       else os.path.relpath(path))
        key = "%s_%s_%s:%s" % (mode, hosts, tasks, short(p["kernel"]))
        idx["entries"][key] = p
        print(key, "launches/round %.1f" % p["launches_per_round"], p.get("lib_sha256", "?")[:12])
    with open(out_path, "w") as f:
        json.dump(idx, f, indent=1)


if __name__ == "__main__":
    main()
