#!/usr/bin/env python3
"""Collect tools/pmc_profile.py outputs into the index bench.py reads (profiles/<name>.json):
    python tools/pmc_index.py profiles/r02_score_pmc.json ca_bf:1000000:10000:1024:gpurun_out/pmc_r02_ca_bf.json ...
Each argument after the output is mode:hosts:tasks:window_tasks:pmc_json; candidates per launch
of the profiled probe = window_tasks x hosts."""
import json
import os
import sys

out_path = sys.argv[1]
idx = {"configs": {}}
if os.path.exists(out_path):
    idx = json.load(open(out_path))
for spec in sys.argv[2:]:
    mode, hosts, tasks, wt, path = spec.split(":", 4)
    p = json.load(open(path))
    p["candidates_per_launch"] = float(wt) * float(hosts)
    p["source"] = path
    idx["configs"]["%s_%s_%s" % (mode, hosts, tasks)] = p
json.dump(idx, open(out_path, "w"), indent=1)
print("wrote", out_path, sorted(idx["configs"]))
