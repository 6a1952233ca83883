#!/usr/bin/env python3
"""Convert the reference's bundled DATA files into the JSON tables this package ships.

Run in the build container only (it reads /root/reference, which does not exist on the GPU
box). Outputs are committed data, not code:

- ``pivot_place/data/locality.json``: zone list in ``locality.yml`` order and the region-pair
  (cost, bw) table in ``meta`` order. The reference expands the latter into zone pairs and
  jitters every bw by U(.95, 1.05) in that order (resources/__init__.py:571-589); the
  expansion is redone by ``pivot_place.locality``.
- ``pivot_place/data/task_demands.json``: the (cpus, mem) pairs of every task row of the seven
  bundled job files with their multiplicity, used by the synthetic configs.
"""
import collections
import json
import os
import sys

import yaml

REF = os.environ.get("PIVOT_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pivot-scheduling_amd",
                   "pivot_place", "data")
Loader = getattr(yaml, "CSafeLoader", yaml.SafeLoader)


def locality():
    with open(os.path.join(REF, "resources", "locality.yml")) as f:
        doc = yaml.load(f, Loader=Loader)
    regions = []
    for cloud, regs in doc["locality"].items():
        for region, zones in regs.items():
            regions.append({"cloud": cloud, "region": region, "zones": list(zones)})
    meta = []
    for key, vals in doc["meta"].items():
        src, dst = key.split("--")
        meta.append({"src": src, "dst": dst, "cost": vals["cost"], "bw": vals["bw"]})
    return {"regions": regions, "meta": meta}


def demands():
    counts = collections.Counter()
    jobdir = os.path.join(REF, "alibaba", "jobs")
    for fn in sorted(os.listdir(jobdir)):
        with open(os.path.join(jobdir, fn)) as f:
            for j in yaml.load(f, Loader=Loader):
                for t in j["tasks"]:
                    counts[(float(t["cpus"]), float(t["mem"]))] += 1
    rows = sorted(counts.items())
    return {"columns": ["cpus", "mem_trace", "count"],
            "rows": [[c, m, n] for (c, m), n in rows]}


def main():
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "locality.json"), "w") as f:
        json.dump(locality(), f, indent=1)
    with open(os.path.join(OUT, "task_demands.json"), "w") as f:
        json.dump(demands(), f)
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
