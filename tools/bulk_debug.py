#!/usr/bin/env python3
"""Diagnostic: the first task where the resident walk's bulk runs (default) and the walk without
them (PVT_RWALK=5) differ on a golden round, with its run context."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import golden_io  # noqa: E402
from oracle import oracle  # noqa: E402
from pivot_place.engine import PlacementEngine  # noqa: E402

name, idx = sys.argv[1], int(sys.argv[2])
case = golden_io.load(name)
r = golden_io.run_arrays(case, case["runs"][idx])
eng = PlacementEngine(0)
os.environ["PVT_RWALK"] = "5"
eng_nb = PlacementEngine(0)
got = eng.place_batch([r])[0]
nob = eng_nb.place_batch([r])[0]
ref = oracle.place(r)
print("bulk == oracle", np.array_equal(got.placement, ref.placement),
      "no-bulk == oracle", np.array_equal(nob.placement, ref.placement))
order = ref.order
pos = [i for i, t in enumerate(order) if got.placement[t] != ref.placement[t]]
print("mismatches", len(pos), "first positions", pos[:10])
if pos:
    p0 = pos[0]
    anc = r.group_anchor[r.task_group[order]]
    for i in range(max(0, p0 - 12), min(len(order), p0 + 6)):
        t = order[i]
        print("%5d task %5d batch %2d.%2d anc %2d grp %3d dem %s  ref %4d got %4d" % (
            i, t, i // 64, i % 64, anc[i], r.task_group[t], r.dem[:, t], ref.placement[t], got.placement[t]))
    h1, h2 = ref.placement[order[p0]], got.placement[order[p0]]
    print("zones ref host %d: %d, got host %d: %d" % (h1, r.zone[h1], h2, r.zone[h2]))
    print("avail0 ref host", r.avail[:, h1], "got host", r.avail[:, h2])
