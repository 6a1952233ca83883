#!/usr/bin/env python3
"""Diagnostic: one small batch per mode through the resident 4-wave path with bulk sticky runs on
(PVT_RWALK=0) against the CPU restatement, printing as it goes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]
t0 = time.time()
print("importing torch", flush=True)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from oracle import oracle  # noqa: E402
from pivot_place import _abi, synthetic  # noqa: E402
from pivot_place.engine import PlacementEngine  # noqa: E402
print("imported %.1f s" % (time.time() - t0), flush=True)
os.environ["PVT_RWALK"] = sys.argv[1] if len(sys.argv) > 1 else "0"
eng = PlacementEngine(0)
print("engine up", flush=True)
bad = 0
for mode in (_abi.PVT_VBP_BF, _abi.PVT_VBP_FF, _abi.PVT_CA_FF, _abi.PVT_CA_BF):
    rounds = [synthetic.make_round(mode, 300, 600, seed=900 + s) for s in range(2)]
    rounds[1].dem[0], rounds[1].dem[1] = 0.5, 2048.0
    got = eng.place_batch(rounds)
    for i, (r, g) in enumerate(zip(rounds, got)):
        ref = oracle.place(r)
        d = int((g.placement != ref.placement).sum())
        bad += d
        print("mode %d round %d: %d placements differ" % (mode, i, d), flush=True)
sys.exit(1 if bad else 0)
