#!/usr/bin/env python3
"""Diagnostic: phases of the fused host-batch kernel (PVT_STAMPS build, `make stamps`) over the
recorded config-1 drop-in rounds (block 0: stage in, anchors, grouping, placement, results out),
cycles per round. usage: fused_stamps.py [SIM_NAME]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from pivot_place.engine import PlacementEngine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sim_c1_cost_aware"
eng = PlacementEngine(0, lib_path=os.environ.get("STAMPS_LIB") or os.path.join(
    ROOT, "pivot-scheduling_amd", "diag", "libpivot_place_stamps.so"))
f = eng.lib.pvt_debug_commit_stamps
f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
buf = (ctypes.c_uint64 * 32)()
assert f(eng.ctx, buf, 32) == 0          # allocates and zeroes the device counters
secs, cand, nr, ok, _ = bench._replay(name, eng)
assert f(eng.ctx, buf, 32) == 0
names = ["stage in", "anchors", "grouping", "placement", "results out"]
tot = sum(buf[16 + k] for k in range(5))
print("%s: %d rounds, parity %s, %.0f cycles per round in the fused kernel (block 0)" % (name, nr, ok, tot / max(nr, 1)))
for k, nm in enumerate(names):
    print("  %-12s %6.1f%%  %8.0f cycles/round" % (nm, 100.0 * buf[16 + k] / max(tot, 1), buf[16 + k] / max(nr, 1)))
