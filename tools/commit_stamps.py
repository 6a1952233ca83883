#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of the commit walk (PVT_STAMPS build, `make stamps`).
Read the SHARES, not the absolute time: stamps serialise the walk."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]
import torch  # noqa: E402
from pivot_place import synthetic  # noqa: E402
from pivot_place.engine import DeviceRound, PlacementEngine  # noqa: E402

mode = int(sys.argv[1]) if len(sys.argv) > 1 else 1
H = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
T = int(sys.argv[3]) if len(sys.argv) > 3 else 10_000
eng = PlacementEngine(0, lib_path=os.environ.get("STAMPS_LIB") or os.path.join(
    ROOT, "pivot-scheduling_amd", "diag", "libpivot_place_stamps.so"))
f = eng.lib.pvt_debug_commit_stamps
f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
buf = (ctypes.c_uint64 * 16)()
assert f(eng.ctx, buf, 16) == 0         # allocates and zeroes the device counters
r = synthetic.make_round(mode, H, T)
dr = DeviceRound(r, eng.device)
eng.run(dr)
torch.cuda.synchronize()
assert f(eng.ctx, buf, 16) == 0
if mode == 2:
    # speculative range walk (pvt_opp.hip): counts per range, draws, candidates, verified walk
    # stamp 2 holds only pass 3's last part (5 and 6 are its first two)
    names = [(0, "pass1-counts"), (1, "pass2-draws"), (5, "pass3a-select+load"),
             (6, "pass3b-candidates"), (2, "pass3c-capacities"), (9, "pass4-setup"),
             (8, "pass4-loop"), (3, "pass4-commits")]
    tot = sum(buf[k] for k, _ in names)
    print("opportunistic H=%d T=%d tasks=%d ranges=%d stats=%s"
          % (H, T, buf[7], buf[4], eng.last_stats()))
    for k, nm in names:
        print("  %-20s %6.1f%%  %8.0f cycles/task" % (nm, 100.0 * buf[k] / max(tot, 1),
                                                      buf[k] / max(buf[7], 1)))
    print("  pass-4 commits %d: lost to a later task %d, among a later task's candidates' id "
          "range %d" % (buf[13], buf[11], buf[12]))
    sys.exit(0)
if mode == 3 or os.environ.get("ZWALK"):
    # frontier walk (pvt_zwalk.hip; vbp first-fit: ordered frontier attempts): prologue
    # (window build, certificates, suffix minima), walk, chunk visits per task
    print("frontier walk mode %d H=%d T=%d tasks=%d stats=%s %s" % (mode, H, T, buf[3], eng.last_stats(),
                                                                    eng.epoch_stats()))
    print("  prologue cycles total %.0f  walk cycles/task %.0f  chunk visits/task %.2f  anchor switches %d"
          % (buf[0], buf[1] / max(buf[3], 1), buf[2] / max(buf[3], 1), buf[4]))
    sys.exit(0)
names = ["wait-prefetch", "hash-lookup", "untouched-pick", "touched-rescore", "commit"]
tot = sum(buf[k] for k in range(5))
print("mode %d H=%d T=%d tasks walked=%d stats=%s mean live touched=%.1f"
      % (mode, H, T, buf[5], eng.last_stats(), buf[6] / max(buf[5], 1)))
for k in range(5):
    print("  %-16s %6.1f%%  %8.0f cycles/task" % (names[k], 100.0 * buf[k] / tot, buf[k] / max(buf[5], 1)))
