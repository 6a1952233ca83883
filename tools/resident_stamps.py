#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of the resident kernel (pvt_batch.hip) at config 4
(PVT_STAMPS build, `make stamps`): block 0, wave 0 of a B-scenario batch. Read the SHARES and
the per-task cycles relative to each other: the stamps serialise the wave they time.
usage: resident_stamps.py MODE [B H T]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]
import torch  # noqa: E402
from pivot_place import _abi, synthetic  # noqa: E402
from pivot_place.engine import DeviceBatch, PlacementEngine  # noqa: E402

MODES = {"ca_ff": _abi.PVT_CA_FF, "ca_bf": _abi.PVT_CA_BF, "opp": _abi.PVT_OPP,
         "vbp_ff": _abi.PVT_VBP_FF, "vbp_bf": _abi.PVT_VBP_BF}
mode = sys.argv[1] if len(sys.argv) > 1 else "ca_bf"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
H = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
T = int(sys.argv[4]) if len(sys.argv) > 4 else 1000
eng = PlacementEngine(0, lib_path=os.environ.get("STAMPS_LIB") or os.path.join(
    ROOT, "pivot-scheduling_amd", "diag", "libpivot_place_stamps.so"))
f = eng.lib.pvt_debug_commit_stamps
f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
NW = 32 + 4096
buf = (ctypes.c_uint64 * NW)()
assert f(eng.ctx, buf, NW) == 0          # allocates and zeroes the device counters
rounds = [synthetic.make_round(MODES[mode], H, T, seed=1 + s) for s in range(B)]
db = DeviceBatch(rounds, eng.device)
eng.run_batch(db)
torch.cuda.synchronize()
assert f(eng.ctx, buf, NW) == 0
names = ["anchor rows", "slot scan", "wave reduction", "exchange", "full path", "commit"]
tot = sum(buf[k] for k in range(6))
n = max(buf[6], 1)
print("%s B=%d H=%d T=%d tasks=%d full-path tasks=%d (PVT_RES_WAVES=%s)"
      % (mode, B, H, T, buf[6], buf[7], os.environ.get("PVT_RES_WAVES", "default")))
for k, nm in enumerate(names):
    print("  %-16s %6.1f%%  %8.0f cycles/task" % (nm, 100.0 * buf[k] / max(tot, 1), buf[k] / n))
print("  %-16s %6.1f%%  %8.0f cycles/task" % ("total", 100.0, tot / n))
if buf[8] or buf[9]:
    print("  resident walk: %d of %d tasks walked, %.0f cycles (%.0f per walked task; the 4-wave "
          "phases above time the rest)" % (buf[8], T, buf[9], buf[9] / max(buf[8], 1)))
    print("  walk: %d LDS chunk probes, %d register-chunk advances, %d keyed key passes"
          % (buf[10], buf[11], buf[12]))
    print("  walk: %.0f cycles per task in the task bodies, %.0f per task for wave 0's whole walk "
          "(the rest of the walk total: the prologue of all waves)"
          % (buf[13] / max(buf[8], 1), buf[14] / max(buf[8], 1)))
    print("  walk: %d bulk runs placed %d tasks (%.1f per run)" % (buf[24], buf[25], buf[25] / max(buf[24], 1)))
cyc = sorted(buf[32 + k] for k in range(min(B, 4096)))
if cyc and cyc[-1]:
    import statistics
    q = lambda p: cyc[min(len(cyc) - 1, int(p * len(cyc)))]
    print("  per round (whole workgroup, cycles): min %d  p25 %d  median %d  p75 %d  p90 %d  max %d"
          % (cyc[0], q(0.25), q(0.5), q(0.75), q(0.9), cyc[-1]))
    per = [(buf[32 + k], k) for k in range(min(B, 4096))]
    per.sort(reverse=True)
    print("  slowest rounds:", ", ".join("%d (%d)" % (k, c) for c, k in per[:8]))

