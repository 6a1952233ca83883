#!/usr/bin/env python3
"""Diagnostic: cycles of the zero-cost frontier walk (PVT_STAMPS build, `make stamps`):
prologue (certificates + window) and walk per chain, chunks scanned per task."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]
import torch  # noqa: E402
from pivot_place import _abi, synthetic  # noqa: E402
from pivot_place.engine import DeviceRound, PlacementEngine  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000
lib = sys.argv[3] if len(sys.argv) > 3 else "libpivot_place_stamps.so"
MODES = {"ca_ff": _abi.PVT_CA_FF, "ca_bf": _abi.PVT_CA_BF, "vbp_ff": _abi.PVT_VBP_FF}
mode = sys.argv[4] if len(sys.argv) > 4 else "ca_bf"
eng = PlacementEngine(0, lib_path=os.path.join(ROOT, "pivot-scheduling_amd", "diag", lib))
f = eng.lib.pvt_debug_commit_stamps
f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
buf = (ctypes.c_uint64 * 32)()
assert f(eng.ctx, buf, 32) == 0
r = synthetic.make_round(MODES[mode], H, T)
dr = DeviceRound(r, eng.device)
eng.run(dr)
torch.cuda.synchronize()
assert f(eng.ctx, buf, 32) == 0
st = eng.epoch_stats()
nch = max(st["frontier_chains"] + st["list_chains"], 1)
print("%s H=%d T=%d stats=%s" % (mode, H, T, st))
print("  prologue   %10.0f cycles per chain" % (buf[0] / nch))
print("    tables + demand scan %.0f, window ids %.0f, window capacities %.0f, suffix minima %.0f"
      % tuple(buf[20 + k] / nch for k in range(4)))
print("  walk       %10.0f cycles per chain, %.0f per task" % (buf[1] / nch, buf[1] / max(buf[3], 1)))
print("  chunks     %10.2f per task" % (buf[2] / max(buf[3], 1)))
print("  tasks      %10d, anchor switches %d" % (buf[3], buf[4]))
print("  bulk runs  %10d runs placed %d tasks (%.1f per run)" % (buf[6], buf[5], buf[5] / max(buf[6], 1)))
print("  run search %10.0f cycles per run, %.2f LDS chunk probes per run" % (buf[7] / max(buf[6], 1), buf[10] / max(buf[6], 1)))
print("  pass 1     %10.0f cycles per bulk call, %.1f iterations" % (buf[8] / max(buf[6], 1), buf[11] / max(buf[6], 1)))
print("  pass 2     %10.0f cycles per bulk call" % (buf[9] / max(buf[6], 1)))
print("    per run: setup %.0f, pass-1 loop %.0f, who loop + host ids %.0f, replay %.0f"
      % tuple(buf[24 + k] / max(buf[6], 1) for k in range(4)))
print("    runs counted in closed form: %d of %d" % (buf[28], buf[6]))
print("  batches    %10.0f cycles per task (records, run masks, log flush)" % (buf[12] / max(buf[3], 1)))
print("  single     %10d tasks on the one-task hot path" % buf[13])
