#!/usr/bin/env python3
"""Diagnostic: phase cycles of the vbp best-fit one-wave list walk (pvt_lwalk.hip; PVT_STAMPS
build, `make stamps`). Stamps serialise the walk: read the shares.
    python tools/lwalk_stamps.py [H] [T]"""
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
eng = PlacementEngine(0, lib_path=os.path.join(ROOT, "pivot-scheduling_amd", "diag",
                                               "libpivot_place_stamps.so"))
f = eng.lib.pvt_debug_commit_stamps
f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
buf = (ctypes.c_uint64 * 16)()
assert f(eng.ctx, buf, 16) == 0
eng.set_pipeline(False)          # (score passes off the walk's time line)
r = synthetic.make_round(_abi.PVT_VBP_BF, H, T)
dr = DeviceRound(r, eng.device)
eng.run(dr)
torch.cuda.synchronize()
assert f(eng.ctx, buf, 16) == 0
n = max(buf[4], 1)
print("vbp_bf H=%d T=%d: %d task steps (refills re-walk some)" % (H, T, buf[4]))
for k, name in enumerate(("record + list head", "cursor search", "live touched scan", "commit")):
    print("  %-20s %8.0f cycles per task" % (name, buf[k] / n))
print("  chunk loads %.2f per task, live-scan chunks %.2f per task, mean live hosts %.1f, "
      "touched winners %.1f %%" % (buf[5] / n, buf[6] / n, buf[8] / n, 100.0 * buf[7] / n))
