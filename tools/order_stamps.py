#!/usr/bin/env python3
"""Diagnostic: phases of group_sort_gather_kernel (block 0) on the default line's grouped order
(PVT_STAMPS build, `make stamps`): offset prelude, group scan (tasks of the group collected in
LDS), sort, gathered writes -- s_memtime cycles summed over R rounds.
usage: order_stamps.py [H T R]"""
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
R = int(sys.argv[3]) if len(sys.argv) > 3 else 5
eng = PlacementEngine(0, lib_path=os.path.join(ROOT, "pivot-scheduling_amd", "diag", "libpivot_place_stamps.so"))
f = eng.lib.pvt_debug_commit_stamps
f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
buf = (ctypes.c_uint64 * 32)()
assert f(eng.ctx, buf, 32) == 0
dr = DeviceRound(synthetic.make_round(_abi.PVT_CA_BF, H, T), eng.device)
for _ in range(R):
    dr.reset()
    eng.run(dr)
torch.cuda.synchronize()
assert f(eng.ctx, buf, 32) == 0
names = ["prelude", "scan", "sort", "gather"]
tot = sum(buf[16 + k] for k in range(4))
for k, nm in enumerate(names):
    print("  %-8s %5.1f%%  %9.0f cycles per round" % (nm, 100.0 * buf[16 + k] / max(tot, 1), buf[16 + k] / R))
print("  total    %9.0f cycles per round (s_memtime: the shader clock)" % (tot / R))
