#!/usr/bin/env python3
"""Diagnostic: where the lock-step sweep's engine time goes (config 2, bench.py c2_lockstep):
per pvt_place_host_batch call, the Python marshalling before the C call, the C call itself
(staging, launches, one synchronisation) and the unpacking after it; and the C call's share
that is device work (HIP events around it would serialise; instead the C call is timed once
with the rounds' kernels and once as an empty batch)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from pivot_place.engine import PlacementEngine  # noqa: E402

eng = PlacementEngine(0)
lib_call = eng.lib.pvt_place_host_batch
# the C++ marshaller (pivot_place._hostbatch) calls the C function through its address, so
# the C-call split below exists only for the ctypes marshalling (PVT_HOSTBATCH=0)
cxx = __import__("pivot_place.engine", fromlist=["_hostbatch"])._hostbatch() is not None
eng._hb_fn = __import__("ctypes").cast(lib_call, __import__("ctypes").c_void_p).value
acc = {"calls": 0, "rounds": 0, "total": 0.0, "c": 0.0}


class Timed:
    def __init__(self, f):
        self.f = f
        self.argtypes = f.argtypes

    def __call__(self, *a):
        t = time.perf_counter()
        rc = self.f(*a)
        acc["c"] += time.perf_counter() - t
        return rc


eng.lib.pvt_place_host_batch = Timed(lib_call)
orig = eng.place_host_batch


def timed_batch(reqs):
    t = time.perf_counter()
    out = orig(reqs)
    acc["total"] += time.perf_counter() - t
    acc["calls"] += 1
    acc["rounds"] += len(reqs)
    return out


eng.place_host_batch = timed_batch
bench.replay_workloads(eng)            # (warms the fixtures and the engine)
for k in acc:
    acc[k] = 0 if k in ("calls", "rounds") else 0.0
r = bench.lockstep_workload(eng)
n = max(acc["calls"], 1)
print("lockstep: engine_seconds %.3f, cpu engine_seconds %.3f, ticks %d" %
      (r["engine_seconds"], r["cpu_baseline"]["engine_seconds"], r["ticks"]))
print("host batches: %d calls, %.2f rounds per call" % (acc["calls"], acc["rounds"] / n))
if cxx:
    print("  per call: %.1f us total (C++ marshalling; PVT_HOSTBATCH=0 splits out the C call)"
          % (acc["total"] * 1e6 / n))
else:
    print("  per call: %.1f us total, %.1f us in the C call, %.1f us Python marshalling + "
          "unpacking" % (acc["total"] * 1e6 / n, acc["c"] * 1e6 / n,
                         (acc["total"] - acc["c"]) * 1e6 / n))
print("  driver serve time not in the host batch: %.1f us per tick"
      % ((r["engine_seconds"] - acc["total"]) * 1e6 / max(r["ticks"], 1)))
