"""ctypes wrapper of the CPU restatement (oracle/pivot_oracle.c). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It checks the product; the product (pivot_place) never imports it.

Parity is pinned: tests/test_oracle_golden.py runs it against the golden fixtures generated
from the reference itself (tests/golden/make_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libpivot_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.oracle_place.restype = ctypes.c_int
        _lib.oracle_place.argtypes = [ctypes.c_void_p]
        _lib.oracle_norm4.restype = ctypes.c_double
        _lib.oracle_norm4.argtypes = [ctypes.POINTER(ctypes.c_double)]
        _lib.oracle_randint.restype = ctypes.c_uint32
        _lib.oracle_randint.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint64]
        _lib.oracle_place_mt.restype = ctypes.c_int
        _lib.oracle_place_mt.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _lib.oracle_meter.restype = ctypes.c_int
        _lib.oracle_meter.argtypes = [ctypes.c_void_p]
        _lib.oracle_anchor.restype = ctypes.c_int
        _lib.oracle_anchor.argtypes = [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 3 + [
            ctypes.c_int64] + [ctypes.c_void_p] * 3
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def place(r, threads=0):
    """Run one round on the CPU restatement. ``r``: pivot_place._abi.RoundArrays. ``threads``
    > 0 runs the OpenMP variant (oracle_place_mt: same results, host scans split over threads;
    the all-cores CPU baseline of bench.py)."""
    from pivot_place._abi import RoundResult, check_rc, fill_struct
    avail = r.avail.copy()
    T = r.n_tasks
    placement = np.full(T, -1, dtype=np.int32)
    order = np.zeros(T, dtype=np.int32)
    mt = None if r.mt_state is None else r.mt_state.copy()
    s = fill_struct(r)
    s.avail, s.zone, s.tiebreak, s.decay = _ptr(avail), _ptr(r.zone), _ptr(r.tiebreak), _ptr(r.decay)
    s.cost, s.bw, s.dem = _ptr(r.cost), _ptr(r.bw), _ptr(r.dem)
    s.task_group, s.group_anchor = _ptr(r.task_group), _ptr(r.group_anchor)
    s.order, s.placement, s.mt_state = _ptr(order), _ptr(placement), _ptr(mt)
    s.rt_bw = _ptr(r.rt_bw)
    if threads > 0:
        check_rc(lib().oracle_place_mt(ctypes.addressof(s), int(threads)))
    else:
        check_rc(lib().oracle_place(ctypes.addressof(s)))
    return RoundResult(placement=placement, order=order, avail=avail, mt_state=mt)


def norm4(x):
    a = (ctypes.c_double * 4)(*[float(v) for v in x])
    return lib().oracle_norm4(a)


def randint(state, n):
    """numpy RandomState.randint(0, n) on a (625,) uint32 MT state, updated in place."""
    assert state.dtype == np.uint32 and state.flags["C_CONTIGUOUS"]
    return int(lib().oracle_randint(state.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n))


def anchor(off, lst, zone, n_hosts, inst_host=None):
    """Mode-host anchors (scheduler/cost_aware.py:45-58) of the items off[c]..off[c+1] of
    ``lst``. Returns (mode_host, anchor_zone, rc); rc = PVT_EINVAL (-1) on an invalid item."""
    off = np.ascontiguousarray(off, dtype=np.int64)
    lst = np.ascontiguousarray(lst, dtype=np.int32)
    zone = np.ascontiguousarray(zone, dtype=np.int32)
    ih = None if inst_host is None else np.ascontiguousarray(inst_host, dtype=np.int32)
    C = len(off) - 1
    mode = np.zeros(C, dtype=np.int32)
    az = np.zeros(C, dtype=np.int32)
    rc = lib().oracle_anchor(C, int(n_hosts), _ptr(off), _ptr(lst), _ptr(ih),
                             0 if ih is None else len(ih), _ptr(zone), _ptr(mode), _ptr(az))
    return mode, az, rc


def meter(log):
    """Reference-order aggregates of a pivot_place.meter.MeterLog: (dict of arrays, rc)."""
    S = log.n_scen
    out = {k: np.zeros(max(S, 1)) for k in ("instance_hours", "egress_cost", "congestion_delay")}
    arrs = [np.ascontiguousarray(a) for _, a in log.arrays()]
    m = log.fill(lambda a: a.ctypes.data if a.size else None, [o.ctypes.data for o in out.values()])
    rc = lib().oracle_meter(ctypes.addressof(m))
    del arrs
    return {k: v[:S] for k, v in out.items()}, rc
