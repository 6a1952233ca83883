"""GPU parity of the frontier walk's bulk runs (pvt_zwalk.hip run_bulk / run step) and of the vbp
best-fit representative lists (pvt_band.hip band_runs_kernel + pvt_lwalk.hip), on rounds built so that
long runs of equal demands fill hosts in index order across chunk boundaries.

Reference order: each task takes the lowest-index fitting host (vbp first-fit, scheduler/vbp.py
:19-24; cost_aware first-fit, cost_aware.py:118-127; cost_aware best-fit's zero-cost winners,
cost_aware.py:85-97) and commits by subtraction. A run places several equal tasks at once by
replaying the same subtractions, so placements, order and final availability must equal the CPU
restatement bit for bit -- at the fit boundary (>= for vbp and best-fit, > for cost_aware
first-fit: capacities that are exact multiples of the demand), with hosts that absorb 0, 1 or
many copies, with disk / gpus demands of +0, -0 and > 0 (the two- and four-dimension loops),
and with the frontier walk switched off for comparison."""
import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu

WALK_MODES = [_abi.PVT_VBP_FF, _abi.PVT_CA_FF, _abi.PVT_CA_BF]


def _place(engine, r, zero_walk=True):
    try:
        engine.set_resident(0)
        engine.set_zero_walk(zero_walk)
        return engine.place(r)
    finally:
        engine.set_zero_walk(True)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)


def _same(res, ref, what=""):
    np.testing.assert_array_equal(res.order, ref.order, err_msg=what)
    np.testing.assert_array_equal(res.placement, ref.placement, err_msg=what)
    a = np.ascontiguousarray(res.avail).view(np.int64)
    b = np.ascontiguousarray(ref.avail).view(np.int64)
    bad = np.nonzero((a != b).any(axis=0))[0]
    assert bad.size == 0, "%s: availability differs (bitwise) on hosts %s" % (what, bad[:10])


def _run_round(mode, H, T, seed, rows, per_host, sort_hosts=True):
    """A round whose tasks use only the given (cpus, mem) demand rows -- so the sorted order has
    long runs of equal demands -- on hosts holding 0..per_host copies of a row's cpus exactly."""
    r = synthetic.make_round(mode, H, T, seed=seed, sort_hosts=sort_hosts)
    rs = np.random.RandomState(seed)
    pick = rs.randint(0, len(rows), size=T)
    r.dem[0] = np.array([rows[k][0] for k in pick])
    r.dem[1] = np.array([rows[k][1] for k in pick])
    r.avail[0] = 0.5 * rs.randint(0, 2 * per_host + 1, size=H)
    r.avail[1] = rs.uniform(0, 4e4, size=H)
    return r


@pytest.mark.parametrize("mode", WALK_MODES, ids=lambda m: _abi.MODE_NAMES[m])
@pytest.mark.parametrize("per_host", [1, 3, 12])
def test_runs_fill_hosts_in_order(engine, mode, per_host):
    """Three demand rows, hosts that take 0..per_host copies of the cpus demand exactly: runs
    fill several hosts, cross 64-host chunks, and stop at the exact-fit boundary."""
    rows = [(0.5, 100.0), (1.0, 250.0), (0.5, 37.5)]
    r = _run_round(mode, 20_000, 3000, 11 + per_host, rows, per_host)
    ref = oracle.place(r, threads=8)
    res = _place(engine, r)
    _same(res, ref, "runs mode %d per_host %d" % (mode, per_host))
    if mode != _abi.PVT_CA_FF or per_host > 1:   # (one strict copy per host: keyed walks stop at once)
        assert engine.epoch_stats()["frontier_chains"] > 0
    _same(_place(engine, r, zero_walk=False), ref, "frontier walk off")


@pytest.mark.parametrize("mode", WALK_MODES, ids=lambda m: _abi.MODE_NAMES[m])
def test_runs_unsorted_hosts(engine, mode):
    """cost_aware first-fit without sort_hosts (the ordered walk, strict fit) and the others on
    the same kind of round."""
    rows = [(1.0, 500.0), (0.5, 500.0)]
    r = _run_round(mode, 9000, 2500, 5, rows, 4, sort_hosts=False)
    _same(_place(engine, r), oracle.place(r, threads=8))


@pytest.mark.parametrize("mode", WALK_MODES, ids=lambda m: _abi.MODE_NAMES[m])
@pytest.mark.parametrize("disk,gpus", [(0.0, 0.0), (-0.0, 0.0), (0.0, -0.0), (5.0, 0.0),
                                       (0.0, 0.25), (25.0, 0.5)])
def test_runs_disk_and_gpus_demands(engine, mode, disk, gpus):
    """Disk / gpus demands of +0 use the two-dimension loop; -0 and positive ones the
    four-dimension loop (where disk or gpus can be what stops a host)."""
    rows = [(0.5, 120.0), (1.5, 90.0)]
    r = _run_round(mode, 12_000, 2000, 23, rows, 6)
    r.dem[2, :] = disk
    r.dem[3, :] = gpus
    r.avail[2] = 100.0
    r.avail[3] = 1.0
    ref = oracle.place(r, threads=8)
    _same(_place(engine, r), ref, "disk %r gpus %r" % (disk, gpus))


@pytest.mark.parametrize("mode", WALK_MODES, ids=lambda m: _abi.MODE_NAMES[m])
def test_one_long_run(engine, mode):
    """Every task has the same demand: one run per 64-task batch, hosts absorbing many copies
    (and the last hosts of the window running dry)."""
    r = _run_round(mode, 30_000, 4000, 31, [(0.5, 10.0)], 20)
    _same(_place(engine, r), oracle.place(r, threads=8))


@pytest.mark.parametrize("window", [0, 53, 400])
def test_vbp_bf_representative_lists(engine, window):
    """vbp best-fit band lists with few distinct demands: each window scores one list per run of
    equal demands; the walk maps every task to its run's list. Windows of 53 / 400 tasks cut runs
    and force refills; hosts that fit a few copies keep touched hosts live."""
    rows = [(0.5, 100.0), (1.0, 250.0), (2.0, 1000.0), (0.5, 37.5)]
    r = _run_round(_abi.PVT_VBP_BF, 80_000, 3000, 41, rows, 3)
    ref = oracle.place(r, threads=8)
    try:
        engine.set_resident(0)
        engine.set_band(1)
        engine.set_window(window)
        res = engine.place(r)
    finally:
        engine.set_band(65536)
        engine.set_window(0)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)
    _same(res, ref, "vbp_bf window %d" % window)
