"""GPU parity of the ordered frontier walk (pvt_capi.hip ordered_frontier over pvt_zwalk.hip's
keyed mode): vbp first-fit (fit >=, reference scheduler/vbp.py) and cost_aware first-fit without
sort_hosts (strict fit, reference scheduler/cost_aware.py) take the first host in index order
that fits; the walk does that over a window of the first 1024 hosts that fit the smallest
remaining demand and stops at the first task none of them fits, where a list window takes over.

Cases make the window stop and rebuild on purpose: hosts that fit exactly once (each commit
kills its host), demands equal to capacities (the >= / > boundary), a crowded cluster whose
first hosts fill up, tasks that fit nowhere, and demands far above most hosts (a sparse alive
set). Placements, order and final availability must equal the CPU restatement bit for bit, and
equal the engine with the frontier walk switched off."""
import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu

FF_MODES = [_abi.PVT_VBP_FF, _abi.PVT_CA_FF]


def _unsorted(r):
    if r.mode == _abi.PVT_CA_FF:
        r.sort_hosts = False
    return r


def _run(engine, r, zero_walk=True):
    try:
        engine.set_resident(0)
        engine.set_zero_walk(zero_walk)
        return engine.place(r)
    finally:
        engine.set_zero_walk(True)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)


def _check(engine, r):
    ref = oracle.place(r)
    res = _run(engine, r)
    walks = engine.epoch_stats()["frontier_chains"]
    np.testing.assert_array_equal(res.placement, ref.placement)
    np.testing.assert_array_equal(res.order, ref.order)
    bad = np.nonzero((res.avail != ref.avail).any(axis=0))[0]
    assert bad.size == 0, "availability differs on hosts %s" % bad[:10]
    off = _run(engine, r, zero_walk=False)
    np.testing.assert_array_equal(off.placement, ref.placement)
    return ref, walks


@pytest.mark.parametrize("mode", FF_MODES)
@pytest.mark.parametrize("H,T,seed", [(100_000, 2600, 1), (5000, 3000, 2), (70_000, 120, 3),
                                      (1_000_000, 2000, 4)])
def test_synthetic_rounds(engine, mode, H, T, seed):
    _, walks = _check(engine, _unsorted(synthetic.make_round(mode, H, T, seed=seed)))
    assert walks > 0


@pytest.mark.parametrize("mode", FF_MODES)
@pytest.mark.parametrize("H", [64, 700, 1024, 1025, 3000])
def test_exact_fit_each_commit_kills_its_host(engine, mode, H):
    """Demand == capacity: vbp (>=) fills each host once and moves on; cost_aware (>) never
    fits such a host at all."""
    r = _unsorted(synthetic.make_round(mode, H, H + 200, seed=H))
    r.avail[0, :] = 2.0
    r.avail[1, :] = 1e9
    r.dem[0, :] = 2.0
    r.dem[1, :] = 1.0
    ref, _ = _check(engine, r)
    expect = H if mode == _abi.PVT_VBP_FF else 0
    assert (ref.placement >= 0).sum() == expect


@pytest.mark.parametrize("mode", FF_MODES)
def test_crowded_first_hosts_fill_up(engine, mode):
    """Small hosts: the window's hosts fill within a few hundred tasks and the walk rebuilds
    its window further along the index order, again and again."""
    r = _unsorted(synthetic.make_round(mode, 50_000, 4000, seed=7))
    rs = np.random.RandomState(7)
    r.avail[0, :] = 0.5 * rs.randint(1, 6, size=r.avail.shape[1])
    r.avail[1, :] = rs.uniform(1e4, 1e5, size=r.avail.shape[1])
    _check(engine, r)


@pytest.mark.parametrize("mode", FF_MODES)
def test_tasks_that_fit_nowhere_and_sparse_alive_hosts(engine, mode):
    """Every 5th task fits no host (the walk stops there and a list window places it as
    unplaceable); big hosts are one in 400, so the alive set is sparse in index order."""
    r = _unsorted(synthetic.make_round(mode, 200_000, 3000, seed=9))
    r.avail[0, :] = 1.0
    r.avail[0, ::400] = 512.0
    r.avail[1, ::400] = 1e9
    r.dem[0, :] = 1.5
    r.dem[0, ::5] = 1e6
    ref, _ = _check(engine, r)
    assert (ref.placement < 0).sum() >= 600


@pytest.mark.parametrize("mode", FF_MODES)
@pytest.mark.parametrize("window", [32, 96, 333])
def test_small_list_windows_between_walks(engine, mode, window):
    r = _unsorted(synthetic.make_round(mode, 20_000, 3000, seed=11))
    r.avail[0, :] = 3.0
    ref = oracle.place(r)
    try:
        engine.set_resident(0)
        engine.set_window(window)
        res = engine.place(r)
    finally:
        engine.set_window(0)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)
    np.testing.assert_array_equal(res.placement, ref.placement)
    assert (res.avail == ref.avail).all()


@pytest.mark.parametrize("mode", FF_MODES)
@pytest.mark.parametrize("full", [70_000, 140_000, 299_990])
def test_first_hosts_full_window_span_grows(engine, mode, full):
    """The first `full` hosts have no capacity: the window's first host span (65,536 hosts)
    holds no alive host, and the span doubles until it reaches hosts that fit."""
    r = _unsorted(synthetic.make_round(mode, 300_000, 2000, seed=full))
    r.avail[:, :full] = 0.0
    ref, _ = _check(engine, r)
    assert (ref.placement >= 0).sum() > 0
