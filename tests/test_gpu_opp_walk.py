"""GPU parity of the opportunistic commit walk's speculative ranges (pvt_opp.hip) against the CPU
restatement (oracle/, pinned to the reference's golden runs; reference
scheduler/opportunistic.py:11-20).

The walk draws every task of a range on the range-start state and verifies the draws in order;
these cases make the speculation fail on purpose: hosts that fit exactly once (every commit
removes its host from every later task, so n falls by one per task and crosses powers of two),
feasible sets that run dry inside a range, few hosts per super-chunk (candidate lists shorter
than the shift), windows of every size up to the 256-task limit, pipelined and sequential
windows, and clusters above 1,048,576 hosts (more super-chunks than lanes). Placements, final
availability and the MT19937 state must equal the oracle's bit for bit."""
import contextlib

import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def windowed(engine, window=0, pipeline=True):
    engine.set_resident(0)
    engine.set_window(window)
    engine.set_pipeline(pipeline)
    try:
        yield
    finally:
        engine.set_window(0)
        engine.set_pipeline(True)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)


def _check(engine, r, **kw):
    ref = oracle.place(r)
    with windowed(engine, **kw):
        res = engine.place(r)
    np.testing.assert_array_equal(res.placement, ref.placement)
    bad = np.nonzero((res.avail != ref.avail).any(axis=0))[0]
    assert bad.size == 0, "availability differs on hosts %s" % bad[:10]
    np.testing.assert_array_equal(res.mt_state, ref.mt_state)
    return ref


def _exact_once(H, T, seed, cpus=1.0):
    """Every host fits one task: each commit takes its host away from every later task."""
    r = synthetic.make_round(_abi.PVT_OPP, H, T, seed=seed)
    r.avail[0, :] = cpus
    r.avail[1, :] = 1e9
    r.dem[0, :] = cpus
    r.dem[1, :] = 1.0
    return r


@pytest.mark.parametrize("pipeline", [True, False])
@pytest.mark.parametrize("window", [0, 1, 7, 64, 100, 256])
def test_exact_fit_every_commit_loses_its_host(engine, window, pipeline):
    # n falls 1000 -> 0 one task at a time (crossing 512, 256, ...), then the rest find nothing
    ref = _check(engine, _exact_once(1000, 1300, seed=3), window=window, pipeline=pipeline)
    assert (ref.placement >= 0).sum() == 1000


@pytest.mark.parametrize("H", [65, 129, 1025, 20000])
def test_exact_fit_small_clusters(engine, H):
    _check(engine, _exact_once(H, min(H + 50, 3000), seed=H))


@pytest.mark.parametrize("window", [0, 64, 256])
def test_crowded_mixed_demands(engine, window):
    """Nearly full hosts and mixed demands: many hosts stop fitting some later tasks but not
    others (candidate shifts below and among a task's candidates)."""
    r = synthetic.make_round(_abi.PVT_OPP, 5000, 4000, seed=17)
    rs = np.random.RandomState(5)
    r.avail[0, :] = 0.5 * rs.randint(1, 9, size=r.avail.shape[1])
    r.avail[1, :] = rs.uniform(1e4, 2e5, size=r.avail.shape[1])
    _check(engine, r, window=window)


def test_sparse_feasible_hosts_short_candidate_lists(engine):
    """One feasible host in 300: a super-chunk holds ~55 candidates, lists end early."""
    H, T = 200_000, 1500
    r = synthetic.make_round(_abi.PVT_OPP, H, T, seed=23)
    r.avail[0, :] = 0.0
    r.avail[0, ::300] = 64.0
    r.avail[1, ::300] = 1e9
    _check(engine, r)


@pytest.mark.parametrize("window", [0, 256])
def test_more_super_chunks_than_lanes(engine, window):
    """H > 64 super-chunks of 16384 hosts: counts are summed and searched 64 at a time."""
    r = synthetic.make_round(_abi.PVT_OPP, 1_100_000, 600, seed=29)
    _check(engine, r, window=window)


def test_config5_opportunistic_all_window_sizes(engine):
    r = synthetic.make_round(_abi.PVT_OPP, 1_000_000, 2000, seed=31)
    ref = oracle.place(r, threads=8)
    for window in (32, 128, 256):
        with windowed(engine, window=window):
            res = engine.place(r)
        np.testing.assert_array_equal(res.placement, ref.placement)
        np.testing.assert_array_equal(res.mt_state, ref.mt_state)
        assert (res.avail == ref.avail).all()
