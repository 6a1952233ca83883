"""Bulk sticky runs and run lists in the resident kernel's 4-wave path (pvt_batch.hip
resident_round): when a run of equal demand rows starts, the winner's copies are counted in one
step (fits, subtract, in order) instead of one loop iteration per task, and (vbp best-fit) when
the winner runs out with at least RES_LIST_MIN tasks of the run left, the rest goes down per-wave
lists of the best fitting hosts by the full path's key, merged on the fly. Every round must equal the CPU restatement, and
the same batch with both off (PVT_RWALK=16, A/B) too: runs longer than the 256-row staging chunk,
demands that are not exactly representable (the copy count comes from the sequential roundings),
winners that run out mid-run, lists used up (rebuilt) and lists that run dry (every head a host
that does not fit: the run's other tasks stay waiting), runs split by the anchor or the group, all-zero rows, and
realtime bandwidths (runs split by group)."""
import os

import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic
from pivot_place.engine import PlacementEngine

pytestmark = pytest.mark.gpu

MODES = [(_abi.PVT_CA_FF, True), (_abi.PVT_CA_FF, False), (_abi.PVT_CA_BF, True),
         (_abi.PVT_VBP_FF, True), (_abi.PVT_VBP_BF, True)]


def _engine(rwalk):
    old = os.environ.get("PVT_RWALK")
    os.environ["PVT_RWALK"] = rwalk
    try:
        return PlacementEngine(0)
    finally:
        if old is None:
            del os.environ["PVT_RWALK"]
        else:
            os.environ["PVT_RWALK"] = old


@pytest.fixture(scope="module", params=["0", "32"])
def engines(request):
    # "0": no one-wave walks, every task on the 4-wave path, bulk sticky runs and run lists on;
    # "32": bulk sticky runs without run lists; "16": the per-task sticky rule only
    return _engine(request.param), _engine("16")


def _same(got, ref, what):
    np.testing.assert_array_equal(got.placement, ref.placement, err_msg=what)
    np.testing.assert_array_equal(got.order, ref.order, err_msg=what)
    assert np.array_equal(got.avail, ref.avail), what


def _check(engines, rounds, what):
    on, off = engines
    got = on.place_batch(rounds)
    base = off.place_batch(rounds)
    for i, (r, g, b) in enumerate(zip(rounds, got, base)):
        ref = oracle.place(r)
        _same(g, ref, "%s round %d (bulk sticky)" % (what, i))
        _same(b, ref, "%s round %d (per-task sticky)" % (what, i))


@pytest.mark.parametrize("mode,sort_hosts", MODES)
def test_sticky_runs_match_oracle(engines, mode, sort_hosts):
    rounds = []
    for s in range(6):
        r = synthetic.make_round(mode, 700, 1300, seed=500 + s, sort_hosts=sort_hosts)
        rs = np.random.RandomState(600 + s)
        if s == 0:                               # two rows only: runs of hundreds of tasks
            rows = np.array([[0.5, 2048.0], [0.25, 1024.0]])
            pick = rs.randint(0, 2, size=r.n_tasks)
            r.dem[0], r.dem[1] = rows[pick, 0], rows[pick, 1]
        elif s == 1:                             # not exactly representable, tight hosts
            r.dem[0] = 0.1
            r.dem[1] = 0.3 * 1024.0
            r.avail[0] = 0.1 * rs.randint(1, 30, size=r.n_hosts) + 0.05 * (s % 2)
        elif s == 2:                             # all-zero rows between the others
            r.dem[:, ::3] = 0.0
        elif s == 3:                             # one row, few hosts: winners run out mid-run
            r.dem[0], r.dem[1] = 1.5, 3000.0
            r.avail[0] = np.minimum(r.avail[0], 4.5)
        elif s == 4:                             # exact fits (strict modes: the last copy fails)
            r.dem[0], r.dem[1] = 0.5, 2048.0
            r.avail[0] = 0.5 * rs.randint(0, 6, size=r.n_hosts)
            r.avail[1] = 2048.0 * rs.randint(0, 6, size=r.n_hosts)
        else:                                    # fewer distinct rows: longer runs
            r.dem[0] = np.round(r.dem[0] * 4) / 4
            r.dem[1] = np.round(r.dem[1] / 4096.0) * 4096.0
        rounds.append(r)
    _check(engines, rounds, "sticky runs mode %d sort_hosts=%s" % (mode, sort_hosts))


@pytest.mark.parametrize("mode", [_abi.PVT_CA_FF, _abi.PVT_CA_BF])
def test_sticky_runs_realtime_bw(engines, mode):
    """Realtime bandwidths (cost_aware.py:79,112): the bandwidth row is the group's, so a run
    ends where the group changes even when anchor and demand repeat."""
    rounds = []
    for s in range(3):
        r = synthetic.make_round(mode, 800, 900, seed=700 + s)
        r.cost = r.cost + 0.001
        r.dem[0] = np.round(r.dem[0] * 2) / 2
        r.dem[1] = np.round(r.dem[1] / 8192.0) * 8192.0
        rs = np.random.RandomState(700 + s)
        bsum = r.bw + r.bw.T
        a = r.group_anchor
        r.rt_bw = (bsum[a][:, r.zone] / rs.randint(1, 4, size=(len(a), r.n_hosts))).astype(np.float64)
        rounds.append(r)
    _check(engines, rounds, "sticky runs realtime bw mode %d" % mode)
