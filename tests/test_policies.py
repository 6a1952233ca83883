"""The drop-in policies (pivot_place.policies) against the reference's recorded schedule() runs.

These tests exercise the Python side of the boundary exactly as the reference's round loop
calls it (scheduler/__init__.py:100-103): _update_resource_info(), then schedule(ready_q).
They check placements, the returned task order, the snapshot arrays mutated in place, the
RandomState advanced by exactly the reference's draws, and the reference's error behaviour.

The CPU variant swaps the engine for the CPU restatement (a test double with the same
``place()`` contract) to check the host logic (grouping, anchors, RNG, marshalling) without a
GPU; the gpu variant runs the real HIP engine.
"""
import numpy as np
import pytest

import fakes
import golden_io
from oracle import oracle
from pivot_place import policies


class OracleEngine:
    """Test double: the CPU restatement behind PlacementEngine.place()'s contract."""

    def place(self, r):
        return oracle.place(r)

    def anchor(self, off, lst, zone, inst_host=None):
        mode, az, rc = oracle.anchor(off, lst, zone, len(zone), inst_host)
        assert rc == 0
        return mode, az


CLASSES = {
    "cost_aware": policies.CostAwareGlobalScheduler,
    "opportunistic": policies.OpportunisticGlobalScheduler,
    "vbp_ff": policies.FirstFitGlobalScheduler,
    "vbp_bf": policies.BestFitGlobalScheduler,
}


def _run(name, idx, engine):
    case = golden_io.load(name)
    run = case["runs"][idx]
    cluster, tasks = fakes.build(case)
    sched = CLASSES[run["policy"]](None, cluster, seed=run["seed"], **run["kwargs"])
    sched.engine = engine
    sched._update_resource_info()
    resc = sched.resource_info
    err = None
    try:
        out = sched.schedule(list(tasks))
    except Exception as e:   # the reference's own failure modes (cost_aware.py:26,81)
        err = type(e).__name__
        out = []
    assert err == run["error"]
    hidx = {h.id: i for i, h in enumerate(cluster.hosts)}
    placement = np.array([-1 if t.placement is None else hidx[t.placement] for t in tasks])
    np.testing.assert_array_equal(placement, np.array(run["placement"]))
    pos = {id(t): i for i, t in enumerate(tasks)}
    assert [pos[id(t)] for t in out] == run["order"]
    after = np.array([resc[h.id] for h in cluster.hosts], dtype=np.float64).T
    _, _, avail, _ = golden_io.expected(case, run)
    assert np.array_equal(after, avail)
    st = sched.randomizer.get_state()
    ref = golden_io.mt_state(run["seed"], run["rng_draws"])
    assert list(st[1]) == list(ref[:624]) and st[2] == ref[624]


@pytest.mark.parametrize("name,idx", golden_io.all_runs(skip_errors=False))
def test_policy_host_logic(name, idx):
    _run(name, idx, OracleEngine())


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx", golden_io.all_runs(skip_errors=False))
def test_policy_on_engine(engine, name, idx):
    _run(name, idx, engine)


def _rt_case():
    """A recorded realtime_bw state (storage <-> host routes with queued packets)."""
    case = golden_io.load("rt_h12")
    run = next(r for r in case["runs"] if r["kwargs"].get("realtime_bw"))
    return case, run


@pytest.mark.parametrize("algo,sort_hosts,raises", [("first-fit", False, False),
                                                   ("first-fit", True, True),
                                                   ("best-fit", False, True)])
def test_realtime_bw_missing_route(algo, sort_hosts, raises):
    """realtime_bw with one storage <-> host route missing: the reference reads routes only in
    host_score_func (best-fit, and first-fit with sort_hosts; cost_aware.py:69-83, 104-119), so
    unsorted first-fit places as usual while the other two raise AttributeError."""
    case, run = _rt_case()
    cluster, tasks = fakes.build(case)
    h0 = cluster.hosts[0].id
    for s in cluster.storage:
        cluster._routes.pop((s.id, h0), None)
    sched = policies.CostAwareGlobalScheduler(None, cluster, seed=run["seed"],
                                              bin_pack_algo=algo, sort_tasks=True,
                                              sort_hosts=sort_hosts, realtime_bw=True)
    sched.engine = OracleEngine()
    sched._update_resource_info()
    if raises:
        with pytest.raises(AttributeError):
            sched.schedule(list(tasks))
    else:
        sched.schedule(list(tasks))
        assert any(t.placement is not None for t in tasks)


def test_realtime_rows_shared_by_anchor():
    """Groups of one anchor storage share one realtime row, read from the cluster's route
    objects once per round (the queues do not move inside schedule())."""
    case, run = _rt_case()
    cluster, tasks = fakes.build(case)
    sched = policies.CostAwareGlobalScheduler(None, cluster, seed=run["seed"], **run["kwargs"])
    memo = {}
    a = cluster.storage[0]
    row = sched._realtime_row(a, memo)
    assert sched._realtime_row(a, memo) is row
    want = [cluster.get_route(a.id, h.id).realtime_bw + cluster.get_route(h.id, a.id).realtime_bw
            for h in cluster.hosts]
    assert row.tolist() == want


def test_realtime_rows_see_replaced_routes():
    """A route replaced between rounds (the reference's cluster.add_route overwrites the
    (src, dst) entry, resources/__init__.py:106-109) is read in the next round: routes are
    looked up per schedule() call, never cached across rounds."""
    case, run = _rt_case()
    cluster, tasks = fakes.build(case)
    sched = policies.CostAwareGlobalScheduler(None, cluster, seed=run["seed"], **run["kwargs"])
    a, h0 = cluster.storage[0], cluster.hosts[0]
    first = sched._realtime_row(a, {})
    old = cluster.get_route(a.id, h0.id)
    cluster._routes[(a.id, h0.id)] = fakes.Route(old.bw, old.realtime_bw * 0.5 + 1.0)
    second = sched._realtime_row(a, {})
    assert second[0] == (old.realtime_bw * 0.5 + 1.0) + cluster.get_route(h0.id, a.id).realtime_bw
    assert second[0] != first[0]
    assert second[1:].tolist() == first[1:].tolist()
