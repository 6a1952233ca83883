"""The drop-in cost_aware round in ONE device round trip (pvt_place_host with pvt_ca_items):
grouping, mode-host anchors, the randomizer draws of application groups and the placement all
on the device. Checked against the reference's recorded schedule() runs (placements, returned
order, snapshot arrays, RandomState after the draws) with a spy that proves the fused path ran
(no silent fallback to the two-call path), and against the two-call path on whole recorded
simulations."""
import numpy as np
import pytest

import fakes
import golden_io
from pivot_place import policies

pytestmark = pytest.mark.gpu


class Spy:
    """The GPU engine, counting fused rounds; the two-call entry points fail the test."""

    def __init__(self, eng, allow_two_call=False):
        self.eng = eng
        self.fused = 0
        self.allow = allow_two_call

    def place_cost_aware(self, *a, **k):
        got = self.eng.place_cost_aware(*a, **k)
        assert got is not None
        self.fused += 1
        return got

    def place(self, r):
        assert self.allow, "two-call path taken"
        return self.eng.place(r)

    def anchor(self, *a, **k):
        assert self.allow, "two-call path taken"
        return self.eng.anchor(*a, **k)


def _cost_aware_runs():
    out = []
    for name, idx in golden_io.all_runs(skip_errors=False):
        run = golden_io.load(name)["runs"][idx]
        kw = run["kwargs"]
        if (run["policy"] == "cost_aware" and not kw.get("realtime_bw")
                and kw.get("bin_pack_algo", "first-fit") in ("first-fit", "best-fit")
                and not (kw.get("bin_pack_algo") == "best-fit" and kw.get("host_decay"))):
            out.append((name, idx))
    return out


@pytest.mark.parametrize("name,idx", _cost_aware_runs())
def test_fused_round_matches_reference(engine, name, idx):
    case = golden_io.load(name)
    run = case["runs"][idx]
    cluster, tasks = fakes.build(case)
    sched = policies.CostAwareGlobalScheduler(None, cluster, seed=run["seed"], **run["kwargs"])
    spy = Spy(engine)
    sched.engine = spy
    sched._update_resource_info()
    resc = sched.resource_info
    err = None
    try:
        sched.schedule(list(tasks))
    except Exception as e:
        err = type(e).__name__
    assert err == run["error"]
    if err is None and tasks:
        assert spy.fused == 1
    hidx = {h.id: i for i, h in enumerate(cluster.hosts)}
    placement = np.array([-1 if t.placement is None else hidx[t.placement] for t in tasks])
    np.testing.assert_array_equal(placement, np.array(run["placement"]))
    after = np.array([resc[h.id] for h in cluster.hosts], dtype=np.float64).T
    _, _, avail, _ = golden_io.expected(case, run)
    if err is None:
        assert np.array_equal(after, avail)
        st = sched.randomizer.get_state()
        ref = golden_io.mt_state(run["seed"], run["rng_draws"])
        assert list(st[1]) == list(ref[:624]) and st[2] == ref[624]


@pytest.mark.parametrize("name", ["sim_c1_cost_aware", "sim_c2a1000_cost_aware"])
def test_fused_replay_equals_reference_rounds(engine, name):
    """Every round of a recorded reference simulation through the fused path: the reference's
    placements in every round, and every non-empty round fused."""
    tr, cases = golden_io.sim_rounds(name)
    cluster, _ = fakes.build(cases[0])
    sched = policies.CostAwareGlobalScheduler(None, cluster, seed=tr["seed"], **tr["kwargs"])
    spy = Spy(engine)
    sched.engine = spy
    hidx = {h.id: i for i, h in enumerate(cluster.hosts)}
    nonempty = 0
    for case in cases:
        fakes.refresh(cluster, case)
        tasks = fakes.build_tasks(case, cluster)
        nonempty += bool(tasks)
        sched._update_resource_info()
        sched.schedule(list(tasks))
        got = [-1 if t.placement is None else hidx[t.placement] for t in tasks]
        assert got == case["runs"][0]["placement"]
    assert spy.fused == nonempty
