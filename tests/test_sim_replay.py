"""Every round of the reference's end-to-end Alibaba simulations, replayed through the drop-in
policies (BASELINE.json config 1 and the config-2 shape).

``tests/golden/sim_*.json.gz`` hold each non-empty ``schedule()`` round of the reference's own
simulation (alibaba/runner.py:27-51 driven by ``pivot_place.des``; tests/golden/
make_golden_sim.py): the snapshot the policy saw, the ready queue with predecessor placements,
and the reference's placements, returned order, snapshot updates and RandomState draws. The
replay drives one policy object per round the way the round loop does
(scheduler/__init__.py:100-103) and carries ONE RandomState through the rounds, as the
simulation's scheduler does. A replay that matches every round reproduces the whole simulated
trajectory, and with it the end-to-end numbers recorded beside the rounds (makespan, average
application runtime, instance hours, egress cost).

CPU variant: the CPU restatement behind the engine contract (host logic: grouping, anchors,
RNG, marshalling). gpu variant: the HIP engine.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import fakes
import golden_io
from oracle import oracle
from pivot_place import policies

CLASSES = {
    "cost_aware": policies.CostAwareGlobalScheduler,
    "opportunistic": policies.OpportunisticGlobalScheduler,
    "vbp_ff": policies.FirstFitGlobalScheduler,
    "vbp_bf": policies.BestFitGlobalScheduler,
}
TRACES = golden_io.sim_traces()
REF = os.environ.get("PIVOT_REFERENCE", "/root/reference")
MAKE_SIM = os.path.join(golden_io.GOLDEN, "make_golden_sim.py")


class OracleEngine:
    def place(self, r):
        return oracle.place(r)

    def anchor(self, off, lst, zone, inst_host=None):
        mode, az, rc = oracle.anchor(off, lst, zone, len(zone), inst_host)
        assert rc == 0
        return mode, az


def _replay(name, engine):
    tr, cases = golden_io.sim_rounds(name)
    cls = CLASSES[tr["policy"]]
    carried = np.random.RandomState(tr["seed"])    # the scheduler's own RNG, across rounds
    shadow = np.random.RandomState(tr["seed"])
    placed = 0
    for k, case in enumerate(cases):
        run = case["runs"][0]
        cluster, tasks = fakes.build(case)
        sched = cls(None, cluster, seed=tr["seed"], **tr["kwargs"])
        sched.randomizer.set_state(carried.get_state())
        sched.engine = engine
        sched._update_resource_info()
        resc = sched.resource_info
        out = sched.schedule(list(tasks))
        hidx = {h.id: i for i, h in enumerate(cluster.hosts)}
        placement = [-1 if t.placement is None else hidx[t.placement] for t in tasks]
        assert placement == run["placement"], "round %d (t=%s)" % (k, case["time"])
        pos = {id(t): i for i, t in enumerate(tasks)}
        assert [pos[id(t)] for t in out] == run["order"], "round %d order" % k
        after = np.array([resc[h.id] for h in cluster.hosts], dtype=np.float64).T
        _, _, avail, _ = golden_io.expected(case, run)
        assert np.array_equal(after, avail), "round %d availability" % k
        for _ in range(run["rng_draws"]):
            shadow.randint(0, 1 << 32, dtype=np.uint32)
        st, ref = sched.randomizer.get_state(), shadow.get_state()
        assert st[2] == ref[2] and np.array_equal(st[1], ref[1]), "round %d RNG" % k
        carried.set_state(st)
        placed += sum(p >= 0 for p in placement)
    assert placed == tr["e2e"]["tasks_placed"]
    return tr


def test_traces_present():
    names = set(TRACES)
    for cfg in ("c1", "h12"):
        for pol in ("opportunistic", "vbp_ff", "cost_aware", "cost_aware_bf", "vbp_bf"):
            assert "sim_%s_%s" % (cfg, pol) in names
    for pol in ("opportunistic", "vbp_ff", "cost_aware"):
        assert "sim_c2_%s" % pol in names


def test_trace_consistency():
    """Each trace's rounds account for the whole workload (every task placed once; the
    contention traces retry unplaced tasks in later rounds)."""
    for name in TRACES:
        tr, cases = golden_io.sim_rounds(name)
        e = tr["e2e"]
        assert e["n_apps_finished"] == tr["n_apps"]
        assert len(cases) == e["rounds"] - e["empty_rounds"]
        times = [c["time"] for c in cases]
        assert times == sorted(times) and len(set(times)) == len(times)
        assert all(t % 5 == times[0] % 5 for t in times)    # rounds every interval=5


@pytest.mark.parametrize("name", TRACES)
def test_sim_replay_host_logic(name):
    _replay(name, OracleEngine())


@pytest.mark.gpu
@pytest.mark.parametrize("name", TRACES)
def test_sim_replay_on_engine(engine, name):
    _replay(name, engine)


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference sources (build container)")
@pytest.mark.parametrize("name", ["sim_h12_cost_aware", "sim_h12_cost_aware_bf",
                                  "sim_h12_opportunistic", "sim_h12_vbp_ff", "sim_h12_vbp_bf"])
def test_dropin_inside_reference_simulator(name):
    """The drop-in mixins on the reference's own GlobalSchedulerBase, plugged into the
    reference's simulator on ``pivot_place.des``, with the CPU restatement
    behind the engine contract: the end-to-end results equal the reference policies' run —
    makespan, average application runtime, instance hours, egress cost (exact)."""
    out = subprocess.run([sys.executable, MAKE_SIM, "--dropin", name], capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    got = json.loads(out.stdout.strip().splitlines()[-1])
    want = golden_io.load(name)["e2e"]
    for k, v in want.items():
        if k != "reference_wall_s":
            assert got[k] == v, (k, got[k], v)
