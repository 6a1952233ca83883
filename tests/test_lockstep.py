"""Lock-step batched-scenario driver (pivot_place.lockstep).

Several simulations run side by side; every engine call their drop-in policies make is served
in batches -- every waiting round that fits the resident kernel, of every policy, in one
pvt_place_host_batch (the rest one by one) -- whenever every live simulation waits on the engine.

* replay (CPU restatement / GPU engine): recorded reference simulations (tests/golden/sim_*)
  replayed concurrently through the driver, every round compared with the reference's;
  duplicated traces make same-mode rounds share launches.
* whole simulations (build container only, needs the reference sources): the reference's own
  simulator on pivot_place.des, several simulations in lock-step through the driver; each
  one's end-to-end results (makespan, runtimes, instance hours, egress cost, rounds) equal its
  standalone run (reference scheduler/__init__.py:87-116, alibaba/runner.py:27-44).
"""
import json
import os
import subprocess
import sys

import pytest

import golden_io
from oracle import oracle
from pivot_place.lockstep import LockstepDriver
from test_sim_replay import MAKE_SIM, REF, _replay

REPLAY = ["sim_h12_cost_aware", "sim_h12_cost_aware", "sim_h12_cost_aware_bf",
          "sim_h12_opportunistic", "sim_h12_opportunistic", "sim_h12_vbp_ff", "sim_h12_vbp_bf",
          "sim_h12_vbp_bf", "sim_c1_cost_aware", "sim_c1_vbp_ff"]


class BatchOracle:
    """The CPU restatement behind the batched engine contract."""

    def place(self, r):
        return oracle.place(r)

    def place_batch(self, rounds):
        return [oracle.place(r) for r in rounds]

    def anchor(self, off, lst, zone, inst_host=None):
        mode, az, rc = oracle.anchor(off, lst, zone, len(zone), inst_host)
        assert rc == 0
        return mode, az


def _lockstep_replay(engine):
    driver = LockstepDriver(engine)
    traces = driver.run([lambda eng, n=n: _replay(n, eng) for n in REPLAY])
    assert [t["name"] for t in traces] == REPLAY
    st = driver.stats
    assert st["place_calls"] > st["place_launches"], st     # rounds shared launches
    assert st["max_rounds_per_launch"] >= 2, st
    return st


def test_lockstep_replay_host_logic():
    st = _lockstep_replay(BatchOracle())
    # (no fused path on the restatement: cost_aware rounds anchor first, in shared calls)
    assert st["anchor_calls"] > st["anchor_launches"], st


@pytest.mark.gpu
def test_lockstep_replay_on_engine(engine):
    """On the GPU engine every tick's rounds -- four policies, cost_aware grouping fused -- go
    to one pvt_place_host_batch: rounds of different policies share a launch."""
    st = _lockstep_replay(engine)
    assert st["host_batch_rounds"] == st["place_calls"], st
    assert st["fused_rounds"] > 0 and st["anchor_calls"] == 0, st
    assert st["max_rounds_per_launch"] >= 6, st


@pytest.mark.gpu
def test_lockstep_replay_resident_off(engine):
    """With the resident kernel switched off (set_resident(0)) host_batch_fits must refuse every
    round pvt_place_host_batch would reject, so the driver serves them one by one (fused
    cost_aware calls and windowed rounds) -- every round still bit-exact, no error."""
    from pivot_place import _abi
    engine.set_resident(0)
    try:
        driver = LockstepDriver(engine)
        traces = driver.run([lambda eng, n=n: _replay(n, eng) for n in REPLAY])
        assert [t["name"] for t in traces] == REPLAY
        assert driver.stats["host_batch_rounds"] == 0, driver.stats
    finally:
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)


def test_driver_propagates_errors():
    class Boom(BatchOracle):
        def place_batch(self, rounds):
            raise RuntimeError("engine failed")

    def sim(eng):
        from pivot_place import synthetic, _abi
        return eng.place(synthetic.make_round(_abi.PVT_VBP_FF, 50, 10, seed=1))

    with pytest.raises(RuntimeError, match="engine failed"):
        LockstepDriver(Boom()).run([sim, sim])


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference sources (build container)")
def test_lockstep_whole_simulations_equal_standalone():
    names = ["sim_h12_cost_aware", "sim_h12_cost_aware", "sim_h12_opportunistic",
             "sim_h12_vbp_ff", "sim_h12_vbp_bf", "sim_h12_cost_aware_bf"]
    out = subprocess.run([sys.executable, MAKE_SIM, "--lockstep"] + names, capture_output=True,
                         text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-2000:]
    got = json.loads(out.stdout.strip().splitlines()[-1])
    assert got["names"] == names
    for name, e2e in zip(names, got["e2e"]):
        want = golden_io.load(name)["e2e"]
        for k, v in want.items():
            if k != "reference_wall_s":
                assert e2e[k] == v, (name, k, e2e[k], v)
    st = got["stats"]
    assert st["max_rounds_per_launch"] >= 2 and st["place_calls"] > st["place_launches"], st
