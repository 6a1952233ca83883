"""GPU parity at the benchmark sizes (BASELINE.json configs 4 and 5).

The round bench.py times -- 1M hosts x 10k ready tasks, 20 zones, seed 20261015 -- is placed
by the HIP engine (through the C ABI) for every policy and compared with the CPU restatement
(oracle/pivot_oracle.c, itself pinned to the reference's golden runs) bit for bit: placement,
processing order and final availability (and the MT19937 state for opportunistic). This is
where the engine's size-dependent heuristics are active: 16 host segments, 1000-task windows,
adaptive refills, the 4-tasks-per-wave score instance of cost_aware best-fit (>= 262144 hosts).

Config 4 at its per-GPU size: 512 scenarios x (1000 hosts x 1000 tasks), one pvt_place_batch
launch per policy, every scenario against the oracle.

Reference loops: scheduler/cost_aware.py:63-127, scheduler/opportunistic.py:11-20,
scheduler/vbp.py:13-50.
"""
import os

import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu

H5, T5, SEED5 = 1_000_000, 10_000, 20261015
ALL_MODES = [_abi.PVT_CA_FF, _abi.PVT_CA_BF, _abi.PVT_OPP, _abi.PVT_VBP_FF, _abi.PVT_VBP_BF]


def oracle_threads():
    """The CPU share of this job (16 per GPU on the box; OMP_NUM_THREADS is set there)."""
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env else min(16, os.cpu_count() or 1)


_cache = {}


def headline(mode):
    """(round, oracle result) of the config-5 round for ``mode``, computed once per session."""
    if mode not in _cache:
        r = synthetic.make_round(mode, H5, T5, seed=SEED5)
        _cache[mode] = (r, oracle.place(r, threads=oracle_threads()))
    return _cache[mode]


def assert_same(res, ref, what):
    np.testing.assert_array_equal(res.order, ref.order, err_msg=what + ": order")
    bad = np.nonzero(res.placement != ref.placement)[0]
    assert bad.size == 0, "%s: %d placements differ, first at processing position(s) %s" % (
        what, bad.size, bad[:5])
    bad = np.nonzero((res.avail != ref.avail).any(axis=0))[0]
    assert bad.size == 0, "%s: availability differs on hosts %s" % (what, bad[:10])
    if ref.mt_state is not None:
        np.testing.assert_array_equal(res.mt_state, ref.mt_state, err_msg=what + ": RNG state")


@pytest.mark.parametrize("mode", ALL_MODES, ids=lambda m: _abi.MODE_NAMES[m])
def test_config5_round_matches_oracle(engine, mode):
    r, ref = headline(mode)
    assert (ref.placement >= 0).sum() > 0
    assert_same(engine.place(r), ref, "config 5 %s" % _abi.MODE_NAMES[mode])


@pytest.mark.parametrize("tw", [2, 4])
@pytest.mark.parametrize("mode", [_abi.PVT_CA_BF, _abi.PVT_VBP_BF], ids=lambda m: _abi.MODE_NAMES[m])
def test_config5_both_score_instances(engine, mode, tw):
    """The score kernel's 2- and 4-tasks-per-wave instances (pvt_set_score_tw) at 1M hosts."""
    r, ref = headline(mode)
    try:
        engine.set_score_tw(tw)
        engine.set_band(0)      # vbp best-fit: the streaming score pass (band lists: default)
        res = engine.place(r)
    finally:
        engine.set_score_tw(0)
        engine.set_band(65536)
    assert_same(res, ref, "config 5 %s tw=%d" % (_abi.MODE_NAMES[mode], tw))


def test_config5_sequential_windows(engine):
    """The same headline round with the window pipeline off (strictly sequential windows)."""
    r, ref = headline(_abi.PVT_CA_BF)
    try:
        engine.set_pipeline(False)
        res = engine.place(r)
    finally:
        engine.set_pipeline(True)
    assert_same(res, ref, "config 5 cost_aware_bf sequential")


@pytest.mark.parametrize("mode", ALL_MODES, ids=lambda m: _abi.MODE_NAMES[m])
def test_config4_batch_per_gpu_matches_oracle(engine, mode):
    """512 independent scenarios of 1000 hosts x 1000 tasks in one pvt_place_batch launch."""
    rounds = [synthetic.make_round(mode, 1000, 1000, seed=SEED5 + s) for s in range(512)]
    got = engine.place_batch(rounds)
    for s, (r, res) in enumerate(zip(rounds, got)):
        assert_same(res, oracle.place(r), "config 4 %s scenario %d" % (_abi.MODE_NAMES[mode], s))


@pytest.fixture(scope="module")
def shard_engines():
    from pivot_place.engine import PlacementEngine
    return [PlacementEngine(0) for _ in range(8)]


@pytest.mark.parametrize("mode", ALL_MODES, ids=lambda m: _abi.MODE_NAMES[m])
def test_config5_host_sharded_world8(shard_engines, mode):
    """BASELINE config 5 as written: the host dimension split 8 ways (8 contexts in lock-step on
    one GPU, exchange by concatenation -- the same packages an RCCL all-gather carries). cost_aware
    best-fit runs frontier-walked epochs, first-fit the keyed / ordered frontier walks, the others
    their list windows; every rank equals the oracle."""
    from pivot_place.sharded import place_lockstep
    r, ref = headline(mode)
    outs = place_lockstep(shard_engines, r)
    for k, o in enumerate(outs):
        assert_same(o, ref, "config 5 %s host-sharded rank %d/8" % (_abi.MODE_NAMES[mode], k))
    if mode in (_abi.PVT_CA_BF, _abi.PVT_CA_FF, _abi.PVT_VBP_FF):
        st = shard_engines[0].epoch_stats()
        assert st["frontier_chains"] > 0, st
