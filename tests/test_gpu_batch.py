"""Scenario batches through pvt_place_batch (resident kernel, one workgroup per round): every
round of a batch must equal the CPU restatement run on that round alone (placement, order,
final availability and MT19937 state bit for bit), whatever the batch mixes."""
import numpy as np
import pytest

import golden_io
from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu

ALL_MODES = [_abi.PVT_CA_FF, _abi.PVT_CA_BF, _abi.PVT_OPP, _abi.PVT_VBP_FF, _abi.PVT_VBP_BF]


def _assert_same(res, ref, tag=""):
    np.testing.assert_array_equal(res.placement, ref.placement, err_msg=tag)
    np.testing.assert_array_equal(res.order, ref.order, err_msg=tag)
    same = (res.avail == ref.avail) | (np.isnan(res.avail) & np.isnan(ref.avail))
    bad = np.nonzero((~same).any(axis=0))[0]
    assert bad.size == 0, "%s: availability differs on hosts %s" % (tag, bad[:10])
    if ref.mt_state is not None:
        np.testing.assert_array_equal(res.mt_state, ref.mt_state, err_msg=tag)


@pytest.mark.parametrize("mode", ALL_MODES)
def test_batch_of_scenarios_matches_oracle(engine, mode):
    """64 independent scenarios (seed per scenario, config 4 shape scaled down) in one launch."""
    rounds = [synthetic.make_round(mode, 1000, 300, seed=100 + s) for s in range(64)]
    got = engine.place_batch(rounds)
    for s, (r, res) in enumerate(zip(rounds, got)):
        _assert_same(res, oracle.place(r), "scenario %d" % s)


@pytest.mark.parametrize("mode", ALL_MODES)
def test_batch_mixed_shapes(engine, mode):
    """Rounds of different sizes share one launch (registers sized for the largest; padding
    hosts never fit, shorter task lists end early), including empty and single-host rounds."""
    shapes = [(1, 5), (7, 0), (64, 2000), (100, 1), (4096, 300), (257, 4096), (1000, 1000),
              (3, 3)]
    rounds = [synthetic.make_round(mode, H, T, seed=7 + i) for i, (H, T) in enumerate(shapes)]
    got = engine.place_batch(rounds)
    for (H, T), r, res in zip(shapes, rounds, got):
        _assert_same(res, oracle.place(r), "H=%d T=%d" % (H, T))


@pytest.mark.parametrize("mode", ALL_MODES)
def test_batch_crowded_and_tied(engine, mode):
    """Identical nearly full hosts: ties everywhere, exhaustion, unplaceable tasks."""
    rounds = []
    for s in range(16):
        r = synthetic.make_round(mode, 500, 1200, seed=40 + s)
        r.avail[0, :] = 4.0
        r.avail[1, :] = 40000.0
        r.avail[0, s::7] = 0.5
        rounds.append(r)
    got = engine.place_batch(rounds)
    for s, (r, res) in enumerate(zip(rounds, got)):
        _assert_same(res, oracle.place(r), "scenario %d" % s)


@pytest.mark.parametrize("resident", [True, False])
def test_ca_bf_zero_scores_and_underflow(engine, resident):
    """cost_aware best-fit scores of exactly 0 (free zone pairs, exact fits in costly zones) and
    scores that underflow to 0 from a subnormal egress cost: ties at 0 go to the lowest host."""
    rounds = []
    for s in range(8):
        r = synthetic.make_round(_abi.PVT_CA_BF, 600, 400, seed=70 + s)
        r.cost = r.cost.copy()
        r.cost[:, 1] = 5e-324 if s % 2 else 1e-300      # zone 1: (sub)normal tiny egress cost
        r.cost[1, :] = 0.0 if s % 3 else r.cost[1, :]
        # exact fits: some hosts hold exactly the demand of some tasks
        for k in range(0, 600, 37):
            t = (k * 7 + s) % r.n_tasks
            r.avail[:, k] = r.dem[:, t]
        rounds.append(r)
    if resident:
        got = engine.place_batch(rounds)
    else:
        engine.set_resident(0)
        try:
            got = [engine.place(r) for r in rounds]
        finally:
            engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)
    for s, (r, res) in enumerate(zip(rounds, got)):
        _assert_same(res, oracle.place(r), "scenario %d" % s)


def test_ca_bf_range_edges(engine):
    """Resident cost_aware best-fit at the edges of its fast winner's safe range: capacities and
    demands beyond 2^498, residuals of 2^-300 and just below (near-exact fits, exact fits in the
    other dimensions) and negative demands that grow a host past 2^498.
    (Magnitudes stay below ~1e153 so no residual norm overflows: a NaN score -- 0 * inf -- is
    outside the engine's numerics, DESIGN.md "Numerics".)"""
    rounds = []
    for s in range(8):
        r = synthetic.make_round(_abi.PVT_CA_BF, 700, 500, seed=90 + s)
        r.avail = r.avail.copy()
        r.dem = r.dem.copy()
        r.avail[:, 3::41] = 1e152                       # insane hosts (> 2^498 ~ 8.2e149)
        r.avail[1, 5::43] = 2.0 ** 499
        for k in range(7, 700, 29):                     # one residual 2^-300 / just under, rest 0
            t = (k * 3 + s) % r.n_tasks
            dim = (k // 2) % 2                          # (cpu or memory)
            r.dem[dim, t] = 0.0
            r.avail[:, k] = r.dem[:, t]
            r.avail[dim, k] = 2.0 ** -300 if k % 2 else 2.0 ** -301
        r.dem[:, 11::97] = -1e151                       # out-of-range (negative) demands
        r.dem[2, 13::89] = 1e151
        rounds.append(r)
    got = engine.place_batch(rounds)
    for s, (r, res) in enumerate(zip(rounds, got)):
        _assert_same(res, oracle.place(r), "scenario %d" % s)


@pytest.mark.parametrize("mode", ALL_MODES)
def test_resident_dim_edges(engine, mode):
    """Demands in the third / fourth dimensions (growing, negative, exactly the capacity), a NaN
    capacity, and -inf demands against padded lanes (H not a multiple of the lanes: padding
    slots must never fit)."""
    rounds = []
    for s in range(12):
        H = 700 + 37 * s
        r = synthetic.make_round(mode, H, 600, seed=300 + s)
        r.avail = r.avail.copy()
        r.dem = r.dem.copy()
        rs = np.random.RandomState(s)
        if s % 4 == 0:
            r.dem[2] = rs.uniform(0, 0.5, r.n_tasks)          # the bound shrinks every commit
        elif s % 4 == 1:
            r.dem[3, ::3] = -rs.uniform(0, 0.01, len(r.dem[3, ::3]))   # negative: bound kept
            r.dem[2, ::7] = 30.0                                  # above some hosts' capacity
            r.avail[2, ::5] = 20.0
        elif s % 4 == 2:
            r.avail[3, 11] = np.nan                               # the bounds are void
            r.dem[3] = rs.uniform(0, 0.001, r.n_tasks)
        else:
            if mode in (_abi.PVT_VBP_FF, _abi.PVT_OPP, _abi.PVT_CA_FF):
                r.dem[0, 5::50] = -np.inf                         # fits every real host
                r.dem[1, 5::50] = -np.inf
            r.dem[2, 9::11] = 100.0                               # exactly the capacity
        rounds.append(r)
    got = engine.place_batch(rounds)
    for s, (r, res) in enumerate(zip(rounds, got)):
        _assert_same(res, oracle.place(r), "scenario %d" % s)


def test_batch_golden_runs(engine):
    """Every golden run (reference schedule() calls) batched per policy configuration."""
    by_mode = {}
    for name, idx in golden_io.all_runs():
        case = golden_io.load(name)
        run = case["runs"][idx]
        r = golden_io.run_arrays(case, run)
        by_mode.setdefault(r.mode, []).append((r, golden_io.expected(case, run), "%s#%d" % (name, idx)))
    for mode, items in by_mode.items():
        got = engine.place_batch([r for r, _, _ in items])
        for (r, exp, tag), res in zip(items, got):
            placement, order, avail = exp[:3]
            np.testing.assert_array_equal(res.placement, placement, err_msg=tag)
            np.testing.assert_array_equal(res.order, order, err_msg=tag)
            assert np.array_equal(res.avail, avail), tag
            if len(exp) > 3 and exp[3] is not None:
                np.testing.assert_array_equal(res.mt_state, exp[3], err_msg=tag)


def test_batch_limits_and_errors(engine):
    r_big = synthetic.make_round(_abi.PVT_CA_BF, _abi.PVT_RESIDENT_MAX_HOSTS + 1, 10, seed=1)
    with pytest.raises(RuntimeError, match="EUNSUPPORTED"):
        engine.place_batch([r_big])
    # pvt_place takes the windowed path for it and still matches
    _assert_same(engine.place(r_big), oracle.place(r_big), "H=4097 via pvt_place")
    r_long = synthetic.make_round(_abi.PVT_VBP_BF, 100, _abi.PVT_RESIDENT_MAX_TASKS + 1, seed=2)
    with pytest.raises(RuntimeError, match="EUNSUPPORTED"):
        engine.place_batch([r_long])
    _assert_same(engine.place(r_long), oracle.place(r_long), "T=4097 via pvt_place")
    mixed = [synthetic.make_round(_abi.PVT_CA_BF, 100, 10, seed=3),
             synthetic.make_round(_abi.PVT_VBP_FF, 100, 10, seed=3)]
    with pytest.raises(RuntimeError, match="EINVAL"):
        engine.place_batch(mixed)
    assert engine.place_batch([]) == []


def test_batch_repeated_runs_are_identical(engine):
    """A resident batch reset and re-run gives the same results (no state leaks between runs)."""
    from pivot_place.engine import DeviceBatch
    rounds = [synthetic.make_round(_abi.PVT_OPP, 800, 900, seed=60 + s) for s in range(8)]
    b = DeviceBatch(rounds, engine.device)
    engine.run_batch(b)
    first = b.results()
    b.reset()
    engine.run_batch(b)
    for a, c in zip(first, b.results()):
        _assert_same(c, a)


@pytest.mark.parametrize("mode", ALL_MODES)
def test_scenario_driver_on_gpu(engine, mode):
    """pivot_place.scenarios.run_block on the GPU engine (batched launches) equals the CPU
    restatement run scenario by scenario (per-scenario digests of placements + availability)."""
    from pivot_place import scenarios

    class Cpu:
        def place(self, r):
            return oracle.place(r)

    seeds = list(range(500, 540))
    assert scenarios.run_block(engine, mode, 700, 250, seeds, batch=16) == \
        scenarios.run_block(Cpu(), mode, 700, 250, seeds)
