"""The one-wave resident walk (pvt_batch.hip resident_walk): cost_aware best-fit rounds of up to
1024 hosts (score-0 winners) are walked by one wave over their hosts in LDS, and the 4-wave path
takes over where the walk stops. (The walk also handles keyed / unsorted cost_aware first-fit and
vbp first-fit, but those modes run the 4-wave path, measured faster; their cases stay here as
resident-path checks of the same shapes.) Every round must equal the CPU restatement, including rounds
built to stop the walk: no score-0 host (anchor zones without capacity), subnormal egress costs
(risky scores), zero-key hosts running out inside a keyed group (the group's frozen keys are
handed over), unplaceable tasks; and the same batch with the walk off (PVT_RWALK=0)."""
import os

import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic
from pivot_place.engine import PlacementEngine

pytestmark = pytest.mark.gpu

WALKED = [_abi.PVT_CA_BF, _abi.PVT_CA_FF, _abi.PVT_VBP_FF]


def _same(got, ref, what):
    np.testing.assert_array_equal(got.placement, ref.placement, err_msg=what)
    np.testing.assert_array_equal(got.order, ref.order, err_msg=what)
    assert np.array_equal(got.avail, ref.avail), what


@pytest.fixture(scope="module")
def engine_nowalk():
    old = os.environ.get("PVT_RWALK")
    os.environ["PVT_RWALK"] = "0"
    try:
        eng = PlacementEngine(0)
    finally:
        if old is None:
            del os.environ["PVT_RWALK"]
        else:
            os.environ["PVT_RWALK"] = old
    return eng


def _check(engine, engine_nowalk, rounds, what):
    got = engine.place_batch(rounds)
    off = engine_nowalk.place_batch(rounds)
    for i, (r, g, o) in enumerate(zip(rounds, got, off)):
        ref = oracle.place(r)
        _same(g, ref, "%s round %d (walk)" % (what, i))
        _same(o, ref, "%s round %d (no walk)" % (what, i))


@pytest.mark.parametrize("mode", WALKED)
@pytest.mark.parametrize("H,T", [(1000, 1000), (1, 7), (64, 300), (65, 65), (1024, 4096), (700, 2000)])
def test_walked_rounds_match_oracle(engine, engine_nowalk, mode, H, T):
    rounds = [synthetic.make_round(mode, H, T, seed=11 + s) for s in range(6)]
    _check(engine, engine_nowalk, rounds, "mode %d H=%d T=%d" % (mode, H, T))


@pytest.mark.parametrize("sort_hosts", [True, False])
def test_cost_aware_first_fit_both_orders(engine, engine_nowalk, sort_hosts):
    rounds = [synthetic.make_round(_abi.PVT_CA_FF, 900, 1500, seed=40 + s, sort_hosts=sort_hosts)
              for s in range(4)]
    _check(engine, engine_nowalk, rounds, "ca_ff sort_hosts=%s" % sort_hosts)


@pytest.mark.parametrize("mode", [_abi.PVT_CA_BF, _abi.PVT_CA_FF])
def test_walk_stops_without_zero_class_host(engine, engine_nowalk, mode):
    """Zones 0-11 hold no capacity: groups anchored there find no score-0 / key-0 host, the walk
    stops (for keyed first-fit inside the group, whose frozen keys the 4-wave path takes over)."""
    rounds = []
    for s in range(5):
        r = synthetic.make_round(mode, 1000, 1200, seed=60 + s)
        r.avail[:2, r.zone < 12] = 0.0
        rounds.append(r)
    _check(engine, engine_nowalk, rounds, "no zero-class hosts mode %d" % mode)


def test_keyed_zero_hosts_run_out_inside_a_group(engine, engine_nowalk):
    """Few zero-key hosts with little memory: they fill in the middle of a group, so the walk
    stops there and the 4-wave path goes on with the group's keys frozen at its start."""
    rounds = []
    for s in range(5):
        r = synthetic.make_round(_abi.PVT_CA_FF, 1000, 2000, seed=80 + s)
        r.avail[1] = np.minimum(r.avail[1], 9000.0)
        rounds.append(r)
    _check(engine, engine_nowalk, rounds, "keyed run-out")


def test_best_fit_risky_scores(engine, engine_nowalk):
    """Subnormal egress costs: a fitting host may score 0 by underflow (risky): the walk stops
    before letting a later host win."""
    rounds = []
    for s in range(4):
        r = synthetic.make_round(_abi.PVT_CA_BF, 800, 800, seed=90 + s)
        r.cost = r.cost.copy()
        r.cost[r.cost > 0] = 1e-310
        rounds.append(r)
    _check(engine, engine_nowalk, rounds, "risky")


def test_vbp_first_fit_unplaceable_tasks(engine, engine_nowalk):
    rounds = []
    for s in range(4):
        r = synthetic.make_round(_abi.PVT_VBP_FF, 500, 3000, seed=100 + s)
        r.dem[0, ::7] = 100.0                       # every 7th task fits no host
        rounds.append(r)
    _check(engine, engine_nowalk, rounds, "unplaceable")


def test_mixed_host_batch_walks(engine):
    """pvt_place_host_batch with every policy: the walked modes and the others in one launch."""
    modes = [_abi.PVT_CA_FF, _abi.PVT_CA_BF, _abi.PVT_OPP, _abi.PVT_VBP_FF, _abi.PVT_VBP_BF]
    rounds = [synthetic.make_round(modes[i % 5], 1000, 200 + 13 * i, seed=120 + i) for i in range(15)]
    got = engine.place_host_batch([(r, None) for r in rounds])
    for i, (r, g) in enumerate(zip(rounds, got)):
        ref = oracle.place(r)
        _same(g, ref, "mixed %d" % i)
        if ref.mt_state is not None:
            assert np.array_equal(g.mt_state, ref.mt_state)


@pytest.mark.parametrize("mode", [_abi.PVT_CA_BF, _abi.PVT_CA_FF, _abi.PVT_VBP_FF, _abi.PVT_VBP_BF,
                                  _abi.PVT_OPP])
def test_sticky_runs_of_equal_demands(engine, engine_nowalk, mode):
    """Long runs of bit-identical demands on hosts that take an exact number of copies (capacity
    a multiple of the demand: the last copy leaves exactly 0, which fits a >= policy once more
    and a strict one not): the sticky winner must hand over to the next host exactly where the
    sequential loop does; a run with a negative demand component keeps the full selection."""
    rounds = []
    for s in range(4):
        r = synthetic.make_round(mode, 600, 900, seed=140 + s)
        rows = np.array([[0.5, 2048.0], [1.0, 4096.0], [0.25, 1024.0]])
        pick = np.sort(np.random.RandomState(s).randint(0, 3, size=r.n_tasks))
        r.dem[0], r.dem[1] = rows[pick, 0], rows[pick, 1]
        r.avail[0] = 0.5 * np.random.RandomState(50 + s).randint(0, 9, size=r.n_hosts)
        r.avail[1] = 2048.0 * np.random.RandomState(60 + s).randint(0, 9, size=r.n_hosts)
        if s == 3:
            r.dem[2, 100:140] = -1.0                # (a run with a negative demand component)
        rounds.append(r)
    _check(engine, engine_nowalk, rounds, "sticky runs mode %d" % mode)


def test_negative_egress_cost_is_refused(engine):
    """Egress costs are prices: include/pivot_place.h requires cost[a][z] + cost[z][a] >= +0
    (and bw sums > 0) -- the engine orders cost_aware scores >= +0 by their bits and keeps a
    best-fit winner while its residual shrinks. Host-array calls check the contract and refuse a
    round that breaks it (PVT_EINVAL) instead of placing it differently from the reference."""
    for mode in (_abi.PVT_CA_BF, _abi.PVT_CA_FF):
        for H in (600, 20_000):                   # the resident kernel and the windowed engine
            r = synthetic.make_round(mode, H, 300, seed=160)
            r.cost = np.where(r.cost > 0, -r.cost, 0.0)
            with pytest.raises(Exception, match="cost sum"):
                engine.place(r)
            r.cost = np.where(r.cost < 0, 0.0, r.cost)
            r.bw = np.zeros_like(r.bw)
            with pytest.raises(Exception, match="bw sum"):
                engine.place(r)


def test_zero_cost_window_certificates(engine, engine_nowalk):
    """The walk's zero-cost window (dense chunks of the anchor's zero-cost hosts) is used only
    under its certificates: rounds where other hosts fit some tasks exactly (score 0 outside the
    window: certificate (ii) fails), where they have residuals below 2^-300 (risky), and where
    the window runs dry mid-group (the 4-wave path takes over with positive scores)."""
    rounds = []
    for s in range(6):
        r = synthetic.make_round(_abi.PVT_CA_BF, 900, 1200, seed=200 + s)
        if s % 3 == 0:                          # exact fits on hosts of every zone
            r.avail[:, ::7] = r.dem[:, (np.arange(r.n_hosts)[::7] * 13) % r.n_tasks]
        elif s % 3 == 1:                        # residuals below 2^-300 on some hosts
            k = (np.arange(r.n_hosts)[::11] * 7) % r.n_tasks
            r.avail[:, ::11] = r.dem[:, k] + 1e-310
        else:                                   # little zero-cost capacity: windows run dry
            r.avail[0] = np.minimum(r.avail[0], 2.0)
        rounds.append(r)
    _check(engine, engine_nowalk, rounds, "zero-cost window certificates")


@pytest.mark.parametrize("mode,sort_hosts", [(_abi.PVT_CA_BF, True), (_abi.PVT_VBP_FF, True),
                                             (_abi.PVT_CA_FF, False)])
def test_bulk_runs_in_the_walk(engine, engine_nowalk, mode, sort_hosts):
    """Runs of equal demands placed in one step on the walk's register chunk -- cost_aware best-fit
    (zero-cost window) and first fit by index (vbp first-fit, unsorted cost_aware first-fit,
    strict) -- (every fitting lane
    counts its copies, the lanes take the run in order and replay their subtractions): runs of up
    to a whole batch over hosts that take an exact number of copies, demands that are not exactly
    representable (0.1 cpus: the copy counts come from the sequential roundings), all-zero demand
    rows (a lane takes every copy), and hosts above 2^500 (no bulk step, the per-task stop; below
    ~1e154, where a zero-cost score would be 0 * inf)."""
    rounds = []
    for s in range(6):
        r = synthetic.make_round(mode, 900, 1500, seed=220 + s, sort_hosts=sort_hosts)
        rs = np.random.RandomState(300 + s)
        if s in (0, 1):
            rows = np.array([[0.5, 2048.0], [1.0, 4096.0], [0.25, 1024.0]])
            pick = np.sort(rs.randint(0, 3, size=r.n_tasks))
            r.dem[0], r.dem[1] = rows[pick, 0], rows[pick, 1]
            r.avail[0] = 0.5 * rs.randint(0, 40, size=r.n_hosts)
            r.avail[1] = 2048.0 * rs.randint(0, 40, size=r.n_hosts)
        elif s == 2:
            r.dem[0] = 0.1
            r.dem[1] = 0.3 * 1024.0
            r.avail[0] = 0.1 * rs.randint(1, 30, size=r.n_hosts) + 0.05 * (s % 2)
        elif s == 3:
            r.dem[:, ::3] = 0.0                  # all-zero rows between the others
        elif s == 4:
            r.avail[:, ::5] = 1e151              # beyond 2^500 (squares still finite): the walk's
                                                 # per-task stop
        else:
            r.dem[0] = np.round(r.dem[0] * 4) / 4   # fewer distinct rows: longer runs
            r.dem[1] = np.round(r.dem[1] / 4096.0) * 4096.0
        rounds.append(r)
    _check(engine, engine_nowalk, rounds, "bulk runs mode %d" % mode)
