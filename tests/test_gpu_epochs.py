"""GPU parity of the group-parallel speculative epochs (cost_aware best-fit, pvt_epoch.hip):
groups of distinct anchor zones are walked side by side on the epoch's start state and only the
exact prefix is kept. Placements, order and availability must equal the CPU restatement and the
sequential engine (pvt_set_epochs(0)) -- including rounds built so that groups DO collide
(spill into other zones, exact fits, repeated anchors), which exercises rejection."""
import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("zero_walk")]


@pytest.fixture(params=[True, False], ids=["frontier", "lists"])
def zero_walk(engine, request):
    """Every epoch test runs with the zero-cost frontier walk (pvt_zwalk.hip) and without it
    (every chain on the list walk)."""
    engine.set_zero_walk(request.param)
    yield request.param
    engine.set_zero_walk(True)


def _same(res, ref):
    np.testing.assert_array_equal(res.placement, ref.placement)
    np.testing.assert_array_equal(res.order, ref.order)
    bad = np.nonzero((res.avail != ref.avail).any(axis=0))[0]
    assert bad.size == 0, "availability differs on hosts %s" % bad[:10]


def _place(engine, r, epochs=True):
    try:
        engine.set_resident(0)
        engine.set_epochs(epochs)
        res = engine.place(r)
        st = engine.epoch_stats()
    finally:
        engine.set_epochs(True)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)
    return res, st


def _regroup(r, anchors):
    """Tasks grouped by the given per-task anchors (first-seen group order)."""
    first = {}
    for a in anchors:
        first.setdefault(int(a), len(first))
    r.task_group = np.array([first[int(a)] for a in anchors], dtype=np.int32)
    r.group_anchor = np.array(list(first.keys()), dtype=np.int32)
    return r


@pytest.mark.parametrize("H,T,seed", [(5000, 300, 1), (70_000, 2600, 2), (200_000, 12_000, 3),
                                      (9000, 4000, 4)])
def test_epochs_match_oracle(engine, zero_walk, H, T, seed):
    r = synthetic.make_round(_abi.PVT_CA_BF, H, T, seed=seed)
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)
    assert st["epochs"] >= 1 and st["segments"] >= 2
    if zero_walk:       # plenty of zero-cost capacity: the frontier walk proves every chain
        assert st["frontier_chains"] > 0 and st["list_chains"] == 0, st
    else:
        assert st["frontier_chains"] == 0, st
    seq, st0 = _place(engine, r, epochs=False)
    _same(seq, ref)
    assert st0["epochs"] == 0


@pytest.mark.parametrize("cpus,seed", [(1.0, 5), (2.0, 6), (4.0, 7)])
def test_epochs_crowded_groups(engine, cpus, seed):
    """Few small hosts: zones fill up, many tasks find no host; placements stay exact."""
    r = synthetic.make_round(_abi.PVT_CA_BF, 8000, 6000, seed=seed)
    r.avail[0, :] = cpus
    r.avail[1, :] = 50000.0
    ref = oracle.place(r, threads=8)
    res, _ = _place(engine, r)
    _same(res, ref)


@pytest.mark.parametrize("seed", [10, 11])
def test_epochs_groups_spill_and_collide(engine, seed):
    """Zones 0-9 have no capacity: groups anchored there spill into zones 10-19, onto hosts the
    groups anchored there want too -- speculation must be rejected and redone."""
    r = synthetic.make_round(_abi.PVT_CA_BF, 20_000, 6000, seed=seed)
    r.avail[:2, r.zone < 10] = 0.0
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)
    assert st["rejected"] > 0, st


def test_epochs_repeated_anchor_zones(engine):
    """40 groups over 20 zones (each zone anchors two groups): groups of one zero-cost
    component share a chain walk, in order."""
    r = synthetic.make_round(_abi.PVT_CA_BF, 60_000, 8000, seed=8)
    rs = np.random.RandomState(8)
    groups = rs.randint(0, 40, size=r.n_tasks)
    first = {}
    for g in groups:
        first.setdefault(int(g), len(first))
    r.task_group = np.array([first[int(g)] for g in groups], dtype=np.int32)
    r.group_anchor = np.array([g % 20 for g in first.keys()], dtype=np.int32)
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)
    assert st["segments"] >= 40


def test_epochs_exact_fits_tie_at_zero(engine):
    """Hosts of other zones that fit a task exactly score 0 and win ties by index: the
    validation must see a foreign host that an earlier group filled to an exact fit."""
    r = synthetic.make_round(_abi.PVT_CA_BF, 6000, 3000, seed=9)
    r.avail[0, :] = 1.0
    r.avail[1, :] = 7864.32
    r.avail[2, :] = 0.0
    r.avail[3, :] = 0.0
    r.dem[0, :] = 0.5
    r.dem[1, :] = 3932.16
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)
    # once hosts were filled to 0.5 cpus (an exact fit) no capacity dimension separates hosts
    # from tasks: the frontier walk cannot rule out a score-0 host outside its zones and leaves
    # those epochs' chains to the lists
    assert st["list_chains"] > 0, st


def test_epochs_long_chains_split(engine):
    """40 groups anchored alternately in two zero-cost components (zones 0-2 and 3-5): each
    component's chain exceeds a walk's cap, so epochs split inside the chain sequence."""
    r = synthetic.make_round(_abi.PVT_CA_BF, 30_000, 8000, seed=12)
    rs = np.random.RandomState(12)
    groups = np.sort(rs.randint(0, 40, size=r.n_tasks))
    first = {}
    for g in groups:
        first.setdefault(int(g), len(first))
    r.task_group = np.array([first[int(g)] for g in groups], dtype=np.int32)
    r.group_anchor = np.array([(g % 2) * 3 + (g // 2) % 3 for g in first.keys()], dtype=np.int32)
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)
    assert st["epochs"] >= 2


def test_zero_walk_non_transitive_zero_cost(engine, zero_walk):
    """Zones 0-1 and 1-2 exchange data for free but 0-2 do not: one component {0, 1, 2} whose
    window holds zone-2 hosts that score > 0 for anchor 0 (scored exactly, never taken as 0)."""
    r = synthetic.make_round(_abi.PVT_CA_BF, 40_000, 5000, seed=13)
    cost = np.array(r.cost, dtype=np.float64)
    for a, b in ((0, 1), (1, 2)):
        cost[a, b] = cost[b, a] = 0.0
    cost[0, 2], cost[2, 0] = 0.03, 0.02
    r.cost = cost
    # zone-1 hosts nearly full, so anchor-0 tasks must look past them
    r.avail[0, r.zone == 1] = 0.5
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)
    if zero_walk:
        assert st["frontier_chains"] > 0, st


def test_zero_walk_exact_fit_hosts_elsewhere(engine, zero_walk):
    """A few hosts of other components fit some tasks exactly (score 0 at a lower index than
    the zero-cost winner): the frontier walk must hand such chains to the lists."""
    r = synthetic.make_round(_abi.PVT_CA_BF, 30_000, 4000, seed=14)
    # disk / gpus of every host 0 (tasks ask for 0): only cpus / mem could separate, and some
    # hosts take the exact (cpus, mem) of a task
    r.avail[2, :] = 0.0
    r.avail[3, :] = 0.0
    for k, h in enumerate(range(3, 400, 7)):
        r.avail[0, h] = r.dem[0, k * 11]
        r.avail[1, h] = r.dem[1, k * 11]
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)


def test_zero_walk_window_exhausted(engine, zero_walk):
    """Zero-cost capacity runs out inside the 1024-host window: chains fall back to the lists
    (positive-score hosts, then no host at all) and stay exact."""
    r = synthetic.make_round(_abi.PVT_CA_BF, 6000, 5000, seed=15)
    r.avail[0, :] = 0.5         # one small task per host; larger tasks fit nowhere
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)
    if zero_walk:
        assert st["list_chains"] > 0, st


def test_zero_walk_tiny_egress_costs(engine, zero_walk):
    """Subnormal egress costs to some zones: a positive score can round to 0 there, so the
    frontier walk leaves those anchors' chains to the lists."""
    r = synthetic.make_round(_abi.PVT_CA_BF, 20_000, 3000, seed=16)
    cost = np.array(r.cost, dtype=np.float64)
    cost[5, 11] = cost[11, 5] = 5e-324
    r.cost = cost
    ref = oracle.place(r, threads=8)
    res, _ = _place(engine, r)
    _same(res, ref)


def test_zero_walk_run_stops_at_segment_start(engine, zero_walk):
    """Two groups anchored in zone 0 walk in one chain, back to back in one 64-task batch, with
    the same demand: the frontier walk's run of equal demands must stop at the second group's
    start (a host whose copies straddle the boundary logs its capacities after the first group's
    last copy). The group between them (zone 1, no capacity there) leaves its chain unproven, so
    the epoch accepts the first group only and applies that group's final entries."""
    H = 4000
    r = synthetic.make_round(_abi.PVT_CA_BF, H, 77, seed=17)
    cost = np.full((20, 20), 0.01)
    np.fill_diagonal(cost, 0.0)
    r.cost = cost
    r.avail[0, :] = 16.0
    r.avail[1, :] = 131072.0
    r.avail[2, :] = 100.0
    r.avail[3, :] = 1.0
    z0 = r.zone == 0
    r.avail[0, z0] = 4.0        # four copies of (1, 1000) per zone-0 host: 42 = 10 x 4 + 2
    r.avail[1, z0] = 4000.0
    r.avail[:2, r.zone == 1] = 0.0
    r.dem[:, :] = 0.0
    r.dem[0, :] = 1.0
    r.dem[1, :] = 1000.0
    r.task_group = np.array([0] * 42 + [1] * 5 + [2] * 30, dtype=np.int32)
    r.group_anchor = np.array([0, 1, 0], dtype=np.int32)
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)
    if zero_walk:
        assert st["frontier_chains"] > 0, st


@pytest.mark.parametrize("H,T,seed", [(200_000, 6000, 24), (1_000_000, 10_000, 20261015)])
def test_zero_walk_large_window_retry(engine, zero_walk, H, T, seed):
    """Every host holds at most 1 cpu (bench.py's loaded config 5): chains need more than the
    1024-host window, report it exhausted, and are walked again with the 3072-host window
    before any falls back to the lists; placements stay exact."""
    r = synthetic.make_round(_abi.PVT_CA_BF, H, T, seed=seed)
    r.avail[0] = np.minimum(r.avail[0], 1.0)
    ref = oracle.place(r, threads=8)
    res, st = _place(engine, r)
    _same(res, ref)
    if zero_walk:
        assert st["frontier_chains"] > 0, st
