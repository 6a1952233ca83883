"""GPU parity: the HIP engine (through the C ABI) against the reference's golden runs and the
CPU restatement. Integer/index outputs and fp64 availability must match bit for bit.

Rounds small enough for the resident kernel (<= 4096 hosts and tasks) run there by default;
``path`` runs each such test on both engines: "resident" (pvt_place -> resident kernel) and
"windowed" (pvt_set_resident(0): score/merge/commit-walk windows)."""
import contextlib

import numpy as np
import pytest

import golden_io
from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu

ALL_MODES = [_abi.PVT_CA_FF, _abi.PVT_CA_BF, _abi.PVT_OPP, _abi.PVT_VBP_FF, _abi.PVT_VBP_BF]


@contextlib.contextmanager
def on_path(engine, path):
    engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS if path == "resident" else 0)
    try:
        yield
    finally:
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)


PATHS = ["resident", "windowed"]


def _assert_same(res, placement, order, avail, mt=None):
    np.testing.assert_array_equal(res.placement, placement)
    np.testing.assert_array_equal(res.order, order)
    bad = np.nonzero((res.avail != avail).any(axis=0))[0]
    assert bad.size == 0, "availability differs on hosts %s" % bad[:10]
    if mt is not None:
        np.testing.assert_array_equal(res.mt_state, mt)


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("name,idx", golden_io.all_runs())
def test_engine_matches_reference(engine, name, idx, path):
    case = golden_io.load(name)
    run = case["runs"][idx]
    with on_path(engine, path):
        res = engine.place(golden_io.run_arrays(case, run))
    _assert_same(res, *golden_io.expected(case, run))


@pytest.mark.parametrize("window", [1, 7, 64])
@pytest.mark.parametrize("name", ["saturate", "c1_sim_h100"])
def test_small_windows_force_refills(engine, name, window):
    """Tiny windows make every list-exhaustion / refill path run; results must not change."""
    case = golden_io.load(name)
    try:
        engine.set_resident(0)
        engine.set_window(window)
        for run in case["runs"]:
            if run["error"]:
                continue
            res = engine.place(golden_io.run_arrays(case, run))
            _assert_same(res, *golden_io.expected(case, run))
    finally:
        engine.set_window(0)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("mode", ALL_MODES)
@pytest.mark.parametrize("H,T,seed", [(5000, 300, 1), (70000, 120, 2), (1, 5, 3), (64, 2000, 4),
                                      (4096, 700, 5), (1000, 4096, 6)])
def test_engine_matches_oracle_synthetic(engine, mode, H, T, seed, path):
    r = synthetic.make_round(mode, H, T, seed=seed)
    ref = oracle.place(r)
    with on_path(engine, path):
        res = engine.place(r)
    _assert_same(res, ref.placement, ref.order, ref.avail, ref.mt_state)


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("mode", ALL_MODES)
def test_engine_crowded_hosts(engine, mode, path):
    """Few, nearly full hosts with identical states: ties, exhaustion and unplaceable tasks."""
    r = synthetic.make_round(mode, 300, 1500, seed=11)
    r.avail[0, :] = 4.0
    r.avail[1, :] = 40000.0
    r.avail[0, ::7] = 0.5
    ref = oracle.place(r)
    with on_path(engine, path):
        res = engine.place(r)
    _assert_same(res, ref.placement, ref.order, ref.avail, ref.mt_state)


@pytest.mark.parametrize("path", PATHS)
def test_sqrt_and_division_are_correctly_rounded(engine, path):
    """Best-fit scores need IEEE sqrt and division: compare scores on many random residuals by
    running vbp best-fit with one task against hosts whose residual norms nearly tie."""
    rs = np.random.RandomState(9)
    H = 4096
    base = rs.uniform(1, 1e6, size=H)
    r = synthetic.make_round(_abi.PVT_VBP_BF, H, 1, seed=9)
    r.avail[1, :] = base
    r.avail[1, 1::2] = np.nextafter(base[1::2], np.inf)
    r.dem[:, 0] = [0.5, 1.0, 0.0, 0.0]
    ref = oracle.place(r)
    with on_path(engine, path):
        res = engine.place(r)
    _assert_same(res, ref.placement, ref.order, ref.avail)


@pytest.mark.parametrize("mode", [_abi.PVT_CA_FF, _abi.PVT_CA_BF, _abi.PVT_VBP_FF, _abi.PVT_VBP_BF])
def test_pipelined_windows_match_oracle(engine, mode):
    """Several full windows, each scored while the previous one is walked (inherited touched
    hosts), must equal the CPU restatement and the strictly sequential schedule."""
    r = synthetic.make_round(mode, 100_000, 2600, seed=21)
    ref = oracle.place(r)
    res = engine.place(r)
    _assert_same(res, ref.placement, ref.order, ref.avail)
    try:
        engine.set_pipeline(False)
        seq = engine.place(r)
    finally:
        engine.set_pipeline(True)
    _assert_same(seq, ref.placement, ref.order, ref.avail)


@pytest.mark.parametrize("mode", [_abi.PVT_CA_BF, _abi.PVT_VBP_BF, _abi.PVT_CA_FF])
@pytest.mark.parametrize("window", [96, 333])
def test_pipelined_crowded_small_windows(engine, mode, window):
    """Crowded hosts and short windows: many windows inherit many touched hosts."""
    r = synthetic.make_round(mode, 2000, 4000, seed=13)
    r.avail[0, :] = 6.0
    r.avail[1, :] = 60000.0
    ref = oracle.place(r)
    try:
        engine.set_resident(0)
        engine.set_window(window)
        res = engine.place(r)
    finally:
        engine.set_window(0)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)
    _assert_same(res, ref.placement, ref.order, ref.avail)


@pytest.mark.parametrize("pipeline", [True, False])
@pytest.mark.parametrize("H,cpus", [(30000, 1.0), (25000, 1.5), (1500, 2.0)])
def test_keyed_first_fit_zero_key_prefix_runs_dry(engine, pipeline, H, cpus):
    """cost_aware first-fit with sort_hosts, one group: the anchor zone's hosts (key 0, listed
    first in host order without a sort) fill up, walks stop on empty prefix lists, and the
    engine completes the order with the full sort mid-group; placements equal the oracle's."""
    r = synthetic.make_round(_abi.PVT_CA_FF, H, 5000, seed=17)
    r.task_group = np.zeros(r.n_tasks, dtype=np.int32)
    r.group_anchor = np.array([3], dtype=np.int32)
    r.avail[0, :] = cpus
    ref = oracle.place(r)
    try:
        engine.set_resident(0)
        engine.set_pipeline(pipeline)
        res = engine.place(r)
    finally:
        engine.set_pipeline(True)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)
    assert (ref.placement >= 0).sum() > 0
    _assert_same(res, ref.placement, ref.order, ref.avail)


@pytest.mark.parametrize("tw", [2, 4])
@pytest.mark.parametrize("mode", [_abi.PVT_CA_BF, _abi.PVT_VBP_BF])
@pytest.mark.parametrize("H,T,window", [(100_000, 2600, 0), (20_000, 900, 96), (2000, 3000, 333)])
def test_score_instances_both_tasks_per_wave(engine, mode, tw, H, T, window):
    """pvt_set_score_tw forces the score kernel's 2- or 4-tasks-per-wave instance, so both stay
    under parity at every host count (the default picks by policy and host count)."""
    r = synthetic.make_round(mode, H, T, seed=31 + tw)
    if H <= 2000:
        r.avail[0, :] = 6.0
    ref = oracle.place(r)
    try:
        engine.set_resident(0)
        engine.set_score_tw(tw)
        engine.set_window(window)
        res = engine.place(r)
    finally:
        engine.set_window(0)
        engine.set_score_tw(0)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)
    _assert_same(res, ref.placement, ref.order, ref.avail)


@pytest.mark.parametrize("mode", [_abi.PVT_CA_FF, _abi.PVT_CA_BF])
@pytest.mark.parametrize("H,T,epochs", [(3000, 400, True), (20_000, 1500, True), (20_000, 1500, False),
                                         (70_000, 3000, True)])
def test_realtime_bw_synthetic(engine, mode, H, T, epochs):
    """cost_aware with realtime_bw (cost_aware.py:79,112): a bandwidth per (group, host) -- here
    the static one scaled by random queue factors -- through the resident kernel (3000 hosts),
    the windowed engine and the epochs; equal to the CPU restatement."""
    r = synthetic.make_round(mode, H, T, seed=41)
    r.cost = r.cost + 0.001            # no free-egress zone: every score depends on the bandwidth
    rs = np.random.RandomState(41)
    bsum = r.bw + r.bw.T
    a = r.group_anchor
    r.rt_bw = (bsum[a][:, r.zone] / rs.randint(1, 4, size=(len(a), H))).astype(np.float64)
    ref = oracle.place(r)
    try:
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS if H <= 4096 else 0)
        engine.set_epochs(epochs)
        res = engine.place(r)
    finally:
        engine.set_epochs(True)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)
    _assert_same(res, ref.placement, ref.order, ref.avail)
