"""GPU parity of the vbp best-fit band lists (pvt_band.hip; reference scheduler/vbp.py:39-50).

Hosts are sorted once per round by snapshot memory; each task's lists come from the band of the
sorted copy around its memory demand plus the hosts committed to since the snapshot (touched,
scanned live). Placements, order and availability must equal the CPU restatement -- with the
band forced on small rounds, on rounds built to stress it (identical memory values, hosts that
fill after one task, tasks that fit nowhere, tiny windows with refills, pipeline on and off) and
against the streaming score pass (pvt_set_band(0)).
"""
import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu


def _same(res, ref):
    np.testing.assert_array_equal(res.order, ref.order)
    np.testing.assert_array_equal(res.placement, ref.placement)
    bad = np.nonzero((res.avail != ref.avail).any(axis=0))[0]
    assert bad.size == 0, "availability differs on hosts %s" % bad[:10]


def _place(engine, r, band=1, window=0, pipeline=True):
    try:
        engine.set_resident(0)
        engine.set_band(band)
        engine.set_window(window)
        engine.set_pipeline(pipeline)
        return engine.place(r)
    finally:
        engine.set_band(65536)
        engine.set_window(0)
        engine.set_pipeline(True)
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)


@pytest.mark.parametrize("H,T,seed", [(300, 200, 1), (5000, 1200, 2), (70_000, 2600, 3),
                                      (200_000, 3000, 4)])
def test_band_matches_oracle(engine, H, T, seed):
    r = synthetic.make_round(_abi.PVT_VBP_BF, H, T, seed=seed)
    ref = oracle.place(r, threads=8)
    _same(_place(engine, r), ref)


@pytest.mark.parametrize("pipeline", [True, False])
@pytest.mark.parametrize("window", [0, 37, 333])
def test_band_windows_and_refills(engine, window, pipeline):
    """Hosts that fit one task each: every commit kills a host, lists run dry, windows refill,
    and later windows see many touched hosts (scanned live, skipped in the sorted copy)."""
    r = synthetic.make_round(_abi.PVT_VBP_BF, 20_000, 4000, seed=5)
    r.avail[0, :] = 1.5
    ref = oracle.place(r, threads=8)
    _same(_place(engine, r, window=window, pipeline=pipeline), ref)


def test_band_identical_memory(engine):
    """Runs of hosts with equal memory (stable sort, ties broken by host-id rank) and tasks that
    fit nowhere (memory above every host)."""
    r = synthetic.make_round(_abi.PVT_VBP_BF, 30_000, 2500, seed=6)
    r.avail[1, :] = np.round(r.avail[1, :] / 4096.0) * 4096.0
    r.dem[1, ::97] = 200_000.0
    ref = oracle.place(r, threads=8)
    assert (ref.placement < 0).sum() > 0
    _same(_place(engine, r), ref)


def test_band_equals_streaming(engine):
    """Band lists and the streaming score pass give the same round."""
    r = synthetic.make_round(_abi.PVT_VBP_BF, 100_000, 2000, seed=7)
    _same(_place(engine, r, band=1), _place(engine, r, band=0))


@pytest.mark.parametrize("world", [1, 3])
def test_band_host_sharded(world):
    """Host-sharded vbp best-fit with band lists on every rank (its own range sorted; touched
    hosts of its range scanned live)."""
    from pivot_place.engine import PlacementEngine
    from pivot_place.sharded import place_lockstep
    engines = [PlacementEngine(0) for _ in range(world)]
    for e in engines:
        e.set_band(1)
    r = synthetic.make_round(_abi.PVT_VBP_BF, 60_000, 1500, seed=8)
    ref = oracle.place(r, threads=8)
    for o in place_lockstep(engines, r):
        _same(o, ref)


@pytest.mark.parametrize("H,T,seed", [(70_000, 2600, 9), (20_000, 4000, 10)])
def test_one_wave_list_walk_equals_list_walk(H, T, seed):
    """vbp best-fit windows walked by the one-wave list walk with list cursors (pvt_lwalk.hip,
    the default) and by the scout list walk (PVT_LWALK=0) give the oracle's round; the second
    case has hosts that fit one task each (every commit kills its host, lists run deep)."""
    import os
    from pivot_place.engine import PlacementEngine
    r = synthetic.make_round(_abi.PVT_VBP_BF, H, T, seed=seed)
    if seed == 10:
        r.avail[0, :] = 1.5
    ref = oracle.place(r, threads=8)
    old = os.environ.get("PVT_LWALK")
    try:
        os.environ["PVT_LWALK"] = "0"
        scout = PlacementEngine(0)
    finally:
        if old is None:
            os.environ.pop("PVT_LWALK", None)
        else:
            os.environ["PVT_LWALK"] = old
    one = PlacementEngine(0)
    for e in (scout, one):
        e.set_resident(0)
        e.set_band(1)
    _same(one.place(r), ref)
    _same(scout.place(r), ref)


@pytest.mark.parametrize("H,T,seed,one_fit", [(70_000, 2600, 11, False), (300_000, 5000, 12, False),
                                              (20_000, 4000, 13, True)])
def test_walks_enqueued_ahead(H, T, seed, one_fit):
    """place_ahead (PVT_AHEAD=1, off by default: measured slower): up to 8 vbp best-fit walks
    enqueued at once, each gated on the previous walk's device status slot (skipped after an
    early stop, its owned hosts otherwise inherited). Same round as the oracle, including hosts
    that fit one task each (refills, skipped windows, the inherited-host fallback)."""
    import os
    from pivot_place.engine import PlacementEngine
    r = synthetic.make_round(_abi.PVT_VBP_BF, H, T, seed=seed)
    if one_fit:
        r.avail[0, :] = 1.5
    ref = oracle.place(r, threads=8)
    old = os.environ.get("PVT_AHEAD")
    try:
        os.environ["PVT_AHEAD"] = "1"
        ahead = PlacementEngine(0)
    finally:
        if old is None:
            os.environ.pop("PVT_AHEAD", None)
        else:
            os.environ["PVT_AHEAD"] = old
    ahead.set_resident(0)
    ahead.set_band(1)
    _same(ahead.place(r), ref)
