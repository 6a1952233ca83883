"""GPU parity of host-dimension sharding (include/pivot_place.h pvt_shard_*).

A sharded round must return exactly what the unsharded engine and the CPU restatement return:
placements, processing order, availability after commits. ``place_lockstep`` runs W contexts
in one process (W shards of the host range, the exchange done by concatenation), so world sizes
up to 8 are covered on a single GPU; the two-process test runs the torch.distributed exchange
(gloo, staged through host memory) with both ranks on cuda:0.
"""
import os
import socket
import sys

import numpy as np
import pytest

import golden_io
from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu

SHARDED_MODES = [_abi.PVT_CA_FF, _abi.PVT_CA_BF, _abi.PVT_VBP_FF, _abi.PVT_VBP_BF]
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def engines():
    from pivot_place.engine import PlacementEngine
    return [PlacementEngine(0) for _ in range(8)]


def _assert_same(res, ref):
    np.testing.assert_array_equal(res.placement, ref.placement)
    np.testing.assert_array_equal(res.order, ref.order)
    bad = np.nonzero((res.avail != ref.avail).any(axis=0))[0]
    assert bad.size == 0, "availability differs on hosts %s" % bad[:10]
    if ref.mt_state is not None:
        np.testing.assert_array_equal(res.mt_state, ref.mt_state)


def _lockstep(engines, world, r):
    from pivot_place.sharded import place_lockstep
    outs = place_lockstep(engines[:world], r)
    for o in outs[1:]:                      # every rank holds the same result
        _assert_same(o, outs[0])
    return outs[0]


@pytest.mark.parametrize("mode", SHARDED_MODES)
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("H,T,seed", [(5000, 300, 1), (70000, 120, 2), (5, 40, 3)])
def test_sharded_matches_oracle(engines, mode, world, H, T, seed):
    r = synthetic.make_round(mode, H, T, seed=seed)
    _assert_same(_lockstep(engines, world, r), oracle.place(r))


@pytest.mark.parametrize("pipeline", [True, False])
@pytest.mark.parametrize("mode", SHARDED_MODES)
def test_sharded_crowded_and_refills(engines, mode, pipeline):
    """Nearly full identical hosts + tiny windows: exhausted packages, bounds, refills; with the
    pipeline on, windows scored past a walk that then stops early come back PVT_ESTALE."""
    r = synthetic.make_round(mode, 3000, 1500, seed=11)
    r.avail[0, :] = 4.0
    r.avail[1, :] = 40000.0
    r.avail[0, ::7] = 0.5
    ref = oracle.place(r)
    try:
        for e in engines:
            e.set_window(37)
            e.set_pipeline(pipeline)
        _assert_same(_lockstep(engines, 4, r), ref)
    finally:
        for e in engines:
            e.set_window(0)
            e.set_pipeline(True)


def test_sharded_pipelined_placer_counts_stale_windows(engines):
    """HostShardedPlacer at world 1 (no exchange): every host fits exactly one task, so a
    window's late tasks find every listed host taken and the walk stops early; the window
    scored past it is stale and re-scored. The result equals the oracle."""
    from pivot_place.engine import DeviceRound
    from pivot_place.sharded import HostShardedPlacer
    r = synthetic.make_round(_abi.PVT_VBP_BF, 3000, 2800, seed=11)
    r.avail[0, :] = 1.5
    r.dem[0, :] = 1.0
    placer = HostShardedPlacer(engines[0], 0, 1)
    dr = DeviceRound(r, engines[0].device)
    placer.run(dr)
    _assert_same(dr.result(), oracle.place(r))
    assert placer.stale > 0 and placer.windows > placer.stale


@pytest.mark.parametrize("name,idx", [x for x in golden_io.all_runs() if x[0] in ("c1_sim_h100", "c2_h1000", "decay", "saturate")])
def test_sharded_matches_reference_golden(engines, name, idx):
    case = golden_io.load(name)
    run = case["runs"][idx]
    r = golden_io.run_arrays(case, run)
    placement, order, avail, mt = golden_io.expected(case, run)
    res = _lockstep(engines, 3, r)
    np.testing.assert_array_equal(res.placement, placement)
    np.testing.assert_array_equal(res.order, order)
    np.testing.assert_array_equal(res.avail, avail)
    if mt is not None:
        np.testing.assert_array_equal(res.mt_state, mt)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("H,T,seed", [(5000, 300, 1), (70000, 600, 2), (200_000, 700, 4), (5, 40, 3)])
def test_opportunistic_host_sharded(engines, world, H, T, seed):
    """Per-rank feasible counts of whole 16384-host super-chunks, all-gathered per window;
    every rank draws and selects on the full tables: placements, availability and the MT19937
    state equal the oracle's on every rank (ranks past the last super-chunk count nothing)."""
    r = synthetic.make_round(_abi.PVT_OPP, H, T, seed=seed)
    _assert_same(_lockstep(engines, world, r), oracle.place(r))


def test_opportunistic_shard_must_be_super_chunk_aligned(engines):
    from pivot_place.engine import DeviceRound
    r = synthetic.make_round(_abi.PVT_OPP, 40000, 10, seed=1)
    dr = DeviceRound(r, engines[0].device)
    with pytest.raises(RuntimeError, match="EINVAL"):
        engines[0].shard_begin(dr, 0, 20000, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, mode, out_q):
    sys.path[:0] = [os.path.join(os.path.dirname(HERE), "pivot-scheduling_amd"), os.path.dirname(HERE)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from pivot_place.engine import PlacementEngine
    from pivot_place.sharded import HostShardedPlacer
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        placer = HostShardedPlacer.from_process_group(PlacementEngine(0))
        res = placer.place(synthetic.make_round(mode, 20000, 400, seed=5))
        out_q.put((rank, res.placement.tolist(), res.avail.tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", [_abi.PVT_CA_BF, _abi.PVT_VBP_FF, _abi.PVT_OPP])
def test_two_process_group_on_one_gpu(mode):
    import torch.multiprocessing as mp
    ref = oracle.place(synthetic.make_round(mode, 20000, 400, seed=5))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(k, 2, port, mode, q)) for k in range(2)]
    for p in procs:
        p.start()
    got = dict((k, (pl, av)) for k, pl, av in (q.get(timeout=100) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in range(2):
        assert got[k][0] == ref.placement.tolist()
        assert got[k][1] == ref.avail.tobytes()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_keyed_prefix_runs_dry(engines, world):
    """Keyed first-fit, one group: every rank's zero-key prefix (the anchor zone's hosts of its
    range, listed without a sort) fills up, the replicated walk stops on empty lists, and every
    rank completes its order with the full sort; all ranks equal the oracle."""
    r = synthetic.make_round(_abi.PVT_CA_FF, 60000, 4000, seed=19)
    r.task_group = np.zeros(r.n_tasks, dtype=np.int32)
    r.group_anchor = np.array([5], dtype=np.int32)
    r.avail[0, :] = 1.0
    ref = oracle.place(r)
    assert (ref.placement >= 0).sum() > 0
    _assert_same(_lockstep(engines, world, r), ref)


def _frontier_round(kind, H, T, seed):
    if kind == "ca_ff_unsorted":
        return synthetic.make_round(_abi.PVT_CA_FF, H, T, seed=seed, sort_hosts=False)
    return synthetic.make_round({"ca_bf": _abi.PVT_CA_BF, "ca_ff": _abi.PVT_CA_FF,
                                 "vbp_ff": _abi.PVT_VBP_FF}[kind], H, T, seed=seed)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("kind", ["ca_bf", "ca_ff", "vbp_ff", "ca_ff_unsorted"])
def test_sharded_frontier_walks(engines, kind, world):
    """The frontier walks on a host-sharded round: cost_aware best-fit epochs (every rank packs
    its first hosts of each chain's zero-cost zones + its host minima), the keyed walk at each
    cost_aware first-fit group start (its first zero-key hosts) and the ordered walk of vbp /
    unsorted cost_aware first-fit (its first alive hosts). After the all-gather every rank walks
    the merged window; all ranks equal the oracle, and the walks did place tasks on every rank."""
    r = _frontier_round(kind, 40_000, 2600, seed=21)
    ref = oracle.place(r, threads=8)
    _assert_same(_lockstep(engines, world, r), ref)
    for e in engines[:world]:
        st = e.epoch_stats()
        assert st["frontier_chains"] > 0, (kind, world, st)
        if kind == "ca_bf":
            assert st["epochs"] >= 1 and st["list_chains"] == 0, st


def _loaded(case, seed):
    r = synthetic.make_round(_abi.PVT_CA_BF, 20_000, 6000, seed=seed)
    if case == "spill":          # zones 0-9 empty: groups spill and collide (rejected segments)
        r.avail[:2, r.zone < 10] = 0.0
    elif case == "window":       # one small task per host: chains outgrow the 1024-host window
        r.avail[0, :] = 0.5
    elif case == "exact":        # exact fits in other zones: certificate 2 fails -> lists
        r.avail[2, :] = 0.0
        r.avail[3, :] = 0.0
        for k, h in enumerate(range(3, 400, 7)):
            r.avail[0, h] = r.dem[0, k * 11]
            r.avail[1, h] = r.dem[1, k * 11]
    return r


@pytest.mark.parametrize("world", [1, 3, 8])
@pytest.mark.parametrize("case", ["spill", "window", "exact"])
def test_sharded_epochs_fall_back_to_lists(engines, case, world):
    """Sharded cost_aware best-fit rounds the frontier walk cannot carry alone: rejected
    segments are walked again, unproven chains go to list windows up to the end of their epoch
    and the frontier epochs resume after them. Equal to the oracle on every rank."""
    r = _loaded(case, 30 + world)
    _assert_same(_lockstep(engines, world, r), oracle.place(r, threads=8))


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_ordered_frontier_empty_ranks(engines, world):
    """vbp first-fit where only the last ranks' hosts are alive at first (the first span holds
    no alive host: the span doubles) and ranks past the span pack nothing."""
    r = synthetic.make_round(_abi.PVT_VBP_FF, 200_000, 3000, seed=23)
    r.avail[0, :150_000] = 0.0
    _assert_same(_lockstep(engines, world, r), oracle.place(r, threads=8))
