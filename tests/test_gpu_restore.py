"""pvt_restore_hosts (PlacementEngine.restore): after a round is placed, restoring the hosts its
placement names gives back the snapshot bit for bit -- for every policy, on the resident kernel
and the windowed engines (epochs, frontier walks, band lists, opportunistic windows) -- so a
replayed round (bench.py's steps) sees the same input each time."""
import numpy as np
import pytest

from pivot_place import _abi, synthetic
from pivot_place.engine import DeviceRound

pytestmark = pytest.mark.gpu

MODES = [_abi.PVT_CA_BF, _abi.PVT_CA_FF, _abi.PVT_OPP, _abi.PVT_VBP_FF, _abi.PVT_VBP_BF]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("H,T", [(1000, 1000), (100000, 1000), (300000, 3000)])
def test_restore_gives_back_the_snapshot(engine, mode, H, T):
    import torch
    r = synthetic.make_round(mode, H, T, seed=5)
    dr = DeviceRound(r, engine.device)
    engine.run(dr)
    torch.cuda.synchronize()
    first = dr.result()
    assert (first.placement >= 0).any()
    engine.restore(dr)
    torch.cuda.synchronize()
    a, a0 = dr.avail.cpu().numpy(), dr.avail0.cpu().numpy()
    assert np.array_equal(a.view(np.int64), a0.view(np.int64)), "mode %d" % mode
    engine.run(dr)                       # the same round again: the same result
    torch.cuda.synchronize()
    again = dr.result()
    np.testing.assert_array_equal(again.placement, first.placement)
    assert np.array_equal(again.avail.view(np.int64), first.avail.view(np.int64))
    if first.mt_state is not None:
        assert np.array_equal(again.mt_state, first.mt_state)


NAMED = ("band_score_kernel", "commit_kernel", "lwalk_kernel", "opp_commit_kernel",
         "opp_count_kernel", "ordered_kernel", "perm_scan_kernel", "resident_kernel",
         "score_kernel", "zwalk_kernel", "merge_kernel", "merge_small_kernel", "merge_pkg_kernel",
         "merge_path_kernel")


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("H,T,batch", [(100000, 1000, 0), (1000, 1000, 8)])
def test_walk_probe_step_is_bench_step(engine, mode, H, T, batch):
    """tools/walk_probe.py (the program the PMC profiles in profiles/ are collected on) must
    price exactly bench.py's step: the same reset (a single round restores the hosts the last
    step placed on -- no 32 MB snapshot copy --, a batch copies its snapshot back) and the same
    named-kernel launches."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import bench
    import walk_probe
    from pivot_place.engine import DeviceBatch

    def measure(make_step, dr):
        calls = {"copy": 0, "restore": 0}
        full, part = dr.reset, engine.restore
        dr.reset = lambda: (calls.__setitem__("copy", calls["copy"] + 1), full())
        engine.restore = lambda d: (calls.__setitem__("restore", calls["restore"] + 1), part(d))
        try:
            step = make_step()
            engine.reset_kstats()
            engine.set_profiling(True)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            engine.set_profiling(False)
        finally:
            del dr.reset
            del engine.restore
        return calls, {n: engine.kernel_kstats(n)["launches"] for n in NAMED}

    def make(kind):
        if batch:
            rounds = [synthetic.make_round(mode, H, T, seed=7 + s) for s in range(batch)]
            dr, run = DeviceBatch(rounds, engine.device), engine.run_batch
        else:
            dr, run = DeviceRound(synthetic.make_round(mode, H, T, seed=7), engine.device), engine.run
        if kind == "bench":
            def mk():
                reset = bench.step_reset(engine, dr, bool(batch))

                def step():
                    reset()
                    run(dr)
                return step
        else:
            def mk():
                return walk_probe.probe_step(engine, dr, run, bool(batch))
        return measure(mk, dr)

    engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS if batch else 0)
    try:
        b_calls, b_k = make("bench")
        p_calls, p_k = make("probe")
    finally:
        engine.set_resident(_abi.PVT_RESIDENT_MAX_HOSTS)
    assert p_calls == b_calls
    assert b_calls == ({"copy": 3, "restore": 0} if batch else {"copy": 0, "restore": 3})
    assert p_k == b_k and sum(b_k.values()) > 0, (p_k, b_k)
