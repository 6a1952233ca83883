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
