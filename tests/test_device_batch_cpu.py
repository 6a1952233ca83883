"""DeviceBatch / DeviceRound bookkeeping on CPU tensors (no GPU call): the packed layouts, the
MT19937 states of an all-opportunistic batch kept as one device tensor, reset, and the empty
batch -- the parts of the scenario-batch path that need no kernel."""
import numpy as np

from pivot_place import _abi, synthetic
from pivot_place.engine import DeviceBatch


def test_empty_batch():
    b = DeviceBatch([], "cpu")
    assert len(b) == 0 and b.mt_dev is None and b.results() == []


def test_opportunistic_batch_keeps_states_as_one_tensor():
    rounds = [synthetic.make_round(_abi.PVT_OPP, 50, 20, seed=s) for s in range(3)]
    b = DeviceBatch(rounds, "cpu")
    assert b.mt_dev is not None and tuple(b.mt_dev.shape) == (3, 625)
    np.testing.assert_array_equal(b.mt_dev.numpy().view(np.uint32)[1], rounds[1].mt_state)
    b.mt_dev[0, 0] = 7
    b.reset()
    np.testing.assert_array_equal(b.mt_dev.numpy().view(np.uint32)[0], rounds[0].mt_state)
    res = b.results()
    np.testing.assert_array_equal(res[2].mt_state, rounds[2].mt_state)
    np.testing.assert_array_equal(res[0].avail, rounds[0].avail)


def test_mixed_batch_has_host_states():
    rounds = [synthetic.make_round(_abi.PVT_CA_BF, 50, 20, seed=1),
              synthetic.make_round(_abi.PVT_CA_BF, 60, 10, seed=2)]
    b = DeviceBatch(rounds, "cpu")
    assert b.mt_dev is None
    assert b.structs[1].n_hosts == 60 and b.structs[1].n_tasks == 10
