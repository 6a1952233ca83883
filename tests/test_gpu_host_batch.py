"""pvt_place_host_batch: independent drop-in rounds of DIFFERENT policies from host memory in one
round trip (one staging copy each way, one resident launch whose workgroups branch on their
round's mode). Every round must equal the CPU restatement and the same round through
pvt_place_host alone: placements, order, availability and MT19937 state."""
import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu

MODES = [_abi.PVT_CA_FF, _abi.PVT_CA_BF, _abi.PVT_OPP, _abi.PVT_VBP_FF, _abi.PVT_VBP_BF]


def _same(got, ref, what):
    np.testing.assert_array_equal(got.placement, ref.placement, err_msg=what)
    np.testing.assert_array_equal(got.order, ref.order, err_msg=what)
    assert np.array_equal(got.avail, ref.avail), what
    if ref.mt_state is not None:
        assert np.array_equal(got.mt_state, ref.mt_state), what


def _rounds(specs):
    return [synthetic.make_round(m, H, T, seed=s) for m, H, T, s in specs]


@pytest.mark.parametrize("specs", [
    [(m, 1000, 40 + 7 * i, 100 + i) for i, m in enumerate(MODES)],            # one of each
    [(MODES[i % 5], 1000, 1 + (37 * i) % 300, 200 + i) for i in range(23)],    # a config-2 tick
    [(MODES[i % 5], H, T, 300 + i) for i, (H, T) in
     enumerate([(1, 1), (2, 5), (64, 64), (100, 18), (4096, 100), (3000, 4096), (513, 0),
                (1000, 1)])],                                                   # shape edges
])
def test_mixed_batch_matches_oracle(engine, specs):
    rounds = _rounds(specs)
    got = engine.place_host_batch([(r, None) for r in rounds])
    assert len(got) == len(rounds)
    for i, (r, g) in enumerate(zip(rounds, got)):
        _same(g, oracle.place(r), "round %d mode %d H=%d T=%d" % (i, r.mode, r.n_hosts, r.n_tasks))


def test_one_policy_batch_equals_single_rounds(engine):
    """Rounds of one policy take the per-mode kernel; each equals its pvt_place_host run."""
    rounds = _rounds([(_abi.PVT_OPP, 700, 150, 400 + i) for i in range(9)])
    got = engine.place_host_batch([(r, None) for r in rounds])
    for r, g in zip(rounds, got):
        _same(g, engine.place(r), "opp batch")


def test_batch_beyond_resident_limits_is_refused(engine):
    r = synthetic.make_round(_abi.PVT_VBP_FF, 5000, 10, seed=1)
    assert not engine.host_batch_fits(r)
    with pytest.raises(Exception):
        engine.place_host_batch([(r, None)])


def test_zone_table_cache_follows_the_tables(engine):
    """Host-array rounds keep their zone tables on the device between calls (the drop-in rounds
    of one cluster pass the same tables every time); a round whose tables differ -- other costs,
    other bandwidths, another zone count -- must be staged and refresh the cache, in single
    calls and inside a batch whose rounds carry different tables."""
    base = [synthetic.make_round(m, 800, 120, seed=400 + i) for i, m in
            enumerate([_abi.PVT_CA_BF, _abi.PVT_CA_FF, _abi.PVT_CA_BF])]
    other = synthetic.make_round(_abi.PVT_CA_BF, 800, 120, seed=410)
    other.cost = other.cost * 2.0 + 0.5
    bw = synthetic.make_round(_abi.PVT_CA_FF, 800, 120, seed=411)
    bw.bw = bw.bw * 0.5
    small = synthetic.make_round(_abi.PVT_CA_BF, 600, 100, seed=412, n_zones=7)
    seq = [base[0], other, base[1], bw, small, base[2], base[0]]
    for i, r in enumerate(seq):                     # one round per call
        _same(engine.place(r), oracle.place(r), "single call %d" % i)
    got = engine.place_host_batch([(r, None) for r in seq])   # mixed tables in one call
    for i, (r, g) in enumerate(zip(seq, got)):
        _same(g, oracle.place(r), "batch round %d" % i)
