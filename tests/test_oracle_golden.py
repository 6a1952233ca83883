"""Pin the CPU restatement (oracle/) to the reference's own outputs (tests/golden/).

Every run recorded from the reference policies must be reproduced bit for bit: placement per
task, processing order, final availability of every host, and MT19937 state.
"""
import numpy as np
import pytest

import golden_io
from oracle import oracle


@pytest.mark.parametrize("name,idx", golden_io.all_runs())
def test_oracle_matches_reference(name, idx):
    case = golden_io.load(name)
    run = case["runs"][idx]
    r = golden_io.run_arrays(case, run)
    res = oracle.place(r)
    placement, order, avail, mt = golden_io.expected(case, run)
    np.testing.assert_array_equal(res.placement, placement)
    np.testing.assert_array_equal(res.order, order)
    assert np.array_equal(res.avail, avail), "final availability differs"
    if mt is not None:
        np.testing.assert_array_equal(res.mt_state, mt)


def test_norm_is_the_ddot_fma_chain():
    """la.norm(x, 2) == sqrt(fma-chain) on random trace-like vectors."""
    import numpy.linalg as la
    rs = np.random.RandomState(3)
    M = 7.68 * 1024
    for _ in range(5000):
        x = np.array([0.5 * rs.randint(-32, 33), rs.uniform(-131072, 131072),
                      float(rs.randint(0, 101)), float(rs.randint(0, 2))])
        if rs.rand() < 0.5:
            x[1] = round(rs.uniform(0, 3), 2) * M
        assert oracle.norm4(x) == la.norm(x, 2)


def test_randint_matches_numpy():
    """Legacy RandomState.randint(0, n): masked rejection, no draw for n == 1."""
    for seed in (0, 7, 12345):
        rs = np.random.RandomState(seed)
        st = golden_io.mt_state(seed)
        for n in [1, 2, 3, 5, 20, 31, 64, 100, 1000, 65537, 1 << 20, 3000000000]:
            for _ in range(50):
                assert oracle.randint(st, n) == rs.randint(0, n)
        ref = rs.get_state()
        assert list(st[:624]) == list(ref[1]) and st[624] == ref[2]


def test_choice_is_randint():
    """RandomState.choice(list) draws randint(0, len) (opportunistic.py:17, cost_aware.py:39)."""
    for n in (1, 2, 7, 31, 100):
        a, b = np.random.RandomState(5), np.random.RandomState(5)
        for _ in range(100):
            assert a.choice(list(range(n))) == b.randint(0, n)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_multithreaded_baseline_equals_oracle(threads):
    """oracle_place_mt (the all-cores CPU baseline bench.py times) returns exactly what the
    single-threaded restatement returns: golden runs and synthetic rounds of every policy."""
    from pivot_place import synthetic
    rounds = []
    for name, idx in golden_io.all_runs():
        case = golden_io.load(name)
        rounds.append(golden_io.run_arrays(case, case["runs"][idx]))
    for mode in range(5):
        rounds.append(synthetic.make_round(mode, 3000, 200, seed=40 + mode))
        crowded = synthetic.make_round(mode, 300, 600, seed=50 + mode)
        crowded.avail[0, :] = 4.0
        crowded.avail[1, :] = 40000.0
        rounds.append(crowded)
    for r in rounds:
        a, b = oracle.place(r), oracle.place(r, threads=threads)
        np.testing.assert_array_equal(a.placement, b.placement)
        np.testing.assert_array_equal(a.order, b.order)
        assert np.array_equal(a.avail, b.avail)
        if a.mt_state is not None:
            np.testing.assert_array_equal(a.mt_state, b.mt_state)
