"""GPU: the grouped processing order (launch_order_prep, group_sort_gather_kernel /
group_sort_kernel, pvt_kernels.hip) against the CPU restatement's, for group sizes on both sides
of every sort path's threshold: rank by counting (<= 128 tasks), the bitonic network with 1-4
elements per thread in registers (129..4096) and the radix-pass fallback (> 4096 tasks in a
group), on both grouped-order paths: the compacting sort-and-gather launch (at most GCOMPACT_MAX
= 64 groups) and the scatter + sort + gather launches (more groups). Demands take few distinct
values, so most sort keys tie and the task-index tie-break (the reference's stable sorts,
scheduler/cost_aware.py:37-42) decides the order."""
import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, synthetic

pytestmark = pytest.mark.gpu

EDGES = [1, 2, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1000, 1023, 1024, 1025, 2047, 2048,
         2049, 3000, 4095, 4096]

MANY = [int(x) for x in np.random.RandomState(5).randint(1, 300, size=100)]   # > GCOMPACT_MAX groups


@pytest.mark.parametrize("sizes", [EDGES, [4097, 5, 300], [1500] * 7, MANY],
                         ids=["edges", "radix", "even", "many"])
@pytest.mark.parametrize("sort_tasks", [True, False])
@pytest.mark.parametrize("mode", [_abi.PVT_CA_BF, _abi.PVT_CA_FF])
def test_grouped_order_matches_oracle(engine, mode, sort_tasks, sizes):
    T = int(sum(sizes))
    r = synthetic.make_round(mode, 5000, T, seed=T % 97, sort_tasks=sort_tasks)
    rs = np.random.RandomState(len(sizes))
    grp = np.repeat(np.arange(len(sizes)), sizes)
    rs.shuffle(grp)                           # groups interleaved in task order
    r.task_group = grp.astype(np.int32)
    r.group_anchor = rs.randint(0, r.n_zones, size=len(sizes)).astype(np.int32)
    r.dem[0] = rs.choice([0.5, 1.0, 2.0], size=T)
    r.dem[1] = rs.choice([512.0, 1024.0], size=T)
    ref = oracle.place(r)
    res = engine.place(r)
    np.testing.assert_array_equal(res.order, ref.order)
    np.testing.assert_array_equal(res.placement, ref.placement)
    assert (res.avail == ref.avail).all()
