"""Synthetic rounds for the large configs (BASELINE.json configs 3-5).

The reference cannot build these sizes (it creates O(H^2) route objects, resources/gen.py:61-74),
so they are defined here from its data:

- zones: the first ``n_zones`` (default 20) zones of locality.yml order, cost table as is,
  bw x U(.95, 1.05) jitter with seed 0 (pivot_place.locality).
- hosts: capacity (16, 131072, 100, 1) like sim.py's defaults (alibaba/sim.py:23-32), zone
  i % Z (resources/gen.py:46); availability from RandomState(seed): cpus = 0.5 * randint(0, 33),
  mem = uniform(0, 131072), disk = 100, gpus = 1.
- tasks: (cpus, mem) rows drawn with replacement from every task row of the seven bundled
  job files, mem x 7.68 * 1024 (alibaba/runner.py:69,97), disk = gpus = 0.
- cost_aware: anchor zone uniform in [0, Z); tasks grouped by anchor in first-seen order, task
  order within a group = draw order (the shape cost_aware.py:45-58 produces).
- vbp best-fit: host-id ranks are a random permutation (ids are uuid prefixes in the reference).
- opportunistic: MT19937 state of RandomState(seed + 1).
Draw order from RandomState(seed): cpus[H], mem[H], task rows[T], anchors[T], ranks[H].
"""
import functools
import json
import os

import numpy as np

from . import _abi
from ._abi import RoundArrays
from .locality import zone_tables

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
MEM_SCALE_FACTOR = 7.68 * 1024


@functools.lru_cache(maxsize=None)
def demand_rows():
    with open(os.path.join(DATA, "task_demands.json")) as f:
        rows = json.load(f)["rows"]
    cpus = np.array([r[0] for r in rows], dtype=np.float64)
    mem = np.array([r[1] for r in rows], dtype=np.float64)
    cnt = np.array([r[2] for r in rows], dtype=np.int64)
    return cpus, mem, np.cumsum(cnt)


def mt_state_of(seed):
    st = np.random.RandomState(seed).get_state()
    out = np.empty(625, dtype=np.uint32)
    out[:624] = st[1]
    out[624] = st[2]
    return out


def make_round(mode, n_hosts, n_tasks, seed=20261015, n_zones=20, sort_tasks=None,
               sort_hosts=True):
    """One synthetic round for ``mode`` (a PVT_* constant) as host arrays."""
    rs = np.random.RandomState(seed)
    H, T = int(n_hosts), int(n_tasks)
    avail = np.empty((4, H), dtype=np.float64)
    avail[0] = 0.5 * rs.randint(0, 33, size=H)
    avail[1] = rs.uniform(0, 131072, size=H)
    avail[2] = 100.0
    avail[3] = 1.0
    zone = (np.arange(H) % n_zones).astype(np.int32)
    cpus, mem, cum = demand_rows()
    rows = np.searchsorted(cum, rs.randint(0, int(cum[-1]), size=T), side="right")
    dem = np.zeros((4, T), dtype=np.float64)
    dem[0] = cpus[rows]
    dem[1] = mem[rows] * MEM_SCALE_FACTOR
    anchors = rs.randint(0, n_zones, size=T)
    rank = rs.permutation(H).astype(np.uint32)
    cost, bw = zone_tables(0, n_zones)
    kw = {}
    if mode in (_abi.PVT_CA_FF, _abi.PVT_CA_BF):
        first = {}
        for a in anchors:
            first.setdefault(int(a), len(first))
        kw["task_group"] = np.array([first[int(a)] for a in anchors], dtype=np.int32)
        kw["group_anchor"] = np.array(list(first.keys()), dtype=np.int32)
        kw["sort_tasks"] = True if sort_tasks is None else sort_tasks
        kw["sort_hosts"] = sort_hosts
    elif mode in (_abi.PVT_VBP_FF, _abi.PVT_VBP_BF):
        kw["sort_tasks"] = True if sort_tasks is None else sort_tasks
        kw["tiebreak"] = rank
    elif mode == _abi.PVT_OPP:
        kw["mt_state"] = mt_state_of(seed + 1)
    return RoundArrays(mode=mode, avail=avail, zone=zone, dem=dem, cost=cost, bw=bw, **kw)


def subset_tasks(r: RoundArrays, n):
    """The first ``n`` tasks of a round (a bounded CPU-baseline sample of the same workload)."""
    kw = dict(mode=r.mode, avail=r.avail.copy(), zone=r.zone, dem=r.dem[:, :n].copy(), cost=r.cost,
              bw=r.bw, tiebreak=r.tiebreak, decay=r.decay, sort_tasks=r.sort_tasks,
              sort_hosts=r.sort_hosts, mt_state=None if r.mt_state is None else r.mt_state.copy())
    if r.task_group is not None:
        kw["task_group"] = r.task_group[:n].copy()
        kw["group_anchor"] = r.group_anchor
    return RoundArrays(**kw)
