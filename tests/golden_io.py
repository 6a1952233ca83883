"""Readers for the golden fixtures (tests/golden/*.json.gz, made by tests/golden/make_golden.py).

Every fixture is one frozen cluster state plus several reference ``schedule()`` runs on it.
This module turns a (state, run) pair into the engine's ABI input (``RoundArrays``, using the
group structure the reference itself produced) and into the expected outputs.
"""
import functools
import gzip
import json
import os

import numpy as np

from pivot_place import _abi
from pivot_place._abi import RoundArrays

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["empty", "one_host", "ties", "exact_fit", "opp_single", "saturate", "pred_ties", "decay",
         "c1_sim_h100", "c2_h1000", "rt_c1_h100", "rt_h12"]


@functools.lru_cache(maxsize=None)
def load(name):
    with gzip.open(os.path.join(GOLDEN, name + ".json.gz"), "rt") as f:
        return json.load(f)


@functools.lru_cache(maxsize=None)
def zones():
    with open(os.path.join(GOLDEN, "zones_seed0.json")) as f:
        z = json.load(f)
    return np.array(z["cost"], dtype=np.float64), np.array(z["bw"], dtype=np.float64), z["zones"]


def mt_state(seed, draws=0):
    """(625,) uint32 MT19937 state of RandomState(seed) advanced by ``draws`` 32-bit outputs."""
    rs = np.random.RandomState(seed)
    for _ in range(draws):
        rs.randint(0, 1 << 32, dtype=np.uint32)
    st = rs.get_state()
    out = np.empty(625, dtype=np.uint32)
    out[:624] = st[1]
    out[624] = st[2]
    return out


def mode_of(run):
    p, k = run["policy"], run["kwargs"]
    if p == "cost_aware":
        return _abi.PVT_CA_BF if k.get("bin_pack_algo") == "best-fit" else _abi.PVT_CA_FF
    return {"opportunistic": _abi.PVT_OPP, "vbp_ff": _abi.PVT_VBP_FF, "vbp_bf": _abi.PVT_VBP_BF}[p]


def host_avail(case):
    a = np.array(case["avail"], dtype=np.float64).reshape(-1, 4)
    return np.ascontiguousarray(a.T)


def run_arrays(case, run):
    """ABI input for a run. cost_aware groups come from the reference's own recording."""
    mode = mode_of(run)
    cost, bw, _ = zones()
    dem = np.array(case["tasks"]["dem"], dtype=np.float64).reshape(-1, 4).T
    k = run["kwargs"]
    kw = dict(mode=mode, avail=host_avail(case), zone=np.array(case["zone"], dtype=np.int32),
              dem=dem, cost=cost, bw=bw)
    if mode in (_abi.PVT_CA_FF, _abi.PVT_CA_BF):
        T = dem.shape[1]
        tg = np.full(T, -1, dtype=np.int32)
        ga = []
        for g, grp in enumerate(run["groups"]):
            ga.append(grp["anchor_zone"])
            for t in grp["tasks"]:
                tg[t] = g
        kw["task_group"] = tg if T else np.zeros(0, dtype=np.int32)
        kw["group_anchor"] = np.array(ga if ga else [0], dtype=np.int32)
        kw["sort_tasks"] = bool(k.get("sort_tasks", False))
        kw["sort_hosts"] = bool(k.get("sort_hosts", False))
        if k.get("host_decay"):
            kw["decay"] = np.maximum(np.array(case["n_running"], dtype=np.int32), 1)
        if k.get("realtime_bw"):
            kw["rt_bw"] = realtime_rows(case, ga if ga else [0])
    elif mode in (_abi.PVT_VBP_FF, _abi.PVT_VBP_BF):
        kw["sort_tasks"] = bool(str(k.get("decreasing", False)))
        kw["tiebreak"] = np.array(case["id_rank"], dtype=np.uint32)
    else:
        kw["mt_state"] = mt_state(run["seed"])
    return RoundArrays(**kw)


def realtime_rows(case, anchor_zones):
    """(G, H) realtime bandwidth per group: in_route.realtime_bw + out_route.realtime_bw of the
    group's anchor storage (the storage of its anchor zone; cost_aware.py:73-79) and each host."""
    sz = case["storage_zone"]
    rt_in, rt_out = case["rt_in"], case["rt_out"]
    rows = []
    for z in anchor_zones:
        k = sz.index(z)
        rows.append([a + b for a, b in zip(rt_in[k], rt_out[k])])
    return np.array(rows, dtype=np.float64).reshape(len(anchor_zones), -1)


def expected(case, run):
    """(placement, processing order, final avail (4,H), MT state after or None)."""
    placement = np.array(run["placement"], dtype=np.int32)
    avail = host_avail(case).copy()
    for row in run["changed_avail"]:
        avail[:, row[0]] = row[1:]
    mode = mode_of(run)
    if mode in (_abi.PVT_CA_FF, _abi.PVT_CA_BF):
        order = [t for g in run["groups"] for t in g["tasks"]]
    else:
        order = run["order"]
    mt = mt_state(run["seed"], run["rng_draws"]) if mode == _abi.PVT_OPP else None
    return placement, np.array(order, dtype=np.int32), avail, mt


def all_runs(skip_errors=True):
    """(case name, run index) of every recorded run (runs that raised are skipped)."""
    out = []
    for name in CASES:
        case = load(name)
        for i, run in enumerate(case["runs"]):
            if skip_errors and run["error"]:
                continue
            out.append((name, i))
    return out


# ---------------------------------------------------------------------------------------
# Whole-simulation traces (tests/golden/sim_*.json.gz, made by make_golden_sim.py)
# ---------------------------------------------------------------------------------------
def sim_traces():
    """Names of the recorded reference simulations, e.g. ``sim_c1_cost_aware``."""
    return sorted(f[:-len(".json.gz")] for f in os.listdir(GOLDEN)
                  if f.startswith("sim_") and f.endswith(".json.gz"))


def sim_rounds(name):
    """(trace, [case, ...]): every recorded non-empty round expanded to the per-state schema of
    ``load()`` (one run per case), so ``fakes.build`` and ``expected`` apply unchanged."""
    tr = load(name)
    cases, avail, nrun = [], None, None
    for r in tr["rounds"]:
        if avail is None:
            avail = [None] * tr["n_hosts"]
            nrun = [0] * tr["n_hosts"]
        for row in r["avail_delta"]:
            avail[row[0]] = row[1:]
        for h, k in r["n_running_delta"]:
            nrun[h] = k
        case = {"n_hosts": tr["n_hosts"], "avail": [list(a) for a in avail], "zone": tr["zone"],
                "id_rank": tr["id_rank"], "n_running": list(nrun),
                "storage_zone": tr["storage_zone"], "tasks": r["tasks"],
                "containers": r["containers"], "runs": r["runs"], "time": r["time"]}
        cases.append(case)
    return tr, cases
