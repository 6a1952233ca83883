"""Meter aggregates (reference resources/meter.py:31-53).

Pinned against the reference: tests/golden/make_meter_logs.py ran three whole reference
simulations (config 1 cost_aware, 12-host opportunistic, config 1 vbp best-fit) and recorded
the reference Meter's raw logs with its own aggregate values. The CPU restatement
(oracle_meter) reproduces them bit for bit; the GPU batch reduction (pvt_meter) is within the
north star's 1e-9 relative bound (written in each assertion) of them and of the restatement on
large synthetic batches.
"""
import gzip
import json
import os

import numpy as np
import pytest

from oracle import oracle
from pivot_place import _abi, meter

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KEYS = {"instance_hours": "cumulative_instance_hours", "egress_cost": "total_network_traffic_cost",
        "congestion_delay": "average_congestion_delay"}
RTOL = 1e-9     # BASELINE.json north star: aggregate cost / makespan within 1e-9 relative


def _fixture():
    with gzip.open(os.path.join(GOLDEN, "meter_logs.json.gz"), "rt") as f:
        runs = json.load(f)
    scen = [{"hosts": [h["intervals"] for h in r["hosts"]],
             "routes": [(rt["cost"], rt["packets"]) for rt in r["routes"]]} for r in runs]
    return runs, scen


def _synthetic(n_scen, seed, max_hosts=200, max_routes=300):
    rng = np.random.default_rng(seed)
    out = []
    for s in range(n_scen):
        hosts = []
        for _ in range(int(rng.integers(0, max_hosts))):
            t = np.cumsum(rng.integers(0, 500, size=2 * int(rng.integers(0, 6))))
            hosts.append([[float(t[2 * i]), float(t[2 * i + 1])] for i in range(len(t) // 2)])
        routes = []
        for _ in range(int(rng.integers(0, max_routes))):
            pkts = []
            for _ in range(int(rng.integers(0, 5))):
                t = np.cumsum(rng.random(2 * int(rng.integers(1, 4))) * 3.0)
                pkts.append([(float(t[2 * i]), float(t[2 * i + 1]), float(rng.integers(1, 1001)))
                             for i in range(len(t) // 2)])
            routes.append((float(rng.choice([0.0, 0.01, 0.02, 0.05, 0.08, 0.12])), pkts))
        out.append({"hosts": hosts, "routes": routes})
    return out


def test_oracle_meter_matches_reference_bit_for_bit():
    runs, scen = _fixture()
    got, rc = oracle.meter(meter.pack(scen))
    assert rc == 0
    for i, r in enumerate(runs):
        for k, ref_k in KEYS.items():
            assert got[k][i] == r["want"][ref_k], (r["name"], k)


def test_pack_layout():
    log = meter.pack([{"hosts": [[[0, 5], [7, 9]], []], "routes": [(0.5, [[(0, 1, 10), (2, 3, 5)]])]},
                      {"hosts": [], "routes": []}])
    assert log.host_off.tolist() == [0, 2, 2] and log.iv_off.tolist() == [0, 2, 2]
    assert log.route_off.tolist() == [0, 1, 1] and log.pkt_off.tolist() == [0, 1]
    assert log.tr_off.tolist() == [0, 2]
    got, rc = oracle.meter(log)
    assert rc == 0
    assert got["instance_hours"].tolist() == [7 / 3600, 0.0]
    assert got["egress_cost"].tolist() == [0.5 * 15 / 8000, 0.0]
    assert got["congestion_delay"].tolist() == [1.0, 0.0]


def test_oracle_meter_rejects_bad_offsets():
    log = meter.pack(_synthetic(2, 1))
    log.iv_off = log.iv_off.copy()
    log.iv_off[1] = 10 ** 9
    assert oracle.meter(log)[1] == _abi.PVT_EINVAL


def test_meter_struct_layout_matches_header():
    import re
    text = open(os.path.join(os.path.dirname(GOLDEN), "..", "include", "pivot_place.h")).read()
    body = re.search(r"typedef struct pvt_meter_log \{(.*?)\} pvt_meter_log;", text,
                     flags=re.S).group(1)
    fields = re.findall(r"\b(\w+)\s*(?:,|;)", body)
    assert [f for f, _ in _abi.pvt_meter_log._fields_] == fields


# ------------------------------------------------------------------ GPU (pvt_meter)
@pytest.mark.gpu
def test_gpu_meter_reference_runs(engine):
    runs, scen = _fixture()
    got = engine.meter(meter.pack(scen))
    for i, r in enumerate(runs):
        for k, ref_k in KEYS.items():
            np.testing.assert_allclose(got[k][i], r["want"][ref_k], rtol=RTOL, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("n_scen,seed", [(1, 0), (7, 1), (512, 2), (4096, 3)])
def test_gpu_meter_batches(engine, n_scen, seed):
    scen = _synthetic(n_scen, seed, max_hosts=60 if n_scen > 100 else 400,
                      max_routes=40 if n_scen > 100 else 900)
    log = meter.pack(scen)
    want, rc = oracle.meter(log)
    assert rc == 0
    got = engine.meter(log)
    for k in KEYS:
        np.testing.assert_allclose(got[k], want[k], rtol=RTOL, atol=0)


@pytest.mark.gpu
def test_gpu_meter_rejects_bad_offsets(engine):
    log = meter.pack(_synthetic(3, 4))
    log.tr_off = log.tr_off.copy()
    log.tr_off[-1] = len(log.tr_size) + 5
    with pytest.raises(RuntimeError, match="EINVAL"):
        engine.meter(log)


@pytest.mark.gpu
def test_gpu_meter_dropin_mixin(engine):
    """MeterAggregatesMixin in front of a Meter-shaped object: the reference's property names
    return the GPU values."""
    runs, scen = _fixture()

    class Loc:
        def __init__(self, i):
            self.i = i

    class Node:
        def __init__(self, loc):
            self.locality = loc

    class Route:
        def __init__(self, a, b):
            self.src, self.dst = Node(a), Node(b)

    class Meta:
        def __init__(self):
            self.cost = {}

    class FakeMeter(meter.MeterAggregatesMixin):
        def __init__(self, r):
            self.engine = engine
            self._Meter__meta = Meta()
            self._Meter__hosts = {("h", i): [list(v) for v in h["intervals"]]
                                  for i, h in enumerate(r["hosts"])}
            self._Meter__routes = {}
            for j, rt in enumerate(r["routes"]):
                ro = Route(Loc(2 * j), Loc(2 * j + 1))
                self._Meter__meta.cost[ro.src.locality, ro.dst.locality] = rt["cost"]
                self._Meter__routes[ro] = {k: p for k, p in enumerate(rt["packets"])}

    for r in runs:
        m = FakeMeter(r)
        for k, ref_k in KEYS.items():
            np.testing.assert_allclose(getattr(m, ref_k), r["want"][ref_k], rtol=RTOL, atol=0)
