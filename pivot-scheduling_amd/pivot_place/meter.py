"""Meter aggregates on the GPU (reference resources/meter.py:31-53).

The reference Meter logs host check-ins / check-outs and per-route packet transfers during a
simulation, and its three aggregate properties fold those logs with Python sums:

    cumulative_instance_hours    sum_h sum_intervals (end - start) / 3600        (:31-33)
    total_network_traffic_cost   sum_routes cost[src, dst] * sum sizes / 8000     (:35-42)
    average_congestion_delay     mean gap between a packet's consecutive transfers (:44-53)

``MeterLog`` packs the logs of any number of scenarios into nested CSR arrays (the layout of
``pvt_meter_log`` in include/pivot_place.h); ``PlacementEngine.meter`` reduces a whole batch
in one launch (one workgroup per scenario). ``MeterAggregatesMixin`` is the drop-in: mixed in
front of the reference's Meter, its three properties come from the GPU. fp64 throughout;
within 1e-9 relative of the reference's left-to-right sums (tests/test_meter.py).
"""
import dataclasses

import numpy as np

from . import _abi


@dataclasses.dataclass
class MeterLog:
    host_off: np.ndarray    # [S+1] int64
    iv_off: np.ndarray      # [n_host_rows+1] int64
    iv_start: np.ndarray    # [n_iv] float64
    iv_end: np.ndarray
    route_off: np.ndarray   # [S+1] int64
    route_cost: np.ndarray  # [n_routes] float64
    pkt_off: np.ndarray     # [n_routes+1] int64
    tr_off: np.ndarray      # [n_pkts+1] int64
    tr_start: np.ndarray    # [n_tr] float64
    tr_end: np.ndarray
    tr_size: np.ndarray

    @property
    def n_scen(self):
        return len(self.host_off) - 1

    def arrays(self):
        return [(f.name, getattr(self, f.name)) for f in dataclasses.fields(self)]

    def fill(self, ptr, out):
        """A pvt_meter_log over this log; ``ptr(array)`` gives each array's address and
        ``out`` holds the three [S] float64 result arrays' addresses."""
        m = _abi.pvt_meter_log()
        m.n_scen = self.n_scen
        m.reserved = 0
        m.n_host_rows = len(self.iv_off) - 1
        m.n_iv = len(self.iv_start)
        m.n_routes = len(self.route_cost)
        m.n_pkts = len(self.tr_off) - 1
        m.n_tr = len(self.tr_size)
        for name, a in self.arrays():
            setattr(m, name, ptr(a))
        m.instance_hours, m.egress_cost, m.congestion_delay = out
        return m


def pack(scenarios) -> MeterLog:
    """``scenarios``: one dict per scenario with ``hosts`` = [[[start, end], ...] per host] and
    ``routes`` = [(cost, [[(start, end, size), ...] per packet]) per route], both in the
    reference meter's dict order."""
    host_off, iv_off, iv_s, iv_e = [0], [0], [], []
    route_off, rcost, pkt_off, tr_off, ts, te, tz = [0], [], [0], [0], [], [], []
    for sc in scenarios:
        for ivs in sc["hosts"]:
            for v in ivs:
                iv_s.append(v[0])
                iv_e.append(v[1])
            iv_off.append(len(iv_s))
        host_off.append(len(iv_off) - 1)
        for cost, pkts in sc["routes"]:
            rcost.append(cost)
            for trans in pkts:
                for t in trans:
                    ts.append(t[0])
                    te.append(t[1])
                    tz.append(t[2])
                tr_off.append(len(tz))
            pkt_off.append(len(tr_off) - 1)
        route_off.append(len(rcost))
    i64 = lambda x: np.array(x, dtype=np.int64)
    f64 = lambda x: np.array(x, dtype=np.float64)
    return MeterLog(i64(host_off), i64(iv_off), f64(iv_s), f64(iv_e), i64(route_off), f64(rcost),
                    i64(pkt_off), i64(tr_off), f64(ts), f64(te), f64(tz))


def scenario_of(meter):
    """The logs of a reference ``resources.meter.Meter`` (its private dicts, in their order)."""
    meta = meter._Meter__meta
    hosts = [[list(v) for v in vals] for vals in meter._Meter__hosts.values()]
    routes = [(meta.cost[r.src.locality, r.dst.locality],
               [[tuple(t) for t in trans] for trans in pkts.values()])
              for r, pkts in meter._Meter__routes.items()]
    return {"hosts": hosts, "routes": routes}


class MeterAggregatesMixin:
    """Mixed in front of the reference's ``Meter``: the three aggregates come from the GPU."""

    engine = None

    def _pvt_aggregates(self):
        if self.engine is None:
            from .engine import default_engine
            eng = default_engine(0)
        else:
            eng = self.engine
        return eng.meter(pack([scenario_of(self)]))

    @property
    def cumulative_instance_hours(self):
        return float(self._pvt_aggregates()["instance_hours"][0])

    @property
    def total_network_traffic_cost(self):
        return float(self._pvt_aggregates()["egress_cost"][0])

    @property
    def average_congestion_delay(self):
        return float(self._pvt_aggregates()["congestion_delay"][0])
