#!/usr/bin/env python3
"""Meter logs of REFERENCE simulations (test-only).

Runs reference simulations exactly as make_golden_sim.py does (its ``simulate``), then writes
the reference Meter's raw logs (resources/meter.py:15-24,55-83) and its own aggregates:

* ``hosts``: the meter's ``__hosts`` dict in its order — per host the [check-in, check-out]
  intervals (host_check_in / host_check_out, :55-76);
* ``routes``: the ``__routes`` dict in its order — per route the zone indices of its src / dst
  locality, ``cost[src.locality, dst.locality]`` from the meter's own ResourceMetadata, and per
  packet (dict order) its [start, end, size] transfers (route_check_in / _out, :78-83);
* ``want``: ``cumulative_instance_hours`` (:31-33), ``total_network_traffic_cost`` (:35-42,
  with ResourceMetadata.calc_network_traffic_cost, resources/__init__.py:565-569) and
  ``average_congestion_delay`` (:44-53), as the reference computes them.

Output: tests/golden/meter_logs.json.gz. Only the fixture travels.
"""
import gzip
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
RUNS = [("sim_c1_cost_aware", "cost_aware", {"bin_pack_algo": "first-fit", "sort_tasks": True,
                                             "sort_hosts": True}, 100, 100,
         "jobs-5000-200-172800-259200.yaml"),
        ("sim_h12_opportunistic", "opportunistic", {}, 12, 100,
         "jobs-5000-200-172800-259200.yaml"),
        ("sim_c1_vbp_bf", "vbp_bf", {"decreasing": True}, 100, 100,
         "jobs-5000-200-172800-259200.yaml")]


def main():
    if os.environ.get("PYTHONHASHSEED") != "0":
        env = dict(os.environ, PYTHONHASHSEED="0")
        sys.exit(subprocess.call([sys.executable] + sys.argv, env=env))
    sys.path.insert(0, HERE)
    import make_golden_sim as mgs
    from pivot_place import des
    des.install(force=True)
    import make_golden as mg
    mg._install_compat()
    import logging
    logging.disable(logging.CRITICAL)
    world = mg.World()
    out = []
    for label, policy, kwargs, n_hosts, n_apps, job in RUNS:
        got = []
        mgs.simulate(mg, world, label, policy, kwargs, n_hosts, n_apps, job, meter_out=got)
        meter, cluster = got[0]
        meta = meter._Meter__meta
        zones = list(meta.zones)
        zi = {z: i for i, z in enumerate(zones)}
        hidx = {id(h): i for i, h in enumerate(cluster.hosts)}
        hosts = [{"host": hidx[id(h)], "intervals": [list(v) for v in vals]}
                 for h, vals in meter._Meter__hosts.items()]
        routes = []
        for r, pkts in meter._Meter__routes.items():
            routes.append({"src": zi[r.src.locality], "dst": zi[r.dst.locality],
                           "cost": meta.cost[r.src.locality, r.dst.locality],
                           "packets": [[list(t) for t in trans] for trans in pkts.values()]})
        out.append({"name": label, "hosts": hosts, "routes": routes, "want": {
            "cumulative_instance_hours": meter.cumulative_instance_hours,
            "total_network_traffic_cost": meter.total_network_traffic_cost,
            "average_congestion_delay": meter.average_congestion_delay}})
        print(label, len(hosts), len(routes), sum(len(r["packets"]) for r in routes),
              out[-1]["want"])
    with gzip.open(os.path.join(HERE, "meter_logs.json.gz"), "wt") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
