"""Reference-shaped stand-ins built from a golden fixture, for the drop-in policy tests.

The drop-in policies read only what the reference's policies read:
cluster.hosts / storage / get_host / get_storage_by_locality / meta.{zones,cost,bw},
h.id / h.locality / h.tasks / h.resource.*_available, and t.cpus / mem / disk / gpus /
container.application.get_predecessors(c.id) / predecessor tasks' placement. These classes
provide exactly that, like the reference's own MockScheduler fake (test/test_resource.py:13-41).
"""
import numpy as np

import golden_io


class Locality:
    def __init__(self, name):
        self.name = name

    def __hash__(self):
        return hash(self.name)

    def __eq__(self, other):
        return isinstance(other, Locality) and other.name == self.name

    def __repr__(self):
        return self.name


class Resource:
    def __init__(self, a):
        self.cpus_available, self.mem_available, self.disk_available, self.gpus_available = (
            float(a[0]), float(a[1]), float(a[2]), float(a[3]))


class Host:
    def __init__(self, hid, locality, avail, n_running):
        self.id = hid
        self.locality = locality
        self.resource = Resource(avail)
        self.tasks = [("running", i) for i in range(n_running)]


class Storage:
    def __init__(self, sid, locality):
        self.id = sid
        self.locality = locality


class Meta:
    def __init__(self, zones, cost, bw):
        self.zones = zones
        self.cost = {(a, b): float(cost[i][j]) for i, a in enumerate(zones) for j, b in enumerate(zones)}
        self.bw = {(a, b): float(bw[i][j]) for i, a in enumerate(zones) for j, b in enumerate(zones)}


class Route:
    def __init__(self, bw, realtime_bw):
        self.bw = bw
        self.realtime_bw = realtime_bw


class Cluster:
    def __init__(self, hosts, storage, meta, routes=None):
        self.hosts = hosts
        self.storage = storage
        self.meta = meta
        self._by_id = {h.id: h for h in hosts}
        self._storage_by_loc = {s.locality: s for s in storage}
        self._routes = routes or {}

    def get_route(self, src_id, dst_id):
        return self._routes.get((src_id, dst_id))

    def get_host(self, hid):
        return self._by_id.get(hid)

    def get_storage_by_locality(self, loc):
        return self._storage_by_loc.get(loc)


class Task:
    def __init__(self, container, d):
        self.container = container
        self.cpus, self.mem, self.disk, self.gpus = d
        self.placement = None


class Container:
    def __init__(self, cid, app):
        self.id = cid
        self.application = app
        self.tasks = []


class Application:
    def __init__(self, aid):
        self.id = aid
        self.preds = {}

    def get_predecessors(self, cid):
        return self.preds.get(cid, [])


def refresh(cluster, case):
    """Set the hosts of a cluster built for an earlier round of the same simulation to this
    round's state (availability, running tasks)."""
    for h, a, nr in zip(cluster.hosts, case["avail"], case["n_running"]):
        h.resource = Resource(a)
        if len(h.tasks) != nr:
            h.tasks = [("running", i) for i in range(nr)]


def build_tasks(case, cluster):
    """The ready tasks of a fixture's round (containers, predecessor placements) on ``cluster``."""
    hosts = cluster.hosts
    apps, conts = {}, []
    for k, c in enumerate(case["containers"]):
        app = apps.setdefault(c["app"], Application("app%d" % c["app"]))
        cont = Container("c%d" % k, app)
        pred = Container("p%d" % k, app)
        for hi in c["pred_hosts"]:
            t = Task(pred, (1, 1.0, 0, 0))
            t.placement = hosts[hi].id
            pred.tasks.append(t)
        app.preds[cont.id] = [pred] if c["pred_hosts"] else []
        conts.append(cont)
    return [Task(conts[ci], tuple(d)) for d, ci in zip(case["tasks"]["dem"], case["tasks"]["container"])]


def build(case):
    """(cluster, tasks) reproducing a fixture's state."""
    cost, bw, names = golden_io.zones()
    zones = [Locality(n) for n in names]
    # host-id strings whose sort order reproduces the recorded ranks
    rank = case["id_rank"]
    ids = ["h%05d" % r for r in rank]
    hosts = [Host(ids[i], zones[z], a, nr) for i, (z, a, nr) in
             enumerate(zip(case["zone"], case["avail"], case["n_running"]))]
    storage = [Storage("s%02d" % k, zones[z]) for k, z in enumerate(case["storage_zone"])]
    routes = {}
    if "rt_in" in case:     # storage <-> host routes with the recorded realtime bandwidths
        for k, s in enumerate(storage):
            for j, h in enumerate(hosts):
                zs, zh = names.index(s.locality.name), names.index(h.locality.name)
                routes[(s.id, h.id)] = Route(float(bw[zs][zh]), case["rt_in"][k][j])
                routes[(h.id, s.id)] = Route(float(bw[zh][zs]), case["rt_out"][k][j])
    cluster = Cluster(hosts, storage, Meta(zones, cost, bw), routes)
    return cluster, build_tasks(case, cluster)
