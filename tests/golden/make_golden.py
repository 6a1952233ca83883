#!/usr/bin/env python3
"""Generate the golden placement fixtures by running the REFERENCE policies (test-only).

This script is test infrastructure. It runs only in the build container, where the reference
is mounted read-only at /root/reference. It is never imported by the product, and nothing here
travels to the GPU box except the JSON fixtures it writes (``tests/golden/*.json.gz``).

How the reference is run:
- SimPy 3.0.11 is not installed and cannot be installed offline. A
  minimal stand-in ``simpy`` module is registered below. It provides constructors only. No
  event ever runs, because ``schedule()`` is a synchronous call that takes zero simulated time
  (reference scheduler/__init__.py:103).
- Python 3.10 removed ``collections.Iterable`` (reference application/__init__.py:7,
  resources/__init__.py:12), so an alias is installed.
- PyYAML 6 needs an explicit Loader (reference resources/__init__.py:574,
  alibaba/runner.py:89), so ``yaml.load`` defaults to the C safe loader.

Every nondeterminism knob is pinned (SURVEY.md §7 hard part 3):
- PYTHONHASHSEED=0, so ``set()`` storage order is fixed (reference resources/gen.py:58-59).
  The script re-launches itself with it.
- ``np.random.seed(0)`` runs before the first ``ResourceMetadata()``. That pins the bw jitter
  (reference resources/__init__.py:589).
- ``uuid.uuid4`` is seeded, which pins host ids (reference resources/__init__.py:170).
- Each scheduler gets an explicit ``seed=`` (reference scheduler/__init__.py:31).

Each fixture records one frozen cluster state plus several ``schedule()`` runs on it. Hosts are
referred to by their index in ``cluster.hosts`` order. Recorded per state: host availability,
zone index, host-id string rank, running-task count, the storage zone order, and the ready tasks with their container's predecessor
placements. Recorded per run: policy kwargs, seed, placement per task (-1 = None), returned
order, the processing order with its anchor zone per group (CA only), the hosts whose
availability changed with their final values, and the number of 32-bit MT19937 outputs the
run consumed from ``RandomState(seed)``. The zone tables (cost, jittered bw) are shared by all
fixtures and written once to ``zones_seed0.json``.
"""
import collections
import collections.abc
import gzip
import json
import os
import random
import subprocess
import sys
import types
import uuid

REF = os.environ.get("PIVOT_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


# ---------------------------------------------------------------------------------------
# Test-only stand-ins. Constructors and attributes only; no event semantics.
# ---------------------------------------------------------------------------------------
def _install_simpy_stub():
    m = types.ModuleType("simpy")

    class Event:
        def __init__(self, env=None):
            self.env = env

        def succeed(self, value=None):
            return self

    class Environment:
        def __init__(self, initial_time=0):
            self.now = initial_time

        def process(self, gen):
            return Event(self)

        def event(self):
            return Event(self)

        def timeout(self, delay=0, value=None):
            return Event(self)

        def run(self, until=None):
            raise NotImplementedError("stub simpy has no event loop")

    class Store:
        def __init__(self, env, capacity=float("inf")):
            self.env, self.capacity, self.items = env, capacity, []

        def put(self, item):
            self.items.append(item)
            return Event(self.env)

        def get(self):
            return Event(self.env)

    class Container:
        def __init__(self, env, capacity=float("inf"), init=0):
            self.env, self.capacity, self.level = env, capacity, init

        def get(self, amount):
            self.level -= amount
            return Event(self.env)

        def put(self, amount):
            self.level += amount
            return Event(self.env)

    class _Req:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    class Resource:
        def __init__(self, env, capacity=1):
            self.env = env

        def request(self):
            return _Req()

    m.Environment, m.Event, m.Store, m.Container, m.Resource = (
        Environment, Event, Store, Container, Resource)
    sys.modules["simpy"] = m
    return m


def _install_compat():
    collections.Iterable = collections.abc.Iterable
    import yaml
    loader = getattr(yaml, "CSafeLoader", yaml.SafeLoader)
    orig = yaml.load

    def load(stream, Loader=None):
        return orig(stream, Loader=Loader or loader)

    yaml.load = load


def _seed_uuid(seed):
    rng = random.Random(seed)
    uuid.uuid4 = lambda: uuid.UUID(int=rng.getrandbits(128), version=4)


# ---------------------------------------------------------------------------------------
# State builders (use the reference's own classes under the stand-ins)
# ---------------------------------------------------------------------------------------
class World:
    """Imports the reference modules once. The jitter is pinned by np.random.seed(0)."""

    def __init__(self):
        import numpy as np
        sys.path.insert(0, REF)
        np.random.seed(0)
        import resources  # noqa: F401
        from resources import ResourceMetadata, Cluster, Host, Storage
        from resources.gen import RandomClusterGenerator
        from resources.network import NetworkRoute
        from application import Application, Container, TaskState
        import scheduler.cost_aware as ca
        import scheduler.opportunistic as op
        import scheduler.vbp as vbp
        from alibaba.runner import TraceBasedApplicationGenerator
        self.np = np
        self.meta = ResourceMetadata()          # draws the 961 jitters now, seed 0
        self.Cluster, self.Host, self.Storage = Cluster, Host, Storage
        self.RandomClusterGenerator, self.NetworkRoute = RandomClusterGenerator, NetworkRoute
        self.Application, self.Container, self.TaskState = Application, Container, TaskState
        self.ca, self.op, self.vbp = ca, op, vbp
        self.TraceGen = TraceBasedApplicationGenerator
        self.simpy = sys.modules["simpy"]
        self.zones = self.meta.zones
        self._apps_cache = {}

    def zone_index(self, loc):
        return self.zones.index(loc)

    def tables(self):
        Z, cost, bw = len(self.zones), self.meta.cost, self.meta.bw
        c = [[cost[(a, b)] for b in self.zones] for a in self.zones]
        w = [[bw[(a, b)] for b in self.zones] for a in self.zones]
        assert len(c) == Z
        return c, w

    def cluster(self, env, n_hosts, full_routes, zones=None, caps=(16, 131072, 100, 1)):
        """Build a cluster the way sim.py does (reference alibaba/sim.py:174).

        ``full_routes`` uses RandomClusterGenerator.generate (all H^2 routes). Otherwise only
        the storage<->host routes that the policies read are built (resources/gen.py:70-74).
        ``zones`` restricts hosts to the given zone indices (host i gets zones[i % len]).
        """
        cpus, mem, disk, gpus = caps
        gen = self.RandomClusterGenerator(env, cpus, cpus, mem, mem, disk, disk, gpus, gpus,
                                          meter=None, seed=0)
        if full_routes and zones is None:
            return gen.generate(n_hosts)
        if zones is None:
            hosts = gen._generate_hosts(n_hosts)
        else:
            hosts = [self.Host(env, cpus, mem, disk, gpus, locality=self.zones[zones[i % len(zones)]])
                     for i in range(n_hosts)]
        storage = gen._generate_storage(hosts)
        routes = []
        for h in hosts:
            for s in storage:
                routes += [self.NetworkRoute(env, h, s, self.meta.bw[(h.locality, s.locality)]),
                           self.NetworkRoute(env, s, h, self.meta.bw[(s.locality, h.locality)])]
        return self.Cluster(env, hosts=hosts, storage=storage, routes=routes, meta=self.meta)

    def apps(self, env, job_file, n_apps):
        """First ``n_apps`` by submit time, loaded by the reference's trace loader."""
        gen = self.TraceGen(env, os.path.join(REF, "alibaba", "jobs", job_file), None, 1000,
                            n_apps)
        return gen.apps[:n_apps]


def fill_hosts(world, cluster, rs, frac_free=0.1, frac_drained=0.05):
    """Partially fill hosts like a running simulation would.

    Container levels are decremented by sequential gets, as SimPy Container.get does
    (reference resources/__init__.py:443-449). Trace-like demands are used, so mem values are
    inexact binary fractions.
    """
    M = 7.68 * 1024
    for h in cluster.hosts:
        r = h.resource
        cpus_c, mem_c = r._HostResource__cpus, r._HostResource__mem
        u = rs.random_sample()
        if u < frac_free:
            continue
        if u < frac_free + frac_drained:
            cpus_c.level = 0
            continue
        n = rs.randint(1, 40)
        for _ in range(n):
            c = 0.5 * rs.randint(1, 4)
            m = round(rs.uniform(0.05, 2.0), 2) * M
            if cpus_c.level - c < 0 or mem_c.level - m < 0:
                break
            cpus_c.get(c)
            mem_c.get(m)


def add_running(cluster, rs, max_tasks=6):
    """Give hosts fake running-task sets: host_decay reads len(h.tasks) (cost_aware.py:115)."""
    counts = []
    for h in cluster.hosts:
        k = int(rs.randint(0, max_tasks))
        s = h._Host__tasks
        for i in range(k):
            s.add(("running", h.id, i))
        counts.append(k)
    return counts


def make_ready(world, apps, cluster, rs, max_tasks):
    """Choose a frontier per app: finished containers (tasks placed on random hosts) and the
    ready containers whose nascent tasks form the ready queue. Placements are drawn from a small
    host subset so the mode-host tie-break (cost_aware.py:52) is exercised."""
    hosts = cluster.hosts
    ready = []
    for app in apps:
        dag_order = list(app.containers)
        finished = set()
        # walk containers in a topological order and finish a random prefix
        order = []
        remaining = {c.id: c for c in dag_order}
        while remaining:
            for cid in list(remaining):
                c = remaining[cid]
                if all(p.id in finished or p.id in [o.id for o in order]
                       for p in app.get_predecessors(cid)):
                    order.append(c)
                    del remaining[cid]
        cut = rs.randint(0, len(order) + 1)
        subset = [hosts[i] for i in rs.choice(len(hosts), size=min(len(hosts), rs.randint(1, 5)),
                                              replace=False)]
        for c in order[:cut]:
            for t in c.generate_tasks():
                t.placement = subset[rs.randint(0, len(subset))].id
                t.state = world.TaskState.FINISHED
            finished.add(c.id)
        for c in order[cut:]:
            if c.id in finished:
                continue
            preds = app.get_predecessors(c.id)
            if all(p.id in finished for p in preds):
                ready.extend(list(c.generate_tasks()))
    # interleave like the LIFO submit queue: shuffle blocks of tasks
    rs.shuffle(ready)
    return ready[:max_tasks]


# ---------------------------------------------------------------------------------------
# Recording runs
# ---------------------------------------------------------------------------------------
POLICIES = {
    "cost_aware": lambda w: w.ca.CostAwareGlobalScheduler,
    "opportunistic": lambda w: w.op.OpportunisticGlobalScheduler,
    "vbp_ff": lambda w: w.vbp.FirstFitGlobalScheduler,
    "vbp_bf": lambda w: w.vbp.BestFitGlobalScheduler,
}


def _draws_between(seed, after):
    """Number of 32-bit MT19937 outputs consumed between RandomState(seed) and ``after``.

    Storing the count (not the 624-word key) keeps fixtures small; tests rebuild the state by
    advancing RandomState(seed) by that many raw 32-bit draws."""
    import numpy as np
    rs = np.random.RandomState(seed)
    for n in range(1 << 22):
        st = rs.get_state()
        if st[2] == after[2] and (st[1] == after[1]).all():
            return n
        rs.randint(0, 1 << 32, dtype=np.uint32)
    raise RuntimeError("RNG advanced by more than 4M draws")


def record_state(world, cluster, tasks, running):
    hosts = cluster.hosts
    hidx = {h.id: i for i, h in enumerate(hosts)}
    ids = [h.id for h in hosts]
    rank = {hid: r for r, hid in enumerate(sorted(ids))}
    avail = [[h.resource.cpus_available, h.resource.mem_available, h.resource.disk_available,
              h.resource.gpus_available] for h in hosts]
    # containers of the ready tasks, with predecessor task placements in reference order
    cont_key, containers, task_cont, dem = {}, [], [], []
    for t in tasks:
        c = t.container
        key = (c.application.id, c.id)
        if key not in cont_key:
            app = c.application
            preds = [p for pc in app.get_predecessors(c.id) for p in pc.tasks]
            cont_key[key] = len(containers)
            containers.append({"app": len(set(k[0] for k in cont_key)) - 1,
                               "app_id": c.application.id, "id": c.id,
                               "pred_hosts": [hidx[p.placement] for p in preds]})
        task_cont.append(cont_key[key])
        dem.append([t.cpus, t.mem, t.disk, t.gpus])
    # stable app numbering in first-seen order
    app_num = {}
    for c in containers:
        c["app"] = app_num.setdefault(c["app_id"], len(app_num))
        del c["app_id"]
    return {
        "n_hosts": len(hosts),
        "avail": avail,
        "zone": [world.zone_index(h.locality) for h in hosts],
        "id_rank": [rank[h] for h in ids],
        "n_running": running,
        "storage_zone": [world.zone_index(s.locality) for s in cluster.storage],
        "tasks": {"dem": dem, "container": task_cont},
        "containers": containers,
    }


def run_policy(world, env, cluster, tasks, policy, kwargs, seed):
    cls = POLICIES[policy](world)
    hosts = cluster.hosts
    hidx = {h.id: i for i, h in enumerate(hosts)}
    tpos = {id(t): i for i, t in enumerate(tasks)}
    groups = []

    if policy == "cost_aware":
        zone_of = world.zone_index

        class Recording(cls):
            def _first_fit(self, hosts_, task_group, anchor, resc):
                groups.append({"anchor_zone": zone_of(anchor.locality),
                               "tasks": [tpos[id(t)] for t in task_group]})
                return super()._first_fit(hosts_, task_group, anchor, resc)

            def _best_fit(self, hosts_, task_group, anchor, resc):
                groups.append({"anchor_zone": zone_of(anchor.locality),
                               "tasks": [tpos[id(t)] for t in task_group]})
                return super()._best_fit(hosts_, task_group, anchor, resc)
        cls = Recording

    for t in tasks:
        t.placement = None
    sched = cls(env, cluster, seed=seed, **kwargs)
    sched._update_resource_info()
    before = {hid: a.copy() for hid, a in sched.resource_info.items()}
    assert (sched.randomizer.get_state()[1] == world.np.random.RandomState(seed).get_state()[1]).all()
    err = None
    try:
        out = list(sched.schedule(list(tasks)))
    except Exception as e:  # e.g. best-fit + host_decay (cost_aware.py:26,67,81)
        err = type(e).__name__
        out = []
    after = sched.resource_info
    changed = []
    for hid, a in after.items():
        if not (a == before[hid]).all():
            changed.append([hidx[hid]] + [float(x) for x in a])
    changed.sort()
    run = {
        "policy": policy, "kwargs": kwargs, "seed": seed,
        "error": err,
        "placement": [-1 if t.placement is None else hidx[t.placement] for t in tasks],
        "order": [tpos[id(t)] for t in out],
        "changed_avail": changed,
        "rng_draws": _draws_between(seed, sched.randomizer.get_state()),
    }
    if policy == "cost_aware":
        run["groups"] = groups
    for t in tasks:
        t.placement = None
    return run


SIM_RUNS = [
    ("cost_aware", {"bin_pack_algo": "first-fit", "sort_tasks": True, "sort_hosts": True}, 0),
    ("cost_aware", {"bin_pack_algo": "first-fit", "sort_tasks": False, "sort_hosts": True}, 1),
    ("cost_aware", {"bin_pack_algo": "first-fit", "sort_tasks": True, "sort_hosts": False}, 2),
    ("cost_aware", {"bin_pack_algo": "first-fit", "sort_tasks": True, "sort_hosts": True,
                    "host_decay": True}, 3),
    ("cost_aware", {"bin_pack_algo": "best-fit", "sort_tasks": True}, 4),
    ("cost_aware", {"bin_pack_algo": "best-fit", "sort_tasks": False}, 5),
    ("cost_aware", {"bin_pack_algo": "best-fit", "host_decay": True}, 6),
    ("opportunistic", {}, 0),
    ("opportunistic", {}, 12345),
    ("vbp_ff", {"decreasing": True}, 0),
    ("vbp_ff", {"decreasing": False}, 0),
    ("vbp_bf", {"decreasing": True}, 0),
]


def case_trace(world, name, n_hosts, n_apps, job_file, max_tasks, seed, full_routes, runs):
    env = world.simpy.Environment()
    cluster = world.cluster(env, n_hosts, full_routes)
    rs = world.np.random.RandomState(seed)
    fill_hosts(world, cluster, rs)
    running = add_running(cluster, rs)
    apps = world.apps(env, job_file, n_apps)
    tasks = make_ready(world, apps, cluster, rs, max_tasks)
    state = record_state(world, cluster, tasks, running)
    state["name"] = name
    state["runs"] = [run_policy(world, env, cluster, tasks, p, dict(k), s) for p, k, s in runs]
    return state


# realtime_bw=True (cost_aware.py:17,79,112): the bandwidth of a storage<->host pair is each
# route's realtime_bw (resources/network.py:70-73), 1 / ((queued MB + 1) / bw) -- so routes get
# queued packets here, and the fixture records every route's realtime_bw as the policy read it.
RT_RUNS = [
    ("cost_aware", {"bin_pack_algo": "first-fit", "sort_tasks": True, "sort_hosts": True,
                    "realtime_bw": True}, 0),
    ("cost_aware", {"bin_pack_algo": "first-fit", "sort_tasks": False, "sort_hosts": True,
                    "realtime_bw": True}, 1),
    ("cost_aware", {"bin_pack_algo": "first-fit", "sort_tasks": True, "sort_hosts": True,
                    "realtime_bw": True, "host_decay": True}, 3),
    ("cost_aware", {"bin_pack_algo": "best-fit", "sort_tasks": True, "realtime_bw": True}, 4),
    ("cost_aware", {"bin_pack_algo": "best-fit", "sort_tasks": False, "realtime_bw": True}, 5),
    ("cost_aware", {"bin_pack_algo": "best-fit", "sort_tasks": True}, 4),
]


def queue_packets(world, cluster, rs, frac=0.4, max_pkts=3):
    """Queue packets (1..max_pkts, uniform sizes up to 4000 MB) on a fraction of the
    storage<->host routes, as in-flight data pulls would (resources/network.py:82-100)."""
    from resources.network import Packet
    env = world.simpy.Environment()
    for s in cluster.storage:
        for h in cluster.hosts:
            for r in (cluster.get_route(s.id, h.id), cluster.get_route(h.id, s.id)):
                if rs.random_sample() < frac:
                    for _ in range(rs.randint(1, max_pkts + 1)):
                        r._NetworkRoute__pkts.items.append(Packet(float(rs.uniform(1, 4000)), env.event()))


def record_realtime(cluster):
    """Every storage<->host route's realtime_bw, as the policy reads it: rt_in[k][h] for
    storage k -> host h, rt_out[k][h] for host h -> storage k."""
    rt_in = [[cluster.get_route(s.id, h.id).realtime_bw for h in cluster.hosts] for s in cluster.storage]
    rt_out = [[cluster.get_route(h.id, s.id).realtime_bw for h in cluster.hosts] for s in cluster.storage]
    return rt_in, rt_out


def case_realtime(world, name, n_hosts, n_apps, job_file, max_tasks, seed, runs):
    """A config-1-shaped state (storage<->host routes only) with queued packets on its routes."""
    env = world.simpy.Environment()
    cluster = world.cluster(env, n_hosts, False)
    rs = world.np.random.RandomState(seed)
    fill_hosts(world, cluster, rs)
    running = add_running(cluster, rs)
    apps = world.apps(env, job_file, n_apps)
    tasks = make_ready(world, apps, cluster, rs, max_tasks)
    queue_packets(world, cluster, rs)
    state = record_state(world, cluster, tasks, running)
    state["name"] = name
    state["rt_in"], state["rt_out"] = record_realtime(cluster)
    state["runs"] = [run_policy(world, env, cluster, tasks, p, dict(k), s) for p, k, s in runs]
    return state


class _Cont:
    """A ready task's container for hand-built edge cases (no predecessors)."""


def case_synthetic(world, name, avail, zones, dems, seed, runs, n_running=None, pred=None):
    """Hand-built state: explicit availability and demands, one app per task (sources), or
    predecessor placements given as host indices (``pred``: per task list or None)."""
    env = world.simpy.Environment()
    H = len(avail)
    cluster = world.cluster(env, H, False, zones=zones, caps=(16, 131072, 100, 1))
    for h, a in zip(cluster.hosts, avail):
        r = h.resource
        r._HostResource__cpus.level = a[0]
        r._HostResource__mem.level = a[1]
        r._HostResource__disk.level = a[2]
        r._HostResource__gpus.level = a[3]
    running = [0] * H if n_running is None else n_running
    for h, k in zip(cluster.hosts, running):
        for i in range(k):
            h._Host__tasks.add(("running", h.id, i))
    tasks = []
    hosts = cluster.hosts
    for i, d in enumerate(dems):
        apps_pred = pred[i] if pred is not None else None
        if apps_pred:
            pc = world.Container(env, "p", cpus=1, mem=1.0)
            c = world.Container(env, "c", cpus=d[0], mem=d[1], disk=d[2], gpus=d[3],
                                dependencies=["p"])
            world.Application(env, "app%d" % i, [pc, c])
            pc._Container__instances = len(apps_pred)
            for t, hi in zip(pc.generate_tasks(), apps_pred):
                t.placement = hosts[hi].id
                t.state = world.TaskState.FINISHED
        else:
            c = world.Container(env, "c", cpus=d[0], mem=d[1], disk=d[2], gpus=d[3])
            world.Application(env, "app%d" % i, [c])
        tasks.extend(list(c.generate_tasks()))
    state = record_state(world, cluster, tasks, running)
    state["name"] = name
    state["runs"] = [run_policy(world, env, cluster, tasks, p, dict(k), s) for p, k, s in runs]
    return state


def edge_cases(world):
    np = world.np
    M = 7.68 * 1024
    out = []
    full = [16.0, 131072.0, 100.0, 1.0]
    # 1. empty ready queue
    out.append(case_synthetic(world, "empty", [full] * 4, [0, 1, 2, 3], [], 0, SIM_RUNS))
    # 2. one host; some tasks fit, some do not; demand == availability on cpus
    out.append(case_synthetic(world, "one_host", [[4.0, 8000.0, 100.0, 1.0]], [5],
                              [[2.0, 0.39 * M, 0, 0], [2.0, 0.2 * M, 0, 0], [0.5, 0.1 * M, 0, 0],
                               [20.0, 1.0, 0, 0]], 0, SIM_RUNS))
    # 3. identical free hosts: every score ties (VBP-BF tie-break by host-id string, others idx)
    out.append(case_synthetic(world, "ties", [full] * 12, list(range(0, 31, 3)),
                              [[0.5, 0.2 * M, 0, 0]] * 7 + [[1.0, 0.5 * M, 0, 0]] * 5, 0, SIM_RUNS))
    # 4. demand exactly equal to availability: >= places, > does not
    out.append(case_synthetic(world, "exact_fit", [[2.0, 1000.0, 0.0, 0.0], [3.0, 2000.0, 1.0, 1.0],
                                                   [2.0, 1000.0, 0.0, 0.0]], [0, 7, 14],
                              [[2.0, 1000.0, 0, 0], [2.0, 1000.0, 0, 0], [1.0, 500.0, 0, 0]],
                              0, SIM_RUNS))
    # 5. opportunistic n == 1 (no draw) and n == 0
    out.append(case_synthetic(world, "opp_single", [[1.0, 100.0, 1, 1], [8.0, 9000.0, 1, 1],
                                                    [1.0, 100.0, 1, 1]], [1, 2, 3],
                              [[4.0, 5000.0, 0, 0], [4.0, 5000.0, 0, 0], [4.0, 5000.0, 0, 0]],
                              0, SIM_RUNS))
    # 6. saturation: far more demand than capacity, many unplaced; hosts drain fully
    rs = np.random.RandomState(77)
    H = 64
    av = [[float(0.5 * rs.randint(0, 33)), float(rs.uniform(0, 131072)), 100.0, 1.0] for _ in range(H)]
    dm = [[0.5 * rs.randint(1, 9), round(rs.uniform(0.05, 3.0), 2) * M, 0, 0] for _ in range(700)]
    zs = list(range(31))
    out.append(case_synthetic(world, "saturate", av, zs, dm, 0, SIM_RUNS))
    # 7. predecessor placements with ties in the mode host (first-seen wins)
    rs = np.random.RandomState(5)
    H = 40
    av = [[float(0.5 * rs.randint(4, 33)), float(rs.uniform(20000, 131072)), 100.0, 1.0] for _ in range(H)]
    dm, pr = [], []
    for i in range(120):
        dm.append([0.5 * rs.randint(1, 5), round(rs.uniform(0.05, 1.0), 2) * M, 0, 0])
        k = rs.randint(0, 6)
        pr.append([int(x) for x in rs.randint(0, H, size=k)] if k else None)
    out.append(case_synthetic(world, "pred_ties", av, list(range(31)), dm, 0, SIM_RUNS, pred=pr))
    # 8. host_decay counts and zero-cost regions in first-fit keys
    rs = np.random.RandomState(9)
    H = 50
    av = [[float(0.5 * rs.randint(2, 33)), float(rs.uniform(5000, 131072)), 100.0, 1.0] for _ in range(H)]
    dm = [[0.5 * rs.randint(1, 4), round(rs.uniform(0.05, 1.5), 2) * M, 0, 0] for _ in range(150)]
    nr = [int(x) for x in rs.randint(0, 5, size=H)]
    out.append(case_synthetic(world, "decay", av, list(range(31)), dm, 0, SIM_RUNS, n_running=nr))
    return out


def main():
    if os.environ.get("PYTHONHASHSEED") != "0":
        env = dict(os.environ, PYTHONHASHSEED="0")
        sys.exit(subprocess.call([sys.executable] + sys.argv, env=env))
    _install_simpy_stub()
    _install_compat()
    _seed_uuid(20261015)
    import logging
    logging.disable(logging.CRITICAL)
    world = World()
    only = sys.argv[1:]
    if only:      # e.g. `make_golden.py rt_c1_h100`: the realtime_bw fixtures alone
        cases = [c for c in realtime_cases(world) if c["name"] in only]
        write_cases(cases)
        return
    cases = []
    cases += edge_cases(world)
    cases.append(case_trace(world, "c1_sim_h100", 100, 100, "jobs-5000-200-172800-259200.yaml",
                            800, 42, True, SIM_RUNS))
    cases.append(case_trace(world, "c2_h1000", 1000, 200, "jobs-5000-200-86400-172800.yaml",
                            1500, 43, False, SIM_RUNS))
    cases += realtime_cases(world)
    cost, bw = world.tables()
    with open(os.path.join(HERE, "zones_seed0.json"), "w") as f:
        json.dump({"zones": [repr(z) for z in world.zones], "cost": cost, "bw": bw}, f)
    write_cases(cases)


def realtime_cases(world):
    return [case_realtime(world, "rt_c1_h100", 100, 100, "jobs-5000-200-172800-259200.yaml", 800,
                          44, RT_RUNS),
            case_realtime(world, "rt_h12", 12, 100, "jobs-5000-200-172800-259200.yaml", 300, 45,
                          RT_RUNS)]


def write_cases(cases):
    for c in cases:
        fn = os.path.join(HERE, "%s.json.gz" % c["name"])
        with gzip.open(fn, "wt") as f:
            json.dump(c, f, separators=(",", ":"))
        nplaced = [sum(p >= 0 for p in r["placement"]) for r in c["runs"]]
        print("%-14s H=%-5d T=%-5d placed per run %s" % (c["name"], c["n_hosts"],
                                                       len(c["tasks"]["dem"]), nplaced))


if __name__ == "__main__":
    main()
