"""Drop-in GPU policies with the reference's plugin contract.

A reference policy subclasses ``GlobalSchedulerBase`` and overrides ``schedule(self, tasks)``
(reference scheduler/__init__.py:79-80), called once per round at scheduler/__init__.py:103.
The mixins below keep that contract and the reference's constructor kwargs. Their
``schedule()`` marshals the round into the engine's SoA layout and calls ``pvt_place``:

=============================  =======================================================
reference class                drop-in here
=============================  =======================================================
CostAwareGlobalScheduler       ``CostAwarePlacement``    (scheduler/cost_aware.py:11-127)
OpportunisticGlobalScheduler   ``OpportunisticPlacement`` (scheduler/opportunistic.py:8-20)
FirstFitGlobalScheduler        ``FirstFitPlacement``     (scheduler/vbp.py:6-29)
BestFitGlobalScheduler         ``BestFitPlacement``      (scheduler/vbp.py:32-50)
=============================  =======================================================

Each mixin needs only what the reference base provides: ``self.cluster`` (hosts, storage,
get_host, get_storage_by_locality, meta), ``self.resource_info`` (the round snapshot, whose
arrays it updates in place like the reference's ``resc[h.id] -= t_demand``) and
``self.randomizer`` (numpy RandomState, advanced exactly as the reference advances it). So a
maintainer combines a mixin with the reference base unchanged, or uses the
ready-made classes at the bottom, built on ``GlobalSchedulerBase`` in this module (the
attributes of reference scheduler/__init__.py:14-85, without the SimPy loop).

What stays on the host, as in the reference: cost_aware grouping and anchor choice
(cost_aware.py:45-58, the ``randomizer.choice(storage)`` at :38-39), because it reads the
application DAG and advances the RNG.
"""
from collections import OrderedDict

import numpy as np
import numpy.random as rnd

from . import _abi
from ._abi import RoundArrays


class GlobalSchedulerBase:
    """The parts of reference scheduler/__init__.py:14-85 that ``schedule()`` relies on."""

    def __init__(self, env, cluster, interval=5, seed=None, meter=None, *args, **kwargs):
        assert isinstance(interval, int)
        self.__env = env
        self.__cluster = cluster
        self.__interval = interval
        self.__resource_info = {}
        self.__randomizer = rnd.RandomState(seed)
        self.__meter = meter

    @property
    def env(self):
        return self.__env

    @property
    def cluster(self):
        return self.__cluster

    @property
    def resource_info(self):
        return dict(self.__resource_info)

    @property
    def randomizer(self):
        return self.__randomizer

    def schedule(self, tasks):
        raise NotImplementedError

    def _update_resource_info(self):
        self.__resource_info = {h.id: np.array([h.resource.cpus_available, h.resource.mem_available,
                                                h.resource.disk_available, h.resource.gpus_available])
                                for h in self.cluster.hosts}


class _ClusterTables:
    """Per-cluster static arrays: zone index per host, host-id ranks, Z x Z cost / bw."""

    def __init__(self, cluster):
        meta = cluster.meta
        hosts = cluster.hosts
        self.n_hosts = len(hosts)
        self.host_ids = [h.id for h in hosts]
        self.host_index = {hid: i for i, hid in enumerate(self.host_ids)}
        self.zones = list(meta.zones) if meta is not None else []
        self.zone_of = {z: i for i, z in enumerate(self.zones)}
        self.zone = np.array([self.zone_of.get(h.locality, 0) for h in hosts], dtype=np.int32)
        order = sorted(range(len(hosts)), key=lambda i: self.host_ids[i])
        self.rank = np.empty(len(hosts), dtype=np.uint32)
        self.rank[order] = np.arange(len(hosts), dtype=np.uint32)
        if meta is not None and self.zones:
            cost, bw = meta.cost, meta.bw
            Z = len(self.zones)
            self.cost = np.array([[cost[(a, b)] for b in self.zones] for a in self.zones],
                                 dtype=np.float64).reshape(Z, Z)
            self.bw = np.array([[bw[(a, b)] for b in self.zones] for a in self.zones],
                               dtype=np.float64).reshape(Z, Z)
        else:
            self.cost = np.zeros((1, 1))
            self.bw = np.ones((1, 1))
        self._storage_key = None

    def storage_tables(self, cluster):
        """(storage_zone[S], zone_storage[Z]) for the device grouping: the zone of each storage in
        cluster.storage order, and the index of get_storage_by_locality(zone) in that list (-1:
        None), rebuilt when the storage list changes."""
        storage = cluster.storage
        key = (id(storage), len(storage), tuple(id(x) for x in storage))
        if self._storage_key != key:
            pos = {id(x): i for i, x in enumerate(storage)}
            self._storage_zone = np.array([self.zone_of.get(x.locality, -1) for x in storage],
                                          dtype=np.int32)
            zs = []
            for z in self.zones:
                st = cluster.get_storage_by_locality(z)
                zs.append(-1 if st is None else pos.get(id(st), -1))
            self._zone_storage = np.array(zs, dtype=np.int32)
            self._storage_key = key
        return self._storage_zone, self._zone_storage

    def routes_of(self, cluster, anchor):
        """(in routes, out routes) between storage ``anchor`` and every host, in host order,
        looked up afresh in every schedule() call (the caller memoises per call): the
        reference's cluster.add_route may replace a (src, dst) route between rounds
        (resources/__init__.py:106-109), and its get_route then returns the new object. A
        missing route raises what the reference's host_score_func raises reading it
        (cost_aware.py:73-79, 106-112)."""
        get_route = cluster.get_route
        ins = [get_route(anchor.id, h) for h in self.host_ids]
        outs = [get_route(h, anchor.id) for h in self.host_ids]
        if any(x is None for x in ins) or any(x is None for x in outs):
            raise AttributeError("'NoneType' object has no attribute 'realtime_bw'")
        return ins, outs

    def matches(self, cluster):
        hosts = cluster.hosts
        return len(hosts) == self.n_hosts and all(h.id == i for h, i in zip(hosts, self.host_ids))


class PlacementMixin:
    """Shared marshalling: snapshot -> SoA, engine call, results -> tasks and resc."""

    engine = None          # set to a PlacementEngine to pin a device; default: cuda:0

    def _engine(self):
        if self.engine is None:
            from .engine import default_engine
            return default_engine(0)
        return self.engine

    def _tables(self):
        cl = self.cluster
        tab = getattr(self, "_pvt_tables", None)
        if tab is None or not tab.matches(cl):
            tab = _ClusterTables(cl)
            self._pvt_tables = tab
        return tab

    def _snapshot(self, resc):
        """The round snapshot as SoA avail[4][H] (one stack of the per-host arrays)."""
        ids = self._tables().host_ids
        if not ids:
            return np.empty((4, 0), dtype=np.float64)
        return np.ascontiguousarray(np.stack([resc[i] for i in ids], axis=1), dtype=np.float64)

    @staticmethod
    def _demand(tasks):
        if not tasks:
            return np.empty((4, 0), dtype=np.float64)
        return np.array([(t.cpus, t.mem, t.disk, t.gpus) for t in tasks], dtype=np.float64).T.copy()

    def _apply(self, tasks, hosts, resc, res, before):
        ids = self._tables().host_ids
        for j in np.nonzero(res.placement >= 0)[0]:
            tasks[j].placement = ids[res.placement[j]]
        changed = np.nonzero((res.avail != before).any(axis=0))[0]
        for j in changed:
            resc[ids[j]][:] = res.avail[:, j]


class CostAwarePlacement(PlacementMixin):
    """PIVOT's cost-aware policy (reference scheduler/cost_aware.py:11-127)."""

    def __init__(self, *args, **kwargs):
        bin_pack_algo = str(kwargs.pop('bin_pack_algo', 'first-fit'))
        sort_tasks = bool(kwargs.pop('sort_tasks', False))
        sort_hosts = bool(kwargs.pop('sort_hosts', False))
        realtime_bw = kwargs.pop('realtime_bw', False)
        host_decay = kwargs.pop('host_decay', False)
        super().__init__(*args, **kwargs)
        self._pvt_algo = bin_pack_algo
        self._pvt_sort_tasks = sort_tasks
        self._pvt_sort_hosts = sort_hosts
        self._pvt_realtime_bw = realtime_bw
        self._pvt_host_decay = host_decay

    def _pred_tasks(self, c):
        """The predecessor tasks of container c, flattened in the reference's order
        (cost_aware.py:50: [t for p in app.get_predecessors(c.id) for t in p.tasks]); the DAG
        is static, so the list is kept per container (their placements are read every round)."""
        cache = self.__dict__.setdefault("_pvt_preds", {})
        e = cache.get(id(c))
        if e is None or e[0] is not c:
            e = cache[id(c)] = (c, [p for pc in c.application.get_predecessors(c.id) for p in pc.tasks])
        return e[1]

    def _items(self, tasks):
        """One item per distinct container of the ready tasks (first-seen order): its
        predecessor placements as host indices (-1: not a host), CSR."""
        idx = self._tables().host_index
        items, item_of, off, lst = [], [], [0], []
        memo = {}
        for t in tasks:
            c = t.container
            i = memo.get(id(c))
            if i is None:
                i = memo[id(c)] = len(items)
                items.append(c)
                lst.extend([idx.get(p.placement, -1) for p in self._pred_tasks(c)])
                off.append(len(lst))
            item_of.append(i)
        return items, item_of, off, lst

    def _group_tasks(self, tasks):
        """Groups keyed by anchor storage, or by application for source tasks, in first-seen
        order (reference cost_aware.py:45-58). The anchor of a task with predecessors is the
        zone of the MODE host of all predecessor task placements (first seen wins ties); the
        mode is computed on the GPU (pvt_anchor), one item per distinct container."""
        cluster = self.cluster
        tab = self._tables()
        items, item_of, off, lst = self._items(tasks)
        zones = None
        if lst:
            _, zones = self._engine().anchor(np.array(off, dtype=np.int64),
                                             np.array(lst, dtype=np.int32), tab.zone)
        groups = OrderedDict()
        for t, i in zip(tasks, item_of):
            z = -1 if zones is None else int(zones[i])
            if z == _abi.ANCHOR_NO_PREDS:
                key = ('app', items[i].application)
            elif z >= 0:
                key = ('storage', cluster.get_storage_by_locality(tab.zones[z]))
            else:   # the mode placement is not a host of the cluster (get_host -> None)
                raise AttributeError("'NoneType' object has no attribute 'locality'")
            groups.setdefault(key, []).append(t)
        return groups

    def _realtime_row(self, anchor, memo):
        """realtime_bw=True (cost_aware.py:73-79, :106-112): per host, the bandwidth the
        reference's host_score_func uses, in_route.realtime_bw + out_route.realtime_bw of the
        routes between the anchor storage and the host (resources/network.py:70-73), read from
        the cluster's own route objects (looked up once per call) and summed elementwise in
        the reference's order. Queues do not move inside schedule(), so groups sharing an
        anchor share the row."""
        row = memo.get(anchor.id)
        if row is None:
            ins, outs = self._tables().routes_of(self.cluster, anchor)
            row = memo[anchor.id] = (np.array([x.realtime_bw for x in ins], dtype=np.float64)
                                     + np.array([x.realtime_bw for x in outs], dtype=np.float64))
        return row

    def _schedule_fused(self, tasks, resc, best_fit):
        """The whole round -- grouping, anchors, draws and placement -- in ONE device round trip
        (engine.place_cost_aware); False when the engine or the round cannot take it."""
        eng = self._engine()
        if not hasattr(eng, "place_cost_aware") or not tasks:
            return False
        tab = self._tables()
        items, item_of, off, lst = self._items(tasks)
        apps = {}
        item_app = [apps.setdefault(id(c.application), len(apps)) for c in items]
        storage_zone, zone_storage = tab.storage_tables(self.cluster)
        avail = self._snapshot(resc)
        decay = None
        if self._pvt_host_decay:
            decay = np.array([max(len(h.tasks), 1) for h in self.cluster.hosts], dtype=np.int32)
        r = RoundArrays(mode=_abi.PVT_CA_BF if best_fit else _abi.PVT_CA_FF, avail=avail,
                        zone=tab.zone, dem=self._demand(tasks), cost=tab.cost, bw=tab.bw,
                        decay=decay, sort_tasks=self._pvt_sort_tasks,
                        sort_hosts=self._pvt_sort_hosts)
        st = self.randomizer.get_state()
        mt = np.empty(625, dtype=np.uint32)
        mt[:624] = st[1]
        mt[624] = st[2]
        got = eng.place_cost_aware(r, item_of, off, lst, item_app, len(apps), storage_zone,
                                   zone_storage, mt)
        if got is None:
            return False
        res, _, mt = got
        self.randomizer.set_state((st[0], mt[:624].copy(), int(mt[624]), st[3], st[4]))
        self._apply(tasks, self.cluster.hosts, resc, res, avail)
        return True

    def schedule(self, tasks):
        algo = self._pvt_algo
        if algo not in ('first-fit', 'best-fit'):
            if tasks:   # the reference calls the str (cost_aware.py:42)
                raise TypeError("'str' object is not callable")
            return tasks
        storage, hosts = self.cluster.storage, self.cluster.hosts
        resc = self.resource_info
        best_fit = algo == 'best-fit'
        # one round trip when nothing needs the groups on the host: realtime_bw reads routes per
        # group anchor, and best-fit with host_decay raises mid-loop (cost_aware.py:26,81)
        if (not self._pvt_realtime_bw and not (best_fit and self._pvt_host_decay)
                and self._schedule_fused(tasks, resc, best_fit)):
            return tasks
        tab = self._tables()
        groups = self._group_tasks(tasks)
        task_pos = {id(t): i for i, t in enumerate(tasks)}
        T = len(tasks)
        task_group = np.zeros(T, dtype=np.int32)
        anchors, rt_rows = [], []
        avail = self._snapshot(resc)
        dem = self._demand(tasks)
        # the reference reads routes only through host_score_func: best-fit, and first-fit with
        # sort_hosts (cost_aware.py:92, 118-119); unsorted first-fit never does
        rt = self._pvt_realtime_bw and (best_fit or self._pvt_sort_hosts)
        rt_memo = {}
        for g, ((kind, obj), members) in enumerate(groups.items()):
            anchor = self.randomizer.choice(storage) if kind == 'app' else obj
            if best_fit and self._pvt_host_decay:
                # the reference reads None[h.id] on the first candidate (cost_aware.py:26,81)
                idx = [task_pos[id(t)] for t in members]
                if any(((avail >= dem[:, [i]]).all(axis=0)).any() for i in idx):
                    raise TypeError("'NoneType' object is not subscriptable")
            anchors.append(tab.zone_of[anchor.locality])
            for t in members:
                task_group[task_pos[id(t)]] = g
            if rt:
                rt_rows.append(self._realtime_row(anchor, rt_memo))
        if best_fit and self._pvt_host_decay:
            return tasks
        decay = None
        if self._pvt_host_decay:
            decay = np.array([max(len(h.tasks), 1) for h in hosts], dtype=np.int32)
        r = RoundArrays(mode=_abi.PVT_CA_BF if best_fit else _abi.PVT_CA_FF, avail=avail,
                        zone=tab.zone, dem=dem, cost=tab.cost, bw=tab.bw, decay=decay,
                        task_group=task_group, group_anchor=np.array(anchors, dtype=np.int32),
                        sort_tasks=self._pvt_sort_tasks, sort_hosts=self._pvt_sort_hosts,
                        rt_bw=np.stack(rt_rows) if rt_rows else None)
        if T:
            res = self._engine().place(r)
            self._apply(tasks, hosts, resc, res, avail)
        return tasks


class OpportunisticPlacement(PlacementMixin):
    """Uniform random feasible host (reference scheduler/opportunistic.py:11-20)."""

    def schedule(self, tasks):
        hosts = self.cluster.hosts
        resc = self.resource_info
        if not tasks:
            return list(tasks)
        tab = self._tables()
        st = self.randomizer.get_state()
        mt = np.empty(625, dtype=np.uint32)
        mt[:624] = st[1]
        mt[624] = st[2]
        avail = self._snapshot(resc)
        r = RoundArrays(mode=_abi.PVT_OPP, avail=avail, zone=tab.zone, dem=self._demand(tasks),
                        mt_state=mt)
        res = self._engine().place(r)
        self.randomizer.set_state((st[0], res.mt_state[:624].copy(), int(res.mt_state[624]),
                                   st[3], st[4]))
        self._apply(tasks, hosts, resc, res, avail)
        return list(tasks)


class _VbpPlacement(PlacementMixin):
    _mode = None

    def __init__(self, *args, **kwargs):
        # str(False) is truthy: the reference always sorts (scheduler/vbp.py:9,35)
        decreasing = str(kwargs.pop('decreasing', False))
        super().__init__(*args, **kwargs)
        self._pvt_decreasing = decreasing

    def schedule(self, tasks):
        hosts = self.cluster.hosts
        resc = self.resource_info
        if not tasks:
            return list(tasks) if self._pvt_decreasing else tasks
        tab = self._tables()
        avail = self._snapshot(resc)
        r = RoundArrays(mode=self._mode, avail=avail, zone=tab.zone, dem=self._demand(tasks),
                        tiebreak=tab.rank, sort_tasks=bool(self._pvt_decreasing))
        res = self._engine().place(r)
        self._apply(tasks, hosts, resc, res, avail)
        return [tasks[i] for i in res.order]


class FirstFitPlacement(_VbpPlacement):
    """Vector bin packing, first fit (reference scheduler/vbp.py:6-29)."""
    _mode = _abi.PVT_VBP_FF


class BestFitPlacement(_VbpPlacement):
    """Vector bin packing, best fit, ties by host-id string (reference scheduler/vbp.py:32-50)."""
    _mode = _abi.PVT_VBP_BF


class CostAwareGlobalScheduler(CostAwarePlacement, GlobalSchedulerBase):
    pass


class OpportunisticGlobalScheduler(OpportunisticPlacement, GlobalSchedulerBase):
    pass


class FirstFitGlobalScheduler(FirstFitPlacement, GlobalSchedulerBase):
    pass


class BestFitGlobalScheduler(BestFitPlacement, GlobalSchedulerBase):
    pass
