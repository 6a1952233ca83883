"""Trace loader -> SoA, with the predecessor-instance table resident in HBM (SURVEY.md §8(f)
rank 3: "anchor/predecessor gather on GPU (a3) + trace loader -> SoA").

The reference loads an Alibaba job YAML into Application / Container objects
(alibaba/runner.py:86-102) and, every cost_aware round, walks Python objects to collect the
predecessor task placements of each ready task (scheduler/cost_aware.py:49-51):

    preds = [t for p in app.get_predecessors(c.id) for t in p.tasks]

Everything in that list except the placements is static for a trace, so it is flattened once:

* applications in submission order (``_bin_insert`` by submit_time, ties in file order,
  alibaba/runner.py:104-152); containers by application, then in ``Application.containers`` order (the dict
  ``{c.id: c}`` of application/__init__.py:20: first position of an id, last definition wins);
* ``pred_off`` / ``pred``: each container's predecessor containers in networkx
  ``DiGraph.predecessors`` order = the order edges into it were added = its ``dependencies``
  order without repeats (application/__init__.py:87-92,137-145);
* instances: container c owns instance indices ``inst_base[c] .. inst_base[c] + n_inst[c])``,
  in ``Container.generate_tasks`` order (application/__init__.py:309-315: Task(len(tasks), ...));
* ``pinst_off`` / ``pinst``: per container, the instance indices of all its predecessors' tasks
  in exactly the reference's iteration order — the list whose placements are counted.

``DeviceTrace`` keeps ``pinst`` and a per-instance host table ``inst_host`` in HBM. A round
records its placements with one scatter and resolves every ready container's anchor with one
``pvt_anchor`` launch that reads the rows of the resident table (``item`` form), so nothing
but the ready containers' row numbers crosses PCIe.

Demands follow alibaba/runner.py:93-100: cpus as in the trace, mem x MEM_SCALE_FACTOR
(7.68 * 1024), output_size = mem x the run's output-size scale factor, disk = gpus = 0.
"""
import dataclasses
import gzip
from typing import List

import numpy as np
import yaml

MEM_SCALE_FACTOR = 7.68 * 1024          # alibaba/runner.py:69


def _loader():
    return getattr(yaml, "CSafeLoader", yaml.SafeLoader)


def load_jobs(path):
    """The job list of an Alibaba trace YAML (plain or .gz)."""
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "rt") as f:
        return yaml.load(f, Loader=_loader())


@dataclasses.dataclass
class TraceArrays:
    app_ids: List[str]
    submit_time: np.ndarray     # [A] float64
    file_index: np.ndarray      # [A] int32: position of the job in the YAML
    app_off: np.ndarray         # [A+1] int64: containers of app a
    cont_ids: List[str]
    cont_app: np.ndarray        # [C] int32
    cpus: np.ndarray            # [C] float64
    mem: np.ndarray             # [C] float64 (scaled)
    output_size: np.ndarray     # [C] float64
    runtime: np.ndarray         # [C] float64
    n_inst: np.ndarray          # [C] int32
    inst_base: np.ndarray       # [C+1] int64
    pred_off: np.ndarray        # [C+1] int64
    pred: np.ndarray            # [E] int32 (global container index)
    pinst_off: np.ndarray       # [C+1] int64
    pinst: np.ndarray           # [P] int32 (instance index)

    @property
    def n_apps(self):
        return len(self.app_ids)

    @property
    def n_containers(self):
        return len(self.cont_ids)

    @property
    def n_instances(self):
        return int(self.inst_base[-1])

    def container_index(self, app, cid):
        """Global index of container ``cid`` (str) of application index ``app``."""
        lo, hi = int(self.app_off[app]), int(self.app_off[app + 1])
        return lo + self.cont_ids[lo:hi].index(str(cid))

    def instance_of(self, c):
        """Global instance index of the tasks of container c (np.arange)."""
        return np.arange(self.inst_base[c], self.inst_base[c + 1], dtype=np.int64)


def from_jobs(jobs, output_size_scale_factor=1000.0, n_apps=None) -> TraceArrays:
    """Flatten a job list (the YAML's schema: id, submit_time, tasks[id, cpus, mem, runtime,
    n_instances, dependencies]). ``n_apps`` keeps the first n applications in submission
    order, as TraceBasedApplicationGenerator does (alibaba/runner.py:121-136)."""
    ts = np.array([float(j["submit_time"]) for j in jobs], dtype=np.float64)
    order = np.argsort(ts, kind="stable")          # _bin_insert: by time, ties in file order
    if n_apps:
        order = order[:n_apps]
    app_ids, submit, app_off = [], [], [0]
    cont_ids, cont_app, cpus, mem, osz, rt, ninst = [], [], [], [], [], [], []
    pred_off, pred = [0], []
    scale = np.float64(MEM_SCALE_FACTOR)
    oscale = np.float64(output_size_scale_factor)
    for a, ji in enumerate(order):                 # applications in submission order
        j = jobs[ji]
        app_ids.append(str(j["id"]))
        submit.append(float(j["submit_time"]))
        defs = {}
        for t in j["tasks"]:                       # {c.id: c}: first position, last value
            defs[str(t["id"])] = t
        base = len(cont_ids)
        idx = {cid: base + k for k, cid in enumerate(defs)}
        for cid, t in defs.items():
            cont_ids.append(cid)
            cont_app.append(a)
            cpus.append(float(t["cpus"]))
            m = np.float64(t["mem"])
            mem.append(m * scale)
            osz.append(m * oscale)
            rt.append(float(t["runtime"]))
            ninst.append(int(t["n_instances"]))
        for cid, t in defs.items():
            seen = set()
            for d in t["dependencies"]:
                d = str(d)
                if d in seen:
                    continue
                seen.add(d)
                pred.append(idx[d])                # KeyError like the reference's _create_dag
            pred_off.append(len(pred))
        app_off.append(len(cont_ids))
    n_inst = np.array(ninst, dtype=np.int32)
    inst_base = np.concatenate([[0], np.cumsum(n_inst, dtype=np.int64)]).astype(np.int64)
    pred_off = np.array(pred_off, dtype=np.int64)
    pred = np.array(pred, dtype=np.int32)
    # per-container predecessor instance lists, vectorised: for every (container, pred) edge
    # the pred's instance range, concatenated in edge order
    cnt = n_inst[pred].astype(np.int64)
    cs = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    edge_start = inst_base[:-1][pred]
    pinst = (np.repeat(edge_start - cs[:-1], cnt)
             + np.arange(int(cs[-1]), dtype=np.int64)).astype(np.int32)
    pinst_off = cs[pred_off]                       # edges are in container order
    return TraceArrays(app_ids=app_ids, submit_time=np.array(submit, dtype=np.float64),
                       file_index=order.astype(np.int32),
                       app_off=np.array(app_off, dtype=np.int64), cont_ids=cont_ids,
                       cont_app=np.array(cont_app, dtype=np.int32),
                       cpus=np.array(cpus, dtype=np.float64), mem=np.array(mem, dtype=np.float64),
                       output_size=np.array(osz, dtype=np.float64),
                       runtime=np.array(rt, dtype=np.float64), n_inst=n_inst,
                       inst_base=inst_base, pred_off=pred_off, pred=pred,
                       pinst_off=pinst_off, pinst=pinst)


def load(path, output_size_scale_factor=1000.0, n_apps=None) -> TraceArrays:
    return from_jobs(load_jobs(path), output_size_scale_factor, n_apps)


class DeviceTrace:
    """A trace's predecessor-instance table and per-instance placements, resident in HBM."""

    def __init__(self, trace: TraceArrays, zone, engine):
        import torch
        self.trace = trace
        self.engine = engine
        dev = engine.device
        self.device = dev
        self.pinst_off = torch.from_numpy(trace.pinst_off).to(dev)
        self.pinst = torch.from_numpy(trace.pinst).to(dev)
        self.zone = torch.from_numpy(np.ascontiguousarray(zone, dtype=np.int32)).to(dev)
        self.inst_host = torch.full((max(trace.n_instances, 1),), -1, dtype=torch.int32,
                                    device=dev)

    def reset(self):
        self.inst_host.fill_(-1)

    def record(self, instances, hosts):
        """Placements of this round: inst_host[instances] = hosts (device or host arrays)."""
        import torch
        i = torch.as_tensor(np.asarray(instances, dtype=np.int64) if not torch.is_tensor(instances)
                            else instances, device=self.device).long()
        h = torch.as_tensor(np.asarray(hosts, dtype=np.int32) if not torch.is_tensor(hosts)
                            else hosts, device=self.device).int()
        self.inst_host.index_copy_(0, i, h)

    def anchors(self, containers):
        """(mode_host, anchor_zone) device tensors for the given container rows."""
        import torch
        item = torch.as_tensor(np.asarray(containers, dtype=np.int32) if not torch.is_tensor(
            containers) else containers, device=self.device).int()
        C = item.numel()
        mode = torch.empty(C, dtype=torch.int32, device=self.device)
        az = torch.empty(C, dtype=torch.int32, device=self.device)
        self.engine.anchor_device(self.pinst_off, self.pinst, self.zone, mode, az,
                                  inst_host=self.inst_host[:self.trace.n_instances] if
                                  self.trace.n_instances else None, item=item)
        return mode, az
