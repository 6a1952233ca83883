"""ctypes mirror of ``include/pivot_place.h`` (the engine's C ABI).

The reference has no native code, so this module is the binding a maintainer would add next to
its scheduler package. ``RoundArrays`` is the numpy-side description of one
round; ``pvt_round`` is the C struct it is marshalled into.
"""
import ctypes
import dataclasses
from typing import Optional

import numpy as np

PVT_ABI_VERSION = 3

PVT_OK = 0
PVT_EINVAL = -1
PVT_ENODEV = -2
PVT_EHIP = -3
PVT_ENOMEM = -4
PVT_EUNSUPPORTED = -5
PVT_ESTALE = -6
ERRORS = {PVT_EINVAL: "EINVAL", PVT_ENODEV: "ENODEV", PVT_EHIP: "EHIP", PVT_ENOMEM: "ENOMEM",
          PVT_EUNSUPPORTED: "EUNSUPPORTED", PVT_ESTALE: "ESTALE"}

PVT_CA_FF, PVT_CA_BF, PVT_OPP, PVT_VBP_FF, PVT_VBP_BF = range(5)
MODE_NAMES = {PVT_CA_FF: "cost_aware_ff", PVT_CA_BF: "cost_aware_bf", PVT_OPP: "opportunistic",
              PVT_VBP_FF: "vbp_ff", PVT_VBP_BF: "vbp_bf"}

PVT_K_SCORE, PVT_K_MERGE, PVT_K_COMMIT, PVT_K_OTHER = range(4)

# Resident rounds / scenario batches (pvt_place_batch).
PVT_RESIDENT_MAX_HOSTS = 4096
PVT_RESIDENT_MAX_TASKS = 4096

# Algorithmic bytes per (task, host) candidate, SURVEY.md §8(d).
BYTES_PER_CANDIDATE = {PVT_CA_FF: 36, PVT_CA_BF: 36, PVT_OPP: 32, PVT_VBP_FF: 32, PVT_VBP_BF: 36}


class pvt_round(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("n_hosts", ctypes.c_int32),
        ("n_tasks", ctypes.c_int32),
        ("n_zones", ctypes.c_int32),
        ("n_groups", ctypes.c_int32),
        ("sort_tasks", ctypes.c_int32),
        ("sort_hosts", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("avail", ctypes.c_void_p),
        ("zone", ctypes.c_void_p),
        ("tiebreak", ctypes.c_void_p),
        ("decay", ctypes.c_void_p),
        ("cost", ctypes.c_void_p),
        ("bw", ctypes.c_void_p),
        ("dem", ctypes.c_void_p),
        ("task_group", ctypes.c_void_p),
        ("group_anchor", ctypes.c_void_p),
        ("order", ctypes.c_void_p),
        ("placement", ctypes.c_void_p),
        ("mt_state", ctypes.c_void_p),
        ("rt_bw", ctypes.c_void_p),
    ]


class pvt_anchor_args(ctypes.Structure):
    _fields_ = [
        ("n_items", ctypes.c_int32),
        ("n_hosts", ctypes.c_int32),
        ("n_pred", ctypes.c_int64),
        ("n_inst", ctypes.c_int64),
        ("off", ctypes.c_void_p),
        ("list", ctypes.c_void_p),
        ("inst_host", ctypes.c_void_p),
        ("zone", ctypes.c_void_p),
        ("mode_host", ctypes.c_void_p),
        ("anchor_zone", ctypes.c_void_p),
        ("item", ctypes.c_void_p),
        ("n_rows", ctypes.c_int64),
    ]


class pvt_meter_log(ctypes.Structure):
    _fields_ = [("n_scen", ctypes.c_int32), ("reserved", ctypes.c_int32)] + [
        (n, ctypes.c_int64) for n in ("n_host_rows", "n_iv", "n_routes", "n_pkts", "n_tr")] + [
        (n, ctypes.c_void_p) for n in ("host_off", "iv_off", "iv_start", "iv_end", "route_off",
                                       "route_cost", "pkt_off", "tr_off", "tr_start", "tr_end",
                                       "tr_size", "instance_hours", "egress_cost",
                                       "congestion_delay")]


class pvt_ca_items(ctypes.Structure):
    _fields_ = [
        ("n_items", ctypes.c_int32),
        ("n_apps", ctypes.c_int32),
        ("n_pred", ctypes.c_int64),
        ("task_item", ctypes.c_void_p),
        ("pred_off", ctypes.c_void_p),
        ("pred_host", ctypes.c_void_p),
        ("item_app", ctypes.c_void_p),
        ("n_storage", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("storage_zone", ctypes.c_void_p),
        ("zone_storage", ctypes.c_void_p),
        ("mt_state", ctypes.c_void_p),
        ("status", ctypes.c_void_p),
    ]


# pvt_place_host grouping error kinds (pvt_ca_items.status[1])
GROUP_OK, GROUP_UNPLACED, GROUP_NO_STORAGE, GROUP_INVALID = 0, 1, 2, 3
# fused grouping limits (csrc/pvt_groups.h): tasks of a round, storages + applications
GRP_MAX_TASKS, GRP_MAX_KEYS = 16384, 8192

# pvt_anchor anchor_zone codes (include/pivot_place.h)
ANCHOR_NO_PREDS, ANCHOR_UNPLACED, ANCHOR_INVALID = -1, -2, -3


class pvt_kstats(ctypes.Structure):
    _fields_ = [("launches", ctypes.c_int64), ("ms", ctypes.c_double),
                ("candidates", ctypes.c_double), ("bytes", ctypes.c_double)]


@dataclasses.dataclass
class RoundArrays:
    """One scheduling round in the engine's SoA layout (host numpy arrays).

    avail (4, H) f64 · zone (H,) i32 · dem (4, T) f64 · cost/bw (Z, Z) f64 · optional
    tiebreak (H,) u32, decay (H,) i32, task_group (T,) i32 + group_anchor (G,) i32,
    mt_state (625,) u32 (MT19937 key + pos), rt_bw (G, H) f64 (cost_aware realtime_bw: in +
    out realtime bandwidth per group and host; row 0 without task_group).
    """
    mode: int
    avail: np.ndarray
    zone: np.ndarray
    dem: np.ndarray
    cost: Optional[np.ndarray] = None
    bw: Optional[np.ndarray] = None
    tiebreak: Optional[np.ndarray] = None
    decay: Optional[np.ndarray] = None
    task_group: Optional[np.ndarray] = None
    group_anchor: Optional[np.ndarray] = None
    sort_tasks: bool = False
    sort_hosts: bool = False
    mt_state: Optional[np.ndarray] = None
    rt_bw: Optional[np.ndarray] = None

    def __post_init__(self):
        self.avail = np.ascontiguousarray(self.avail, dtype=np.float64).reshape(4, -1)
        self.zone = np.ascontiguousarray(self.zone, dtype=np.int32)
        self.dem = np.ascontiguousarray(self.dem, dtype=np.float64).reshape(4, -1)
        if self.cost is None:
            self.cost = np.zeros((1, 1))
        if self.bw is None:
            self.bw = np.ones((1, 1))
        self.cost = np.ascontiguousarray(self.cost, dtype=np.float64)
        self.bw = np.ascontiguousarray(self.bw, dtype=np.float64)
        for name, dt in (("tiebreak", np.uint32), ("decay", np.int32), ("task_group", np.int32),
                         ("group_anchor", np.int32), ("mt_state", np.uint32),
                         ("rt_bw", np.float64)):
            v = getattr(self, name)
            if v is not None:
                setattr(self, name, np.ascontiguousarray(v, dtype=dt))

    @property
    def n_hosts(self):
        return self.avail.shape[1]

    @property
    def n_tasks(self):
        return self.dem.shape[1]

    @property
    def n_zones(self):
        return self.cost.shape[0]

    @property
    def n_groups(self):
        return 0 if self.group_anchor is None else len(self.group_anchor)

    def copy(self):
        return dataclasses.replace(self, **{f.name: (getattr(self, f.name).copy()
                                                      if isinstance(getattr(self, f.name), np.ndarray)
                                                      else getattr(self, f.name))
                                             for f in dataclasses.fields(self)})


@dataclasses.dataclass
class RoundResult:
    placement: np.ndarray      # (T,) i32 host index, -1 = not placed
    order: np.ndarray          # (T,) i32 processing order
    avail: np.ndarray          # (4, H) f64 after commits
    mt_state: Optional[np.ndarray] = None


def fill_struct(r: RoundArrays) -> pvt_round:
    """A pvt_round with the scalar fields of ``r`` set; the caller fills the array pointers
    (host pointers for the CPU oracle, device pointers for the engine)."""
    s = pvt_round()
    s.mode = r.mode
    s.n_hosts = r.n_hosts
    s.n_tasks = r.n_tasks
    s.n_zones = r.n_zones
    s.n_groups = r.n_groups
    s.sort_tasks = int(bool(r.sort_tasks))
    s.sort_hosts = int(bool(r.sort_hosts))
    s.reserved = 0
    return s


def check_rc(rc, lib_error=""):
    if rc != PVT_OK:
        raise RuntimeError("pivot_place error %s (%d): %s" % (ERRORS.get(rc, "?"), rc, lib_error))
