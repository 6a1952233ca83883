"""PlacementEngine: the Python side of the C ABI (libpivot_place.so, gfx950 only).

The engine owns one ``pvt_ctx`` per GPU. ``place()`` takes a round as host numpy arrays
(``RoundArrays``), stages them in HBM as torch-ROCm tensors, calls ``pvt_place`` and returns
host copies. ``DeviceRound`` keeps a round resident in HBM for repeated calls (bench, multi-GPU).

There is no CPU fallback: if the HIP library is missing or no gfx950 device is visible, the
constructor raises. The CPU restatement under oracle/ is test infrastructure and is never
reached from here.
"""
import ctypes
import os

import numpy as np

from . import _abi
from ._abi import RoundArrays, RoundResult

LIB_NAME = "libpivot_place.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

_lib = None


def load_library(path=None):
    """Load libpivot_place.so (raises OSError when it was not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("PIVOT_PLACE_LIB") or LIB_PATH   # env: diagnostic builds
    if not os.path.exists(p):
        raise OSError("pivot_place: %s not found; build it with `make -C pivot-scheduling_amd` "
                      "(there is no CPU fallback)" % p)
    lib = ctypes.CDLL(p)
    c_int, c_void_p = ctypes.c_int, ctypes.c_void_p
    sig = {
        "pvt_abi_version": ([], c_int),
        "pvt_ctx_create": ([c_int, ctypes.POINTER(c_void_p)], c_int),
        "pvt_ctx_destroy": ([c_void_p], c_int),
        "pvt_ctx_set_stream": ([c_void_p, c_void_p], c_int),
        "pvt_place": ([c_void_p, c_void_p], c_int),
        "pvt_set_profiling": ([c_void_p, c_int], c_int),
        "pvt_set_profiling_kernel": ([c_void_p, ctypes.c_char_p], c_int),
        "pvt_reset_kstats": ([c_void_p], c_int),
        "pvt_get_kstats": ([c_void_p, c_int, ctypes.POINTER(_abi.pvt_kstats)], c_int),
        "pvt_get_kernel_kstats": ([c_void_p, ctypes.c_char_p, ctypes.POINTER(_abi.pvt_kstats)], c_int),
        "pvt_place_host": ([c_void_p, ctypes.POINTER(_abi.pvt_round), ctypes.POINTER(_abi.pvt_ca_items)], c_int),
        "pvt_place_host_batch": ([c_void_p, ctypes.POINTER(_abi.pvt_round),
                                  ctypes.POINTER(ctypes.POINTER(_abi.pvt_ca_items)), ctypes.c_int32,
                                  ctypes.POINTER(ctypes.c_int32)], c_int),
        "pvt_place_batch_mt": ([c_void_p, c_void_p, ctypes.c_int32, c_void_p], c_int),
        "pvt_restore_hosts": ([c_void_p, c_void_p, c_void_p, ctypes.c_int32, c_void_p, ctypes.c_int32], c_int),
        "pvt_set_window": ([c_void_p, c_int], c_int),
        "pvt_set_pipeline": ([c_void_p, c_int], c_int),
        "pvt_set_score_tw": ([c_void_p, c_int], c_int),
        "pvt_set_epochs": ([c_void_p, c_int], c_int),
        "pvt_set_zero_walk": ([c_void_p, c_int], c_int),
        "pvt_set_band": ([c_void_p, ctypes.c_int32], c_int),
        "pvt_zero_walk_stats": ([c_void_p] + [ctypes.POINTER(ctypes.c_int64)] * 3, c_int),
        "pvt_epoch_stats": ([c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                             ctypes.POINTER(ctypes.c_int64)], c_int),
        "pvt_last_stats": ([c_void_p, ctypes.POINTER(ctypes.c_int64),
                            ctypes.POINTER(ctypes.c_int64)], c_int),
        "pvt_last_error": ([c_void_p], ctypes.c_char_p),
        "pvt_shard_begin": ([c_void_p, c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                             ctypes.POINTER(ctypes.c_int64)], c_int),
        "pvt_shard_score": ([c_void_p, c_void_p, ctypes.POINTER(ctypes.c_int32),
                             ctypes.POINTER(ctypes.c_int64)], c_int),
        "pvt_shard_commit": ([c_void_p, c_void_p], c_int),
        "pvt_place_batch": ([c_void_p, c_void_p, ctypes.c_int32], c_int),
        "pvt_set_resident": ([c_void_p, ctypes.c_int32], c_int),
        "pvt_anchor": ([c_void_p, c_void_p], c_int),
        "pvt_meter": ([c_void_p, c_void_p], c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes, f.restype = args, res
    if lib.pvt_abi_version() != _abi.PVT_ABI_VERSION:
        raise OSError("pivot_place ABI mismatch: library %d, binding %d"
                      % (lib.pvt_abi_version(), _abi.PVT_ABI_VERSION))
    if path is None:
        _lib = lib
    return lib


def _torch():
    import torch
    return torch


_HB = []


def _hostbatch():
    """pivot_place._hostbatch, the C++ marshaller of place_host_batch (built next to
    libpivot_place.so by the Makefile), or None when it is absent or PVT_HOSTBATCH=0 -- then
    the ctypes marshalling builds the same descriptors for the same C call."""
    if not _HB:
        mod = None
        if os.environ.get("PVT_HOSTBATCH", "1") != "0":
            try:
                from . import _hostbatch as mod
            except ImportError:
                mod = None
        _HB.append(mod)
    return _HB[0]


class DeviceRound:
    """A round resident in HBM: torch tensors plus the pvt_round struct that points at them.

    ``reset()`` restores the pristine availability (one D2D copy), so the same round can be
    placed repeatedly (one bench step = reset + place)."""

    def __init__(self, r: RoundArrays, device):
        torch = _torch()
        self.arrays = r
        dev = torch.device(device)

        def up(a):
            return None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)

        self.avail0 = up(r.avail)
        self.avail = self.avail0.clone()
        self.zone, self.tiebreak, self.decay = up(r.zone), up(r.tiebreak), up(r.decay)
        self.cost, self.bw, self.dem = up(r.cost), up(r.bw), up(r.dem)
        self.task_group, self.group_anchor = up(r.task_group), up(r.group_anchor)
        self.rt_bw = up(r.rt_bw)
        T = r.n_tasks
        self.order = torch.empty(max(T, 1), dtype=torch.int32, device=dev)
        self.placement = torch.full((max(T, 1),), -1, dtype=torch.int32, device=dev)
        self.mt0 = None if r.mt_state is None else r.mt_state.copy()
        self.mt = None if r.mt_state is None else r.mt_state.copy()
        s = _abi.fill_struct(r)

        def dp(t):
            return None if t is None else t.data_ptr()

        s.avail, s.zone, s.tiebreak, s.decay = dp(self.avail), dp(self.zone), dp(self.tiebreak), dp(self.decay)
        s.cost, s.bw, s.dem = dp(self.cost), dp(self.bw), dp(self.dem)
        s.task_group, s.group_anchor = dp(self.task_group), dp(self.group_anchor)
        s.order, s.placement = dp(self.order), dp(self.placement)
        s.rt_bw = dp(self.rt_bw)
        s.mt_state = None if self.mt is None else self.mt.ctypes.data
        self.struct = s

    def reset(self):
        self.avail.copy_(self.avail0)
        if self.mt is not None:
            self.mt[:] = self.mt0

    def result(self) -> RoundResult:
        T = self.arrays.n_tasks
        return RoundResult(placement=self.placement[:T].cpu().numpy(),
                           order=self.order[:T].cpu().numpy(),
                           avail=self.avail.cpu().numpy(),
                           mt_state=None if self.mt is None else self.mt.copy())


class DeviceBatch:
    """Independent rounds resident in HBM for pvt_place_batch, packed field by field into flat
    device buffers (round i's arrays are slices at fixed offsets), so ``reset()`` restores every
    round's snapshot with one D2D copy; ``structs`` is the pvt_round[n] array the call takes."""

    _FIELDS = (("avail", np.float64), ("zone", np.int32), ("tiebreak", np.uint32),
               ("decay", np.int32), ("cost", np.float64), ("bw", np.float64),
               ("dem", np.float64), ("task_group", np.int32), ("group_anchor", np.int32),
               ("rt_bw", np.float64))

    def __init__(self, rounds, device):
        torch = _torch()
        dev = torch.device(device)
        self.arrays = list(rounds)
        n = len(self.arrays)
        self.structs = (_abi.pvt_round * max(n, 1))()
        self.bufs, offs = {}, {}
        self.mt, self._mt, self._mt0 = [], None, None
        self.mt_dev = self._mt_dev0 = None
        if n == 0:
            return
        for name, dt in self._FIELDS:
            parts = [getattr(r, name) for r in self.arrays]
            if all(p is None for p in parts):
                continue
            sizes = [0 if p is None else p.size for p in parts]
            offs[name] = np.concatenate([[0], np.cumsum(sizes)])
            flat = np.concatenate([np.ascontiguousarray(p, dtype=dt).ravel() for p in parts
                                   if p is not None]) if any(sizes) else np.zeros(1, dtype=dt)
            self.bufs[name] = torch.from_numpy(flat).to(dev)
        self.avail0 = self.bufs["avail"].clone()
        T = [r.n_tasks for r in self.arrays]
        toff = np.concatenate([[0], np.cumsum(T)])
        self.order = torch.empty(max(int(toff[-1]), 1), dtype=torch.int32, device=dev)
        self.placement = torch.empty(max(int(toff[-1]), 1), dtype=torch.int32, device=dev)
        self._toff = toff
        self._hoff = offs["avail"]
        # MT19937 states (opportunistic) packed in one host array: reset is one copy
        has_mt = [r.mt_state is not None for r in self.arrays]
        self._mt0 = np.stack([r.mt_state if r.mt_state is not None else np.zeros(625, np.uint32)
                              for r in self.arrays]).astype(np.uint32) if any(has_mt) else None
        self._mt = None if self._mt0 is None else self._mt0.copy()
        self.mt = [self._mt[i] if has_mt[i] else None for i in range(n)]
        # every round opportunistic: the states stay on the device (pvt_place_batch_mt), reset
        # by a D2D copy, read back by results() only
        self.mt_dev = self._mt_dev0 = None
        if all(has_mt):
            self._mt_dev0 = torch.from_numpy(self._mt0.view(np.int32).copy()).to(dev)
            self.mt_dev = self._mt_dev0.clone()
        for i, r in enumerate(self.arrays):
            st = _abi.fill_struct(r)
            for name, dt in self._FIELDS:
                if name in self.bufs and getattr(r, name) is not None:
                    buf = self.bufs[name]
                    setattr(st, name, buf.data_ptr() + int(offs[name][i]) * buf.element_size())
            st.order = self.order.data_ptr() + int(toff[i]) * 4
            st.placement = self.placement.data_ptr() + int(toff[i]) * 4
            st.mt_state = None if self.mt[i] is None else self.mt[i].ctypes.data
            self.structs[i] = st

    def __len__(self):
        return len(self.arrays)

    def reset(self):
        if not self.arrays:
            return
        self.bufs["avail"].copy_(self.avail0)
        if self.mt_dev is not None:
            self.mt_dev.copy_(self._mt_dev0)
        elif self._mt is not None:
            self._mt[:] = self._mt0

    def placement_of(self, i):
        return self.placement[int(self._toff[i]):int(self._toff[i + 1])]

    def results(self):
        if not self.arrays:
            return []
        pl = self.placement.cpu().numpy()
        od = self.order.cpu().numpy()
        av = self.bufs["avail"].cpu().numpy()
        if self.mt_dev is not None:
            self._mt[:] = self.mt_dev.cpu().numpy().view(np.uint32).reshape(self._mt.shape)
        out = []
        for i, r in enumerate(self.arrays):
            t0, t1 = int(self._toff[i]), int(self._toff[i + 1])
            h0, h1 = int(self._hoff[i]), int(self._hoff[i + 1])
            out.append(RoundResult(placement=pl[t0:t1].copy(), order=od[t0:t1].copy(),
                                   avail=av[h0:h1].reshape(4, -1).copy(),
                                   mt_state=None if self.mt[i] is None else self.mt[i].copy()))
        return out


_PTRS = {}


def _ptr(a):
    """Address of a contiguous numpy array's data (None for None). The cluster tables a policy
    passes every round (zone, cost, bw, tiebreak) are the same objects round after round, so
    their addresses are cached by identity (the cache keeps the array alive); a fresh array
    takes the ctypes buffer path (~0.5 us, against ~2 us for .ctypes.data)."""
    if a is None:
        return None
    e = _PTRS.get(id(a))
    if e is not None and e[0] is a:
        return e[1]
    try:
        p = ctypes.addressof(ctypes.c_char.from_buffer(a))
    except (TypeError, ValueError, BufferError):      # (read-only or empty buffers)
        p = a.__array_interface__["data"][0]
    if len(_PTRS) >= 64:                              # (per-round arrays pass through)
        _PTRS.clear()
    _PTRS[id(a)] = (a, p)
    return p


def _align(n, a=256):
    return (n + a - 1) // a * a


class _Stager:
    """Drop-in rounds (``PlacementEngine.place``): the round's arrays packed into ONE pinned
    host buffer, one asynchronous copy to a persistent device buffer, the round placed there, and
    its results (availability, placement, order -- the front of the buffer) back with one copy into
    pinned memory and one stream synchronisation. Replaces a dozen pageable tensor uploads and
    three synchronous downloads per round, which dominated config 1 / 2 sized rounds."""

    _IN = (("zone", np.int32), ("tiebreak", np.uint32), ("decay", np.int32), ("cost", np.float64),
           ("bw", np.float64), ("dem", np.float64), ("task_group", np.int32),
           ("group_anchor", np.int32), ("rt_bw", np.float64))

    def __init__(self, device):
        self.device = device
        self.cap = 0
        self.hbuf = self.dbuf = None

    def _ensure(self, n):
        if n <= self.cap:
            return
        torch = _torch()
        cap = max(1 << 16, 1 << (int(n) - 1).bit_length())
        self.hbuf = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
        self.dbuf = torch.empty(cap, dtype=torch.uint8, device=self.device)
        self.cap = cap

    def place(self, eng, r: RoundArrays) -> RoundResult:
        torch = _torch()
        H, T = r.n_hosts, r.n_tasks
        # front: avail (updated in place), placement, order -- the part copied back
        o_av = 0
        o_pl = _align(o_av + 32 * H)
        o_or = _align(o_pl + 4 * max(T, 1))
        o = _align(o_or + 4 * max(T, 1))
        n_out = o
        parts = [(o_av, np.ascontiguousarray(r.avail, dtype=np.float64))]
        offs = {}
        for name, dt in self._IN:
            a = getattr(r, name)
            if a is None:
                continue
            a = np.ascontiguousarray(a, dtype=dt)
            offs[name] = o
            parts.append((o, a))
            o = _align(o + a.nbytes)
        self._ensure(o)
        hv = self.hbuf.numpy()
        for off, a in parts:
            if a.nbytes:
                hv[off:off + a.nbytes] = a.reshape(-1).view(np.uint8)
        stream = torch.cuda.current_stream(eng.device)
        self.dbuf[:o].copy_(self.hbuf[:o], non_blocking=True)
        base = self.dbuf.data_ptr()
        st = _abi.fill_struct(r)
        st.avail = base + o_av
        for name, _ in self._IN:
            setattr(st, name, base + offs[name] if name in offs else None)
        st.placement, st.order = base + o_pl, base + o_or
        mt = None if r.mt_state is None else np.array(r.mt_state, dtype=np.uint32)
        st.mt_state = None if mt is None else mt.ctypes.data
        eng._set_stream(stream.cuda_stream)
        eng._check(eng.lib.pvt_place(eng.ctx, ctypes.addressof(st)))
        self.hbuf[:n_out].copy_(self.dbuf[:n_out], non_blocking=True)
        stream.synchronize()
        return RoundResult(
            placement=hv[o_pl:o_pl + 4 * T].view(np.int32).copy(),
            order=hv[o_or:o_or + 4 * T].view(np.int32).copy(),
            avail=hv[o_av:o_av + 32 * H].view(np.float64).reshape(4, H).copy(),
            mt_state=mt)


class PlacementEngine:
    """One pvt_ctx on one gfx950 device."""

    def __init__(self, device=0, window=0, lib_path=None):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError("pivot_place needs a ROCm GPU (gfx950); none is visible")
        self.lib = load_library(lib_path)
        self.device_index = int(device)
        self.device = torch.device("cuda", self.device_index)
        ctx = ctypes.c_void_p()
        rc = self.lib.pvt_ctx_create(self.device_index, ctypes.byref(ctx))
        if rc != _abi.PVT_OK:
            raise RuntimeError("pvt_ctx_create(%d) failed: %s" % (self.device_index,
                                                                  _abi.ERRORS.get(rc, rc)))
        self.ctx = ctx
        if window:
            self.lib.pvt_set_window(self.ctx, int(window))

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.pvt_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != _abi.PVT_OK:
            msg = self.lib.pvt_last_error(self.ctx)
            _abi.check_rc(rc, msg.decode() if msg else "")

    def _bind_stream(self):
        """Bind the context to torch's current stream on this device (the C call only when it
        changed: torch's raw-stream query and one cached pointer, a few microseconds less per
        resident call than a Stream object each time)."""
        torch = _torch()
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:
            idx = self.device.index if isinstance(self.device, torch.device) else torch.device(self.device).index
            ptr = raw(0 if idx is None else idx)
        else:
            ptr = torch.cuda.current_stream(self.device).cuda_stream
        if ptr != getattr(self, "_bound_stream", None):
            self._set_stream(ptr)

    def _set_stream(self, ptr):
        """pvt_ctx_set_stream, remembering the pointer for _bind_stream (every binding of this
        context goes through here)."""
        self._check(self.lib.pvt_ctx_set_stream(self.ctx, ctypes.c_void_p(ptr)))
        self._bound_stream = ptr

    def run(self, dr: DeviceRound):
        """Place a resident round (its avail / placement / order / mt are updated in place)."""
        self._bind_stream()
        self._check(self.lib.pvt_place(self.ctx, ctypes.addressof(dr.struct)))

    def restore(self, dr: DeviceRound):
        """dr.reset() after a placement of dr, restoring only the hosts its placement names (the
        only capacities a round changes; pvt_restore_hosts): one small launch on the current
        stream instead of a copy of the whole snapshot."""
        self._bind_stream()
        T = dr.arrays.n_tasks
        self._check(self.lib.pvt_restore_hosts(self.ctx, dr.avail.data_ptr(), dr.avail0.data_ptr(),
                                               dr.arrays.n_hosts, dr.placement.data_ptr(), T))
        if dr.mt is not None:
            dr.mt[:] = dr.mt0

    def place(self, r: RoundArrays) -> RoundResult:
        """Place a host-array round in one round trip (pvt_place_host: the context stages the
        inputs through one pinned buffer, one copy each way, one synchronisation). A round the
        resident kernel takes goes through the C++ marshaller as a one-round host batch (the
        same kernels, ~20 us less host time than the ctypes structs)."""
        one = self._one_round_cxx(r, None)
        if one is not None:
            (placement, order, avail, mt, _imt, _st), rc = one
            self._check(rc)
            return RoundResult(placement=placement, order=order, avail=avail, mt_state=mt)
        res, rc = self._place_host(r, None)
        self._check(rc)
        return res

    def _one_round_cxx(self, r, ca):
        """(result tuple, round rc) of r as a one-round pvt_place_host_batch through the C++
        marshaller, or None when it does not take the round (no marshaller, beyond the resident
        limits -- including a context whose resident kernel is off)."""
        hb = _hostbatch()
        if hb is None or r.n_tasks == 0 or not self.host_batch_fits(r, ca):
            return None
        fn = getattr(self, "_hb_fn", None)
        if fn is None:
            fn = self._hb_fn = ctypes.cast(self.lib.pvt_place_host_batch, ctypes.c_void_p).value
        rc, results, rcs = hb.place_host_batch(fn, self.ctx.value, [r], [ca])
        if rc == _abi.PVT_EUNSUPPORTED:
            return None
        self._check(rc)
        return results[0], rcs[0]

    def place_staged_torch(self, r: RoundArrays) -> RoundResult:
        """The previous drop-in path (kept for A/B timing): torch-pinned staging + pvt_place."""
        st = getattr(self, "_stager", None)
        if st is None:
            st = self._stager = _Stager(self.device)
        return st.place(self, r)

    @staticmethod
    def _host_struct(r: RoundArrays):
        """(pvt_round over r's host arrays, its RoundResult whose arrays the call fills)."""
        T = r.n_tasks
        s = _abi.fill_struct(r)
        avail = np.array(r.avail, dtype=np.float64, order="C")
        placement = np.empty(T, dtype=np.int32)
        order = np.empty(T, dtype=np.int32)
        mt = None if r.mt_state is None else np.array(r.mt_state, dtype=np.uint32)
        s.avail = _ptr(avail)
        s.zone, s.tiebreak, s.decay = _ptr(r.zone), _ptr(r.tiebreak), _ptr(r.decay)
        s.cost, s.bw, s.dem = _ptr(r.cost), _ptr(r.bw), _ptr(r.dem)
        s.task_group, s.group_anchor, s.rt_bw = _ptr(r.task_group), _ptr(r.group_anchor), _ptr(r.rt_bw)
        s.placement, s.order = _ptr(placement), _ptr(order)
        s.mt_state = _ptr(mt)
        return s, RoundResult(placement=placement, order=order, avail=avail, mt_state=mt)

    def _place_host(self, r: RoundArrays, items):
        s, res = self._host_struct(r)
        rc = self.lib.pvt_place_host(self.ctx, ctypes.byref(s),
                                     None if items is None else ctypes.byref(items))
        return res, rc

    @staticmethod
    def _ca_items(task_item, pred_off, pred_host, item_app, n_apps, storage_zone, zone_storage,
                  mt_state):
        """(pvt_ca_items, the arrays it points at -- kept alive by the caller -- , its MT19937
        state array, its status array)."""
        keep = (np.ascontiguousarray(task_item, dtype=np.int32),
                np.ascontiguousarray(pred_off, dtype=np.int64),
                np.ascontiguousarray(pred_host, dtype=np.int32),
                np.ascontiguousarray(item_app, dtype=np.int32),
                np.ascontiguousarray(storage_zone, dtype=np.int32),
                np.ascontiguousarray(zone_storage, dtype=np.int32))
        ti, off, ph, ia, sz, zs = keep
        mt = np.array(mt_state, dtype=np.uint32)
        status = np.zeros(2, dtype=np.int32)
        it = _abi.pvt_ca_items()
        it.n_items, it.n_apps, it.n_pred = ia.size, int(n_apps), ph.size
        it.task_item, it.pred_off, it.pred_host = _ptr(ti), _ptr(off), _ptr(ph)
        it.item_app = _ptr(ia)
        it.n_storage, it.reserved = sz.size, 0
        it.storage_zone, it.zone_storage = _ptr(sz), _ptr(zs)
        it.mt_state, it.status = _ptr(mt), _ptr(status)
        return it, keep, mt, status

    def _ca_result(self, res, rc, mt, status):
        if rc == _abi.PVT_EUNSUPPORTED:
            return None
        if rc != _abi.PVT_OK and status[1] in (_abi.GROUP_UNPLACED, _abi.GROUP_NO_STORAGE):
            # the reference: cluster.get_host(placement).locality / storage.locality on None
            raise AttributeError("'NoneType' object has no attribute 'locality'")
        self._check(rc)
        return res, int(status[0]), mt

    def place_cost_aware(self, r: RoundArrays, task_item, pred_off, pred_host, item_app, n_apps,
                         storage_zone, zone_storage, mt_state):
        """A cost_aware round whose grouping (scheduler/cost_aware.py:30-58: mode-host anchors,
        first-seen groups, one randomizer.choice(storage) per application group) runs on the
        device in the same round trip as the placement (pvt_place_host with pvt_ca_items).
        Returns (RoundResult, groups, the randomizer's MT19937 state after the draws), or None
        when the round is beyond the fused path's limits (use anchor() + place()). Raises
        AttributeError where the reference does (a mode placement that is no host; an anchor
        zone without storage)."""
        one = self._one_round_cxx(r, (task_item, pred_off, pred_host, item_app, n_apps,
                                      storage_zone, zone_storage, mt_state))
        if one is not None:
            (placement, order, avail, rmt, imt, status), rc = one
            res = RoundResult(placement=placement, order=order, avail=avail, mt_state=rmt)
            return self._ca_result(res, rc, imt, status)
        it, _keep, mt, status = self._ca_items(task_item, pred_off, pred_host, item_app, n_apps,
                                               storage_zone, zone_storage, mt_state)
        res, rc = self._place_host(r, it)
        return self._ca_result(res, rc, mt, status)

    def host_batch_fits(self, r: RoundArrays, ca_args=None):
        """Whether place_host_batch takes this round (resident limits; the fused grouping's)."""
        if r.n_tasks == 0:
            return True
        max_hosts = min(getattr(self, "_resident_max", _abi.PVT_RESIDENT_MAX_HOSTS),
                        _abi.PVT_RESIDENT_MAX_HOSTS)   # the C side's resident_fits limit
        ok = r.n_hosts <= max_hosts and r.n_tasks <= _abi.PVT_RESIDENT_MAX_TASKS
        if ca_args is not None:
            n_storage = len(ca_args[5])
            ok = ok and r.n_tasks <= _abi.GRP_MAX_TASKS and 1 <= n_storage and \
                n_storage + int(ca_args[4]) <= _abi.GRP_MAX_KEYS
        return ok

    def place_host_batch(self, reqs):
        """Independent drop-in rounds, possibly of different policies, in ONE round trip
        (pvt_place_host_batch). ``reqs``: (RoundArrays, ca_args) pairs, ca_args None or the
        arguments of place_cost_aware after the round. Returns, per request, what place() or
        place_cost_aware() would return -- or the exception that call would raise (instances
        of Exception, returned, not raised). Every round must satisfy host_batch_fits()."""
        n = len(reqs)
        if n == 0:
            return []
        hb = _hostbatch()
        if hb is not None:
            return self._place_host_batch_cxx(hb, reqs)
        structs = (_abi.pvt_round * n)()
        items = (ctypes.POINTER(_abi.pvt_ca_items) * n)()
        outs, keep = [], []
        for i, (r, ca) in enumerate(reqs):
            s, res = self._host_struct(r)
            structs[i] = s
            if ca is None:
                items[i] = ctypes.POINTER(_abi.pvt_ca_items)()
                outs.append((res, None))
            else:
                it, k, mt, status = self._ca_items(*ca)
                keep.append((it, k))
                items[i] = ctypes.pointer(it)
                outs.append((res, (mt, status)))
        rcs = (ctypes.c_int32 * n)()
        self._check(self.lib.pvt_place_host_batch(self.ctx, structs, items, n, rcs))
        out = []
        for i, (res, ca) in enumerate(outs):
            if ca is None:
                out.append(res)
                continue
            mt, status = ca
            try:
                out.append(self._ca_result(res, rcs[i], mt, status))
            except Exception as e:     # noqa: BLE001 -- handed to the caller of this round
                out.append(e)
        return out

    def _place_host_batch_cxx(self, hb, reqs):
        """place_host_batch with the descriptors built in C++ (csrc/pvt_hostpy.cpp): the same
        C call, ~4x less host time per round than the ctypes structs above."""
        fn = getattr(self, "_hb_fn", None)
        if fn is None:
            fn = self._hb_fn = ctypes.cast(self.lib.pvt_place_host_batch, ctypes.c_void_p).value
        rc, results, rcs = hb.place_host_batch(fn, self.ctx.value, [r for r, _ in reqs],
                                               [ca for _, ca in reqs])
        self._check(rc)
        out = []
        for (placement, order, avail, mt, imt, status), rci in zip(results, rcs):
            res = RoundResult(placement=placement, order=order, avail=avail, mt_state=mt)
            if status is None:
                out.append(res)
                continue
            try:
                out.append(self._ca_result(res, rci, imt, status))
            except Exception as e:     # noqa: BLE001 -- handed to the caller of this round
                out.append(e)
        return out

    # -- resident rounds and scenario batches (include/pivot_place.h, pvt_place_batch)
    def run_batch(self, batch: "DeviceBatch"):
        """Place every round of a resident batch in ONE launch (one workgroup per round)."""
        self._bind_stream()
        if batch.mt_dev is not None:
            self._check(self.lib.pvt_place_batch_mt(self.ctx, ctypes.addressof(batch.structs),
                                                    len(batch), ctypes.c_void_p(batch.mt_dev.data_ptr())))
        else:
            self._check(self.lib.pvt_place_batch(self.ctx, ctypes.addressof(batch.structs), len(batch)))

    def place_batch(self, rounds) -> list:
        """Place independent rounds of one policy (each <= PVT_RESIDENT_MAX_HOSTS hosts and
        PVT_RESIDENT_MAX_TASKS tasks) together; returns one RoundResult per round."""
        b = DeviceBatch(rounds, self.device)
        self.run_batch(b)
        return b.results()

    def set_resident(self, max_hosts=_abi.PVT_RESIDENT_MAX_HOSTS):
        """pvt_place runs rounds up to ``max_hosts`` hosts on the resident kernel (0: never)."""
        self._check(self.lib.pvt_set_resident(self.ctx, int(max_hosts)))
        self._resident_max = int(max_hosts)   # host_batch_fits mirrors the context's limit

    # -- anchor resolution (include/pivot_place.h, pvt_anchor; reference cost_aware.py:45-58)
    def anchor_device(self, off, lst, zone, mode_host, anchor_zone, inst_host=None, item=None):
        """Mode-host anchors of the items off[c]..off[c+1] of ``lst`` (device int64 / int32
        tensors); writes ``mode_host`` and ``anchor_zone`` (device int32 tensors, one per item).
        ``inst_host``: optional device int32 table that ``lst`` indexes. ``item``: optional
        device int32 row numbers (item c uses row item[c] of ``off``)."""
        torch = _torch()
        stream = torch.cuda.current_stream(self.device)
        self._set_stream(stream.cuda_stream)
        a = _abi.pvt_anchor_args()
        a.n_items = off.numel() - 1 if item is None else item.numel()
        a.n_rows = 0 if item is None else off.numel() - 1
        a.item = None if item is None else item.data_ptr()
        a.n_hosts = zone.numel()
        a.n_pred = lst.numel()
        a.n_inst = 0 if inst_host is None else inst_host.numel()
        a.off, a.list, a.zone = off.data_ptr(), lst.data_ptr(), zone.data_ptr()
        a.inst_host = None if inst_host is None else inst_host.data_ptr()
        a.mode_host, a.anchor_zone = mode_host.data_ptr(), anchor_zone.data_ptr()
        self._check(self.lib.pvt_anchor(self.ctx, ctypes.addressof(a)))

    def anchor(self, off, lst, zone, inst_host=None):
        """Host-array form of anchor_device: returns (mode_host, anchor_zone) numpy arrays. The
        inputs go up in one pinned copy and the outputs (at the buffer's front) come back in one
        (see _Stager)."""
        torch = _torch()
        off = np.ascontiguousarray(off, dtype=np.int64)
        C = off.size - 1
        arrs = [("lst", np.ascontiguousarray(lst, dtype=np.int32)),
                ("zone", np.ascontiguousarray(zone, dtype=np.int32))]
        if inst_host is not None:
            arrs.append(("ih", np.ascontiguousarray(inst_host, dtype=np.int32)))
        o_mode, o_az = 0, _align(4 * max(C, 1))
        o = _align(o_az + 4 * max(C, 1))
        n_out = o
        offs = {"off": o}
        o = _align(o + off.nbytes)
        for name, a in arrs:
            offs[name] = o
            o = _align(o + a.nbytes)
        st = getattr(self, "_stager", None)
        if st is None:
            st = self._stager = _Stager(self.device)
        st._ensure(o)
        hv = st.hbuf.numpy()
        for name, a in [("off", off)] + arrs:
            if a.nbytes:
                hv[offs[name]:offs[name] + a.nbytes] = a.reshape(-1).view(np.uint8)
        st.dbuf[:o].copy_(st.hbuf[:o], non_blocking=True)
        d = st.dbuf

        def view(name, n, dt):
            return d[offs[name]:offs[name] + n * 4 * (2 if dt == torch.int64 else 1)].view(dt)

        off_d = view("off", off.size, torch.int64)
        lst_d = view("lst", arrs[0][1].size, torch.int32)
        zone_d = view("zone", arrs[1][1].size, torch.int32)
        ih = view("ih", arrs[2][1].size, torch.int32) if inst_host is not None else None
        mode = d[o_mode:o_mode + 4 * max(C, 0)].view(torch.int32)
        az = d[o_az:o_az + 4 * max(C, 0)].view(torch.int32)
        self.anchor_device(off_d, lst_d, zone_d, mode, az, ih)
        st.hbuf[:n_out].copy_(d[:n_out], non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return (hv[o_mode:o_mode + 4 * C].view(np.int32).copy(),
                hv[o_az:o_az + 4 * C].view(np.int32).copy())

    # -- meter aggregates (include/pivot_place.h, pvt_meter; reference resources/meter.py:31-53)
    def meter(self, log):
        """Aggregates of every scenario of a ``pivot_place.meter.MeterLog`` in one launch:
        dict of [S] float64 numpy arrays instance_hours / egress_cost / congestion_delay."""
        torch = _torch()
        dev = self.device
        keep = {name: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                for name, a in log.arrays()}
        S = log.n_scen
        out = {k: torch.empty(max(S, 1), dtype=torch.float64, device=dev)
               for k in ("instance_hours", "egress_cost", "congestion_delay")}
        m = log.fill(lambda a: None, [o.data_ptr() for o in out.values()])
        for name, t in keep.items():
            setattr(m, name, t.data_ptr() if t.numel() else None)
        stream = torch.cuda.current_stream(dev)
        self._set_stream(stream.cuda_stream)
        self._check(self.lib.pvt_meter(self.ctx, ctypes.addressof(m)))
        return {k: v[:S].cpu().numpy() for k, v in out.items()}

    # -- host-dimension sharding (include/pivot_place.h, pvt_shard_*); see pivot_place.sharded
    def shard_begin(self, dr: DeviceRound, host_lo, host_hi, world):
        """Start a sharded round on ``dr`` (full replicated availability); returns the largest
        per-rank package in bytes."""
        torch = _torch()
        stream = torch.cuda.current_stream(self.device)
        self._set_stream(stream.cuda_stream)
        mx = ctypes.c_int64()
        self._check(self.lib.pvt_shard_begin(self.ctx, ctypes.addressof(dr.struct), int(host_lo),
                                             int(host_hi), int(world), ctypes.byref(mx)))
        return mx.value

    def shard_score(self, package):
        """Score the next window over this rank's hosts into ``package`` (a device uint8
        tensor). Returns (tasks in the window, package bytes); (0, 0) when the round is done."""
        nt, nb = ctypes.c_int32(), ctypes.c_int64()
        self._check(self.lib.pvt_shard_score(self.ctx, ctypes.c_void_p(package.data_ptr()),
                                             ctypes.byref(nt), ctypes.byref(nb)))
        return nt.value, nb.value

    def shard_commit(self, packages):
        """Merge every rank's package (rank order, contiguous) and launch the commit walk.
        Returns False when the package was scored past a walk that stopped early (PVT_ESTALE:
        every rank gets it together; score again), True otherwise."""
        rc = self.lib.pvt_shard_commit(self.ctx, ctypes.c_void_p(packages.data_ptr()))
        if rc == _abi.PVT_ESTALE:
            return False
        self._check(rc)
        return True

    def set_window(self, tasks):
        self._check(self.lib.pvt_set_window(self.ctx, int(tasks)))

    def set_score_tw(self, tw=0):
        """Score-kernel tasks per wave: 0 = the policy default, 2 or 4 (identical results)."""
        self._check(self.lib.pvt_set_score_tw(self.ctx, int(tw)))

    def set_pipeline(self, on=True):
        self._check(self.lib.pvt_set_pipeline(self.ctx, int(bool(on))))

    def set_epochs(self, on=True):
        """cost_aware best-fit: group-parallel speculative epochs (default on; identical results)."""
        self._check(self.lib.pvt_set_epochs(self.ctx, int(bool(on))))

    def set_band(self, min_hosts=65536):
        """vbp best-fit: band lists over hosts sorted by snapshot memory from ``min_hosts`` hosts
        on (0: the streaming score pass always; identical results)."""
        self._check(self.lib.pvt_set_band(self.ctx, int(min_hosts)))

    def set_zero_walk(self, on=True):
        """Epoch chains: the zero-cost frontier walk where it proves its winners (default on;
        identical results)."""
        self._check(self.lib.pvt_set_zero_walk(self.ctx, int(bool(on))))

    def epoch_stats(self):
        e, s, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.pvt_epoch_stats(self.ctx, ctypes.byref(e), ctypes.byref(s), ctypes.byref(r)))
        zf, zl, zc = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.pvt_zero_walk_stats(self.ctx, ctypes.byref(zf), ctypes.byref(zl),
                                                 ctypes.byref(zc)))
        return {"epochs": e.value, "segments": s.value, "rejected": r.value,
                "frontier_chains": zf.value, "list_chains": zl.value, "longest_chain_tasks": zc.value}

    def set_profiling(self, on=True, kernel=None):
        """True / 1: HIP events around every launch; 2: around the named kernels only -- or, with
        ``kernel``, around that one named kernel only."""
        self._check(self.lib.pvt_set_profiling_kernel(self.ctx, kernel.encode() if kernel else None))
        self._check(self.lib.pvt_set_profiling(self.ctx, 2 if on == 2 else int(bool(on))))

    def reset_kstats(self):
        self._check(self.lib.pvt_reset_kstats(self.ctx))

    def kstats(self, kclass):
        k = _abi.pvt_kstats()
        self._check(self.lib.pvt_get_kstats(self.ctx, int(kclass), ctypes.byref(k)))
        return {"launches": k.launches, "ms": k.ms, "candidates": k.candidates, "bytes": k.bytes}

    def kernel_kstats(self, name):
        """HIP-event timing of one named kernel's launches while profiling was on."""
        k = _abi.pvt_kstats()
        self._check(self.lib.pvt_get_kernel_kstats(self.ctx, name.encode(), ctypes.byref(k)))
        return {"launches": k.launches, "ms": k.ms, "candidates": k.candidates, "bytes": k.bytes}

    def last_stats(self):
        w, r = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.pvt_last_stats(self.ctx, ctypes.byref(w), ctypes.byref(r)))
        return {"windows": w.value, "refills": r.value}


_engines = {}


def default_engine(device=0) -> PlacementEngine:
    """Process-wide engine per device (what the drop-in policies use)."""
    eng = _engines.get(device)
    if eng is None:
        eng = PlacementEngine(device)
        _engines[device] = eng
    return eng
