"""Lock-step batched-scenario driver (BASELINE config 4).

The reference runs one simulation per ``ExperimentRun`` process (alibaba/runner.py:27-44) and
its round loop calls the policy's ``schedule()`` once per ``interval`` tick
(scheduler/__init__.py:87-116): independent scenarios are independent processes, each paying
one engine call per round. Here S simulations run side by side in one process, each in its own
thread, and every engine call a drop-in policy makes -- ``place`` (the round) and ``anchor``
(cost_aware's mode-host anchors) -- goes through a per-simulation proxy that blocks. Whenever
EVERY live simulation is blocked on the engine, the driver serves all waiting calls at once:

* ``place`` / ``place_cost_aware``: every waiting round -- whatever the simulations' policies,
  cost_aware rounds with their grouping fused -- goes to ONE ``pvt_place_host_batch`` (one
  staging copy each way, one resident launch with a workgroup per round) when it fits the
  resident limits; larger rounds go to ``pvt_place_host`` alone. (An engine without the host
  batch -- the CPU restatement in tests -- gets one ``place_batch`` per policy mode.)
* ``anchor``: all items of all simulations in ONE ``pvt_anchor`` call (each simulation's host
  indices offset into one concatenated zone table).

Scenarios share nothing, so serving calls from different simulated times together is exact;
since every simulation's round loop ticks at multiples of ``interval`` from t = 0, the
simulations advance in lock-step and a batch holds one tick of every live scenario. The GPU is
only ever called from the driver's thread (the engine context is not thread-safe).

    driver = LockstepDriver(engine)
    results = driver.run([lambda eng: simulate(..., engine=eng) for ...])
"""
import threading
import time

import numpy as np

from . import _abi


class _Call:
    __slots__ = ("sim", "kind", "args", "result", "error", "done")

    def __init__(self, sim, kind, args):
        self.sim, self.kind, self.args = sim, kind, args
        self.result = self.error = None
        self.done = False


class SimEngine:
    """The engine one simulation's policy sees: ``place`` and ``anchor`` block until the
    driver has served them in a batch."""

    def __init__(self, driver, sim):
        self._driver, self._sim = driver, sim

    def place(self, r):
        return self._driver._call(self._sim, "place", (r,))

    def anchor(self, off, lst, zone, inst_host=None):
        return self._driver._call(self._sim, "anchor", (off, lst, zone, inst_host))

    def place_cost_aware(self, r, *ca_args):
        """The fused cost_aware round (PlacementEngine.place_cost_aware): None when the engine
        has no fused path or the round is beyond it (the policy then uses anchor + place)."""
        return self._driver._call(self._sim, "place_ca", (r,) + tuple(ca_args))


class LockstepDriver:
    """Runs simulations side by side and batches their engine calls (module docstring).
    ``engine``: a PlacementEngine, or any object with ``place``, ``place_batch`` and ``anchor``
    of the same meaning (tests use the CPU restatement)."""

    def __init__(self, engine, max_batch=4096):
        self.engine = engine
        self.max_batch = max_batch
        self._cv = threading.Condition()
        self._pending = []
        self._live = 0
        self.stats = {"batches": 0, "place_calls": 0, "place_launches": 0, "anchor_calls": 0,
                      "anchor_launches": 0, "max_rounds_per_launch": 0, "serve_s": 0.0,
                      "host_batch_rounds": 0, "fused_rounds": 0}

    # -------------------------------------------------------------- simulation side
    def _call(self, sim, kind, args):
        c = _Call(sim, kind, args)
        with self._cv:
            self._pending.append(c)
            self._cv.notify_all()
            while not c.done:
                self._cv.wait()
        if c.error is not None:
            raise c.error
        return c.result

    # -------------------------------------------------------------- driver side
    def run(self, sims):
        """``sims``: callables ``f(engine) -> result``, each running one simulation to the end
        with ``engine`` behind its policy. Returns their results in order (re-raises the first
        simulation error after every simulation has stopped)."""
        n = len(sims)
        results, errors = [None] * n, [None] * n

        def body(i):
            try:
                results[i] = sims[i](SimEngine(self, i))
            except BaseException as e:   # noqa: BLE001 -- re-raised in the driver thread
                errors[i] = e
            finally:
                with self._cv:
                    self._live -= 1
                    self._cv.notify_all()

        threads = [threading.Thread(target=body, args=(i,), daemon=True) for i in range(n)]
        with self._cv:
            self._live = n
        for t in threads:
            t.start()
        with self._cv:
            while True:
                while self._live > 0 and len(self._pending) < self._live:
                    self._cv.wait()
                if self._live == 0 and not self._pending:
                    break
                batch, self._pending = self._pending, []
                self._serve(batch)
                self._cv.notify_all()
        for t in threads:
            t.join()
        for e in errors:
            if e is not None:
                raise e
        return results

    def _serve(self, batch):
        t = time.perf_counter()
        self.stats["batches"] += 1
        anchors = [c for c in batch if c.kind == "anchor"]
        places = [c for c in batch if c.kind in ("place", "place_ca")]
        if anchors:
            self._serve_anchors(anchors)
        if places:
            self._serve_places(places)
        self.stats["serve_s"] += time.perf_counter() - t

    def _serve_anchors(self, calls):
        """One pvt_anchor over every simulation's items: lists are offset into one host space
        (entries -1, a predecessor task without placement, stay -1)."""
        self.stats["anchor_calls"] += len(calls)
        offs, lsts, zones, spans = [np.zeros(1, dtype=np.int64)], [], [], []
        base_item = base_entry = base_host = 0
        for c in calls:
            off, lst, zone, inst_host = c.args
            if inst_host is not None:          # per-instance tables are not concatenated
                try:
                    c.result = self.engine.anchor(off, lst, zone, inst_host)
                except Exception as e:         # noqa: BLE001
                    c.error = e
                c.done = True
                self.stats["anchor_launches"] += 1
                continue
            off = np.asarray(off, dtype=np.int64)
            lst = np.asarray(lst, dtype=np.int32)
            zone = np.asarray(zone, dtype=np.int32)
            n_items = len(off) - 1
            offs.append(off[1:] + base_entry)
            lsts.append(np.where(lst >= 0, lst + base_host, lst).astype(np.int32))
            zones.append(zone)
            spans.append((c, base_item, n_items, base_host))
            base_item += n_items
            base_entry += int(off[-1])
            base_host += len(zone)
        if not spans:
            return
        try:
            mode, az = self.engine.anchor(np.concatenate(offs), np.concatenate(lsts),
                                          np.concatenate(zones))
            self.stats["anchor_launches"] += 1
            mode, az = np.asarray(mode), np.asarray(az)
            for c, b, n, hb in spans:
                m = mode[b:b + n].astype(np.int32)
                c.result = (np.where(m >= 0, m - hb, m).astype(np.int32), az[b:b + n].copy())
                c.done = True
        except Exception as e:                 # noqa: BLE001 -- every caller sees the error
            for c, _, _, _ in spans:
                c.error, c.done = e, True

    def _note_launch(self, rounds):
        self.stats["place_launches"] += 1
        self.stats["max_rounds_per_launch"] = max(self.stats["max_rounds_per_launch"], rounds)

    def _serve_places(self, calls):
        """Every waiting round in ONE pvt_place_host_batch when the engine has it (whatever the
        policies; cost_aware rounds with their fused grouping), the rest as before: rounds of
        one policy mode per pvt_place_batch, larger rounds one by one."""
        self.stats["place_calls"] += len(calls)
        eng = self.engine
        batched, rest = [], []
        for c in calls:
            ca = c.args[1:] if c.kind == "place_ca" else None
            if hasattr(eng, "place_host_batch") and eng.host_batch_fits(c.args[0], ca):
                batched.append(c)
            else:
                rest.append(c)
        for k in range(0, len(batched), self.max_batch):
            part = batched[k:k + self.max_batch]
            try:
                res = eng.place_host_batch([(c.args[0], c.args[1:] if c.kind == "place_ca" else None)
                                            for c in part])
                for c, x in zip(part, res):
                    if isinstance(x, Exception):
                        c.error = x
                    else:
                        c.result = x
            except Exception as e:             # noqa: BLE001 -- every caller sees the error
                for c in part:
                    c.error = e
            for c in part:
                c.done = True
            self._note_launch(len(part))
            self.stats["host_batch_rounds"] += len(part)
            self.stats["fused_rounds"] += sum(c.kind == "place_ca" for c in part)
        by_mode = {}
        for c in rest:
            r = c.args[0]
            if c.kind == "place_ca":           # beyond the batch: the fused call alone, if any
                if hasattr(eng, "place_cost_aware"):
                    try:
                        c.result = eng.place_cost_aware(*c.args)
                    except Exception as e:     # noqa: BLE001
                        c.error = e
                    self.stats["place_launches"] += 1
                c.done = True
                continue
            fits = (r.n_tasks > 0 and r.n_hosts <= _abi.PVT_RESIDENT_MAX_HOSTS
                    and r.n_tasks <= _abi.PVT_RESIDENT_MAX_TASKS)
            if fits:
                by_mode.setdefault(r.mode, []).append(c)
            else:
                try:
                    c.result = self.engine.place(r)
                except Exception as e:         # noqa: BLE001
                    c.error = e
                c.done = True
                self.stats["place_launches"] += 1
        for mode, cs in by_mode.items():
            for k in range(0, len(cs), self.max_batch):
                part = cs[k:k + self.max_batch]
                try:
                    res = self.engine.place_batch([c.args[0] for c in part])
                    for c, x in zip(part, res):
                        c.result = x
                except Exception as e:         # noqa: BLE001
                    for c in part:
                        c.error = e
                for c in part:
                    c.done = True
                self._note_launch(len(part))
