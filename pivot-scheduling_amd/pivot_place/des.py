"""SimPy-3 semantics discrete-event core.

The reference simulator runs on SimPy 3.0.11 (reference requirements.txt:2), which is absent
from this image and cannot be installed offline. This module restates the
published SimPy 3.0.11 algorithm so that the reference's round loop
(scheduler/__init__.py:87-147,185-194), host resources (resources/__init__.py:119-135,244-314,
370-461) and network routes (resources/network.py:43-100) run unchanged on top of it:

    from pivot_place import des
    des.install()           # registers this module as ``simpy`` when SimPy is not importable

What is restated (the subset of the SimPy 3.0.11 API the reference uses, plus conditions and
interrupts so generic SimPy processes behave):

* ``Environment``: a heap of ``(time, priority, eid, event)``; ``eid`` is a global insertion
  counter, so events due at the same time and priority run first-in first-out; ``URGENT`` (0)
  events (process start, interrupts, ``run(until=t)``'s stop event) precede ``NORMAL`` (1)
  ones due at the same time. ``step()`` pops one event and runs its callbacks in order;
  a failed event nobody waited on (not defused) re-raises its exception. ``run(until)`` stops
  at the URGENT stop event scheduled at ``until``, or when the queue is empty.
* ``Event``: PENDING → triggered (``succeed``/``fail``/``trigger`` schedule it now) →
  processed (its callbacks ran; ``callbacks`` is then None).
* ``Timeout``: triggered at creation, scheduled ``delay`` later (NORMAL).
* ``Process``: an event wrapping a generator. It starts through an URGENT ``Initialize``
  event; ``_resume`` sends each yielded event's value back into the generator (or throws its
  exception, defusing it), continuing synchronously while the yielded event is already
  processed, and otherwise registers itself as a callback of that event. The generator's
  return value is the process event's value.
* Resources (``Store``, ``Container``, ``Resource``): put/get queues of request events. A new
  put (get) request is appended to its queue and immediately tries ``_trigger_put``
  (``_trigger_get``); when a put (get) event is *processed*, it tries the opposite queue. A
  trigger pass walks its queue from the head, calling ``_do_put``/``_do_get`` per request,
  removing triggered requests, and stops after a request whose ``_do_*`` returned a false
  value. ``Container._do_*`` return True when they succeed (so one trigger can serve several
  requests); ``Store`` and ``Resource`` return None (one request per pass). A ``Resource``
  request is granted when a user slot is free; a release frees the slot at once and the next
  request is granted when the release event is processed.

Everything is single-threaded and deterministic; no wall-clock time is involved.
"""
import heapq
import itertools
import sys

__all__ = ["Environment", "Event", "Timeout", "Process", "Initialize", "Interruption",
           "Interrupt", "Condition", "AllOf", "AnyOf", "ConditionValue", "Store", "FilterStore",
           "Container", "Resource", "PENDING", "URGENT", "NORMAL", "Infinity", "install"]

Infinity = float("inf")
PENDING = object()
URGENT = 0
NORMAL = 1


class EmptySchedule(Exception):
    """No events left to process."""


class StopSimulation(Exception):
    """Ends ``Environment.run``; carries the ``until`` event's value."""

    @classmethod
    def callback(cls, event):
        if event._ok:
            raise cls(event._value)
        raise event._value


class Interrupt(Exception):
    """Thrown into a process by ``Process.interrupt(cause)``."""

    @property
    def cause(self):
        return self.args[0]


# ---------------------------------------------------------------------------------------
# Events
# ---------------------------------------------------------------------------------------
class Event:
    def __init__(self, env):
        self.env = env
        self.callbacks = []
        self._value = PENDING

    def __repr__(self):
        return "<%s() object at 0x%x>" % (type(self).__name__, id(self))

    @property
    def triggered(self):
        return self._value is not PENDING

    @property
    def processed(self):
        return self.callbacks is None

    @property
    def ok(self):
        return self._ok

    @property
    def defused(self):
        return hasattr(self, "_defused")

    @defused.setter
    def defused(self, value):
        self._defused = True

    @property
    def value(self):
        if self._value is PENDING:
            raise AttributeError("Value of %s is not yet available" % self)
        return self._value

    def trigger(self, event):
        """Take ``event``'s outcome and schedule this event (usable as a callback)."""
        self._ok = event._ok
        self._value = event._value
        self.env.schedule(self)

    def succeed(self, value=None):
        if self._value is not PENDING:
            raise RuntimeError("%s has already been triggered" % self)
        self._ok = True
        self._value = value
        self.env.schedule(self)
        return self

    def fail(self, exception):
        if self._value is not PENDING:
            raise RuntimeError("%s has already been triggered" % self)
        if not isinstance(exception, BaseException):
            raise ValueError("%s is not an exception." % exception)
        self._ok = False
        self._value = exception
        self.env.schedule(self)
        return self

    def __and__(self, other):
        return Condition(self.env, Condition.all_events, [self, other])

    def __or__(self, other):
        return Condition(self.env, Condition.any_events, [self, other])


class Timeout(Event):
    def __init__(self, env, delay, value=None):
        if delay < 0:
            raise ValueError("Negative delay %s" % delay)
        self.env = env
        self.callbacks = []
        self._value = value
        self._delay = delay
        self._ok = True
        env.schedule(self, NORMAL, delay)


class Initialize(Event):
    """Starts a process: URGENT, so it runs before NORMAL events due at the same time."""

    def __init__(self, env, process):
        self.env = env
        self.callbacks = [process._resume]
        self._value = None
        self._ok = True
        env.schedule(self, URGENT)


class Interruption(Event):
    def __init__(self, process, cause):
        self.env = process.env
        self.callbacks = [self._interrupt]
        self._value = Interrupt(cause)
        self._ok = False
        self._defused = True
        if process._value is not PENDING:
            raise RuntimeError("%s has terminated and cannot be interrupted." % process)
        if process is self.env.active_process:
            raise RuntimeError("A process is not allowed to interrupt itself.")
        self.process = process
        self.env.schedule(self, URGENT)

    def _interrupt(self, event):
        if self.process._value is not PENDING:
            return
        self.process._target.callbacks.remove(self.process._resume)
        self.process._resume(self)


class Process(Event):
    def __init__(self, env, generator):
        if not hasattr(generator, "throw"):
            raise ValueError("%s is not a generator." % generator)
        self.env = env
        self.callbacks = []
        self._value = PENDING
        self._generator = generator
        self._target = Initialize(env, self)

    @property
    def target(self):
        return self._target

    @property
    def is_alive(self):
        return self._value is PENDING

    def interrupt(self, cause=None):
        Interruption(self, cause)

    def _resume(self, event):
        env = self.env
        env._active_proc = self
        while True:
            try:
                if event._ok:
                    event = self._generator.send(event._value)
                else:
                    event._defused = True
                    exc = type(event._value)(*event._value.args)
                    exc.__cause__ = event._value
                    event = self._generator.throw(exc)
            except StopIteration as e:
                event = None
                self._ok = True
                self._value = e.args[0] if len(e.args) else None
                env.schedule(self)
                break
            except BaseException as e:
                event = None
                self._ok = False
                self._value = e
                env.schedule(self)
                break
            try:
                if event.callbacks is not None:
                    event.callbacks.append(self._resume)
                    break
            except AttributeError:
                if not hasattr(event, "callbacks"):
                    msg = "Invalid yield value \"%s\"" % (event,)
                    err = RuntimeError(msg)
                    event = None
                    self._ok = False
                    self._value = err
                    env.schedule(self)
                    break
                raise
        self._target = event
        env._active_proc = None


class ConditionValue:
    """Values of the events a condition saw processed, in the condition's event order."""

    def __init__(self):
        self.events = []

    def __getitem__(self, key):
        if key not in self.events:
            raise KeyError(str(key))
        return key._value

    def __contains__(self, key):
        return key in self.events

    def __eq__(self, other):
        if type(other) is ConditionValue:
            return self.events == other.events
        return self.todict() == other

    def keys(self):
        return (e for e in self.events)

    def values(self):
        return (e._value for e in self.events)

    def items(self):
        return ((e, e._value) for e in self.events)

    def todict(self):
        return dict(self.items())


class Condition(Event):
    def __init__(self, env, evaluate, events):
        super().__init__(env)
        self._evaluate = evaluate
        self._events = tuple(events)
        self._count = 0
        if not self._events:
            self.succeed(ConditionValue())
            return
        for e in self._events:
            if self.env != e.env:
                raise ValueError("It is not allowed to mix events from different environments")
        for e in self._events:
            if e.callbacks is None:
                self._check(e)
            else:
                e.callbacks.append(self._check)
        self.callbacks.append(self._build_value)

    def _populate_value(self, value):
        for e in self._events:
            if isinstance(e, Condition):
                e._populate_value(value)
            elif e.callbacks is None:
                value.events.append(e)

    def _build_value(self, event):
        self._remove_check_callbacks()
        if event._ok:
            self._value = ConditionValue()
            self._populate_value(self._value)

    def _remove_check_callbacks(self):
        for e in self._events:
            if e.callbacks and self._check in e.callbacks:
                e.callbacks.remove(self._check)
            if isinstance(e, Condition):
                e._remove_check_callbacks()

    def _check(self, event):
        if self._value is not PENDING:
            return
        self._count += 1
        if not event._ok:
            event._defused = True
            self.fail(event._value)
        elif self._evaluate(self._events, self._count):
            self.succeed()

    @staticmethod
    def all_events(events, count):
        return len(events) == count

    @staticmethod
    def any_events(events, count):
        return count > 0 or len(events) == 0


class AllOf(Condition):
    def __init__(self, env, events):
        super().__init__(env, Condition.all_events, events)


class AnyOf(Condition):
    def __init__(self, env, events):
        super().__init__(env, Condition.any_events, events)


# ---------------------------------------------------------------------------------------
# Environment
# ---------------------------------------------------------------------------------------
class Environment:
    def __init__(self, initial_time=0):
        self._now = initial_time
        self._queue = []
        self._eid = itertools.count()
        self._active_proc = None

    @property
    def now(self):
        return self._now

    @property
    def active_process(self):
        return self._active_proc

    def process(self, generator):
        return Process(self, generator)

    def timeout(self, delay, value=None):
        return Timeout(self, delay, value)

    def event(self):
        return Event(self)

    def all_of(self, events):
        return AllOf(self, events)

    def any_of(self, events):
        return AnyOf(self, events)

    def schedule(self, event, priority=NORMAL, delay=0):
        heapq.heappush(self._queue, (self._now + delay, priority, next(self._eid), event))

    def peek(self):
        try:
            return self._queue[0][0]
        except IndexError:
            return Infinity

    def step(self):
        try:
            self._now, _, _, event = heapq.heappop(self._queue)
        except IndexError:
            raise EmptySchedule()
        callbacks, event.callbacks = event.callbacks, None
        for callback in callbacks:
            callback(event)
        if not event._ok and not hasattr(event, "_defused"):
            exc = type(event._value)(*event._value.args)
            exc.__cause__ = event._value
            raise exc

    def run(self, until=None):
        if until is not None:
            if not isinstance(until, Event):
                at = float(until)
                if at <= self.now:
                    raise ValueError("until(=%s) should be > the current simulation time." % at)
                until = Event(self)
                until._ok = True
                until._value = None
                self.schedule(until, URGENT, at - self.now)
            elif until.callbacks is None:
                return until.value
            until.callbacks.append(StopSimulation.callback)
        try:
            while True:
                self.step()
        except StopSimulation as exc:
            return exc.args[0]
        except EmptySchedule:
            pass


# ---------------------------------------------------------------------------------------
# Resources
# ---------------------------------------------------------------------------------------
class _Put(Event):
    def __init__(self, resource):
        super().__init__(resource._env)
        self.resource = resource
        self.proc = self.env.active_process
        resource.put_queue.append(self)
        self.callbacks.append(resource._trigger_get)
        resource._trigger_put(None)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc_value, traceback):
        self.cancel()

    def cancel(self):
        if not self.triggered:
            self.resource.put_queue.remove(self)


class _Get(Event):
    def __init__(self, resource):
        super().__init__(resource._env)
        self.resource = resource
        self.proc = self.env.active_process
        resource.get_queue.append(self)
        self.callbacks.append(resource._trigger_put)
        resource._trigger_get(None)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc_value, traceback):
        self.cancel()

    def cancel(self):
        if not self.triggered:
            self.resource.get_queue.remove(self)


class _BaseResource:
    def __init__(self, env, capacity):
        self._env = env
        self._capacity = capacity
        self.put_queue = []
        self.get_queue = []

    @property
    def capacity(self):
        return self._capacity

    def _trigger_put(self, get_event):
        q, idx = self.put_queue, 0
        while idx < len(q):
            ev = q[idx]
            proceed = self._do_put(ev)
            if not ev.triggered:
                idx += 1
            elif q.pop(idx) is not ev:
                raise RuntimeError("Put queue invariant violated")
            if not proceed:
                break

    def _trigger_get(self, put_event):
        q, idx = self.get_queue, 0
        while idx < len(q):
            ev = q[idx]
            proceed = self._do_get(ev)
            if not ev.triggered:
                idx += 1
            elif q.pop(idx) is not ev:
                raise RuntimeError("Get queue invariant violated")
            if not proceed:
                break


class StorePut(_Put):
    def __init__(self, store, item):
        self.item = item
        super().__init__(store)


class StoreGet(_Get):
    pass


class FilterStoreGet(_Get):
    def __init__(self, store, filter=lambda item: True):
        self.filter = filter
        super().__init__(store)


class Store(_BaseResource):
    def __init__(self, env, capacity=Infinity):
        if capacity <= 0:
            raise ValueError('"capacity" must be > 0.')
        super().__init__(env, capacity)
        self.items = []

    def put(self, item):
        return StorePut(self, item)

    def get(self):
        return StoreGet(self)

    def _do_put(self, event):
        if len(self.items) < self._capacity:
            self.items.append(event.item)
            event.succeed()

    def _do_get(self, event):
        if self.items:
            event.succeed(self.items.pop(0))


class FilterStore(Store):
    def get(self, filter=lambda item: True):
        return FilterStoreGet(self, filter)

    def _do_get(self, event):
        for item in self.items:
            if event.filter(item):
                self.items.remove(item)
                event.succeed(item)
                break
        return True


class ContainerPut(_Put):
    def __init__(self, container, amount):
        if amount <= 0:
            raise ValueError("amount(=%s) must be > 0." % amount)
        self.amount = amount
        super().__init__(container)


class ContainerGet(_Get):
    def __init__(self, container, amount):
        if amount <= 0:
            raise ValueError("amount(=%s) must be > 0." % amount)
        self.amount = amount
        super().__init__(container)


class Container(_BaseResource):
    def __init__(self, env, capacity=Infinity, init=0):
        if capacity <= 0:
            raise ValueError('"capacity" must be > 0.')
        if init < 0:
            raise ValueError('"init" must be >= 0.')
        if init > capacity:
            raise ValueError('"init" must be <= "capacity".')
        super().__init__(env, capacity)
        self._level = init

    @property
    def level(self):
        return self._level

    def put(self, amount):
        return ContainerPut(self, amount)

    def get(self, amount):
        return ContainerGet(self, amount)

    def _do_put(self, event):
        if self._capacity - self._level >= event.amount:
            self._level += event.amount
            event.succeed()
            return True

    def _do_get(self, event):
        if self._level >= event.amount:
            self._level -= event.amount
            event.succeed()
            return True


class Request(_Put):
    def __exit__(self, exc_type, exc_value, traceback):
        super().__exit__(exc_type, exc_value, traceback)
        self.resource.release(self)


class Release(_Get):
    def __init__(self, resource, request):
        self.request = request
        super().__init__(resource)


class Resource(_BaseResource):
    def __init__(self, env, capacity=1):
        if capacity <= 0:
            raise ValueError('"capacity" must be > 0.')
        super().__init__(env, capacity)
        self.users = []
        self.queue = self.put_queue

    @property
    def count(self):
        return len(self.users)

    def request(self):
        return Request(self)

    def release(self, request):
        return Release(self, request)

    def _do_put(self, event):
        if len(self.users) < self.capacity:
            self.users.append(event)
            event.usage_since = self._env.now
            event.succeed()

    def _do_get(self, event):
        try:
            self.users.remove(event.request)
        except ValueError:
            pass
        event.succeed()


def install(force=False):
    """Register this module as ``simpy`` (and ``simpy.core``/``simpy.events``/``simpy.resources``
    aliases) unless a real SimPy is importable. Returns the module that ``import simpy`` yields."""
    if not force:
        try:
            import simpy  # noqa: F401
            return sys.modules["simpy"]
        except ImportError:
            pass
    mod = sys.modules[__name__]
    for name in ("simpy", "simpy.core", "simpy.events", "simpy.resources"):
        sys.modules[name] = mod
    return mod
