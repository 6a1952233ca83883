"""pivot_place.des: the SimPy 3.0.11 event semantics the reference simulator relies on.

Expected values are SimPy 3's documented behaviour (its tutorial's car process, the ordering
rules of ``Environment.schedule``/``step``, resource queue semantics). The end-to-end check is
test_sim_replay.py: the reference's whole simulator ran on this core to record the traces.
"""
import pytest

from pivot_place import des


def test_car_example():
    """SimPy's tutorial process: park 5, drive 2, until=15."""
    env, log = des.Environment(), []

    def car(env):
        while True:
            log.append(("park", env.now))
            yield env.timeout(5)
            log.append(("drive", env.now))
            yield env.timeout(2)

    env.process(car(env))
    env.run(until=15)
    assert log == [("park", 0), ("drive", 5), ("park", 7), ("drive", 12), ("park", 14)]
    assert env.now == 15


def test_same_time_fifo_and_urgent_start():
    """Events due at the same time run in scheduling order; a process started at time t runs
    (URGENT Initialize) before NORMAL events already due at t."""
    env, log = des.Environment(), []

    def p(name, delay):
        yield env.timeout(delay)
        log.append(name)

    for i in range(5):
        env.process(p(i, 3))
    env.run()
    assert log == [0, 1, 2, 3, 4]

    env, log = des.Environment(), []
    t = env.timeout(0)
    t.callbacks.append(lambda e: log.append("timeout"))

    def starter():
        log.append("started")
        yield env.timeout(0)

    env.process(starter())
    env.run()
    assert log == ["started", "timeout"]


def test_process_value_and_processed_events():
    env = des.Environment()

    def child():
        yield env.timeout(3)
        return 42

    def parent(out):
        v = yield env.process(child())
        out.append((env.now, v))
        ev = env.event().succeed("x")
        yield env.timeout(1)
        # yielding an already-processed event resumes synchronously with its value
        out.append((env.now, (yield ev)))

    out = []
    env.process(parent(out))
    env.run()
    assert out == [(3, 42), (4, "x")]


def test_run_until_checks_and_peek():
    env = des.Environment()
    env.timeout(4)
    assert env.peek() == 4
    env.run(until=2)
    assert env.now == 2
    with pytest.raises(ValueError):
        env.run(until=1)
    env.run()
    assert env.now == 4 and env.peek() == des.Infinity


def test_run_until_event_returns_value():
    env = des.Environment()

    def p():
        yield env.timeout(7)
        return "done"

    assert env.run(env.process(p())) == "done" and env.now == 7


def test_unhandled_failure_raises_and_handled_is_defused():
    env = des.Environment()

    def bad():
        yield env.timeout(1)
        raise KeyError("boom")

    env.process(bad())
    with pytest.raises(KeyError):
        env.run()

    env, seen = des.Environment(), []

    def waiter():
        try:
            yield env.process(bad())
        except KeyError as e:
            seen.append((env.now, e.args[0]))

    env.process(waiter())
    env.run()
    assert seen == [(1, "boom")]


def test_interrupt():
    env, log = des.Environment(), []

    def sleeper():
        try:
            yield env.timeout(10)
        except des.Interrupt as i:
            log.append((env.now, i.cause))

    def waker(p):
        yield env.timeout(3)
        p.interrupt("wake")

    p = env.process(sleeper())
    env.process(waker(p))
    env.run()
    assert log == [(3, "wake")]


def test_conditions():
    env = des.Environment()
    out = []

    def p():
        a, b = env.timeout(1, "a"), env.timeout(2, "b")
        r = yield a & b
        out.append((env.now, sorted(r.todict().values())))
        c, d = env.timeout(5, "c"), env.timeout(3, "d")
        r = yield c | d
        out.append((env.now, list(r.todict().values())))

    env.process(p())
    env.run()
    assert out == [(2, ["a", "b"]), (5, ["d"])]


def test_store_fifo_and_blocking_get():
    env = des.Environment()
    store, got = des.Store(env), []

    def consumer(name):
        while True:
            item = yield store.get()
            got.append((env.now, name, item))

    def producer():
        for i in range(4):
            yield env.timeout(2)
            yield store.put(i)

    env.process(consumer("A"))
    env.process(consumer("B"))
    env.process(producer())
    env.run(until=20)
    # waiting getters are served in request order; each item goes to exactly one getter
    assert got == [(2, "A", 0), (4, "B", 1), (6, "A", 2), (8, "B", 3)]


def test_store_capacity_blocks_put():
    env = des.Environment()
    store, log = des.Store(env, capacity=1), []

    def producer():
        for i in range(3):
            yield store.put(i)
            log.append(("put", i, env.now))

    def consumer():
        yield env.timeout(5)
        while True:
            x = yield store.get()
            log.append(("get", x, env.now))
            yield env.timeout(5)

    env.process(producer())
    env.process(consumer())
    env.run(until=30)
    assert log == [("put", 0, 0), ("get", 0, 5), ("put", 1, 5), ("get", 1, 10), ("put", 2, 10),
                   ("get", 2, 15)]
    assert store.items == []


def test_container_levels_and_blocking():
    env = des.Environment()
    tank, log = des.Container(env, capacity=10, init=4), []

    def taker(n):
        yield tank.get(n)
        log.append(("got", n, env.now, tank.level))

    def filler():
        yield env.timeout(3)
        yield tank.put(6)
        log.append(("put", 6, env.now, tank.level))

    env.process(taker(3))
    env.process(taker(5))      # blocks: level 1 < 5 until the put
    env.process(taker(2))      # FIFO: waits behind the blocked request
    env.process(filler())
    env.run()
    assert log == [("got", 3, 0, 1), ("put", 6, 3, 0), ("got", 5, 3, 0), ("got", 2, 3, 0)]
    with pytest.raises(ValueError):
        des.Container(env, capacity=2, init=3)
    with pytest.raises(ValueError):
        tank.get(0)


def test_resource_mutex():
    env = des.Environment()
    res, log = des.Resource(env, capacity=1), []

    def user(name, hold):
        with res.request() as req:
            yield req
            log.append((name, "in", env.now))
            yield env.timeout(hold)
            log.append((name, "out", env.now))

    for i, hold in enumerate([3, 2, 1]):
        env.process(user(i, hold))
    env.run()
    assert log == [(0, "in", 0), (0, "out", 3), (1, "in", 3), (1, "out", 5), (2, "in", 5),
                   (2, "out", 6)]
    assert res.count == 0 and res.queue == []


def test_host_resource_pattern():
    """The reference's HostResource.subscribe/unsubscribe (resources/__init__.py:433-461): a
    mutex around sequential container gets/puts, all in zero simulated time."""
    env = des.Environment()
    lock = des.Resource(env)
    cpus, mem = des.Container(env, 16, init=16), des.Container(env, 1024, init=1024)

    def subscribe(c, m):
        with lock.request() as req:
            yield req
            yield cpus.get(c)
            yield mem.get(m)
        return True

    def task(c, m, runtime):
        ok = yield env.process(subscribe(c, m))
        assert ok
        yield env.timeout(runtime)
        with lock.request() as req:
            yield req
            yield cpus.put(c)
            yield mem.put(m)

    for i in range(4):
        env.process(task(2 + i, 100.0 * (i + 1), 10 + i))
    env.run(until=1)
    assert cpus.level == 16 - (2 + 3 + 4 + 5) and mem.level == 1024 - 1000.0
    env.run()
    assert cpus.level == 16 and mem.level == 1024 and env.now == 13


def test_install_registers_simpy():
    import sys
    saved = {k: sys.modules.get(k) for k in ("simpy", "simpy.core", "simpy.events", "simpy.resources")}
    try:
        mod = des.install(force=True)
        import simpy
        assert simpy is mod and simpy.Environment is des.Environment
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
