"""Anchor resolution (reference scheduler/cost_aware.py:45-58).

The reference picks, per ready task, the MODE host of its predecessors' task placements with
``max(Counter(placements).items(), key=lambda x: x[1])``: highest count, first seen among equal
counts. The CPU restatement (oracle_anchor) is pinned here against the groups the reference
itself formed in every golden cost_aware run, and against that Counter expression; the gpu tests
check pvt_anchor (pvt_anchor.hip) against the restatement, item for item, including lists longer
than the kernel's LDS tile (sorted in scratch) and the instance-table (inst_host) form.
"""
import collections

import numpy as np
import pytest

import golden_io
from oracle import oracle
from pivot_place import _abi


def counter_mode(placements):
    """The reference expression itself (cost_aware.py:52)."""
    return max(collections.Counter(placements).items(), key=lambda x: x[1])[0]


def fixture_items(st):
    """(off, list) over the fixture's containers: pred_hosts as the reference iterated them."""
    off, lst = [0], []
    for c in st["containers"]:
        lst.extend(c["pred_hosts"])
        off.append(len(lst))
    return np.array(off, dtype=np.int64), np.array(lst, dtype=np.int32)


@pytest.mark.parametrize("case", golden_io.CASES)
def test_oracle_anchor_matches_reference_groups(case):
    st = golden_io.load(case)
    off, lst = fixture_items(st)
    zone = np.array(st["zone"], dtype=np.int32)
    mode, az, rc = oracle.anchor(off, lst, zone, st["n_hosts"])
    assert rc == 0
    for i, c in enumerate(st["containers"]):
        if c["pred_hosts"]:
            assert mode[i] == counter_mode(c["pred_hosts"])
            assert az[i] == zone[mode[i]]
        else:
            assert (mode[i], az[i]) == (-1, _abi.ANCHOR_NO_PREDS)
    task_cont = st["tasks"]["container"]
    checked = 0
    for run in st["runs"]:
        if run["policy"] != "cost_aware" or run["error"] or not run.get("groups"):
            continue
        for g in run["groups"]:
            conts = {task_cont[t] for t in g["tasks"]}
            zs = {int(az[c]) for c in conts}
            if zs == {_abi.ANCHOR_NO_PREDS}:
                continue        # an application group: anchor drawn by randomizer.choice
            assert zs == {g["anchor_zone"]}, (case, g)
            checked += 1
    if any(c["pred_hosts"] for c in st["containers"]) and any(
            r["policy"] == "cost_aware" and not r["error"] for r in st["runs"]):
        assert checked > 0


def random_items(rng, n_items, n_hosts, max_len, unplaced=False):
    off, lst = [0], []
    for _ in range(n_items):
        n = int(rng.integers(0, max_len + 1))
        k = int(rng.integers(1, 6))                    # few distinct hosts: many ties
        pool = rng.integers(-1 if unplaced else 0, n_hosts, size=k)
        lst.extend(int(x) for x in rng.choice(pool, size=n))
        off.append(len(lst))
    return np.array(off, dtype=np.int64), np.array(lst, dtype=np.int32)


def test_oracle_anchor_matches_counter_on_random_lists():
    rng = np.random.default_rng(5)
    H = 50
    zone = (np.arange(H) % 7).astype(np.int32)
    off, lst = random_items(rng, 400, H, 60, unplaced=True)
    mode, az, rc = oracle.anchor(off, lst, zone, H)
    assert rc == 0
    for i in range(len(off) - 1):
        L = lst[off[i]:off[i + 1]].tolist()
        if not L:
            assert az[i] == _abi.ANCHOR_NO_PREDS
            continue
        m = counter_mode(L)
        assert mode[i] == m
        assert az[i] == (zone[m] if m >= 0 else _abi.ANCHOR_UNPLACED)


def test_oracle_anchor_rejects_bad_items():
    zone = np.zeros(4, dtype=np.int32)
    mode, az, rc = oracle.anchor([0, 2, 3], [1, 9, 2], zone, 4)
    assert rc == _abi.PVT_EINVAL and az[0] == _abi.ANCHOR_INVALID and az[1] == zone[2]
    mode, az, rc = oracle.anchor([0, 2], [0, 5], zone, 4, inst_host=[3, 1])
    assert rc == _abi.PVT_EINVAL and az[0] == _abi.ANCHOR_INVALID


# ------------------------------------------------------------------ GPU (pvt_anchor)
@pytest.mark.gpu
@pytest.mark.parametrize("case", golden_io.CASES)
def test_gpu_anchor_fixtures(engine, case):
    st = golden_io.load(case)
    off, lst = fixture_items(st)
    zone = np.array(st["zone"], dtype=np.int32)
    want = oracle.anchor(off, lst, zone, st["n_hosts"])
    got = engine.anchor(off, lst, zone)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


@pytest.mark.gpu
@pytest.mark.parametrize("max_len,n_items,H", [(0, 10, 5), (1, 300, 3), (64, 2000, 100),
                                               (4096, 60, 1000), (5000, 40, 20),
                                               (40000, 6, 100000)])
def test_gpu_anchor_random(engine, max_len, n_items, H):
    rng = np.random.default_rng(max_len + n_items)
    zone = rng.integers(0, 31, size=H).astype(np.int32)
    off, lst = random_items(rng, n_items, H, max_len, unplaced=True)
    want = oracle.anchor(off, lst, zone, H)
    assert want[2] == 0
    got = engine.anchor(off, lst, zone)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


@pytest.mark.gpu
def test_gpu_anchor_distinct_hosts_long_list(engine):
    """All-distinct lists (every count 1: the first entry wins) across every path edge:
    registers (<= 64), wave LDS sort (<= 1024), block LDS sort (<= 8192), LDS histograms."""
    H = 1 << 20
    zone = (np.arange(H) % 20).astype(np.int32)
    rng = np.random.default_rng(11)
    lens = [1, 2, 63, 64, 65, 1023, 1024, 1025, 4095, 4096, 4097, 8192, 8193, 9000, 70000]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    lst = np.concatenate([rng.permutation(H)[:n] for n in lens]).astype(np.int32)
    want = oracle.anchor(off, lst, zone, H)
    got = engine.anchor(off, lst, zone)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[0], lst[off[:-1]])
    assert np.array_equal(got[1], want[1])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [64, 65, 700, 1024, 1025, 3000, 8192, 8193, 20000])
def test_gpu_anchor_tied_lists(engine, n):
    """Every path with heavy ties: two hosts with equal counts, the later-seen one sorted first
    by host index (the first-seen one must win), plus unplaced entries."""
    H = 5000
    zone = (np.arange(H) % 31).astype(np.int32)
    rng = np.random.default_rng(n)
    base = np.where(np.arange(n) % 2 == 0, 4000, 7).astype(np.int32)   # 4000 seen first
    base[rng.random(n) < 0.1] = -1
    rng.shuffle(base[1:])
    off = np.array([0, n, 2 * n], dtype=np.int64)
    lst = np.concatenate([base, base[::-1]]).astype(np.int32)
    want = oracle.anchor(off, lst, zone, H)
    got = engine.anchor(off, lst, zone)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


@pytest.mark.gpu
def test_gpu_anchor_instance_table(engine):
    """inst_host form: entries index a per-instance host table resident in HBM."""
    rng = np.random.default_rng(3)
    H, N = 500, 20000
    zone = rng.integers(0, 20, size=H).astype(np.int32)
    inst_host = rng.integers(-1, 40, size=N).astype(np.int32)
    off, lst = random_items(rng, 700, N, 300)
    want = oracle.anchor(off, lst, zone, H, inst_host=inst_host)
    assert want[2] == 0
    got = engine.anchor(off, lst, zone, inst_host=inst_host)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


@pytest.mark.gpu
def test_gpu_anchor_invalid_items_raise(engine):
    zone = np.zeros(4, dtype=np.int32)
    with pytest.raises(RuntimeError, match="EINVAL"):
        engine.anchor([0, 2, 3], [1, 9, 2], zone)
    with pytest.raises(RuntimeError, match="EINVAL"):
        engine.anchor([0, 2], [0, 5], zone, inst_host=[3, 1])
