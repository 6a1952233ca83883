"""Multi-process path (world_size 2, gloo on CPU): scenario batches sharded over ranks.

Each rank places its contiguous block of scenarios and the final gather gives every rank the
whole batch; the result must equal one process running every scenario. The per-rank engine is
the CPU restatement behind the engine's place() contract (no GPU here); the GPU variant of the
same driver is what bench.py runs for N > 1.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _OracleEngine:
    def place(self, r):
        from oracle import oracle
        return oracle.place(r)


class _OracleBatchEngine(_OracleEngine):
    """Adds the batch entry point (PlacementEngine.place_batch's contract), counting calls."""

    def __init__(self):
        self.batches = []

    def place_batch(self, rounds):
        self.batches.append(len(rounds))
        return [self.place(r) for r in rounds]


def _worker(rank, world, port, mode, seeds, out_q):
    sys.path[:0] = [os.path.join(os.path.dirname(HERE), "pivot-scheduling_amd"),
                    os.path.dirname(HERE), HERE]
    import torch.distributed as dist
    from pivot_place import scenarios
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = scenarios.run_sharded(_OracleEngine(), mode, 300, 40, seeds)
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4])
def test_scenario_batch_two_ranks(mode):
    from pivot_place import scenarios
    seeds = list(range(100, 107))
    ref = scenarios.run_block(_OracleEngine(), mode, 300, 40, seeds)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, seeds, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == ref and got[1] == ref


def test_batched_block_equals_per_round_block():
    """run_block through place_batch (blocks of `batch` rounds) == one place() per scenario."""
    from pivot_place import scenarios
    seeds = list(range(200, 211))
    for mode in (1, 2, 4):
        ref = scenarios.run_block(_OracleEngine(), mode, 200, 30, seeds)
        eng = _OracleBatchEngine()
        assert scenarios.run_block(eng, mode, 200, 30, seeds, batch=4) == ref
        assert eng.batches == [4, 4, 3]
    big = _OracleBatchEngine()
    scenarios.run_block(big, 3, scenarios.RESIDENT_MAX + 1, 2, [1])
    assert big.batches == []          # beyond the resident limits: one place() per round


def test_shard_blocks_cover_everything():
    from pivot_place.scenarios import shard
    for n in (0, 1, 7, 4096):
        for world in (1, 2, 3, 8):
            blocks = [shard(n, world, r) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
            assert max(b - a for a, b in blocks) - min(b - a for a, b in blocks) <= 1


# ---------------------------------------------------------------- host-dimension sharding
class _ProtocolEngine:
    """Stands in for PlacementEngine's pvt_shard_* calls on CPU: rank k's package for window w
    is bytes (k, w, ...); commit checks it received every rank's package in rank order."""

    device = "cpu"

    def __init__(self, rank, world, windows):
        self.rank, self.world, self.windows, self.w = rank, world, windows, 0
        self.seen = []

    def shard_begin(self, dr, lo, hi, world):
        assert world == self.world
        self.range = (lo, hi)
        return 64

    def shard_score(self, send):
        if self.w >= len(self.windows):
            return 0, 0
        nt = self.windows[self.w]
        nb = 4 * nt
        send[:nb] = torch_u8([self.rank, self.w] * (nb // 2))
        return nt, nb

    def shard_commit(self, recv):
        nb = 4 * self.windows[self.w]
        for k in range(self.world):
            assert recv[k * nb:(k + 1) * nb].tolist() == [k, self.w] * (nb // 2)
        self.seen.append(nb)
        self.w += 1
        return True


def torch_u8(vals):
    import torch
    return torch.tensor(vals, dtype=torch.uint8)


class _FakeRound:
    class arrays:
        n_hosts = 1001
        mode = 1      # PVT_CA_BF: an even split


def _shard_worker(rank, world, port, out_q):
    sys.path[:0] = [os.path.join(os.path.dirname(HERE), "pivot-scheduling_amd"),
                    os.path.dirname(HERE), HERE]
    import torch.distributed as dist
    from pivot_place.sharded import HostShardedPlacer
    import test_distributed as td
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = td._ProtocolEngine(rank, world, [5, 16, 3])
        placer = HostShardedPlacer.from_process_group(eng)
        placer.run(td._FakeRound())
        out_q.put((rank, eng.range, eng.seen, placer.windows))
    finally:
        dist.destroy_process_group()


def test_host_sharded_exchange_two_ranks():
    """The sharded driver's per-window all-gather (gloo path) delivers every rank's package in
    rank order, and the ranks split the hosts into contiguous ranges."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] == (0, 501) and got[1][0] == (501, 1001)
    for r in range(2):
        assert got[r][1] == [20, 64, 12] and got[r][2] == 3


def test_opportunistic_shard_ranges_are_whole_super_chunks():
    """Opportunistic host shards: whole 16384-host super-chunks, contiguous, covering [0, H);
    ranks past the last super-chunk get an empty range."""
    from pivot_place import _abi
    from pivot_place.sharded import OPP_SUPER_CHUNK, shard_range
    for H, world in ((1_000_000, 8), (5000, 3), (200_000, 8), (40000, 2)):
        rs = [shard_range(H, world, k, _abi.PVT_OPP) for k in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == H
        for (a, b), (c, d) in zip(rs, rs[1:]):
            assert b == c
        for a, b in rs:
            assert a <= b and (a % OPP_SUPER_CHUNK == 0 or a == H) and (b == H or b % OPP_SUPER_CHUNK == 0)
