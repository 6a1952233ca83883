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


def test_shard_blocks_cover_everything():
    from pivot_place.scenarios import shard
    for n in (0, 1, 7, 4096):
        for world in (1, 2, 3, 8):
            blocks = [shard(n, world, r) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
            assert max(b - a for a, b in blocks) - min(b - a for a, b in blocks) <= 1
