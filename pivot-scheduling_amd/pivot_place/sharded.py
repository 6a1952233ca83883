"""Host-dimension sharding of one round over several GPUs (BASELINE config 5).

Each rank scores a contiguous host range and keeps the whole availability array (32 B per host:
32 MB at 1M hosts), which every rank updates identically because every rank runs the same
commit walk. Per window, the only exchange is one all-gather of per-task candidate packages
(the rank's exact top entries plus a bound, 16 B each; include/pivot_place.h, pvt_shard_*):
over xGMI with RCCL (``torch.distributed`` backend "nccl"), staged through host memory with
gloo. The reference scans every host of the cluster per task (scheduler/cost_aware.py:88-92,
scheduler/vbp.py:19-22, 43-47); a sharded round returns exactly what pvt_place() returns.

Opportunistic rounds shard by whole super-chunks of 16384 hosts (the count pass's unit): each
rank counts the feasible hosts of its super-chunks per task (bitmaps + counts), the window's
packages are all-gathered, and every rank runs the same draw / k-th-host walk on the full
tables (per-rank feasible counts -> all-gather -> draw -> select), so the
MT19937 state and placements agree everywhere (reference scheduler/opportunistic.py:11-20).

``place_lockstep`` drives several contexts in one process (one per shard, same or different
GPUs) with the exchange done by concatenation: the same protocol without a process group.
"""
from . import _abi
from .engine import DeviceRound
from .scenarios import shard

OPP_SUPER_CHUNK = 64 * 256     # hosts per super-chunk of the opportunistic count pass


def shard_range(n_hosts, world, rank, mode):
    """Host range of ``rank``: an even split, or for opportunistic rounds whole super-chunks
    (rank r takes super-chunks [r * P, (r + 1) * P), P = ceil(super-chunks / world))."""
    if mode != _abi.PVT_OPP:
        return shard(n_hosts, world, rank)
    nsq = (n_hosts + OPP_SUPER_CHUNK - 1) // OPP_SUPER_CHUNK
    per = (nsq + world - 1) // world
    return (min(n_hosts, rank * per * OPP_SUPER_CHUNK), min(n_hosts, (rank + 1) * per * OPP_SUPER_CHUNK))


def torch_exchange(group=None):
    """All-gather of the first ``nbytes`` of every rank's package into ``recv`` (rank order)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    nccl = dist.get_backend(group) == "nccl"

    def exchange(send, nbytes, recv):
        if nccl:
            dist.all_gather_into_tensor(recv[:world * nbytes], send[:nbytes], group=group)
            return
        host = send[:nbytes].cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        recv[:world * nbytes].copy_(torch.cat(parts))
    return exchange


class HostShardedPlacer:
    """Rank ``rank`` of ``world``: places rounds whose host dimension is split over the ranks."""

    def __init__(self, engine, rank, world, exchange=None):
        if exchange is None and int(world) != 1:
            raise ValueError("a sharded round over %d ranks needs an exchange" % world)
        self.engine, self.rank, self.world, self.exchange = engine, int(rank), int(world), exchange
        self.windows = 0

    @classmethod
    def from_process_group(cls, engine, group=None):
        import torch.distributed as dist
        return cls(engine, dist.get_rank(group), dist.get_world_size(group), torch_exchange(group))

    def host_range(self, n_hosts, mode=None):
        return shard_range(n_hosts, self.world, self.rank, mode)

    def run(self, dr: DeviceRound):
        """Place a resident round in place (``dr.placement``/``order``/``avail`` as pvt_place).

        The exchange runs on its own stream, so it overlaps the commit walk the engine left in
        flight (pvt_shard_commit returns at once; the next pvt_shard_score scores the following
        window beside it); the context's stream waits for the exchange before the merge."""
        import torch
        eng = self.engine
        lo, hi = self.host_range(dr.arrays.n_hosts, dr.arrays.mode)
        mx = eng.shard_begin(dr, lo, hi, self.world)
        send = torch.empty(max(mx, 1), dtype=torch.uint8, device=eng.device)
        recv = torch.empty(max(mx, 1) * self.world, dtype=torch.uint8, device=eng.device)
        gpu = torch.device(eng.device).type == "cuda"
        cur = torch.cuda.current_stream(eng.device) if gpu else None
        side = torch.cuda.Stream(eng.device) if gpu else None
        self.windows = self.stale = 0
        while True:
            nt, nbytes = eng.shard_score(send)
            if nt == 0:
                return
            if self.exchange is None:          # a single shard: its package is the whole set
                ok = eng.shard_commit(send)
            elif gpu:
                with torch.cuda.stream(side):
                    self.exchange(send, nbytes, recv)
                cur.wait_stream(side)
                ok = eng.shard_commit(recv)
            else:                              # host-side stand-ins (tests)
                self.exchange(send, nbytes, recv)
                ok = eng.shard_commit(recv)
            self.windows += 1
            self.stale += 0 if ok else 1

    def place(self, r):
        dr = DeviceRound(r, self.engine.device)
        self.run(dr)
        return dr.result()


def place_lockstep(engines, r):
    """Run one round split over ``len(engines)`` contexts in this process; returns every
    shard's RoundResult (all equal to pvt_place's)."""
    import torch
    world = len(engines)
    drs = [DeviceRound(r, e.device) for e in engines]
    mx = [e.shard_begin(dr, *shard_range(r.n_hosts, world, k, r.mode), world)
          for k, (e, dr) in enumerate(zip(engines, drs))]
    sends = [torch.empty(max(m, 1), dtype=torch.uint8, device=e.device) for m, e in zip(mx, engines)]
    recvs = [torch.empty(max(m, 1) * world, dtype=torch.uint8, device=e.device)
             for m, e in zip(mx, engines)]
    while True:
        got = [e.shard_score(s) for e, s in zip(engines, sends)]
        if len(set(got)) != 1:
            raise RuntimeError("shards disagree on the window: %s" % (got,))
        nt, nb = got[0]
        if nt == 0:
            break
        for recv in recvs:
            for k, s in enumerate(sends):
                recv[k * nb:(k + 1) * nb].copy_(s[:nb])
        ok = [e.shard_commit(recv) for e, recv in zip(engines, recvs)]
        if len(set(ok)) != 1:
            raise RuntimeError("shards disagree on a stale window: %s" % (ok,))
    return [dr.result() for dr in drs]
