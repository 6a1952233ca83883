"""Scenario batches sharded over GPUs (BASELINE config 4; SURVEY.md §8(e), first row).

Independent simulations (one seed each) share nothing, so the batch is split into contiguous
blocks of seeds, one block per rank, with no collective on the data path. Each rank places its
scenarios on its own GPU; a single gather of small per-scenario summaries at the end gives every
rank the whole batch's results (the "final metrics gather" of §8(e)).

``engine`` is anything with ``place(RoundArrays) -> RoundResult`` (a PlacementEngine on a GPU).
"""
import hashlib

import numpy as np

from . import synthetic


def shard(n_items, world, rank):
    """Contiguous block [lo, hi) of ``n_items`` owned by ``rank`` (sizes differ by at most 1)."""
    base, extra = divmod(int(n_items), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def summarize(seed, res):
    """Per-scenario result: placed count and a digest of placements + final availability."""
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(res.placement, dtype=np.int32).tobytes())
    h.update(np.ascontiguousarray(res.avail, dtype=np.float64).tobytes())
    return {"seed": int(seed), "placed": int((res.placement >= 0).sum()),
            "digest": h.hexdigest()[:16]}


def run_block(engine, mode, n_hosts, n_tasks, seeds):
    out = []
    for s in seeds:
        r = synthetic.make_round(mode, n_hosts, n_tasks, seed=int(s))
        out.append(summarize(s, engine.place(r)))
    return out


def run_sharded(engine, mode, n_hosts, n_tasks, seeds, group=None):
    """Run this rank's block of ``seeds`` and gather every rank's summaries (in seed order)."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    lo, hi = shard(len(seeds), world, rank)
    mine = run_block(engine, mode, n_hosts, n_tasks, seeds[lo:hi])
    if world == 1:
        return mine
    parts = [None] * world
    dist.all_gather_object(parts, mine, group=group)
    return [x for p in parts for x in p]
