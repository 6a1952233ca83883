"""Scenario batches sharded over GPUs (BASELINE config 4; SURVEY.md §8(e), first row).

Independent simulations (one seed each) share nothing, so the batch is split into contiguous
blocks of seeds, one block per rank, with no collective on the data path. Each rank places its
scenarios on its own GPU; a single gather of small per-scenario summaries at the end gives every
rank the whole batch's results (the "final metrics gather" of §8(e)).

``engine`` is anything with ``place(RoundArrays) -> RoundResult`` (a PlacementEngine on a GPU).
When it also has ``place_batch`` and the rounds fit the resident kernel (<= 4096 hosts and
tasks), a rank's block is placed ``batch`` rounds per call: one launch, one workgroup per
scenario (include/pivot_place.h, pvt_place_batch).
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


RESIDENT_MAX = 4096   # pvt_place_batch limits (PVT_RESIDENT_MAX_HOSTS / _TASKS)


def run_block(engine, mode, n_hosts, n_tasks, seeds, batch=512):
    """Place one synthetic round per seed; returns the per-scenario summaries in seed order."""
    seeds = [int(s) for s in seeds]
    batched = (hasattr(engine, "place_batch") and batch > 0 and n_hosts <= RESIDENT_MAX
               and n_tasks <= RESIDENT_MAX)
    out = []
    if not batched:
        for s in seeds:
            out.append(summarize(s, engine.place(synthetic.make_round(mode, n_hosts, n_tasks, seed=s))))
        return out
    for i in range(0, len(seeds), batch):
        block = seeds[i:i + batch]
        rounds = [synthetic.make_round(mode, n_hosts, n_tasks, seed=s) for s in block]
        out.extend(summarize(s, res) for s, res in zip(block, engine.place_batch(rounds)))
    return out


def run_sharded(engine, mode, n_hosts, n_tasks, seeds, group=None, batch=512):
    """Run this rank's block of ``seeds`` and gather every rank's summaries (in seed order)."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    lo, hi = shard(len(seeds), world, rank)
    mine = run_block(engine, mode, n_hosts, n_tasks, seeds[lo:hi], batch=batch)
    if world == 1:
        return mine
    parts = [None] * world
    dist.all_gather_object(parts, mine, group=group)
    return [x for p in parts for x in p]
