#!/usr/bin/env python3
"""Diagnose an epoch mismatch: the zero-score / underflow ca_bf scenario of test_gpu_batch,
placed with epochs off and on; prints the first mismatch in processing order and the epoch
counters."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]
import numpy as np  # noqa: E402


def main():
    from oracle import oracle
    from pivot_place import _abi, synthetic
    from pivot_place.engine import PlacementEngine
    eng = PlacementEngine(0)
    eng.set_resident(0)
    for s in range(8):
        r = synthetic.make_round(_abi.PVT_CA_BF, 600, 400, seed=70 + s)
        r.cost = r.cost.copy()
        r.cost[:, 1] = 5e-324 if s % 2 else 1e-300
        r.cost[1, :] = 0.0 if s % 3 else r.cost[1, :]
        for k in range(0, 600, 37):
            t = (k * 7 + s) % r.n_tasks
            r.avail[:, k] = r.dem[:, t]
        ref = oracle.place(r)
        for ep in (False, True):
            eng.set_epochs(ep)
            res = eng.place(r)
            st = eng.epoch_stats()
            po = ref.order
            bad = np.nonzero(res.placement[po] != ref.placement[po])[0]
            print("scenario %d epochs=%s stats=%s mismatches=%d first=%s" % (
                s, ep, st, bad.size, None if bad.size == 0 else
                (int(bad[0]), int(res.placement[po[bad[0]]]), int(ref.placement[po[bad[0]]]),
                 int(r.task_group[po[bad[0]]]))), flush=True)
            if bad.size and ep:
                tg = r.task_group[po]
                starts = np.nonzero(np.diff(tg))[0] + 1
                print("  group starts (processing order):", starts.tolist()[:30])
                print("  group anchors:", r.group_anchor.tolist())


if __name__ == "__main__":
    main()
