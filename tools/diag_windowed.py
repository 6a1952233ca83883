#!/usr/bin/env python3
"""Diagnose a windowed-engine mismatch (test_gpu_batch zero-score / underflow scenario 7): the
first processing-order mismatch under each knob (merge kernel, tasks per wave, window, pipeline)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]
import numpy as np  # noqa: E402


def scenario(s):
    from pivot_place import _abi, synthetic
    r = synthetic.make_round(_abi.PVT_CA_BF, 600, 400, seed=70 + s)
    r.cost = r.cost.copy()
    r.cost[:, 1] = 5e-324 if s % 2 else 1e-300
    r.cost[1, :] = 0.0 if s % 3 else r.cost[1, :]
    for k in range(0, 600, 37):
        t = (k * 7 + s) % r.n_tasks
        r.avail[:, k] = r.dem[:, t]
    return r


def main():
    if len(sys.argv) == 1:
        for env in ({}, {"PVT_MERGE_SMALL": "0"}):
            e = dict(os.environ, **env)
            print("== env", env, flush=True)
            subprocess.run([sys.executable, __file__, "run"], env=e, check=False)
        return
    from oracle import oracle
    from pivot_place.engine import PlacementEngine
    eng = PlacementEngine(0)
    eng.set_resident(0)
    eng.set_epochs(False)
    for s in (7, 0):
        r = scenario(s)
        ref = oracle.place(r)
        for tw, win, pipe in ((0, 0, 1), (4, 0, 1), (2, 0, 0), (0, 1, 0), (0, 7, 1)):
            eng.set_score_tw(tw)
            eng.set_window(win)
            eng.set_pipeline(bool(pipe))
            res = eng.place(r)
            po = ref.order
            bad = np.nonzero(res.placement[po] != ref.placement[po])[0]
            print("s=%d tw=%d win=%d pipe=%d order_eq=%s mismatches=%d first=%s" % (
                s, tw, win, pipe, np.array_equal(res.order, ref.order), bad.size,
                None if bad.size == 0 else (int(bad[0]), int(res.placement[po[bad[0]]]),
                                            int(ref.placement[po[bad[0]]]))), flush=True)
        eng.set_score_tw(0); eng.set_window(0); eng.set_pipeline(True)


if __name__ == "__main__":
    main()
