#!/usr/bin/env python3
"""Where a drop-in round's time goes (configs 1/2 replays): the recorded reference simulation's
rounds through the drop-in policy class, with the engine call timed apart from the Python
around it, for the GPU engine and for the C restatement.

    python tools/replay_split.py sim_c1_cost_aware [sim_c2a1000_cost_aware ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT, os.path.join(ROOT, "tests")]


class Timed:
    def __init__(self, eng):
        self.eng = eng
        self.secs = 0.0
        self.calls = 0
        if hasattr(eng, "place_cost_aware"):
            self.place_cost_aware = self._wrap(eng.place_cost_aware)
        self.place = self._wrap(eng.place)
        self.anchor = self._wrap(eng.anchor)

    def _wrap(self, f):
        def g(*a, **k):
            t = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                self.secs += time.perf_counter() - t
                self.calls += 1
        return g


def main():
    import bench
    from pivot_place.engine import PlacementEngine
    eng = PlacementEngine(0)
    for name in sys.argv[1:] or ["sim_c1_cost_aware"]:
        for label, e in (("gpu", eng), ("cpu1", bench._OracleEngine(0))):
            bench._replay(name, e)
            t = Timed(e)
            secs, cand, nr, ok, _ = bench._replay(name, t)
            print("%s %s: %d rounds %.3f ms/round, engine calls %d = %.3f ms/round, rest %.3f "
                  "ms/round, parity %s" % (name, label, nr, secs * 1e3 / nr, t.calls,
                                          t.secs * 1e3 / nr, (secs - t.secs) * 1e3 / nr, ok),
                  flush=True)


if __name__ == "__main__":
    main()
