"""Diagnostic: golden runs with small windows, pipelined vs sequential; reports mismatches."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import golden_io
from pivot_place.engine import PlacementEngine
eng = PlacementEngine(0)
for name in sys.argv[1].split(","):
    c = golden_io.load(name)
    for w in (7, 64):
        eng.set_window(w)
        for idx, run in enumerate(c["runs"]):
            if run["error"]:
                continue
            r = golden_io.run_arrays(c, run)
            exp = golden_io.expected(c, run)
            for pipe in (True, False):
                eng.set_pipeline(pipe)
                res = eng.place(r)
                bad = np.nonzero(res.placement[exp[1]] != exp[0][exp[1]])[0]
                if bad.size:
                    print(name, "run", idx, "mode", r.mode, "window", w, "pipe", pipe, "first bad pos", bad[0],
                          "got", res.placement[exp[1]][bad[0]:bad[0] + 4], "want", exp[0][exp[1]][bad[0]:bad[0] + 4])
print("done")
