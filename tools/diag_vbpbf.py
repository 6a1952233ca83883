#!/usr/bin/env python3
"""vbp best-fit diagnosis: one synthetic round placed with band lists on/off and the one-wave
list walk on/off (PVT_LWALK), each compared with the oracle; prints the first mismatches.
    python tools/diag_vbpbf.py --hosts 70000 --tasks 2600 --seed 9"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hosts", type=int, default=70000)
    ap.add_argument("--tasks", type=int, default=2600)
    ap.add_argument("--seed", type=int, default=9)
    ap.add_argument("--pipeline", type=int, default=1)
    a = ap.parse_args()
    import numpy as np
    from oracle import oracle
    from pivot_place import _abi, synthetic
    from pivot_place.engine import PlacementEngine
    r = synthetic.make_round(_abi.PVT_VBP_BF, a.hosts, a.tasks, seed=a.seed)
    ref = oracle.place(r, threads=8)
    pos = {int(t): i for i, t in enumerate(ref.order)}
    for lw in ("1", "0"):
        os.environ["PVT_LWALK"] = lw
        eng = PlacementEngine(0)
        eng.set_resident(0)
        eng.set_pipeline(bool(a.pipeline))
        for band in (1, 0):
            eng.set_band(band)
            got = eng.place(r)
            bad = np.nonzero(got.placement != ref.placement)[0]
            st = eng.last_stats()
            print("lwalk=%s band=%d: %d placements differ, windows=%d refills=%d" %
                  (lw, band, bad.size, st["windows"], st["refills"]), flush=True)
            for t in sorted(bad, key=lambda t: pos[int(t)])[:6]:
                print("   task %d (processing position %d): got %d ref %d demand %s" %
                      (t, pos[int(t)], got.placement[t], ref.placement[t], r.dem[:, t].tolist()))


if __name__ == "__main__":
    main()
