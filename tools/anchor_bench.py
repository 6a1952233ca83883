"""Anchor-resolution throughput (pvt_anchor over a DeviceTrace).

Workload: the 400-job trace sample (tests/golden/jobs_sample.yaml.gz) tiled --copies times
(5000 apps for 12.5 copies ~ one bundled trace file), every instance placed on a random host of
--hosts, every container resolved in one launch per step (item form over the resident table).
Algorithmic bytes per list entry: 4 (pinst) + 4 (inst_host gather) = 8 B.
Prints one JSON line: entries/s, items/s, GB/s, ms per launch (HIP events on the launch stream).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pivot-scheduling_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=13)
    ap.add_argument("--hosts", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from pivot_place import trace
    from pivot_place.engine import PlacementEngine
    jobs = trace.load_jobs(os.path.join(ROOT, "tests", "golden", "jobs_sample.yaml.gz"))
    tiled = [dict(j, id="%s_%d" % (j["id"], k)) for k in range(args.copies) for j in jobs]
    tr = trace.from_jobs(tiled)
    eng = PlacementEngine(0)
    rng = np.random.default_rng(1)
    zone = (np.arange(args.hosts) % 31).astype(np.int32)
    dt = trace.DeviceTrace(tr, zone, eng)
    dt.record(np.arange(tr.n_instances), rng.integers(0, args.hosts, tr.n_instances))
    items = torch.arange(tr.n_containers, dtype=torch.int32, device=eng.device)
    for _ in range(3):
        dt.anchors(items)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(args.steps):
        dt.anchors(items)
    b.record(st)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / args.steps
    P = len(tr.pinst)
    # CPU baseline: the C restatement (oracle_anchor, 1 thread) on the same items
    import time
    sys.path.insert(0, ROOT)
    from oracle import oracle
    ih = dt.inst_host[:tr.n_instances].cpu().numpy()
    t0 = time.perf_counter()
    cref = oracle.anchor(tr.pinst_off, tr.pinst, zone, args.hosts, inst_host=ih)
    cpu_s = time.perf_counter() - t0
    mode, az = dt.anchors(items)
    assert np.array_equal(mode.cpu().numpy(), cref[0]), "GPU anchors differ from the oracle"
    print(json.dumps({"metric": "anchor resolution (pvt_anchor, item form)", "apps": tr.n_apps,
                      "containers": tr.n_containers, "instances": tr.n_instances,
                      "list_entries": P, "hosts": args.hosts, "ms_per_launch": ms,
                      "items_per_s": tr.n_containers / ms * 1e3,
                      "entries_per_s": P / ms * 1e3,
                      "algorithmic_GBps": 8.0 * P / ms * 1e-6,
                      "cpu_baseline": {"items_per_s": tr.n_containers / cpu_s, "cores": 1,
                                       "kind": "port", "sample": "oracle_anchor on all items"},
                      "note": "ms includes the host-side argument checks and the 4-byte "
                              "error-count read-back of each synchronous pvt_anchor call"}))


if __name__ == "__main__":
    main()
