"""Meter-aggregate throughput (pvt_meter over a batch of scenarios).

Workload: --scen synthetic scenarios shaped like the config-1 reference meters
(tests/golden/meter_logs.json.gz: ~15-100 hosts with a few intervals each, ~150-350 routes,
~10k single-transfer packets), resident in HBM; one pvt_meter launch per step reduces all of
them. Algorithmic bytes: 16 B per interval + 24 B per transfer + 8 B per offset entry.
Prints one JSON line with scenarios/s, GB/s and the C restatement's rate on the same batch.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pivot-scheduling_amd"))
sys.path.insert(0, ROOT)


def synthetic(n_scen, seed):
    """Flat CSR logs directly (no per-item Python lists): hosts 64, 4 intervals each; routes
    256, packets 40 each, 1 transfer per packet (as in the reference's meters)."""
    from pivot_place.meter import MeterLog
    rng = np.random.default_rng(seed)
    H, IV, R, PK = 64, 4, 256, 40
    n_h, n_r = n_scen * H, n_scen * R
    n_iv, n_p = n_h * IV, n_r * PK
    st = np.cumsum(rng.integers(0, 300, size=(n_h, 2 * IV)), axis=1).astype(np.float64)
    return MeterLog(host_off=np.arange(0, n_h + 1, H, dtype=np.int64),
                    iv_off=np.arange(0, n_iv + 1, IV, dtype=np.int64),
                    iv_start=st[:, 0::2].ravel().copy(), iv_end=st[:, 1::2].ravel().copy(),
                    route_off=np.arange(0, n_r + 1, R, dtype=np.int64),
                    route_cost=rng.choice([0.0, 0.01, 0.02, 0.05, 0.08], size=n_r),
                    pkt_off=np.arange(0, n_p + 1, PK, dtype=np.int64),
                    tr_off=np.arange(0, n_p + 1, dtype=np.int64),
                    tr_start=rng.random(n_p) * 1e4, tr_end=rng.random(n_p) * 1e4 + 1e4,
                    tr_size=rng.integers(1, 1001, size=n_p).astype(np.float64))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scen", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from oracle import oracle
    from pivot_place import _abi
    from pivot_place.engine import PlacementEngine
    log = synthetic(args.scen, 0)
    eng = PlacementEngine(0)
    dev = eng.device
    d = {k: torch.from_numpy(a).to(dev) for k, a in log.arrays()}
    out = [torch.empty(args.scen, dtype=torch.float64, device=dev) for _ in range(3)]
    m = log.fill(lambda a: None, [o.data_ptr() for o in out])
    for k, t in d.items():
        setattr(m, k, t.data_ptr())
    stream = torch.cuda.current_stream(dev)
    eng._set_stream(stream.cuda_stream)
    for _ in range(3):
        eng._check(eng.lib.pvt_meter(eng.ctx, ctypes.addressof(m)))
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(args.steps):
        eng._check(eng.lib.pvt_meter(eng.ctx, ctypes.addressof(m)))
    b.record(stream)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / args.steps
    t0 = time.perf_counter()
    want, rc = oracle.meter(log)
    cpu_s = time.perf_counter() - t0
    assert rc == _abi.PVT_OK
    for o, k in zip(out, ("instance_hours", "egress_cost", "congestion_delay")):
        np.testing.assert_allclose(o.cpu().numpy(), want[k], rtol=1e-9, atol=0)
    nbytes = (16 * len(log.iv_start) + 24 * len(log.tr_size) + 8 * (len(log.iv_off) +
              len(log.pkt_off) + len(log.tr_off)) + 8 * len(log.route_cost))
    print(json.dumps({"metric": "meter aggregates (pvt_meter)", "scenarios": args.scen,
                      "intervals": len(log.iv_start), "transfers": len(log.tr_size),
                      "ms_per_launch": ms, "scenarios_per_s": args.scen / ms * 1e3,
                      "algorithmic_GBps": nbytes / ms * 1e-6,
                      "cpu_baseline": {"scenarios_per_s": args.scen / cpu_s, "cores": 1,
                                       "kind": "port", "sample": "oracle_meter on the batch"},
                      "note": "ms includes the synchronous call's argument checks and error-"
                              "count read-back"}))


if __name__ == "__main__":
    main()
