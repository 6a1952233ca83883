#!/usr/bin/env python3
"""Diagnostic: the host side of the last N ms of a `rocprofv3 --hip-trace --kernel-trace
--output-format csv` run -- every HIP API call of the main thread in order with its duration and
the host time before it (time spent outside the runtime), plus the kernels that ran meanwhile.
usage: api_timeline.py HIP_API_TRACE_CSV KERNEL_TRACE_CSV [LAST_MS]"""
import csv
import sys

api_path, k_path = sys.argv[1], sys.argv[2]
last_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
api = []
with open(api_path) as f:
    for r in csv.DictReader(f):
        api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r.get("Thread_Id", "")))
ker = []
with open(k_path) as f:
    for r in csv.DictReader(f):
        ker.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40]))
api.sort()
ker.sort()
t_end = max(e for _, e, _, _ in api)
t0 = t_end - last_ms * 1e6
main_tid = max(set(t for _, _, _, t in api), key=lambda t: sum(1 for a in api if a[3] == t))
prev_end = None
host_gap = 0.0
for s, e, fn, tid in api:
    if s < t0 or tid != main_tid:
        continue
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    host_gap += gap
    ks = [k for k in ker if k[0] < e and k[1] > s]
    print("%9.1f us  +%7.1f host  %-32s %8.1f us  %s" % ((s - t0) / 1e3, gap, fn[:32], (e - s) / 1e3,
                                                      ", ".join(k[2] for k in ks)[:80]))
    prev_end = e
print("host time between API calls: %.1f us" % host_gap)
