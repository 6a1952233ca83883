#!/usr/bin/env python3
"""Diagnostic: the device timeline of a `rocprofv3 --kernel-trace --output-format csv` run --
busy time vs span and the largest idle gaps between consecutive kernels (with the kernels on
either side), over the last N ms of the trace (the timed steps).
usage: trace_gaps.py KERNEL_TRACE_CSV [LAST_MS] [TOP] [END_KERNEL]
END_KERNEL: the window ends at the last launch of the kernel whose name contains it (skips what
runs after the timed steps, e.g. the parity check's copies)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
rows.sort()
end_k = sys.argv[4] if len(sys.argv) > 4 else None
if end_k:
    last = max((i for i, r in enumerate(rows) if end_k in r[2]), default=len(rows) - 1)
    rows = rows[:last + 1]
if last_ms > 0 and rows:
    t_end = max(e for _, e, _ in rows)
    rows = [r for r in rows if r[0] >= t_end - last_ms * 1e6]
if not rows:
    sys.exit("no kernels")
span = max(e for _, e, _ in rows) - rows[0][0]
busy = 0
cur_s, cur_e = rows[0][0], rows[0][1]
for s, e, _ in rows[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print("kernels %d  span %.3f ms  busy %.3f ms  idle %.3f ms" % (len(rows), span / 1e6, busy / 1e6,
                                                              (span - busy) / 1e6))
per = defaultdict(lambda: [0, 0.0])
for s, e, n in rows:
    per[n][0] += 1
    per[n][1] += (e - s) / 1e6
for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:top]:
    print("  %-40s %5d launches %9.3f ms" % (n[:40], c, t))
gaps = []
end = rows[0][1]
prev = rows[0][2]
for s, e, n in rows[1:]:
    if s > end:
        gaps.append((s - end, prev, n))
    if e > end:
        end, prev = e, n
gaps.sort(reverse=True)
tot = defaultdict(lambda: [0, 0.0])
for g, a, b in gaps:
    tot[(a, b)][0] += 1
    tot[(a, b)][1] += g / 1e3
print("idle gaps by (before -> after), total us:")
for (a, b), (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:top]:
    print("  %8.1f us  %4d x  %s -> %s" % (t, c, a[:34], b[:34]))
