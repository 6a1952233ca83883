"""Print the key fields of bench.py JSON lines found in the given log files."""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = [x for x in open(f) if x.startswith("{")][-1]
    except (OSError, IndexError):
        print(f, "no bench line")
        continue
    d = json.loads(line)
    k = {a: round(b, 3) for a, b in d.get("kernels_ms_per_step", {}).items()}
    print(f, "%.3g" % d["value"], "%.3f ms" % d["ms_per_step"], k, "windows",
          d.get("windows_per_step"), "refills", d.get("refills_per_step"))
