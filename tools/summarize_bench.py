"""Print one line per bench log under gpurun_out/ (value, ms/step, kernel ms, windows)."""
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench_*.log")):
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no result"); continue
    d = json.loads(lines[-1])
    print("%-34s %7.1f Gcand/s %7.2f ms  %s  win=%d ref=%d" % (
        f.split("/")[-1], d["value"] / 1e9, d["ms_per_step"],
        {k: round(v, 2) for k, v in d["kernels_ms_per_step"].items()}, d["windows_per_step"], d["refills_per_step"]))
