import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out", "bb_*.log"))):
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(os.path.basename(f), "no result"); continue
    d = json.loads(lines[-1])
    print("%-18s %.3g cand/s  ms/step %.3f  kernel %.3f ms" % (os.path.basename(f)[3:-4], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"]))
