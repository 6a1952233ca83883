#!/usr/bin/env python3
"""rocprofv3 PMC profile of one kernel of the engine (run on the GPU box; never touches the GPU
itself: every pass is a child `rocprofv3 --pmc ... -- python <probe>` under a hard time limit).

Passes (one counter set each; gfx950 slot limits, MI355X_MICROARCH.md §rocprofv3 PMC slots:
8 SQ, 4 TCC -- FETCH_SIZE takes 3, WRITE_SIZE 2 --, 2 GRBM per pass):
  a      SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE
         SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE + FETCH_SIZE
  b      SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY
         SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS + WRITE_SIZE
(the older four-pass split sq / sq2 / fetch / write is still accepted by --passes)
Counters missing from `rocprofv3 -L` (gpurun_out/counters.txt, when present) are dropped.

Per dispatch of the kernels whose name contains --kernel, every counter is summed over its rows
(XCDs / instances), then averaged over dispatches. Derived per launch:
  valu_busy_cycles  = SQ_ACTIVE_INST_VALU x 4 (quad-cycles; MI355X_MICROARCH.md constants table)
  lds_busy_cycles   = SQ_LDS_IDX_ACTIVE (LDS-array cycles)
  hbm_bytes         = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B; gfx950 FETCH_SIZE reads half of a
                      wide streaming read, MI355X_MICROARCH.md §HBM)
  clock_ghz         = GRBM_GUI_ACTIVE / 8 / duration (effective clock, §DVFS)
Peaks: 1024 SIMDs x 2.4 GHz of VALU issue cycles; 256 CUs x 2.4 GHz of LDS-array cycles.

    python tools/pmc_profile.py --tag r02 --kernel score_kernel -- tools/score_probe.py --mode ca_bf
Writes gpurun_out/pmc_<tag>_<kernel>.json and .csv for every listed kernel the probe launched.
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pivot-scheduling_amd", "pivot_place", "libpivot_place.so")


def lib_sha256(path=LIB):
    """sha256 of the engine library the probe loads: bench.py uses a PMC profile only for the
    binary it was collected on."""
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()
PASSES = {
    "sq": ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE",
           "SQ_LDS_BANK_CONFLICT", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
    "sq2": ["SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAIT_ANY",
            "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS"],
    "fetch": ["FETCH_SIZE"],
    "write": ["WRITE_SIZE"],
}
PASSES["a"] = PASSES["sq"] + PASSES["fetch"]
PASSES["b"] = PASSES["sq2"] + PASSES["write"]
SIMDS, CUS, CLOCK = 1024, 256, 2.4e9


def known_counters():
    path = os.path.join(ROOT, "gpurun_out", "counters.txt")
    if not os.path.exists(path):
        return None
    return open(path).read()


def run_pass(name, counters, tag, probe, secs):
    out_dir = os.path.join(ROOT, "gpurun_out", "pmc_%s_%s" % (tag, name))
    cmd = ["timeout", "-s", "KILL", str(secs), "rocprofv3", "--pmc"] + counters + [
        "--output-format", "csv", "-d", out_dir, "-o", "pmc", "--", sys.executable] + probe
    print("pass %s: %s" % (name, " ".join(counters)), flush=True)
    subprocess.run(cmd, check=True, env=dict(os.environ, TMPDIR="/tmp"), timeout=secs + 30)
    files = glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise RuntimeError("no counter_collection.csv under %s" % out_dir)
    return files[0]


def base_name(name):
    """The __global__ function's own name: 'void pvt::zwalk_kernel<true, false>(pvt::ZwalkArgs)'
    -> 'zwalk_kernel' (so 'commit_kernel' does not match opp_commit_kernel)."""
    return name.split("(")[0].split("<")[0].split("::")[-1].split(" ")[-1]


def parse(path, kernel):
    """{dispatch: {counter: value summed over rows}}, {dispatch: kernel name}, {dispatch: ns}."""
    vals, names, dur = {}, {}, {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if base_name(name) != kernel:
                continue
            d = row.get("Dispatch_Id")
            c = row.get("Counter_Name")
            vals.setdefault(d, {})
            vals[d][c] = vals[d].get(c, 0.0) + float(row["Counter_Value"])
            names[d] = name
            try:
                dur[d] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
            except (KeyError, ValueError):
                pass
    return vals, names, dur


def summarise(kname, avg, durs, probe, cand):
    dur_s = (sum(durs) / len(durs)) * 1e-9 if durs else None
    out = {"kernel": kname, "probe": probe, "lib_sha256": lib_sha256(), "counters_per_launch": avg,
           "profiled_duration_ms": dur_s * 1e3 if dur_s else None}
    if "SQ_ACTIVE_INST_VALU" in avg:
        out["valu_busy_cycles_per_launch"] = 4.0 * avg["SQ_ACTIVE_INST_VALU"]
    if "SQ_LDS_IDX_ACTIVE" in avg:
        out["lds_busy_cycles_per_launch"] = avg["SQ_LDS_IDX_ACTIVE"]
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        out["hbm_bytes_per_launch"] = (2.0 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
    out["valu_peak_cycles_per_s"] = SIMDS * CLOCK
    out["lds_peak_cycles_per_s"] = CUS * CLOCK
    if dur_s:
        if "GRBM_GUI_ACTIVE" in avg:
            out["clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8.0 / dur_s / 1e9
        for k, peak in (("valu_busy_cycles_per_launch", SIMDS * CLOCK),
                        ("lds_busy_cycles_per_launch", CUS * CLOCK)):
            if k in out:
                out[k.replace("_cycles_per_launch", "_frac_profiled")] = out[k] / dur_s / peak
        if "hbm_bytes_per_launch" in out:
            out["hbm_frac_profiled"] = out["hbm_bytes_per_launch"] / dur_s / 8.0e12
    if cand:
        out["candidates_per_launch"] = cand
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r02")
    ap.add_argument("--kernel", default="score_kernel",
                    help="kernel name substring; several, comma-separated, are taken from the same "
                         "passes (one pmc_<tag>_<kernel>.json each)")
    ap.add_argument("--passes", default="a,b")
    ap.add_argument("--secs", type=int, default=90)
    ap.add_argument("--candidates-per-launch", type=float, default=0.0)
    ap.add_argument("probe", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    probe = [x for x in a.probe if x != "--"]
    probe[0] = os.path.join(ROOT, probe[0]) if not os.path.isabs(probe[0]) else probe[0]
    kernels = a.kernel.split(",")
    listing = known_counters()
    avg = {k: {} for k in kernels}
    kname = {k: None for k in kernels}
    durs = {k: [] for k in kernels}
    for name in a.passes.split(","):
        counters = PASSES[name]
        if listing is not None:
            counters = [c for c in counters if c in listing]
        if not counters:
            continue
        path = run_pass(name, counters, a.tag, probe, a.secs)
        for kern in kernels:
            vals, names, dur = parse(path, kern)
            if not vals:     # (a candidate kernel this workload never launches)
                print("pass %s: no dispatch of %s" % (name, kern), flush=True)
                continue
            kname[kern] = kname[kern] or sorted(set(names.values()))[0]
            for c in counters:
                xs = [v[c] for v in vals.values() if c in v]
                if xs:
                    avg[kern][c] = sum(xs) / len(xs)
            durs[kern] += list(dur.values())
            avg[kern].setdefault("dispatches_" + name, len(vals))
            avg[kern].setdefault("dispatches_sq", len(vals))   # (pmc_index: launches per round)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    if not any(kname.values()):
        raise RuntimeError("no dispatch of any of %s" % a.kernel)
    for kern in kernels:
        if kname[kern] is None:
            continue
        out = summarise(kname[kern], avg[kern], durs[kern], probe, a.candidates_per_launch)
        stem = "pmc_%s_%s" % (a.tag, kern)
        with open(os.path.join(ROOT, "gpurun_out", stem + ".json"), "w") as f:
            json.dump(out, f, indent=1)
        with open(os.path.join(ROOT, "gpurun_out", stem + ".csv"), "w") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "counter", "value_per_launch"])
            for c, v in sorted(avg[kern].items()):
                w.writerow([kname[kern], c, v])
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
