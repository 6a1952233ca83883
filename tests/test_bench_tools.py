"""CPU checks of bench.py's measurement helpers (no GPU): the config-1/2 replay of recorded
reference simulations through the drop-in classes, and the PMC index bench.py reads (entries of
another build are not used)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_replay_config1_on_the_cpu_restatement():
    """Every round of the recorded config-1 simulation through CostAwareGlobalScheduler with the
    C restatement behind the engine contract: the reference's placements in every round."""
    secs, cand, rounds, ok, tr = bench._replay("sim_c1_cost_aware", bench._OracleEngine(0))
    assert ok and rounds == 415 and cand == 7634 * 100
    assert tr["n_hosts"] == 100 and secs > 0


def test_pmc_index_and_binary_check(tmp_path, monkeypatch):
    prof = {"kernel": "pvt::zwalk_kernel<false, false>(pvt::ZwalkArgs)",
            "probe": ["tools/walk_probe.py", "--mode", "ca_bf", "--reps", "3"],
            "lib_sha256": "0" * 64,
            "counters_per_launch": {"SQ_INSTS_VALU": 300.0, "SQ_INSTS_SALU": 100.0,
                                    "SQ_ACTIVE_INST_ANY": 10.0, "SQ_WAVE_CYCLES": 20.0,
                                    "SQ_WAIT_ANY": 5.0, "SQ_WAVES": 32.0, "dispatches_sq": 6}}
    src = tmp_path / "pmc.json"
    src.write_text(json.dumps(prof))
    idx = tmp_path / "index.json"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_index.py"), str(idx),
                          "ca_bf:1000:10:%s" % src], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    entry = json.loads(idx.read_text())["entries"]["ca_bf_1000_10:zwalk_kernel"]
    assert entry["launches_per_round"] == 2.0
    monkeypatch.setattr(bench, "PMC_INDEX", str(idx))
    e, note = bench.pmc_entry(bench.MODES["ca_bf"], 1000, 10, "zwalk_kernel")
    if os.path.exists(bench.LIB):     # another build's profile: not used
        assert e is None and "another build" in note
    monkeypatch.setattr(bench, "lib_sha256", lambda: "0" * 64)
    e, note = bench.pmc_entry(bench.MODES["ca_bf"], 1000, 10, "zwalk_kernel")
    assert e is not None and note is None
    k = {"ms": 1.0, "launches": 1}
    rl = bench.walk_roofline(bench.MODES["ca_bf"], 1000, 10, k, {"longest_chain_tasks": 10}, 1)
    assert rl["instructions_per_task"] == pytest.approx(400.0 * 2 / 10)
    # zwalk_kernel: 4 waves per workgroup, all of them counted and all of them issuing
    assert rl["frac"] == pytest.approx(80.0 * (10 / 1e-3) / (4 * 2.4e9 / 4))
    assert rl["frac_one_wave"] == pytest.approx(80.0 * (10 / 1e-3) / (2.4e9 / 4))
    # the dominant kernel is the one with the most HIP-event time, whatever its class
    ks = {"kernels": {"zwalk_kernel": {"ms": 1.0, "launches": 1},
                      "merge_small_kernel": {"ms": 0.2, "launches": 3}}}
    rl = bench.dominant_roofline(bench.MODES["ca_bf"], 1000, 10, ks, {"longest_chain_tasks": 10}, 1)
    assert rl["kernel"] == "zwalk_kernel" and rl["frac"] == pytest.approx(80.0 * 1e4 / 2.4e9)
    assert rl["dominant_share_of_timed_kernels"] == pytest.approx(1.0 / 1.2)


def test_pmc_index_variant_keys(tmp_path, monkeypatch):
    """Batch (config 4) and loaded (config 5) profiles are indexed under their own keys, and the
    kernel name is matched whole (commit_kernel is not opp_commit_kernel)."""
    idx = tmp_path / "index.json"
    specs = []
    for name, kern in (("a", "void pvt::resident_kernel<1, 4>(pvt::ResidentArgs)"),
                       ("b", "void pvt::opp_commit_kernel(pvt::OppCommitArgs)")):
        src = tmp_path / ("%s.json" % name)
        src.write_text(json.dumps({"kernel": kern, "probe": ["--reps", "2"], "lib_sha256": "1" * 64,
                                   "counters_per_launch": {"dispatches_sq": 2}}))
        specs.append(src)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_index.py"), str(idx),
                          "ca_bf:1000:1000_b512:%s" % specs[0], "opp:100000:1000:%s" % specs[1]],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    keys = set(json.loads(idx.read_text())["entries"])
    assert keys == {"ca_bf_1000_1000_b512:resident_kernel", "opp_100000_1000:opp_commit_kernel"}
    monkeypatch.setattr(bench, "PMC_INDEX", str(idx))
    monkeypatch.setattr(bench, "lib_sha256", lambda: "1" * 64)
    e, _ = bench.pmc_entry(bench.MODES["ca_bf"], 1000, 1000, "resident_kernel", "_b512")
    assert e is not None
    e, _ = bench.pmc_entry(bench.MODES["opp"], 100000, 1000, "commit_kernel")
    assert e is None
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_profile
    assert pmc_profile.base_name("void pvt::opp_commit_kernel(pvt::OppCommitArgs)") == "opp_commit_kernel"
    assert pmc_profile.base_name("void pvt::zwalk_kernel<true, false>(pvt::ZwalkArgs)") == "zwalk_kernel"


def _full_out(world=1):
    """A full-size bench.py result as main() builds it at N = world: every extra line with its
    kernel times, long roofline / CPU-baseline dicts and notes (the sizes of BENCH_r04's)."""
    long_note = "x" * 330
    roof = {"kernel": "zwalk_kernel", "bound": "issue", "unit": "instructions/s (one workgroup)",
            "traffic": 4168352.0, "walk_ms_per_step": 0.18233333333333, "critical_path_tasks": 1525,
            "peak_basis": long_note, "achieved": 3.4123456789e8, "peak": 2.4e9,
            "frac": 0.14212345678, "frac_one_wave": 0.56812345, "cycles_per_task": 291.2345678,
            "latency_floor": {"peak_tasks_per_s": 4.8e7, "achieved_tasks_per_s": 8.37e6,
                              "frac": 0.174}, "instructions_per_task": 40.712345678,
            "pmc_source": "profiles/r05a/pmc_r05a_c5_ca_bf_loaded_zwalk_kernel.json",
            "pmc_lib_sha256": "b" * 64, "issue_active_frac_pmc": 0.43712345,
            "wait_frac_pmc": 0.515123, "waves_per_launch": 32.0,
            "dominant_share_of_timed_kernels": 0.912345678}
    cpu = {"value": 1.75123456789e9, "unit": "candidates/s", "cores": 16, "kind": "port",
           "value_1thread": 1.6123456789e8, "sample": long_note}
    kern = {"zwalk_kernel": 0.18212345, "epoch_validate_kernel": 0.0061234, "score_kernel": 0.1,
            "merge_path_kernel": 0.2, "lwalk_kernel": 0.3}
    extra = {}
    tags = [] if world > 1 else (["c5_%s" % m for m in ("ca_ff", "opp", "vbp_ff", "vbp_bf")] + ["c5_ca_bf_loaded"]
            + ["c3_%s" % m for m in bench.MODES] + ["c4_%s" % m for m in bench.MODES])
    for t in tags:
        extra[t] = {"value": 3.5123456789e13, "ms_per_step": 0.2912345678, "hosts": 1000000,
                    "tasks": 10000, "steps": 5, "parity": True,
                    "kernels_ms_per_step": {"score": 0.1, "merge": 0.2, "commit": 0.3, "other": 0.4},
                    "kernel_ms_per_step": dict(kern),
                    "roofline": dict(roof, pmc_source="profiles/r05a/pmc_r05a_%s_zwalk_kernel.json"
                                     % t), "cpu_baseline": dict(cpu),
                    "hbm_GBs_measured": 15.123456789, "hbm_frac_measured": 0.0019,
                    "hbm_bytes_per_step": 4.1e6, "hbm_pmc_source": "profiles/r05a/x.json"}
    for t in tags:
        if t.startswith("c4"):
            extra[t]["scenarios"] = 512
    for t in ("c1_replay_cost_aware", "c2_replay_cost_aware", "c2_replay_opportunistic",
              "c2_replay_vbp_ff", "c2_lockstep") if world == 1 else ():
        extra[t] = {"workload": long_note, "rounds": 2145, "candidates": 84820000.0,
                    "value": 42338040.15905987, "unit": "candidates/s", "seconds": 2.0033992995,
                    "ms_per_round": 0.9339856874471256, "parity": True, "engine_seconds": 2.2397,
                    "max_rounds_per_launch": 6, "cpu_1thread": {"seconds": 1.9, "value": 4.3e7},
                    "cpu_baseline": dict(cpu), "note": long_note,
                    "roofline": {"kernel": None, "bound": "round trip", "unit": "rounds/s",
                                 "achieved": 1070.68, "peak": 33794.15, "frac": 0.0316824,
                                 "traffic": None, "peak_basis": long_note}}
    if world > 1:
        extra["c4_scenarios_ca_bf_x%d" % world] = {
            "workload": long_note, "value": 5.2e11 * world, "unit": "candidates/s",
            "ms_per_step": 0.97123, "n_gpus": world, "scenarios": 512 * world,
            "scenarios_per_gpu": 512, "hosts": 1000, "tasks": 1000, "steps": 5, "scaling": "weak",
            "timing": long_note, "parity": True, "parity_scope": long_note,
            "kernels_ms_per_step": {"score": 0.1}, "kernel_ms_per_step": dict(kern),
            "roofline": dict(roof, kernel="resident_kernel", bound="valu",
                             pmc_source="profiles/r05a/pmc_r05a_c4_ca_bf_resident_kernel.json")}
    return {"metric": bench.METRIC, "value": 3.6617021276595e13, "unit": "candidates/s",
            "n_gpus": world, "steps": 20, "warmup": 5, "ms_per_step": 0.2731234567,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (SURVEY.md §8(d): trace demand rows, 20 locality.yml zones, seeded)",
            "config": {"workload": "synthetic 1000000 hosts x 10000 ready tasks per round, 20 zones,"
                                   " cost_aware best-fit, one independent scenario per GPU",
                       "scenarios_per_gpu": 1, "hosts": 1000000, "tasks_per_round": 10000,
                       "zones": 20, "policy": "ca_bf",
                       "parallelism": "scenario-sharded x%d (no data-path collective)" % world,
                       "dist_backend": "nccl" if world > 1 else None},
            "roofline": dict(roof), "cpu_baseline": dict(cpu),
            "kernels_ms_per_step": {"score": 0.0, "merge": 0.0, "commit": 0.18, "other": 0.05},
            "kernel_ms_per_step": dict(kern), "walk_us_per_task": 0.0182,
            "windows_per_step": 0, "refills_per_step": 0, "epochs_per_step": 1,
            "segments_per_step": 20, "rejected_segments_per_step": 0,
            "frontier_chains_per_step": 8, "list_chains_per_step": 0, "parity": True,
            "hbm_GBs_measured": 15.26, "hbm_frac_measured": 0.0019, "hbm_bytes_per_step": 4.17e6,
            "hbm_pmc_source": "profiles/r05a/pmc_r05a_c5_ca_bf_step.json", "extra": extra}


@pytest.mark.parametrize("world", [1, 8])
def test_bench_line_fits_the_driver(world):
    """The printed line stays under 8 KB with every extra (a 33 KB line went
    unparsed) and keeps, per extra, value / time / parity / roofline / CPU baseline -- at the
    full level, PMC source included."""
    out = _full_out(world)
    line = bench.compact_line(out, "gpurun_out/bench_full.json")
    assert len(line) <= 8192 and "\n" not in line
    res = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline", "parity", "hbm_GBs_measured"):
        assert k in res, k
    assert res["value"] == out["value"] and res["ms_per_step"] == out["ms_per_step"]
    assert res["full_results"] == "gpurun_out/bench_full.json"
    for k in ("kernel", "bound", "achieved", "peak", "frac", "traffic", "pmc_source"):
        assert k in res["roofline"], k
    assert set(res["extra"]) == set(out["extra"])
    for tag, e in res["extra"].items():
        assert e["parity"] is True and e["value"] > 0, tag
        assert "frac" in e["roofline"], tag
        if out["extra"][tag].get("roofline", {}).get("pmc_source"):
            assert e["roofline"]["pmc_source"].startswith("r05a"), tag
        if "cpu_baseline" in out["extra"][tag]:
            assert e["cpu_baseline"]["value"] > 0 and e["cpu_baseline"]["cores"] == 16, tag
    if world > 1:
        c4 = res["extra"]["c4_scenarios_ca_bf_x%d" % world]
        assert c4["n_gpus"] == world and c4["scenarios"] == 512 * world


def test_bench_line_degrades_instead_of_growing():
    """More extras than the line can hold: the cut gets coarser, the line stays parseable."""
    out = _full_out(1)
    for i in range(60):
        out["extra"]["more_%d" % i] = dict(out["extra"]["c5_opp"])
    line = bench.compact_line(out)
    assert len(line) <= bench.LINE_MAX or len(json.loads(line)["extra"]) == len(out["extra"])
    assert json.loads(line)["extra"]["more_59"]["parity"] is True
