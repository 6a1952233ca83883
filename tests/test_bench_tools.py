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
