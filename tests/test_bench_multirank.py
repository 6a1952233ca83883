"""bench.py's multi-rank path, before an 8-GPU node runs it: two ranks
started by bench.py itself (--gpus 2, no WORLD_SIZE), both on cuda:0 over gloo -- the launcher,
the process group, the barrier + MAX-over-ranks timing and, with --shard hosts, the
torch.distributed exchange of host-sharded packages, and the config-4 scenario line every N > 1
run adds (--c4-batch scenarios per rank, MAX-over-ranks timing, parity MIN-reduced). The JSON
line must report both ranks and parity with the CPU restatement."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("mode", ["ca_bf", "vbp_ff", "opp"])
@pytest.mark.parametrize("shard", ["scenarios", "hosts"])
def test_bench_two_ranks_gloo(shard, mode):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--hosts", "20000", "--tasks", "300", "--mode", mode, "--steps", "2", "--warmup", "1",
           "--shard", shard, "--cpu-baseline-seconds", "0", "--extra", "0", "--c4-batch", "16"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    assert len(lines[0]) <= 8192
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["parity"] is True, res
    assert res["scaling"] == ("strong" if shard == "hosts" else "weak")
    assert res["value"] > 0 and res["config"]["dist_backend"] == "gloo"
    c4 = res["extra"]["c4_scenarios_%s_x2" % mode]
    assert c4["parity"] is True and c4["n_gpus"] == 2 and c4["scenarios"] == 32, c4
    # (roofline.frac: when a PMC profile of this binary covers the config)
    assert c4["value"] > 0 and c4["roofline"].get("kernel") == "resident_kernel"


@pytest.mark.parametrize("mode", ["ca_bf", "vbp_bf", "opp"])
def test_bench_two_ranks_scenario_batch(mode):
    """bench.py --gpus 2 --batch 64: each rank places its own 64 scenarios (1000 x 1000) with one
    pvt_place_batch launch per step -- the config-4 workload as the main line."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--hosts", "1000", "--tasks", "1000", "--batch", "64", "--mode", mode, "--steps", "2",
           "--warmup", "1", "--cpu-baseline-seconds", "0", "--extra", "0"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    assert len(lines[0]) <= 8192
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["parity"] is True and res["scaling"] == "weak", res
    assert res["config"]["scenarios_per_gpu"] == 64
    assert abs(res["value"] * res["ms_per_step"] * 1e-3 - 2 * 64 * 1e6) < 1e-3 * 2 * 64 * 1e6


@pytest.mark.timeout(300)
def test_bench_two_ranks_config4_line_fits():
    """The N > 1 line as the driver's scaling runs print it: the default workload plus the
    config-4 scenario line at its full per-GPU batch (--c4-batch 512, 1024 scenarios over two
    ranks): one JSON line of at most 8 KB that parses, with the c4 extra's roofline and parity."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--hosts", "20000", "--tasks", "300", "--steps", "2", "--warmup", "1",
           "--cpu-baseline-seconds", "0", "--extra", "0", "--c4-batch", "512"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and len(lines[0]) <= 8192, out.stdout[-2000:]
    res = json.loads(lines[0])
    c4 = res["extra"]["c4_scenarios_ca_bf_x2"]
    assert c4["parity"] is True and c4["n_gpus"] == 2 and c4["scenarios"] == 1024, c4
    # (roofline.frac: when a PMC profile of this binary covers the config)
    assert c4["value"] > 0 and c4["roofline"].get("kernel") == "resident_kernel", c4
