"""bench.py's multi-rank path, before an 8-GPU node runs it: two ranks
started by bench.py itself (--gpus 2, no WORLD_SIZE), both on cuda:0 over gloo -- the launcher,
the process group, the barrier + MAX-over-ranks timing and, with --shard hosts, the
torch.distributed exchange of host-sharded packages. The JSON line must report both ranks and
parity with the CPU restatement."""
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
           "--shard", shard, "--cpu-baseline-seconds", "0", "--extra", "0"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["parity"] is True, res
    assert res["scaling"] == ("strong" if shard == "hosts" else "weak")
    assert res["value"] > 0 and res["config"]["dist_backend"] == "gloo"
