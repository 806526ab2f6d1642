"""bench.py's N-rank GPU branch for real on a one-GPU box:
two ranks share device 0 over gloo (SFM_BENCH_SHARED_GPU=1), each runs the
full HIP step on its own pairs, and rank 0 reports the gathered rows.  The
driver's SCALE run uses the same code with RCCL and one GPU per rank; only
the backend and the device index differ (bench.rank_device_index)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(args, shared):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "SFM_BENCH_CPU_STUB"):
        env.pop(k, None)
    if shared:
        env["SFM_BENCH_SHARED_GPU"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_two_ranks_share_the_gpu():
    common = ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-regularize", "--config", "c3"]
    two = _bench(["--gpus", "2"] + common, shared=True)
    assert two["n_gpus"] == 2 and two["dist"]["world_size"] == 2 and two["dist"]["backend"] == "gloo"
    assert "rehearsal" in two
    assert two["config"]["global_batch"] == 8 and two["gathered"]["pairs"] == 8
    assert two["gathered"]["per_rank"] == [4, 4]
    one = _bench(common, shared=False)
    assert "rehearsal" not in one and one["n_gpus"] == 1
    # rank 0's pairs are the single process's pairs (seed 1000 + rank): same inliers
    assert two["inliers"][:4] == one["inliers"]
    assert all(v > 0 for v in two["inliers"])
