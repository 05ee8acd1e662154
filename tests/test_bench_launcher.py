"""bench.py --gpus N launches N ranks by itself (torch.distributed.run as a child process) when it is not
already running under a torch.distributed launcher; RASR_BENCH_LAUNCH_PROBE makes every rank report its
environment and stop before any GPU work, so this runs on CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["RASR_BENCH_LAUNCH_PROBE"] = "1"
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=240)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_starts_n_ranks(n):
    r = _run(["--gpus", str(n), "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == list(range(n))
    assert all(x["world_size"] == n and x["gpus"] == n for x in lines)
    assert sorted(x["local_rank"] for x in lines) == list(range(n))


def test_single_gpu_runs_in_process():
    r = _run(["--gpus", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"rank": 0, "world_size": 1, "local_rank": 0, "gpus": 1}]
