"""bench.py --gpus N launches N ranks by itself (torch.distributed.run as a child process) when it is not
already running under a torch.distributed launcher; RASR_BENCH_LAUNCH_PROBE makes every rank report its
environment and stop before any GPU work, so this runs on CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, probe_dir):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["RASR_BENCH_LAUNCH_PROBE"] = str(probe_dir)  # every rank writes rank<R>.json there
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       env=env, timeout=240)
    recs = [json.loads(p.read_text()) for p in sorted(probe_dir.glob("rank*.json"))]
    return r, recs


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_starts_n_ranks(n, tmp_path):
    r, recs = _run(["--gpus", str(n), "--steps", "1", "--warmup", "0"], tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sorted(x["rank"] for x in recs) == list(range(n))
    assert all(x["world_size"] == n and x["gpus"] == n for x in recs)
    assert sorted(x["local_rank"] for x in recs) == list(range(n))


def test_single_gpu_runs_in_process(tmp_path):
    r, recs = _run(["--gpus", "1"], tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert recs == [{"rank": 0, "world_size": 1, "local_rank": 0, "gpus": 1}]


def test_host_leg_all_ranks_gloo(tmp_path):
    """The N > 1 host leg's aggregation (bench.host_leg_record) over a real gloo process group of 3 ranks: every rank
    sees every rank's rate, the aggregate divides all ranks' frames by the slowest rank's time."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["RASR_BENCH_LAUNCH_PROBE"] = str(tmp_path)
    env["RASR_BENCH_PROBE_HOST_LEG"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], capture_output=True,
                       text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = [json.loads(p.read_text()) for p in sorted(tmp_path.glob("rank*.json"))]
    assert len(recs) == 3
    for x in recs:
        leg = x["host_leg"]
        assert leg["ranks"] == 3 and leg["backend"] == "gloo"
        assert leg["per_rank_frames_per_s"] == pytest.approx([3000 / 0.1, 3000 / 0.2, 3000 / 0.3])
        assert leg["value"] == pytest.approx(3 * 3000 / 0.3)
