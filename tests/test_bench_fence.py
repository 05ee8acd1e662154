"""bench.py --gpus N cannot lose its JSON line to the checks of never-executed multi-GPU paths ("do
this" 1).  RASR_BENCH_FENCE_PROBE=1 runs the real N > 1 orchestration -- the ranks' process group, the fenced
children (the density-sharded check as N fresh ranks, the C-ABI sharded check as one process), their timeouts and
kills, the deadline watchdog and the line -- over gloo on the CPU with a synthetic headline and synthetic check
payloads; RASR_BENCH_INJECT puts a hang or an exception into one rank.  In every case the launcher must print
exactly one line, with the failed check reported as an error, within the bound, and exit 0."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FENCE_S = 12  # RASR_BENCH_FENCE_TIMEOUT_S for these runs


def _run(n, inject=None, deadline=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["RASR_BENCH_FENCE_PROBE"] = "1"
    env["RASR_BENCH_FENCE_TIMEOUT_S"] = str(FENCE_S)
    env.pop("RASR_BENCH_INJECT", None)
    if inject:
        env["RASR_BENCH_INJECT"] = inject
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)]
    if deadline:
        args += ["--deadline", str(deadline)]
    t0 = time.monotonic()
    r = subprocess.run(args, capture_output=True, text=True, env=env, timeout=240)
    dt = time.monotonic() - t0
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    return r, lines, dt


def _line(r, lines):
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["value"] == 1.0 and line["n_gpus"] >= 2
    return line


@pytest.mark.parametrize("n", [2, 3])
def test_fenced_checks_clean(n):
    r, lines, _ = _run(n)
    line = _line(r, lines)
    assert line["density_sharded"]["ranks"] == n and line["density_sharded"]["sum"] == n
    assert line["density_sharded_capi"]["probe"] is True
    assert line["density_sharded_capi"]["devices"] == ",".join(str(d) for d in range(n))
    assert "deadline" not in line


def test_density_check_rank_raises():
    r, lines, dt = _run(2, "raise@1")
    line = _line(r, lines)
    err = line["density_sharded"]["error"]
    assert "rank 1 exited" in err and "injected fault" in err, err
    assert line["density_sharded_capi"]["probe"] is True  # the next check still ran
    assert dt < 120


def test_density_check_rank_hangs():
    r, lines, dt = _run(2, "hang@1")
    line = _line(r, lines)
    err = line["density_sharded"]["error"]
    assert "timed out" in err and "[1]" in err, err
    assert line["density_sharded"]["wall_s"] < FENCE_S + 5
    assert line["density_sharded_capi"]["probe"] is True
    assert dt < FENCE_S + 120


def test_capi_check_hangs():
    r, lines, dt = _run(2, "capi-hang")
    line = _line(r, lines)
    assert line["density_sharded"]["sum"] == 2
    assert "timed out" in line["density_sharded_capi"]["error"]
    assert dt < FENCE_S + 120


def test_deadline_prints_line_when_a_rank_hangs():
    """Rank 1 of the headline's own ranks hangs after the headline (outside any fenced child): rank 0 waits for it
    on the barrier until the deadline, prints the line with every finished record, and all ranks exit 0."""
    r, lines, dt = _run(2, "parent-hang@1", deadline=40)
    line = _line(r, lines)
    assert line["deadline"]["seconds"] == 40
    assert line["density_sharded"]["sum"] == 2 and line["density_sharded_capi"]["probe"] is True
    assert dt < 40 + 60
