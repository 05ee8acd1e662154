"""CPU: the score-only layout (gmm_prepare.cc buildClassLayout: class tiles split by constant parity over lane
groups, then mixed tiles) against the SCORE_ONLY kernel's arithmetic, emulated on the host
(tests/cpp/class_layout_test.cc): every entry placed once, the parity rules of both tile kinds, and the
kernel's minimum equal to the direct min of 2 dot + Q for random quantized frames (SIMD and batch-int constants,
D = 16 / 39 / 45 / 64, ragged, tiny, empty and 160-density mixtures).  The GPU tests check the kernel itself
against the oracle (tests/test_scores_only.py, tests/test_batch_int_score_only.py)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_class_layout_matches_kernel_arithmetic(built):
    exe = os.path.join(ROOT, "build", "tests", "class_layout_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok")
