"""The RASR-side adapter (integration/rasr/Mm/GpuFeatureScorer.{hh,cc}) is real source: it compiles
-fsyntax-only against the reference's own Mm/Core headers with the reference's compiler flags
(`make check-integration`).  Runs where the reference tree is present (this container), skipped elsewhere."""
import os
import subprocess

import numpy as np
import pytest

import oracle
import rasr_amd as ra

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/Mm"), reason="reference tree absent")
def test_adapter_compiles_against_reference_headers():
    r = subprocess.run(["make", "-s", "-C", ROOT, "check-integration"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "adapters compile" in r.stdout


def test_adapter_registers_every_type():
    """Every type the library serves is registered by the adapter (under "gpu-" + the reference name)."""
    from rasr_amd import _capi
    src = open(os.path.join(ROOT, "integration", "rasr", "Mm", "GpuFeatureScorer.cc")).read()
    for name in _capi.SCORER_TYPES:
        assert f'"{name}"' in src, name


@pytest.mark.parametrize("dim", [39, 45, 33])
def test_batch_fast_restatement_is_batch_int_at_48(dim):
    """At padded dimension 48 the unrolled scorer's fixed 48-byte stride equals the layout: batch-int's scores."""
    ms = ra.synthetic_mixture_set(30, ra.ragged_counts(30, 300, low=1, high=20, seed=dim), dim, seed=dim,
                                  weights="random")
    frames = ra.synthetic_frames(50, dim, seed=dim + 2)
    a = oracle.batch_fast_score(ms, frames)
    b = oracle.batch_int_score(ms, frames)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("dim", [16, 32])
def test_batch_fast_restatement_refuses_small_dimensions(dim):
    ms = ra.synthetic_mixture_set(3, 4, dim, seed=1)
    with pytest.raises(ValueError):
        oracle.batch_fast_score(ms, ra.synthetic_frames(2, dim, seed=1))


def test_adapter_linked_and_run_in_plugin_harness():
    """integration/rasr/Mm/GpuFeatureScorer.cc linked with the real host classes inside test doubles of RASR's
    plugin machinery (tests/rasr_harness/include/README) over an oracle-backed stand-in of the C-ABI, and driven
    through FeatureScorerFactory, FeatureScorerScaling, the OfflineRecognizer (search and aligner reads) and
    FeatureScorerNode call sequences at buffer sizes 1, 4, 64 and 512 (make check-integration-link): every scaled
    score and best density equals the oracle's, "density-shard-devices" reaches gmm_scorer_create_sharded, and a
    type without assignments routes bestDensity() to the component's criticalError."""
    r = subprocess.run(["make", "-s", "-C", ROOT, "check-integration-link"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "PASSED (0 failures)" in r.stdout
    assert r.stdout.count("score dump") == 14 and r.stdout.count("recognizer ") == 23 and "DIFFER" not in r.stdout
    assert "density-shard-devices 0,1,2 -> gmm_scorer_create_sharded over 3 devices" in r.stdout
    assert "component criticalError, abort" in r.stdout


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_adapter_over_product_library_on_gpu(gpu):
    """The same adapter and harness linked against the PRODUCT library librasr_gmm.so (the HIP kernels; the oracle
    is only the checker), run on the GPU: registerGpuFeatureScorers -> FeatureScorerFactory -> FeatureScorerScaling,
    the recognizer sequence (search: score(e); aligner: score(e) + bestDensity(e)) and the FeatureScorerNode dump at
    buffer sizes 1, 4, 64 and 512 (512 and 64: the asynchronous prefetch), and density-shard-devices 0,0,0 (three
    density parts on one GPU, the copy exchange).  SIMD and batch-int: every scaled score and best density bit for
    bit; float types within 1e-4 relative, best densities equal except at near ties (both f64 scores within 1e-4)."""
    exe = os.path.join(ROOT, "build", "tests", "rasr_adapter_harness_gpu")
    assert os.path.exists(exe), "build it with make (it travels with the tree)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=540)
    out = r.stdout
    assert r.returncode == 0, out[-4000:] + r.stderr[-3000:]
    assert "adapter over librasr_gmm.so (HIP)" in out
    assert "PASSED (0 failures)" in out and "DIFFER" not in out
    assert out.count("score dump") == 14 and out.count("recognizer ") == 27
    assert out.count("density-shard-devices 0,0,0") == 5
    for t in ("SIMD-diagonal-maximum", "batch-diagonal-maximum-int"):  # the exact types stay exact
        assert all("within" not in line for line in out.splitlines() if f" {t} " in line)
    print(out)
