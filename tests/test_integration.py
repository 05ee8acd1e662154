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
    through FeatureScorerFactory, FeatureScorerScaling, the OfflineRecognizer and FeatureScorerNode call
    sequences at buffer sizes 1, 4 and 64 (make check-integration-link): every scaled score and best density
    equals the oracle's, "density-shard-devices" reaches gmm_scorer_create_sharded, and a type without assignments
    routes bestDensity() to the component's criticalError."""
    r = subprocess.run(["make", "-s", "-C", ROOT, "check-integration-link"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "PASSED (0 failures)" in r.stdout
    assert r.stdout.count("score dump") == 10 and r.stdout.count("recognizer ") == 11 and "DIFFER" not in r.stdout
    assert "density-shard-devices 0,1,2 -> gmm_scorer_create_sharded over 3 devices" in r.stdout
    assert "component criticalError, abort" in r.stdout
