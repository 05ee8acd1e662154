#!/usr/bin/env python3
"""Write tests/golden/*.npz: small models + frames with the oracle's outputs frozen.

These fixtures freeze the CPU restatement (oracle/gmm_oracle.c) as computed on the
machine that generated them; they are regression vectors for the oracle and the
product, NOT reference outputs (the reference cannot be built here; see
oracle/gmm_oracle.h: parity unpinned).  The 1/sqrt(var) table depends on the CPU's
rsqrtss (the reference's -ffast-math build uses it), so the table and the CPU
vendor are stored and tests skip when a different rsqrtss is detected.
"""
import os
import platform
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
import rasr_amd as ra  # noqa: E402

CASES = {
    "d39_m12_k10_uniform": dict(n_mixtures=12, densities_per_mixture=10, dimension=39, seed=101),
    "d45_m9_ragged_random": dict(n_mixtures=9, densities_per_mixture=[1, 3, 16, 17, 5, 33, 2, 8, 12],
                                 dimension=45, seed=102, weights="random"),
    "d39_m8_k6_cov3": dict(n_mixtures=8, densities_per_mixture=6, dimension=39, seed=103, n_covariances=3,
                           weights="random"),
    "d16_m5_k4_uniform": dict(n_mixtures=5, densities_per_mixture=4, dimension=16, seed=104),
}


def cpu_vendor():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("vendor_id"):
                return line.split(":")[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    # default tests/golden; `--out DIR` writes a set for another CPU's rsqrtss (e.g. made on the GPU box
    # into gpurun_out/ and committed as tests/golden/cpu_<vendor>/), so the GPU tests there are not skipped
    out = os.path.join(ROOT, "tests", "golden")
    if "--out" in sys.argv:
        out = os.path.abspath(sys.argv[sys.argv.index("--out") + 1])
    os.makedirs(out, exist_ok=True)
    for name, kw in CASES.items():
        ms = ra.synthetic_mixture_set(**kw)
        frames = ra.synthetic_frames(24, ms.dimension, seed=7)
        frames[0] *= 50.0  # clipping
        o = oracle.OracleSimd(ms)
        s, b, raw = o.score(frames)
        fs, fb = oracle.OracleFloat(ms).score(frames)
        arrays = dict(means=ms.means, variances=ms.variances, density_mean=ms.density_mean,
                      density_covariance=ms.density_covariance, mixture_offsets=ms.mixture_offsets,
                      mixture_densities=ms.mixture_densities, mixture_log_weights=ms.mixture_log_weights,
                      frames=frames, simd_scores=s, simd_best=b, simd_raw=raw, simd_isv=o.isv,
                      simd_scaling=np.float32(o.scaling), simd_prepared_mean=o.prepared_mean,
                      simd_constant_weight=o.constant_weight, float_scores=fs, float_best=fb,
                      cpu_vendor=np.array(cpu_vendor()))
        if ms.n_covariances == 1:
            arrays["batch_int_scores"] = oracle.batch_int_score(ms, frames)
            arrays["batch_float_scores"] = oracle.batch_float_score(ms, frames)
        np.savez_compressed(os.path.join(out, name + ".npz"), **arrays)
        print("wrote", name)


if __name__ == "__main__":
    main()
