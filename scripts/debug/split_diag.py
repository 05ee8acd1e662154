"""Where do split-kernel scores differ from the oracle? (debug helper, GPU)"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import oracle
import rasr_amd as ra

CASES = [(37, "ragged", 45, 1, "random", 777), (100, 10, 45, 1, "uniform", 300),
         (37, "ragged", 39, 1, "random", 777), (64, 16, 16, 1, "random", 513)]
if os.environ.get("QUICK"):
    CASES = CASES[:1]
for (m, k, d, c, w, f) in CASES:
    if k == "ragged":
        k = ra.ragged_counts(m, m * 20, low=1, high=40, seed=7)
    ms = ra.synthetic_mixture_set(m, k, d, seed=7, n_covariances=c, weights=w)
    frames = ra.synthetic_frames(f, d, seed=13)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=8)
    for native in (False, True):
        sc = ra.Scorer(ms, "diagonal-maximum", max_frames=f, native_f32=native)
        s, b = sc.score_host(frames)
        err = np.abs(s.astype(np.float64) - ref_s) / np.maximum(1, np.abs(ref_s))
        bad = np.argwhere(err > 1e-4)
        print(f"D={d} M={m} native={native} kernel={sc.main_kernel()} maxerr={err.max():.3g} nbad={len(bad)}")
        counts = np.diff(ms.mixture_offsets)
        for e, t in bad[:8]:
            print(f"   mix {e} (K={counts[e]}) frame {t}: gpu {s[e,t]:.6f} (dns {b[e,t]}) ref {ref_s[e,t]:.6f} (dns {ref_b[e,t]})")
        if len(bad):
            print("   bad frames:", np.unique(bad[:, 1])[:20], "bad mixtures:", np.unique(bad[:, 0])[:20])
