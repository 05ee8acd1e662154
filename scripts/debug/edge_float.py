import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import rasr_amd as ra, oracle
from tests.test_gpu_parity import _edge_model
ms = _edge_model()
frames = ra.synthetic_frames(130, 39, seed=4)
frames[0] *= 1000.0
frames[2] = ms.means[4]
ref_s, ref_b = oracle.OracleFloat(ms).score(frames)
sc = ra.Scorer(ms, "diagonal-maximum", max_frames=130)
s, b = sc.score_host(frames)
om = oracle.OracleFloat(ms)
isv = 1/np.sqrt(ms.variances[0].astype(np.float64))
lnorm = 39*np.log(2*np.pi) + np.log(ms.variances[0].astype(np.float64)).sum()
def dscore(e, j, t):
    d = ms.mixture_densities[ms.mixture_offsets[e] + j]
    x = frames[t].astype(np.float64); m = ms.means[d].astype(np.float64)
    return 0.5*(-2*ms.mixture_log_weights[ms.mixture_offsets[e]+j] + lnorm + (((m-x)*isv)**2).sum())
mism = np.argwhere(b != ref_b)
print("n mism", len(mism))
for e, t in mism[:25]:
    print(e, t, "gpu", b[e,t], "ref", ref_b[e,t], "gpu_s", s[e,t], "ref_s", ref_s[e,t],
          "f64 gpu-choice", dscore(e, b[e,t], t) if b[e,t] < 1000 else None, "f64 ref-choice", dscore(e, ref_b[e,t], t))
err = np.abs(s.astype(np.float64)-ref_s)/np.maximum(1,np.abs(ref_s)); print("max rel", err.max())
