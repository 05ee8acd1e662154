import os, sys, time, numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import rasr_amd as ra
ms = ra.synthetic_mixture_set(5000, 160, 39, seed=2024)
fr = torch.from_numpy(ra.synthetic_frames(8192, 39, seed=1)).cuda()
out = torch.empty((5000, 8192), dtype=torch.float32, device="cuda"); best = torch.empty((5000, 8192), dtype=torch.int32, device="cuda")
for kind in ["diagonal-maximum", "batch-diagonal-maximum-float"]:
    sc = ra.Scorer(ms, kind, max_frames=8192, reference_order=True)
    sc.score_device(fr, out, best); torch.cuda.synchronize()
    t = time.time(); n = 5
    for _ in range(n): sc.score_device(fr, out, best)
    torch.cuda.synchronize(); dt = (time.time() - t) / n
    print(os.path.basename(os.environ.get("RASR_GMM_LIB", "default")), kind, "%.2f ms per 8192 frames = %.3f M frames/s, checksum %.6f" % (dt * 1e3, 8192 / dt / 1e6, float(out[:, :64].double().sum())))
