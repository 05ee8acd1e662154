import ctypes, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import rasr_amd as ra
lib = ra.load_library()          # our library (and its libamdhip64) first
import torch
print("torch avail", torch.cuda.is_available())
maps = [l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l]
print(sorted(set(maps)))
ms = ra.synthetic_mixture_set(5, 4, 16, seed=1)
try:
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=8)
    print("scorer ok")
except Exception as e:
    print("scorer failed:", e)
