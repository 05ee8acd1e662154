#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary (gmm_score_host): frames copied in, the score table
(and best densities) copied out, synchronously -- the number DESIGN.md quotes beside bench.py's
HBM-resident `value`.  Also the device-resident rate with the table copied to pinned host memory on a
second stream (what a caller overlapping the D2H with the next batch would see)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rasr_amd as ra  # noqa: E402

F, STEPS = 32768, 5
ms = ra.synthetic_mixture_set(5000, 160, 39, seed=2024)
frames = ra.synthetic_frames(F, 39, seed=7)
out = {}
for kind in ("diagonal-maximum", "SIMD-diagonal-maximum"):
    sc = ra.Scorer(ms, kind, max_frames=F)
    for want_best in (True, False):
        sc.score_host(frames, want_best=want_best)
        t0 = time.perf_counter()
        for _ in range(STEPS):
            sc.score_host(frames, want_best=want_best)
        dt = (time.perf_counter() - t0) / STEPS
        out[f"{kind} host best={want_best}"] = {"frames_per_s": F / dt, "ms_per_step": dt * 1e3}
    # device-resident scoring with the score table streamed to pinned host memory on a copy stream
    dev = torch.device("cuda", 0)
    fr = torch.from_numpy(frames).to(dev)
    bufs = [torch.empty((5000, F), dtype=torch.float32, device=dev) for _ in range(2)]
    host = [torch.empty((5000, F), dtype=torch.float32, pin_memory=True) for _ in range(2)]
    copy = torch.cuda.Stream(dev)
    comp = torch.cuda.current_stream(dev)
    done = [torch.cuda.Event() for _ in range(2)]
    for i in range(2):
        sc.score_device(fr, bufs[i], None, comp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(STEPS * 2):
        b = i % 2
        comp.wait_stream(copy)  # the previous copy out of buffer b has finished
        sc.score_device(fr, bufs[b], None, comp)
        done[b].record(comp)
        copy.wait_event(done[b])
        with torch.cuda.stream(copy):
            host[b].copy_(bufs[b], non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (STEPS * 2)
    out[f"{kind} device + overlapped D2H of scores"] = {"frames_per_s": F / dt, "ms_per_step": dt * 1e3}
    del sc
print(json.dumps(out, indent=1))
