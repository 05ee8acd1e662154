#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary (gmm_score_host): frames copied in, the score table
(and best densities) copied out (frame chunks overlapped with the scoring; pageable destinations through
the pinned staging ring, pinned ones by direct DMA) -- the number DESIGN.md quotes beside bench.py's
HBM-resident `value`.  Also the device-resident rate with the table copied to pinned host memory on a
second stream (what a caller overlapping the D2H with the next batch would see)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rasr_amd as ra  # noqa: E402

F, STEPS = 32768, 5
ms = ra.synthetic_mixture_set(5000, 160, 39, seed=2024)
frames = ra.synthetic_frames(F, 39, seed=7)
out = {}
def rate(sc, want_best, outs):
    sc.score_host(frames, want_best=want_best, **outs)
    t0 = time.perf_counter()
    for _ in range(STEPS):
        sc.score_host(frames, want_best=want_best, **outs)
    dt = (time.perf_counter() - t0) / STEPS
    return {"frames_per_s": F / dt, "ms_per_step": dt * 1e3}


for kind in ("diagonal-maximum", "SIMD-diagonal-maximum"):
    # pageable caller buffers (kept across calls, like BatchFeatureScorerBase::scores_): staging ring,
    # copy threads swept; pinned caller buffers (gmm_host_alloc): direct DMA
    page = {"out": np.empty((5000, F), np.float32), "best_out": np.empty((5000, F), np.uint32)}
    pin = {"out": ra.pinned_empty((5000, F), np.float32), "best_out": ra.pinned_empty((5000, F), np.uint32)}
    for threads in (1, 4, 8, 16):
        os.environ["RASR_GMM_HOST_THREADS"] = str(threads)
        sc = ra.Scorer(ms, kind, max_frames=F)
        for want_best in (True, False):
            out[f"{kind} host pageable threads={threads} best={want_best}"] = rate(sc, want_best, page)
        del sc
    sc = ra.Scorer(ms, kind, max_frames=F)
    for want_best in (True, False):
        out[f"{kind} host pinned best={want_best}"] = rate(sc, want_best, pin)
    out[f"{kind} host fresh pageable arrays best=False"] = rate(sc, False, {})
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
