"""A/B: the bench network's layer GEMMs (429-2048x6-5000, 32768 frames, bf16 in, f32 accumulate) on
torch.matmul (hipBLASLt) -- plain GEMM, no bias/activation epilogue -- against bench.py --mode nn's
nnGemm256 number (13.6 M frames/s, profiles/r01/bench_nn_v2_256.log)."""
import json
import torch

F = 32768
dims = [429] + [2048] * 6 + [5000]
dev = torch.device("cuda", 0)
ws = [torch.randn(dims[i], dims[i + 1], device=dev, dtype=torch.bfloat16) for i in range(len(dims) - 1)]
x = torch.randn(F, dims[0], device=dev, dtype=torch.bfloat16)


def fwd():
    h = x
    for w in ws:
        h = h @ w
    return h


for _ in range(5):
    fwd()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
out = {}
for i, w in enumerate(ws):
    a = torch.randn(F, dims[i], device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        a @ w
    s.record()
    for _ in range(20):
        a @ w
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    out[f"layer{i} {dims[i]}x{dims[i+1]}"] = {"ms": ms, "tflops": 2 * F * dims[i] * dims[i + 1] / ms / 1e9}
s.record()
for _ in range(10):
    fwd()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 10
flop = sum(2 * F * dims[i] * dims[i + 1] for i in range(len(ws)))
out["network"] = {"ms": ms, "frames_per_s": F / ms * 1e3, "tflops": flop / ms / 1e9, "frac_bf16_peak": flop / ms / 1e9 / 2516.6}
print(json.dumps(out, indent=1))
