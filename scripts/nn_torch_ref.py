#!/usr/bin/env python3
"""The hybrid-DNN forward pass of the bench (NN_DIMS, 32768 frames, bf16 operands, f32 accumulate) through
PyTorch's own GEMMs (hipBLASLt on ROCm): torch.nn.functional.linear + sigmoid per hidden layer, the output
layer's linear with the prior folded into its bias (as nnGemm8p: no softmax, the hybrid scorer's scores are the
prior-corrected logits).  A yardstick for nnGemm8p's all-layer time (bench.py --mode nn), not a product path.
usage: nn_torch_ref.py [--frames 32768] [--iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch
    dims = [429] + [2048] * 6 + [5000]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(7)
    ws = [(torch.randn(dims[i + 1], dims[i], generator=g) / dims[i] ** 0.5).to(dev, torch.bfloat16)
          for i in range(len(dims) - 1)]
    bs = [torch.zeros(dims[i + 1], device=dev, dtype=torch.bfloat16) for i in range(len(dims) - 1)]
    x = torch.randn(a.frames, dims[0], generator=g).to(dev, torch.bfloat16)

    def forward(h, gemm_only=False):
        for i, (w, b) in enumerate(zip(ws, bs)):
            h = torch.nn.functional.linear(h, w, b)
            if not gemm_only:
                h = torch.sigmoid(h) if i < len(ws) - 1 else h.float()
        return h

    out = {}
    for name, go in (("gemm_bias_activation", False), ("gemm_bias_only", True)):
        for _ in range(3):
            forward(x, go)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            forward(x, go)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        flop = 2.0 * a.frames * sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1))
        out[name] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1), "frac_of_2516": round(flop / ms / 1e9 / 2516.6, 3)}
    print(json.dumps({"frames": a.frames, "torch": torch.__version__, **out}))


if __name__ == "__main__":
    main()
