"""Child process of tests/test_rccl_exchange.py::test_torch_nccl_world1_density_sharded (GPU box only).

torch.distributed over the `nccl` backend (RCCL on ROCm) at world size 1 on cuda:0:
* rasr_amd.parallel.DensityShardedScorer (the layout bench.py --gpus N runs) scores a ragged model; its table must
  equal the unsharded scorer's bit for bit (scores and best densities);
* an in-place all_reduce(MIN) of int64 shard keys -- the per-frame reduce's dtype and op -- must leave the keys
  unchanged on one rank.
Prints one JSON line."""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import rasr_amd as ra
    from rasr_amd import parallel

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    rec = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    try:
        counts = ra.ragged_counts(60, 60 * 14, low=1, high=40, seed=3)
        ms = ra.synthetic_mixture_set(60, counts, 39, seed=5, weights="random")
        F = 257
        frames = ra.synthetic_frames(F, 39, seed=6)
        kind = "SIMD-diagonal-maximum"
        sc = parallel.DensityShardedScorer(ms, kind, F, 0, 1, device=0)
        fr = torch.from_numpy(frames).cuda()
        local_s = torch.zeros((sc.n_local, F), dtype=torch.float32, device="cuda")
        local_b = torch.zeros((sc.n_local, F), dtype=torch.int32, device="cuda")
        full, fullb = sc.score(fr, local_s, local_b)
        torch.cuda.synchronize()
        ref_s, ref_b = ra.Scorer(ms, kind, max_frames=F).score_host(frames)
        s = full.cpu().numpy()
        b = fullb.cpu().numpy().view(np.uint32)
        rec["scores"] = ("bit-exact vs the unsharded scorer"
                         if np.array_equal(s.view(np.uint32), ref_s.view(np.uint32)) else "DIFFER")
        rec["best"] = "equal" if np.array_equal(b, ref_b) else "DIFFER"
        # the per-frame reduce's collective: int64 keys, MIN, in place
        g = torch.Generator().manual_seed(7)
        keys = torch.randint(-(1 << 62), 1 << 62, (7, F), generator=g, dtype=torch.int64).cuda()
        want = keys.clone()
        dist.all_reduce(keys, op=dist.ReduceOp.MIN)
        torch.cuda.synchronize()
        rec["all_reduce_min_int64"] = "ok" if torch.equal(keys, want) else "DIFFER"
    finally:
        dist.destroy_process_group()
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
