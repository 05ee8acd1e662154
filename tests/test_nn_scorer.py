"""Hybrid-DNN scorer (rasr_amd.nn, include/rasr_nn.h): the MI355X drop-in for Nn::BatchFeatureScorer
(src/Nn/BatchFeatureScorer.cc), checked against oracle/nn_oracle.py.

Tolerances (bf16 MFMA, f32 accumulation, BASELINE config 5):
  * against the bf16 contract (oracle.forward_bf16: the same bf16 roundings, exact sums):
    |gpu - ref| <= 2e-3 * (1 + |ref|) -- accumulation order and device exp/tanh only;
  * against the reference's f32 arithmetic (oracle.forward_f32): |gpu - ref| <= 5e-2 * (1 + |ref|),
    the bf16 rounding of weights and activations (measured max printed by the test).
"""
import numpy as np
import pytest

import rasr_amd as ra
from oracle import nn_oracle
from rasr_amd import nn


def _err(a, ref):
    return float((np.abs(a.astype(np.float64) - ref) / (1.0 + np.abs(ref))).max())


def test_oracle_prior_matches_library():
    ms = ra.synthetic_mixture_set(30, ra.ragged_counts(30, 200, low=1, high=12, seed=3), 13, seed=3,
                                  weights="random")
    # unnormalised mixture weights: scale each mixture's weights differently
    ms.mixture_log_weights[:] += np.repeat(np.log(np.arange(1, 31)), np.diff(ms.mixture_offsets))
    assert np.allclose(nn.prior_from_mixture_set(ms), nn_oracle.prior_from_mixture_set(ms), atol=1e-6)


def test_oracle_bf16_close_to_f32():
    layers = nn.synthetic_network([39, 256, 256, 100], "sigmoid", seed=1)
    frames = ra.synthetic_frames(50, 39, seed=2)
    a = nn_oracle.forward_f32(layers, frames)
    b = nn_oracle.forward_bf16(layers, frames)
    assert _err(b, a.astype(np.float64)) < 5e-2
    assert a.shape == (100, 50)


ACTS = ["sigmoid", "tanh", "relu", "elu", "identity"]


@pytest.mark.gpu
@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("dims,frames", [([39, 256, 100], 300), ([429, 1000, 1000, 997], 517),
                                          ([45, 128, 128, 128, 64], 128), ([16, 5000], 33),
                                          # <= 64 frames: nnGemmSmall (16-unit row blocks, 1..4 column blocks)
                                          ([39, 256, 100], 1), ([45, 128, 128, 128, 64], 17),
                                          ([429, 1000, 1000, 997], 64), ([429, 1000, 1000, 997], 128),
                                          # hidden layer on nnGemm8p (Npad 8192: 8 x 32 = 256 tiles of 256, well
                                          # above the 192-workgroup cutoff kNnTile128Wgs), top on nnGemm128
                                          ([64, 2048, 300], 8192)])
def test_nn_scorer_gpu(gpu, act, dims, frames):
    layers = nn.synthetic_network(dims, act, seed=len(dims) + frames)
    x = ra.synthetic_frames(frames, dims[0], seed=frames)
    lp = np.log(np.random.Generator(np.random.PCG64(4)).dirichlet(np.ones(dims[-1]))).astype(np.float32)
    sc = nn.NnScorer(layers, log_prior=lp, prior_scale=0.6, max_frames=frames + 7)
    assert sc.n_classes() == dims[-1] and sc.input_dim() == dims[0]
    s = sc.score_host(x)
    e16 = _err(s, nn_oracle.forward_bf16(layers, x, lp, 0.6).astype(np.float64))
    e32 = _err(s, nn_oracle.forward_f32(layers, x, lp, 0.6).astype(np.float64))
    print(f"{act} {dims}: vs bf16 contract {e16:.2e}, vs f32 {e32:.2e}")
    assert e16 <= 2e-3
    assert e32 <= 5e-2


@pytest.mark.gpu
def test_nn_scorer_bench_shape(gpu):
    """BASELINE config 5's network exactly as bench.py --mode nn builds it (429 -> 2048 x 6 -> 5000, sigmoid),
    on a frame count that is not a multiple of the 256-frame tile; checked against the bf16 contract."""
    dims = [429] + [2048] * 6 + [5000]
    layers = nn.synthetic_network(dims, "sigmoid", seed=5)
    x = ra.synthetic_frames(300, 429, seed=6)
    lp = np.log(np.random.Generator(np.random.PCG64(7)).dirichlet(np.ones(5000))).astype(np.float32)
    sc = nn.NnScorer(layers, log_prior=lp, prior_scale=0.7, max_frames=512)
    s = sc.score_host(x)
    e16 = _err(s, nn_oracle.forward_bf16(layers, x, lp, 0.7).astype(np.float64))
    print(f"bench shape: vs bf16 contract {e16:.2e}")
    assert e16 <= 2e-3


@pytest.mark.gpu
def test_nn_scorer_device_strides_and_errors(gpu):
    import torch
    layers = nn.synthetic_network([39, 300, 200], "sigmoid", seed=9)
    layers[0] = (layers[0][0], layers[0][1], "sigmoid", 0.5)  # SigmoidLayer "gamma"
    layers[1] = (layers[1][0], None, "identity", 1.0)         # top layer without bias
    x = ra.synthetic_frames(130, 39, seed=10)
    sc = nn.NnScorer(layers, max_frames=130)
    ref = nn_oracle.forward_bf16(layers, x).astype(np.float64)
    padded = torch.zeros((130, 48), dtype=torch.float32, device=gpu)
    padded[:, :39] = torch.from_numpy(x).to(gpu)
    out = torch.full((200, 160), 7.0, dtype=torch.float32, device=gpu)
    sc.score_device(padded, out)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert _err(o[:, :130], ref) <= 2e-3
    assert (o[:, 130:] == 7.0).all()  # nothing written past n_frames
    # host path with strided caller buffers: frame rows of 48 floats (39 used, the rest a sentinel that must
    # not be read as features), a score table of 160 columns of which only the first 130 are written
    xs = np.full((130, 48), np.nan, np.float32)
    xs[:, :39] = x
    table = np.full((200, 160), 7.0, np.float32)
    sc.score_host(xs, out=table)
    assert _err(table[:, :130], ref) <= 2e-3
    assert (table[:, 130:] == 7.0).all()
    # the top layer writes 4 frames of a class with one 16-byte store when the table allows it: an odd row
    # stride (133 floats) and a table starting 4 bytes into its allocation take the 4-byte path
    big = torch.full((200, 133), 7.0, dtype=torch.float32, device=gpu)
    view = big[:, 1:]  # row stride 133, first column 4 bytes in
    sc.score_device(padded, view)
    torch.cuda.synchronize()
    b = big.cpu().numpy()
    assert _err(b[:, 1:131], ref) <= 2e-3
    assert (b[:, 0] == 7.0).all() and (b[:, 131:] == 7.0).all()
    with pytest.raises(ra.GmmError):
        sc.score_host(ra.synthetic_frames(131, 39, seed=1))  # more than max_frames
    # caller buffers the C-ABI would overrun: refused before the call
    with pytest.raises(ValueError):
        sc.score_host(x, out=np.empty((199, 160), np.float32))  # fewer rows than classes
    with pytest.raises(ValueError):
        sc.score_host(x, n_frames=131)  # more frames than rows given
    with pytest.raises(ValueError):
        sc.score_host(x[:, :38])  # narrower than the input dimension
    # frame-major host table (NN_HOST_FRAME_MAJOR): row t = frame t's classes, other entries untouched
    fm = np.full((133, 205), 7.0, np.float32)
    sc.score_host(x, out=fm, frame_major=True)
    assert _err(fm[:130, :200].T, ref) <= 2e-3
    assert (fm[130:] == 7.0).all() and (fm[:, 200:] == 7.0).all()
    with pytest.raises(ValueError):
        sc.score_host(x, out=np.empty((130, 199), np.float32), frame_major=True)
    with pytest.raises(ra.GmmError):
        nn.NnScorer([(np.ones((4, 5), np.float32), None, "relu", 1.0),
                     (np.ones((6, 2), np.float32), None, "identity", 1.0)])  # 5 != 6


@pytest.mark.gpu
@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("dims,frames", [([100, 70], 300),      # K 100 -> 2 K-tiles of 64
                                          ([150, 64, 33], 257),  # 3 K-tiles, then 4 (padded 256)
                                          ([64, 600, 10], 513),  # exactly 1 K-tile, then 12
                                          ([1, 5], 3)])          # a 1-wide input
def test_nn_scorer_k_tile_counts(gpu, dims, frames, big):
    # the GEMMs' pipelines have separate paths for the last one and two K-tiles (no later stage to issue,
    # s_waitcnt vmcnt(0) instead of the counted wait): every short K-tile count is exercised, on nnGemm128
    # (these layers' 256-tile grids are small) and, with 49152 more frames (>= 192 tiles of 256), on nnGemm8p
    frames += 49152 if big else 0
    layers = nn.synthetic_network(dims, "tanh", seed=sum(dims))
    x = ra.synthetic_frames(frames, dims[0], seed=frames + 1)
    sc = nn.NnScorer(layers, max_frames=frames)
    s = sc.score_host(x)
    assert _err(s, nn_oracle.forward_bf16(layers, x).astype(np.float64)) <= 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["tanh", "elu", "sigmoid"])
def test_nn_activations_near_zero(gpu, act):
    """Hidden activations of tiny pre-activations (|z| ~ 1e-7 .. 1e-2).  tanh: the reference's std::tanh
    (Math::FastMatrix::tanh, src/Math/FastMatrix.hh:776-780) is accurate there, so the device form must keep its
    RELATIVE accuracy (bf16 keeps a small output to 2^-9 relative), which 1 - 2/(e + 1) alone loses by
    cancellation.  elu: the reference itself forms exp(x) - 1 (FastMatrix.hh:1656-1665), whose absolute error
    (~1e-7) the restatement and the device share: the absolute contract.  The top layer is the identity, so the
    scores are -bf16(act(z)) element by element."""
    rng = np.random.Generator(np.random.PCG64(11))
    d_in, d_h = 64, 128
    w = (rng.standard_normal((d_in, d_h)) * np.logspace(-7, -2, d_h)[None, :] / 8).astype(np.float32)
    layers = [(w, None, act, 1.0), (np.eye(d_h, dtype=np.float32), None, "identity", 1.0)]
    x = ra.synthetic_frames(40, d_in, seed=12)
    sc = nn.NnScorer(layers, max_frames=40)
    s = sc.score_host(x).astype(np.float64)
    ref = nn_oracle.forward_bf16(layers, x).astype(np.float64)
    if act == "tanh":
        rel = np.abs(s - ref) / np.maximum(np.abs(ref), 1e-30)
        print(f"{act}: max relative error {rel.max():.2e} for |ref| in [{np.abs(ref).min():.1e}, {np.abs(ref).max():.1e}]")
        assert rel.max() <= 2 ** -6  # one bf16 ulp (<= 2^-7 relative) of the hidden output, either side, + series
    else:
        assert np.abs(s - ref).max() <= 1e-6 + 2 ** -7 * np.abs(ref).max()  # one bf16 ulp + exp(x) - 1


@pytest.mark.gpu
@pytest.mark.parametrize("frames", [1, 7, 64])
@pytest.mark.parametrize("frame_major", [False, True])
def test_nn_small_host_call_page_locked(gpu, frames, frame_major):
    """nn_score_host_ex with page-locked frames and table (<= 64 frames: the one-stream path without the copy
    engine) equals the pageable call bit for bit; the rest of a strided caller table stays untouched."""
    layers = nn.synthetic_network([39, 256, 300], "sigmoid", seed=frames)
    sc = nn.NnScorer(layers, max_frames=64)
    x = ra.synthetic_frames(frames, 41, seed=frames + 3)  # row stride 41 > input 39
    ref = sc.score_host(x, frame_major=frame_major)
    xp = ra.pinned_empty(x.shape)
    xp[:] = x
    shape = (frames + 2, 300 + 5) if frame_major else (300, frames + 3)
    out = ra.pinned_empty(shape)
    out[:] = -3.0
    sc.score_host(xp, out=out, frame_major=frame_major)
    got = out[:frames, :300] if frame_major else out[:, :frames]
    assert np.array_equal(np.ascontiguousarray(got).view(np.uint32), ref.view(np.uint32))
    rest = np.ones(shape, bool)
    if frame_major:
        rest[:frames, :300] = False
    else:
        rest[:, :frames] = False
    assert (out[rest] == -3.0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["sigmoid", "relu"])
def test_nn_kernel_choice_bit_identical(gpu, act):
    """Between nnGemm8p and UNSPLIT nnGemm128 a frame's scores do not depend on the call size: the first 1600
    frames of an 8192-frame call (every layer on nnGemm8p, 8 x 32 = 256 tiles of 256, well above the
    192-workgroup cutoff; top layer as C^T) equal a 1600-frame call of the same frames (nnGemm128 without K split,
    16 x 14 tiles of 128) bit for bit: same K order per accumulator chain, same epilogue arithmetic.  Smaller
    calls split K (nnSplitReduce) or run nnGemmSmall: their sums differ in rounding only."""
    layers = nn.synthetic_network([64, 2048, 2048], act, seed=21)
    x = ra.synthetic_frames(8192, 64, seed=22)
    sc = nn.NnScorer(layers, max_frames=8192)
    full = sc.score_host(x)
    part = sc.score_host(x[:1600])
    assert np.array_equal(part.view(np.uint32), np.ascontiguousarray(full[:, :1600]).view(np.uint32))
    ref = nn_oracle.forward_bf16(layers, x[:500]).astype(np.float64)
    assert _err(part[:, :500], ref) <= 2e-3
    split = sc.score_host(x[:500])  # 16 x 4 tiles of 128, K split 4 ways
    assert _err(split, ref) <= 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["sigmoid", "tanh", "relu"])
def test_nn_kernel_boundaries_within_contract(gpu, act):
    """The same frames through each kernel the call size picks -- nnGemmSmall (<= 128 frames, K over 8 waves),
    nnGemm128 with a K split (500 frames, nnSplitReduce), unsplit nnGemm128 (1600) and nnGemm8p (8192) -- agree
    with each other within the bf16 contract (their partial sums are added in different orders, so they are not
    bit-identical), and each with the oracle."""
    layers = nn.synthetic_network([429, 2048, 2048, 1000], act, seed=31)
    x = ra.synthetic_frames(8192, 429, seed=32)
    sc = nn.NnScorer(layers, max_frames=8192)
    calls = {n: sc.score_host(x[:n]) for n in (100, 500, 1600, 8192)}
    ref = nn_oracle.forward_bf16(layers, x[:100]).astype(np.float64)
    for n, s in calls.items():
        assert _err(s[:, :100], ref) <= 2e-3, n
        assert _err(s[:, :100], calls[100].astype(np.float64)) <= 4e-3, n
