"""The RASR-side hybrid-DNN adapter (integration/rasr/Nn/GpuBatchFeatureScorer.{hh,cc} and
GpuBatchFeatureScorerNetwork.cc) linked and RUN: registered at the Nn id range (as src/Nn/Module.cc:39-67 registers
nn-batch-feature-scorer), created through Mm::FeatureScorerFactory, its network built by the Nn test doubles from the
configuration (tests/rasr_harness/include/Nn: links, layer types, dimensions, parameter files, "gamma", the prior
from the mixture set or a prior file with "priori-scale", class labels with "disregard-classes"), then driven through
Speech::OfflineRecognizer's addFeature / getScorer / flush sequence over two segments at several buffer sizes
(tests/rasr_harness/nn_harness.cc; the reference's protocol is src/Nn/BatchFeatureScorer.cc:92-171).

* CPU (`rasr_nn_harness`): over the f32 stand-in of the NN C-ABI -- the adapter's own logic (registration, network
  walk, activation-layer fusion, prior removal, label mapping, ring buffer) against oracle/nn_oracle.py forward_f32,
  |got - ref| <= 1e-5 (1 + |ref|) (f32 summation order only).
* GPU (`rasr_nn_harness_gpu`): over the PRODUCT library (nnGemm8p, bf16 MFMA) against forward_bf16 within the bf16
  contract of tests/test_nn_scorer.py, 2e-3 (1 + |ref|), and on the reference's own unit-test networks
  (tests/golden/nn_reference_vectors.json, as tests/test_nn_reference_vectors.py) within their bf16 bounds.
Classes the label wrapper disregards score Core::Type<Score>::max (BatchFeatureScorer.cc:164-170).
"""
import json
import os
import subprocess

import numpy as np
import pytest

import rasr_amd as ra
from oracle import nn_oracle
from rasr_amd import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCORER = "acoustic-model.mixture-set"
FLT_MAX = np.finfo(np.float32).max


def _write_case(d, layers, mixture_logw, frames, buffers, prior_scale=1.0, disregard=(), prior_file=None,
                split_activation=False):
    """layers: [(W [in][out], b [out], activation, gamma)] as rasr_amd.nn takes them; the top one is written as
    linear+softmax.  split_activation: hidden layers as a "linear" layer followed by an activation layer."""
    os.makedirs(d, exist_ok=True)
    acts = {"sigmoid": "sigmoid", "tanh": "tanh", "relu": "rectified", "elu": "elu", "identity": "identity"}
    lines, names = [], []
    for i, (w, b, act, gamma) in enumerate(layers):
        top = i + 1 == len(layers)
        name = f"layer-{len(names)}"
        names.append(name)
        pf = os.path.join(d, f"{name}.bin")
        with open(pf, "wb") as fh:
            fh.write(np.ascontiguousarray(b if b is not None else np.zeros(w.shape[1]), np.float32).tobytes())
            fh.write(np.ascontiguousarray(w, np.float32).tobytes())
        if top:
            ltype = "linear+softmax"
        elif split_activation:
            ltype = "linear"
        else:
            ltype = "linear" if act == "identity" else f"linear+{acts[act]}"
        lines += [f"{SCORER}.{name}.layer-type = {ltype}", f"{SCORER}.{name}.dimension-input = {w.shape[0]}",
                  f"{SCORER}.{name}.dimension-output = {w.shape[1]}", f"{SCORER}.{name}.parameter-file = {pf}"]
        if act == "sigmoid" and not split_activation:
            lines.append(f"{SCORER}.{name}.gamma = {gamma!r}")
        if split_activation and not top and act != "identity":
            aname = f"layer-{len(names)}"
            names.append(aname)
            lines += [f"{SCORER}.{aname}.layer-type = {acts[act]}"]
            if act == "sigmoid":
                lines.append(f"{SCORER}.{aname}.gamma = {gamma!r}")
    lines.append(f"{SCORER}.neural-network.links = 0->{names[0]}:0")
    for a, b in zip(names[:-1], names[1:]):
        lines.append(f"{SCORER}.{a}.links = 0->{b}:0")
    lines.append(f"{SCORER}.priori-scale = {prior_scale!r}")
    if prior_file is not None:
        lines.append(f"{SCORER}.prior-file = {prior_file}")
    if disregard:
        lines.append(f"{SCORER}.class-labels.disregard-classes = {','.join(str(c) for c in disregard)}")
    lines.append(f"harness.buffer-sizes = {','.join(str(b) for b in buffers)}")
    with open(os.path.join(d, "config.txt"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(os.path.join(d, "mixtures.bin"), "wb") as fh:
        fh.write(np.uint32(len(mixture_logw)).tobytes())
        for lw in mixture_logw:
            fh.write(np.uint32(len(lw)).tobytes() + np.asarray(lw, np.float64).tobytes())
    with open(os.path.join(d, "frames.bin"), "wb") as fh:
        fh.write(np.array(frames.shape, np.uint32).tobytes() + np.ascontiguousarray(frames, np.float32).tobytes())


def _run(exe, d, buffers, n_frames, n_classes):
    r = subprocess.run([exe, d], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "PASSED (0 failures)" in r.stdout
    return {b: np.fromfile(os.path.join(d, f"scores_{b}.bin"), np.float32).reshape(n_frames, n_classes)
            for b in buffers}


def _mixtures(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 5))
        w = rng.random(k) + 0.1
        out.append(np.log(w / w.sum() * rng.uniform(0.5, 2.0)))  # unnormalised mixtures: a non-uniform prior
    return out


def _expected_prior(mixture_logw, keep):
    """Prior::setFromMixtureSet over the accumulated classes (Prior.cc:159-190, not compatibility mode): the oracle's
    restatement on the mixture set restricted to those classes, in output order."""
    sub = [mixture_logw[k] for k in keep]
    offs = np.concatenate([[0], np.cumsum([len(w) for w in sub])]).astype(np.uint32)
    ms = ra.MixtureSet(np.zeros((1, 1), np.float32), np.ones((1, 1), np.float32), np.zeros(1, np.uint32),
                       np.zeros(1, np.uint32), offs, np.zeros(int(offs[-1]), np.uint32),
                       np.concatenate(sub).astype(np.float64))
    return nn_oracle.prior_from_mixture_set(ms)


def _table(ref_out, n_classes, keep):
    """[F][M] as the adapter's score(e): the network's -output of the class's output index, FLT_MAX elsewhere."""
    t = np.full((ref_out.shape[1], n_classes), FLT_MAX, np.float32)
    t[:, keep] = ref_out.T
    return t


CASES = {
    # name: (dims, activation, frames, buffers, prior scale, disregarded classes, activation as its own layer)
    "sigmoid": ([39, 96, 64, 40], "sigmoid", 150, [1, 8, 64], 0.6, (), False),
    "tanh-split": ([45, 80, 33], "tanh", 97, [8, 200], 1.0, (), True),
    "relu-disregard": ([16, 50, 30], "relu", 70, [4, 32], 0.8, (2, 9, 29), False),
    "elu-gamma": ([20, 64, 12], "elu", 41, [1, 5], 0.0, (), False),
}


def _case(tmp_path, name, device):
    dims, act, F, buffers, scale, disregard, split = CASES[name]
    n_classes = dims[-1] + len(disregard)
    keep = [k for k in range(n_classes) if k not in disregard]
    layers = nn.synthetic_network(dims, act, seed=len(name))
    if name == "sigmoid":
        layers[0] = (layers[0][0], layers[0][1], "sigmoid", 0.7)  # SigmoidLayer "gamma"
    mix = _mixtures(n_classes, seed=F)
    frames = ra.synthetic_frames(F, dims[0], seed=F + 1)
    d = str(tmp_path / f"{name}-{device}")
    _write_case(d, layers, mix, frames, buffers, prior_scale=scale, disregard=disregard, split_activation=split)
    lp = _expected_prior(mix, keep)
    return d, layers, frames, buffers, n_classes, keep, lp, scale


def _err(a, ref):
    fin = ref != FLT_MAX
    assert np.array_equal(a[~fin], ref[~fin]), "disregarded classes must score Core::Type<Score>::max"
    return float((np.abs(a[fin].astype(np.float64) - ref[fin]) / (1.0 + np.abs(ref[fin].astype(np.float64)))).max())


@pytest.mark.parametrize("name", sorted(CASES))
def test_nn_adapter_cpu_standin(built, tmp_path, name):
    d, layers, frames, buffers, M, keep, lp, scale = _case(tmp_path, name, "cpu")
    got = _run(os.path.join(ROOT, "build", "tests", "rasr_nn_harness"), d, buffers, frames.shape[0], M)
    ref = _table(nn_oracle.forward_f32(layers, frames, lp, scale), M, keep)
    for b, s in got.items():
        assert _err(s, ref) <= 1e-5, (b, _err(s, ref))


def test_nn_adapter_prior_file(built, tmp_path):
    """"prior-file" instead of the mixture set's weights (BatchFeatureScorer.cc:67-71)."""
    d, layers, frames, buffers, M, keep, _, _ = _case(tmp_path, "sigmoid", "file")
    lp = np.log(np.random.default_rng(3).dirichlet(np.ones(M))).astype(np.float32)
    pf = os.path.join(d, "prior.bin")
    lp.tofile(pf)
    with open(os.path.join(d, "config.txt"), "a") as fh:
        fh.write(f"{SCORER}.prior-file = {pf}\n{SCORER}.priori-scale = 0.45\n")
    got = _run(os.path.join(ROOT, "build", "tests", "rasr_nn_harness"), d, buffers, frames.shape[0], M)
    ref = _table(nn_oracle.forward_f32(layers, frames, lp, np.float32(0.45)), M, keep)
    for s in got.values():
        assert _err(s, ref) <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_nn_adapter_over_product_library(gpu, tmp_path, name):
    d, layers, frames, buffers, M, keep, lp, scale = _case(tmp_path, name, "gpu")
    got = _run(os.path.join(ROOT, "build", "tests", "rasr_nn_harness_gpu"), d, buffers, frames.shape[0], M)
    ref = _table(nn_oracle.forward_bf16(layers, frames, lp, scale), M, keep)
    for b, s in got.items():
        e = _err(s, ref)
        print(f"{name} buffer {b}: vs bf16 contract {e:.2e}")
        assert e <= 2e-3, (b, e)


@pytest.mark.gpu
def test_nn_adapter_reference_networks(gpu, tmp_path):
    """The reference's own unit-test networks through the adapter on the GPU (priori-scale 0: the reference tests
    apply no prior): Nn_NeuralNetwork.forward (linear+sigmoid -> linear+softmax, softmax of -score vs the expected
    posteriors, 1e-2 as tests/test_nn_reference_vectors.py) and Nn_LinearAndActivationLayer's linear+softmax layer
    (-score vs its stated pre-activation outputs within the bf16 rounding bound)."""
    from test_nn_reference_vectors import CASES as REF, _linear_bound, _param_layer, _softmax_cols, _two_layer_net
    exe = os.path.join(ROOT, "build", "tests", "rasr_nn_harness_gpu")
    layers, x, expected, _ = _two_layer_net()
    d = str(tmp_path / "ref2")
    _write_case(d, layers, [[0.0], [0.0]], x, [1, 3], prior_scale=0.0)
    for s in _run(exe, d, [1, 3], x.shape[0], 2).values():
        post = _softmax_cols(-s.T.astype(np.float64))
        assert np.abs(post - expected).max() <= 1e-2, np.abs(post - expected).max()
    name = "Nn_LinearAndActivationLayer.LinearAndSoftmaxLayer.forward"
    assert REF[name]["activation"] == "softmax"
    w, b, x, linear, _, _ = _param_layer(name)
    d = str(tmp_path / "ref1")
    _write_case(d, [(w, b, "identity", 1.0)], [[0.0]] * 3, x, [1, 2], prior_scale=0.0)
    for s in _run(exe, d, [1, 2], x.shape[0], 3).values():
        z = -s.T.astype(np.float64)
        assert (np.abs(z - linear) <= _linear_bound(w, b, x)).all()
