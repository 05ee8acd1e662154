"""Pin of the hybrid-DNN oracle (oracle/nn_oracle.py) and of the GPU scorer (nnGemm8p through
include/rasr_nn.h) to the known answers the reference's own unit tests hold:

  * src/Test/Nn_NeuralNetwork.cc:38-119 -- linear+sigmoid -> linear+softmax, 2 -> 2 -> 2, 4 frames;
  * src/Test/Nn_LinearAndActivationLayer.cc:74-175 -- one linear+sigmoid and one linear+softmax layer,
    3 -> 3, 2 frames, parameters [out][bias, in...] (LinearLayer::setParameters, src/Nn/LinearLayer.cc:383-423).

The vectors are transcribed into tests/golden/nn_reference_vectors.json.  The scorer's top layer is
linear+softmax evaluated without the softmax (Nn::BatchFeatureScorer, src/Nn/BatchFeatureScorer.cc:52-79,
148-171: score = -output), so the tests apply the softmax to -score; a sigmoid output layer is restated
as that layer followed by an identity top layer (score = -sigmoid(z)).

Tolerances:
  * oracle (f32) vs the reference's f64 vectors: the reference tests' own 1e-6;
  * GPU vs the oracle's bf16 contract (forward_bf16): 2e-3 * (1 + |ref|), as tests/test_nn_scorer.py;
  * GPU vs the reference's vectors: the bf16 operand rounding bound.  Each bf16 operand carries a relative
    error <= 2^-9 (round to nearest even, 8 significant bits), so a product w*x is off by at most
    |w x| (2^-8 + 2^-18) and a linear output by sum_i |w_i x_i| (2^-8 + 2^-18) + f32 accumulation; the
    test asserts that bound on the pre-activation outputs (the comment vectors `linear`) and carries it
    through the sigmoid / softmax to the posteriors (stated per case below).
"""
import json
import os

import numpy as np
import pytest

from oracle import nn_oracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "nn_reference_vectors.json")) as fh:
    CASES = {c["name"]: c for c in json.load(fh)["networks"]}

U_BF16 = 2.0 ** -9


def _softmax_cols(z):
    z = z.astype(np.float64)
    e = np.exp(z - z.max(axis=0, keepdims=True))
    return e / e.sum(axis=0, keepdims=True)


def _two_layer_net():
    c = CASES["Nn_NeuralNetwork.forward"]
    l1, l2 = c["layers"]
    layers = [(np.array(l1["W"], np.float32), np.array(l1["b"], np.float32), "sigmoid", 1.0),
              (np.array(l2["W"], np.float32), np.array(l2["b"], np.float32), "identity", 1.0)]
    return layers, np.array(c["frames"], np.float32), np.array(c["expected"], np.float64).T, c["tolerance"]


def _param_layer(name):
    c = CASES[name]
    p = np.array(c["parameters"], np.float32)          # [out][bias, in...]
    w = np.ascontiguousarray(p[:, 1:].T)               # weights_.at(r, row) = parameters[row][1 + r]
    b = np.ascontiguousarray(p[:, 0])                  # bias_.at(row) = parameters[row][0]
    return (w, b, np.array(c["frames"], np.float32), np.array(c["linear"], np.float64).T,
            np.array(c["expected"], np.float64).T, c["tolerance"])


def _linear_bound(w, b, x):
    """bf16 rounding bound of each linear output [out][frames]: sum_i |w_i x_i| (2^-8 + 2^-18), plus an f32
    accumulation allowance and the rounding of the bias (kept in f32)."""
    wx = np.abs(w.astype(np.float64)).T @ np.abs(x.astype(np.float64)).T
    return wx * (2 * U_BF16 + U_BF16 ** 2) + 1e-6 * (1.0 + wx + np.abs(b.astype(np.float64))[:, None])


# ----------------------------------------------------------------------------------------------- CPU pins


def test_oracle_two_layer_network_matches_reference():
    layers, x, expected, tol = _two_layer_net()
    post = _softmax_cols(-nn_oracle.forward_f32(layers, x))
    assert post.shape == expected.shape == (2, 4)
    assert np.abs(post - expected).max() <= tol, np.abs(post - expected).max()


@pytest.mark.parametrize("name", ["Nn_LinearAndActivationLayer.LinearAndSigmoidLayer.forward",
                                  "Nn_LinearAndActivationLayer.LinearAndSoftmaxLayer.forward"])
def test_oracle_linear_layer_orientation_and_bias(name):
    w, b, x, linear, expected, tol = _param_layer(name)
    # the pre-activation outputs the reference test states in its comment (:146, :166)
    z = -nn_oracle.forward_f32([(w, b, "identity", 1.0)], x)
    assert np.abs(z - linear).max() <= 1e-5
    if CASES[name]["activation"] == "softmax":
        post = _softmax_cols(z)
    else:
        eye = np.eye(w.shape[1], dtype=np.float32)
        post = -nn_oracle.forward_f32([(w, b, "sigmoid", 1.0), (eye, None, "identity", 1.0)], x).astype(np.float64)
    assert np.abs(post - expected).max() <= tol, np.abs(post - expected).max()


def test_transposed_orientation_would_fail():
    """The pin discriminates: reading the parameter matrix without the row <-> column interchange, or with
    the bias as the last column, misses the reference's linear outputs by far more than the tolerance."""
    w, b, x, linear, _, _ = _param_layer("Nn_LinearAndActivationLayer.LinearAndSoftmaxLayer.forward")
    p = np.array(CASES["Nn_LinearAndActivationLayer.LinearAndSoftmaxLayer.forward"]["parameters"], np.float32)
    wrong = [(np.ascontiguousarray(p[:, 1:]), b), (np.ascontiguousarray(p[:, :3].T), p[:, 3].copy())]
    for ww, bb in wrong:
        z = -nn_oracle.forward_f32([(ww, bb, "identity", 1.0)], x)
        assert np.abs(z - linear).max() > 0.1


# ----------------------------------------------------------------------------------------------- GPU pins


def _gpu_scores(layers, x):
    from rasr_amd import nn
    sc = nn.NnScorer(layers, max_frames=max(8, x.shape[0]))
    return sc.score_host(x).astype(np.float64)


@pytest.mark.gpu
def test_gpu_two_layer_network_matches_reference(gpu):
    layers, x, expected, _ = _two_layer_net()
    s = _gpu_scores(layers, x)
    ref16 = nn_oracle.forward_bf16(layers, x).astype(np.float64)
    assert (np.abs(s - ref16) / (1 + np.abs(ref16))).max() <= 2e-3
    post = _softmax_cols(-s)
    err = np.abs(post - expected).max()
    print(f"Nn_NeuralNetwork.forward on nnGemm8p: max |posterior - reference| = {err:.2e}")
    # logits within the two layers' bf16 bounds (<= ~0.02 here); the softmax of a 2-class logit difference is
    # 1/4-Lipschitz, so 1e-2 is a bound with margin that a wrong orientation or bias (errors ~0.1-1) violates
    assert err <= 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["Nn_LinearAndActivationLayer.LinearAndSigmoidLayer.forward",
                                  "Nn_LinearAndActivationLayer.LinearAndSoftmaxLayer.forward"])
def test_gpu_linear_layer_matches_reference(gpu, name):
    w, b, x, linear, expected, _ = _param_layer(name)
    z = -_gpu_scores([(w, b, "identity", 1.0)], x)
    bound = _linear_bound(w, b, x)
    print(f"{name}: linear |gpu - ref| max {np.abs(z - linear).max():.2e}, bf16 bound max {bound.max():.2e}")
    assert (np.abs(z - linear) <= bound).all()
    if CASES[name]["activation"] == "softmax":
        post = _softmax_cols(z)
    else:
        eye = np.eye(w.shape[1], dtype=np.float32)
        post = -_gpu_scores([(w, b, "sigmoid", 1.0), (eye, None, "identity", 1.0)], x)
    # sigmoid' <= 1/4 and softmax is 1/2-Lipschitz in the max-norm of the logits: the bound carries over
    # scaled by 1/2, plus the bf16 rounding of the sigmoid outputs fed to the identity layer (2^-9 relative)
    assert (np.abs(post - expected) <= 0.5 * bound.max() + U_BF16 * np.abs(expected) + 1e-6).all()
