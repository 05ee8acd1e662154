"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the hybrid-DNN scorer path of the reference
(Nn::BatchFeatureScorer, src/Nn/BatchFeatureScorer.cc), the checker for rasr_amd.nn.

  * LinearLayer::_forward (src/Nn/LinearLayer.cc:297-321): out = W^T in + bias, W [in][out];
  * activation layers (src/Nn/ActivationLayer.cc): sigmoid(gamma x) = 1 / (1 + exp(-gamma x)) (:103-131),
    tanh, rectified max(0, x) (:270), ELU alpha 1 (:333-348), identity;
  * BatchFeatureScorer::init (cc:52-79): the top layer is linear+softmax with the softmax off and
    BiasLayer::removeLogPriorFromBias (LinearLayer.cc:499-518): bias -= prior_scale * log_prior;
  * getScore (cc:148-171): score(e, t) = -output(e, t);
  * Prior::setFromMixtureSet (src/Nn/Prior.cc:159-190).

forward_f32 is the reference arithmetic (f32).  forward_bf16 states the GPU contract: weights and
every layer input rounded to bf16 (round to nearest even), products summed exactly (f64 here,
f32 MFMA accumulation on the GPU), bias / activation / scores in f32.
Parity unpinned: the reference holds no network files or score dumps for this path.
"""
import numpy as np


def bf16(x: np.ndarray) -> np.ndarray:
    """Round f32 to bf16 (nearest even), returned as f32."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def _act(x, act, gamma):
    if act == "sigmoid":
        return (1.0 / (1.0 + np.exp(-np.float32(gamma) * x))).astype(np.float32)
    if act == "tanh":
        return np.tanh(x).astype(np.float32)
    if act == "relu":
        return np.where(x > 0, x, np.float32(0)).astype(np.float32)
    if act == "elu":
        return np.where(x > 0, x, np.exp(x) - np.float32(1)).astype(np.float32)
    return x.astype(np.float32)


def _top_bias(b, n, log_prior, prior_scale):
    b = np.zeros(n, np.float32) if b is None else b.astype(np.float32)
    if log_prior is not None and prior_scale != 0:
        b = (b - np.float32(prior_scale) * log_prior.astype(np.float32)).astype(np.float32)
    return b


def forward_f32(layers, frames, log_prior=None, prior_scale=1.0):
    """Scores [classes][frames] in the reference's f32 arithmetic."""
    h = frames.astype(np.float32).T  # [in][frames], RASR matrices are column-major: one column per frame
    for i, (w, b, act, gamma) in enumerate(layers):
        top = i + 1 == len(layers)
        bias = _top_bias(b, w.shape[1], log_prior, prior_scale) if top else (
            np.zeros(w.shape[1], np.float32) if b is None else b.astype(np.float32))
        z = (w.astype(np.float32).T @ h + bias[:, None]).astype(np.float32)
        h = -z if top else _act(z, act, gamma)
    return h.astype(np.float32)


def forward_bf16(layers, frames, log_prior=None, prior_scale=1.0):
    """Scores [classes][frames] under the GPU's bf16 contract (see module doc)."""
    h = bf16(frames.astype(np.float32)).T.astype(np.float64)
    for i, (w, b, act, gamma) in enumerate(layers):
        top = i + 1 == len(layers)
        bias = _top_bias(b, w.shape[1], log_prior, prior_scale) if top else (
            np.zeros(w.shape[1], np.float32) if b is None else b.astype(np.float32))
        acc = (bf16(w).astype(np.float64).T @ h).astype(np.float32)
        z = (acc + bias[:, None]).astype(np.float32)
        if top:
            return (-z).astype(np.float32)
        h = bf16(_act(z, act, gamma)).astype(np.float64)
    raise ValueError("empty network")


def prior_from_mixture_set(ms) -> np.ndarray:
    """Prior::setFromMixtureSet: f32 per-mixture weight sums (`f32 += Mm::Weight`, an f64 (src/Mm/Types.hh:30):
    the sum formed in f64 and rounded to f32 per density), normalized by their f64-accumulated total
    (std::accumulate with a 0.0 init), std::log."""
    p = np.zeros(ms.n_mixtures, np.float32)
    for m in range(ms.n_mixtures):
        for i in range(int(ms.mixture_offsets[m]), int(ms.mixture_offsets[m + 1])):
            p[m] = np.float32(np.float64(p[m]) + np.exp(np.float64(ms.mixture_log_weights[i])))
    total = np.float32(sum(float(v) for v in p))
    return np.log(p / total).astype(np.float32)
