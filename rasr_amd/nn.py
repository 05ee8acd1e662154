"""ctypes binding of the hybrid-DNN scorer C-ABI (include/rasr_nn.h), the MI355X drop-in for
Nn::BatchFeatureScorer (src/Nn/BatchFeatureScorer.cc): a feed-forward network whose top layer is
linear+softmax evaluated without the softmax, the scaled log prior removed from its bias, and
score(e, t) = -output[e, t].  Computation: one bf16 MFMA GEMM per layer with the bias and the
activation fused (rasr_amd/csrc/nn_kernels.hip); there is no CPU path.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _capi

ACTIVATIONS = {"identity": 0, "sigmoid": 1, "tanh": 2, "relu": 3, "elu": 4}


class NnLayerDesc(ctypes.Structure):
    _fields_ = [
        ("input_dim", ctypes.c_uint32),
        ("output_dim", ctypes.c_uint32),
        ("weights", ctypes.c_void_p),
        ("bias", ctypes.c_void_p),
        ("activation", ctypes.c_int),
        ("gamma", ctypes.c_float),
    ]


class NnNetworkDesc(ctypes.Structure):
    _fields_ = [
        ("n_layers", ctypes.c_uint32),
        ("layers", ctypes.POINTER(NnLayerDesc)),
        ("log_prior", ctypes.c_void_p),
        ("prior_scale", ctypes.c_float),
    ]


_PROTOTYPES = [
    ("nn_prior_from_mixture_set", ctypes.c_int, [ctypes.POINTER(_capi.MixtureSetDesc), ctypes.c_void_p]),
    ("nn_scorer_create", ctypes.c_int,
     [ctypes.POINTER(NnNetworkDesc), ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("nn_scorer_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("nn_scorer_n_classes", ctypes.c_uint32, [ctypes.c_void_p]),
    ("nn_scorer_input_dim", ctypes.c_uint32, [ctypes.c_void_p]),
    ("nn_score_device", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
      ctypes.c_void_p]),
    ("nn_score_host", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]),
    ("nn_score_host_ex", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
      ctypes.c_uint32]),
    ("nn_scorer_set_timing", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("nn_scorer_kernel_time", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]),
    ("nn_last_error", ctypes.c_char_p, []),
]


def _lib():
    lib = _capi.load_library()
    if not getattr(lib, "_nn_bound", False):
        for name, res, args in _PROTOTYPES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        lib._nn_bound = True
    return lib


def _check(rc: int, what: str) -> None:
    if rc != _capi.GMM_OK:
        raise _capi.GmmError(f"{what} failed ({rc}): {_lib().nn_last_error().decode()}")


def prior_from_mixture_set(ms) -> np.ndarray:
    """Prior::setFromMixtureSet (src/Nn/Prior.cc:159-190), one-to-one class labels."""
    out = np.empty(ms.n_mixtures, dtype=np.float32)
    d = ms.desc()
    _check(_lib().nn_prior_from_mixture_set(ctypes.byref(d), out.ctypes.data_as(ctypes.c_void_p)),
           "nn_prior_from_mixture_set")
    return out


class NnScorer:
    """layers: [(W [in][out] f32, b [out] f32 or None, activation name, gamma)], the last one the top
    (linear+softmax) layer; log_prior [classes] or None; prior_scale ("priori-scale")."""

    def __init__(self, layers, log_prior=None, prior_scale: float = 1.0, max_frames: int = 4096, device: int = 0):
        lib = _lib()
        self._keep = []
        descs = (NnLayerDesc * len(layers))()
        for i, (w, b, act, gamma) in enumerate(layers):
            w = np.ascontiguousarray(w, dtype=np.float32)
            self._keep.append(w)
            descs[i].input_dim, descs[i].output_dim = w.shape
            descs[i].weights = w.ctypes.data
            if b is not None:
                b = np.ascontiguousarray(b, dtype=np.float32)
                assert b.shape == (w.shape[1],)
                self._keep.append(b)
                descs[i].bias = b.ctypes.data
            descs[i].activation = ACTIVATIONS[act]
            descs[i].gamma = float(gamma)
        net = NnNetworkDesc()
        net.n_layers = len(layers)
        net.layers = descs
        if log_prior is not None:
            lp = np.ascontiguousarray(log_prior, dtype=np.float32)
            self._keep.append(lp)
            net.log_prior = lp.ctypes.data
        net.prior_scale = float(prior_scale)
        h = ctypes.c_void_p()
        _check(lib.nn_scorer_create(ctypes.byref(net), int(max_frames), int(device), ctypes.byref(h)),
               "nn_scorer_create")
        self._keep = None  # the library copied everything
        self._h = h
        self._l = lib
        self.max_frames = int(max_frames)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._l.nn_scorer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def n_classes(self) -> int:
        return int(self._l.nn_scorer_n_classes(self._h))

    def input_dim(self) -> int:
        return int(self._l.nn_scorer_input_dim(self._h))

    def score_device(self, frames, scores, stream=None, n_frames=None) -> None:
        """frames: torch cuda f32 [F, >=D]; scores: [classes, >=F] f32; asynchronous on `stream`."""
        f = int(frames.shape[0] if n_frames is None else n_frames)
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device)
        s = getattr(stream, "cuda_stream", stream)
        _check(self._l.nn_score_device(self._h, ctypes.c_void_p(frames.data_ptr()), f, int(frames.stride(0)),
                                       ctypes.c_void_p(scores.data_ptr()), int(scores.stride(0)),
                                       ctypes.c_void_p(s) if s else None), "nn_score_device")

    def score_host(self, frames: np.ndarray, out: np.ndarray | None = None, n_frames: int | None = None,
                   frame_major: bool = False) -> np.ndarray:
        """nn_score_host(_ex).  frames: [F][>= input_dim] f32 rows (row stride = frames.shape[1]); out: optional
        caller-kept table, [>= n_classes][>= F] (row stride = out.shape[1]) of which only the first F columns are
        written, or with frame_major [>= F][>= n_classes] of which the first F rows' first n_classes entries are."""
        frames = np.ascontiguousarray(frames, dtype=np.float32)
        if frames.ndim != 2 or frames.shape[1] < self.input_dim():
            raise ValueError("frames must be a 2-d f32 [n_frames][>= input_dim] array")
        f = frames.shape[0] if n_frames is None else int(n_frames)
        if not 0 <= f <= frames.shape[0]:
            raise ValueError(f"n_frames {f} outside [0, {frames.shape[0]}] (the rows of frames)")
        c = self.n_classes()
        shape = (f, c) if frame_major else (c, f)
        scores = np.empty(shape, dtype=np.float32) if out is None else out
        if (scores.dtype != np.float32 or not scores.flags.c_contiguous or scores.ndim != 2
                or scores.shape[0] < shape[0] or scores.shape[1] < shape[1]):
            raise ValueError(f"out must be a C-contiguous f32 [>= {shape[0]}][>= {shape[1]}] array")
        _check(self._l.nn_score_host_ex(self._h, frames.ctypes.data_as(ctypes.c_void_p), f, frames.shape[1],
                                        scores.ctypes.data_as(ctypes.c_void_p), scores.shape[1],
                                        2 if frame_major else 0), "nn_score_host_ex")
        return scores

    def set_timing(self, enable: bool) -> None:
        _check(self._l.nn_scorer_set_timing(self._h, int(bool(enable))), "nn_scorer_set_timing")

    def kernel_time(self, reset: bool = True):
        ms, n = ctypes.c_double(), ctypes.c_uint32()
        _check(self._l.nn_scorer_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(n), int(reset)),
               "nn_scorer_kernel_time")
        return ms.value, n.value


def synthetic_network(dims, activation="sigmoid", seed: int = 0):
    """Random-init feed-forward stack of the given dimensions (input, hidden..., classes):
    W ~ N(0, 1/in) (unit-variance pre-activations), b ~ N(0, 0.1); last layer linear."""
    rng = np.random.Generator(np.random.PCG64(seed))
    layers = []
    for i in range(len(dims) - 1):
        w = (rng.standard_normal((dims[i], dims[i + 1]), dtype=np.float32) / np.sqrt(dims[i])).astype(np.float32)
        b = (0.1 * rng.standard_normal(dims[i + 1], dtype=np.float32)).astype(np.float32)
        layers.append((w, b, activation if i + 2 < len(dims) else "identity", 1.0))
    return layers
