"""TEST INFRASTRUCTURE ONLY -- RASR's binary maximum-likelihood mixture-set estimator files.

* `write_estimator_file`: the byte layout AbstractMixtureSetEstimator::write produces
  (src/Mm/AbstractMixtureSetEstimator.cc:416-420 header, :481-509 body; VectorAccumulator::write,
  GaussDensityEstimator::write, AbstractMixtureEstimator::write): the generator of the test files.
* `estimate`: a pure-Python restatement of what the reference's default reader does with such a file,
  MixtureSetEstimatorReader::read (src/Mm/MixtureSetReader.cc:52-74) = read (cc:433-479) + estimate
  (cc:299-337), written independently of the product reader (rasr_amd/csrc/host/MixtureSetEstimatorFile.cc).
  It returns plain tables; covariance sums run over the covariance's means in mean-index order (the
  reference iterates an unordered_set of pointers, GaussDensityEstimator.hh CovarianceToMeanSetMap).

Parity status: unpinned by the reference (no estimator files or tests ship with it); the generator follows
the writer's code above, the restatement the reader's.
"""
from __future__ import annotations

import math
import struct
import sys

import numpy as np

MAGIC = b"MIXSET\0\0"  # MixtureSetEstimator::magic() (MixtureSetEstimator.hh:36), 8 bytes written


def write_estimator_file(path_or_none, dimension, means, covariances, densities, mixtures, version=2):
    """means / covariances: lists of (sums [size] f64, weight); densities: [(mean index, covariance index)];
    mixtures: [[(density index, weight), ...], ...].  version 0 writes u32 counts instead of f64 weights.
    Returns the bytes (and writes them to path_or_none if given)."""
    le = "<"
    out = bytearray()
    out += MAGIC
    out += struct.pack(le + "I", version)
    out += struct.pack(le + "I", dimension)

    def acc(sums, weight):
        sums = np.asarray(sums, dtype="<f8")
        b = struct.pack(le + "I", len(sums)) + sums.tobytes()
        b += struct.pack(le + "d", weight) if version > 0 else struct.pack(le + "I", int(weight))
        return b

    out += struct.pack(le + "I", len(means))
    for s, w in means:
        out += acc(s, w)
    out += struct.pack(le + "I", len(covariances))
    for s, w in covariances:
        out += acc(s, w)
    out += struct.pack(le + "I", len(densities))
    for m, c in densities:
        out += struct.pack(le + "II", m, c)
    out += struct.pack(le + "I", len(mixtures))
    for mix in mixtures:
        out += struct.pack(le + "I", len(mix))
        for d, w in mix:
            out += struct.pack(le + "I", d)
            out += struct.pack(le + "d", w) if version > 0 else struct.pack(le + "I", int(w))
    data = bytes(out)
    if path_or_none is not None:
        with open(path_or_none, "wb") as f:
            f.write(data)
    return data


class EstimatorError(ValueError):
    pass


def _parse(data: bytes):
    pos = 0

    def take(fmt):
        nonlocal pos
        n = struct.calcsize(fmt)
        if pos + n > len(data):
            raise EstimatorError("truncated")
        v = struct.unpack_from("<" + fmt, data, pos)
        pos += n
        return v

    magic = data[:8]
    if len(magic) < 8 or magic[:7] != b"MIXSET\0":
        raise EstimatorError("magic")
    pos = 8
    (version,) = take("I")
    (dimension,) = take("I")

    def acc():
        (n,) = take("I")
        sums = list(take(f"{n}d")) if n else []
        (w,) = take("d") if version > 0 else take("I")
        return sums, float(w)

    (n_means,) = take("I")
    means = [acc() for _ in range(n_means)]
    (n_covs,) = take("I")
    covs = [acc() for _ in range(n_covs)]
    (n_dens,) = take("I")
    dens = []
    for _ in range(n_dens):
        m, c = take("II")
        if m >= n_means or c >= n_covs:
            raise EstimatorError("density index")
        dens.append((m, c))
    (n_mix,) = take("I")
    mixtures = []
    for _ in range(n_mix):
        (n,) = take("I")
        mix = []
        for _ in range(n):
            (d,) = take("I")
            (w,) = take("d") if version > 0 else take("I")
            if d >= n_dens:
                raise EstimatorError("mixture index")
            mix.append([d, float(w)])
        mixtures.append(mix)
    for s, _ in means + covs:
        if len(s) != dimension:
            raise EstimatorError("size")
    return dimension, means, covs, dens, mixtures


def _ulp_distance(a: float, b: float) -> int:
    ia = struct.unpack("<q", struct.pack("<d", a))[0]
    ib = struct.unpack("<q", struct.pack("<d", b))[0]
    if ia < 0:
        ia = (1 << 63) - ia
    if ib < 0:
        ib = (1 << 63) - ib
    return abs(ia - ib)


def estimate(data: bytes, minimum_observation_weight=5.0, minimum_relative_weight=0.0, minimum_variance=0.0,
             allow_zero_weights=False, normalize_mixture_weights=True) -> dict:
    """Tables of the estimated MixtureSet: dimension, means [n][D] f32, variances [n][D] f32, density_mean,
    density_covariance, mixture_offsets, mixture_densities, mixture_log_weights (f64).  Raises EstimatorError
    where the reference fails (criticalError / verify / a failed stream)."""
    dimension, means, covs, dens, mixtures = _parse(data)

    def mix_weight(mix):
        s = 0.0
        for _, w in mix:
            s += w
        return s

    if not allow_zero_weights:
        for mix in mixtures:
            if mix_weight(mix) == 0:
                raise EstimatorError("zero-weight mixture")
    # covariance -> means of the densities the mixtures reference (before the removal)
    mean_set = {}
    for mix in mixtures:
        for d, _ in mix:
            m, c = dens[d]
            mean_set.setdefault(c, set()).add(m)
    # removeDensitiesWithLowWeight
    for mix in mixtures:
        if not mix:
            raise EstimatorError("empty mixture")
        best = 0
        for j in range(1, len(mix)):
            if mix[j][1] > mix[best][1]:
                best = j
        min_weight = max(minimum_observation_weight, mix_weight(mix) * minimum_relative_weight)
        kept = [e for j, e in enumerate(mix) if j == best or e[1] >= min_weight]
        mix[:] = kept
    # index maps (first appearance)
    mean_idx, cov_idx, dens_idx = {}, {}, {}
    for mix in mixtures:
        for d, _ in mix:
            m, c = dens[d]
            mean_idx.setdefault(m, len(mean_idx))
            cov_idx.setdefault(c, len(cov_idx))
            dens_idx.setdefault(d, len(dens_idx))
    offsets, entries, logw = [0], [], []
    for mix in mixtures:
        lw = [math.log(w) if w > 0 else -sys.float_info.max for _, w in mix]
        if normalize_mixture_weights and lw:
            mx = 0
            for j in range(1, len(lw)):
                if lw[mx] < lw[j]:
                    mx = j
            acc = 0.0
            for j in range(len(lw)):
                if j != mx:
                    acc += math.exp(lw[j] - lw[mx])
            norm = math.log1p(acc) + lw[mx]
            lw = [v - norm for v in lw]
        entries += [dens_idx[d] for d, _ in mix]
        logw += lw
        offsets.append(len(entries))
    order_d = sorted(dens_idx, key=dens_idx.get)
    order_m = sorted(mean_idx, key=mean_idx.get)
    order_c = sorted(cov_idx, key=cov_idx.get)
    D = dimension
    mean_out = np.zeros((len(order_m), D), np.float32)
    for i, m in enumerate(order_m):
        s, w = means[m]
        if w != 0:
            mean_out[i] = np.array([v / w for v in s], np.float64).astype(np.float32)
    var_out = np.ones((len(order_c), D), np.float32)
    for i, c in enumerate(order_c):
        s, w = covs[c]
        if w == 0:
            continue
        wm = [0.0] * D
        ww = 0.0
        for m in sorted(mean_set[c]):
            ms, mw = means[m]
            if mw > 0:
                wm = [wm[k] + ms[k] * ms[k] / mw for k in range(D)]
                ww += mw
        if _ulp_distance(w, ww) > int(1e12):
            raise EstimatorError("covariance weight")
        v = np.array([(s[k] - wm[k]) / w for k in range(D)], np.float64).astype(np.float32)
        mv = np.float32(minimum_variance)
        if mv != 0:
            v = np.where(v < mv, mv, v).astype(np.float32)
        var_out[i] = v
    return {"dimension": D, "means": mean_out, "variances": var_out,
            "density_mean": np.array([mean_idx[dens[d][0]] for d in order_d], np.uint32),
            "density_covariance": np.array([cov_idx[dens[d][1]] for d in order_d], np.uint32),
            "mixture_offsets": np.array(offsets, np.uint32), "mixture_densities": np.array(entries, np.uint32),
            "mixture_log_weights": np.array(logw, np.float64)}


def accumulate_viterbi(frames, assignment, n_means, n_covs, density_mean, density_covariance):
    """Maximum-likelihood (Viterbi) accumulation as the trainer does it (GaussDensityEstimator::accumulate:
    the frame's sum into its density's mean estimator, its square into the covariance estimator, weight 1):
    returns (means, covariances) accumulator lists for write_estimator_file."""
    D = frames.shape[1]
    msum = np.zeros((n_means, D), np.float64)
    mw = np.zeros(n_means, np.float64)
    csum = np.zeros((n_covs, D), np.float64)
    cw = np.zeros(n_covs, np.float64)
    for x, d in zip(frames.astype(np.float64), assignment):
        m, c = density_mean[d], density_covariance[d]
        msum[m] += x
        mw[m] += 1
        csum[c] += x * x
        cw[c] += 1
    return [(msum[i], mw[i]) for i in range(n_means)], [(csum[i], cw[i]) for i in range(n_covs)]
