"""Mixture-set text files (include/rasr_gmm_io.h): the product reader against the
std::istream restatement of MixtureSet::read (oracle/pms_istream.cc), bit-exact
tables, the reference's error behaviour, round trips through the writer, and
(GPU) a model read from file scored against the oracle."""
import gzip
import os
import random
import zlib

import numpy as np
import pytest

import rasr_amd as ra
from rasr_amd import _capi
from oracle import pms

FIELDS = ["means", "variances", "density_mean", "density_covariance", "mixture_offsets", "mixture_densities",
          "mixture_log_weights"]
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(autouse=True)
def _lib(built):
    return built


def _same(ms, tables):
    for f in FIELDS:
        a, b = getattr(ms, f), tables[f]
        assert a.shape == b.shape, f
        assert a.tobytes() == b.tobytes(), f  # bit-exact, NaN payloads and -0 included


def _valid(t):
    """The product additionally rejects what the reference's scorers would index out of range."""
    nm, nc, nd = t["means"].shape[0], t["variances"].shape[0], t["density_mean"].shape[0]
    return bool(np.all(t["density_mean"] < nm) and np.all(t["density_covariance"] < nc)
                and np.all(t["mixture_densities"] < nd))


def _check_file(path, offset=0, reduced=0):
    rc, tables = pms.pms_read(str(path), offset, reduced)
    try:
        ms = ra.read_mixture_set(str(path), offset, reduced)
    except ra.GmmError as e:
        if rc == pms.OK:
            assert not _valid(tables), f"product rejected a file the reference reads: {e}"
        elif rc in (pms.VERSION, pms.COVARIANCE_TYPE):
            assert "(-2)" in str(e)
        return None
    assert rc == pms.OK, f"product read a file the reference rejects (oracle status {rc})"
    _same(ms, tables)
    return ms


def _text(header, mixtures, densities, means, covs, version="2.0", covtype="DiagonalCovariance", sep=" ",
          eol="\n"):
    lines = [f"#Version: {version}", f"#CovarianceType: {covtype}", sep.join(map(str, header))]
    lines += [sep.join(map(str, m)) for m in mixtures]
    lines += [sep.join(map(str, d)) for d in densities]
    lines += [sep.join(map(str, m)) for m in means]
    lines += [" " + sep.join(map(str, c)) for c in covs]
    return eol.join(lines) + eol


TINY = dict(header=(3, 2, 3, 3, 1),
            mixtures=[(2, 0, -0.5, 1, -0.9162907318741551), (1, 2, 0)],
            densities=[(0, 0), (1, 0), (2, 0)],
            means=[(3, 0.25, -1.5, 2), (3, "1e-3", "+4.5E1", ".5"), (3, "5.", "-0", "1.17549435e-38")],
            covs=[(3, 1.5, 1, "0.25", 2, 3, "0.5")])


def test_tiny_file_bit_exact(tmp_path):
    p = tmp_path / "tiny.pms"
    p.write_text(_text(**TINY))
    ms = _check_file(p)
    assert ms is not None and ms.dimension == 3 and ms.n_mixtures == 2 and ms.n_densities == 3
    np.testing.assert_array_equal(ms.variances, np.float32([[1.5, 0.5, 1.5]]))  # variance x feature weight
    np.testing.assert_array_equal(ms.mixture_offsets, [0, 2, 3])
    assert np.signbit(ms.means[2, 1])  # "-0" stays negative zero


def test_golden_fixture(tmp_path):
    """tests/golden/pms/tiny_v2.pms (+ expected tables, written by scripts/make_pms_golden.py)."""
    src = os.path.join(HERE, "golden", "pms", "tiny_v2.pms")
    z = np.load(os.path.join(HERE, "golden", "pms", "tiny_v2_tables.npz"), allow_pickle=False)
    ms = ra.read_mixture_set(src)
    _same(ms, {f: z[f] for f in FIELDS})
    rc, tables = pms.pms_read(src)
    assert rc == pms.OK
    _same(ms, tables)


def test_version_1_linear_weights(tmp_path):
    t = dict(TINY)
    t["mixtures"] = [(2, 0, 0.25, 1, 0.75), (1, 2, 0)]
    p = tmp_path / "v1.pms"
    p.write_text(_text(version="1.0", **t))
    ms = _check_file(p)
    assert ms.mixture_log_weights[0] == np.log(0.25) and ms.mixture_log_weights[2] == -np.finfo(np.float64).max


@pytest.mark.parametrize("offset,reduced", [(0, 2), (1, 2), (1, 3), (0, 5), (2, 0), (3, 1), (4, 1)])
def test_dimension_offset_and_reduction(tmp_path, offset, reduced):
    p = tmp_path / "d.pms"
    p.write_text(_text(**TINY))
    _check_file(p, offset, reduced)


def test_whitespace_variants(tmp_path):
    for i, (sep, eol) in enumerate([("\t", "\n"), ("  ", "\r\n"), (" \v ", "\n\n\f"), ("\n", "\n")]):
        p = tmp_path / f"w{i}.pms"
        body = _text(**TINY, sep=sep, eol=eol)
        # the two header lines are read by getline: keep them '\n'-terminated without '\r'
        head, rest = body.split(eol, 2)[:2], body.split(eol, 2)[2]
        p.write_text(head[0] + "\n" + head[1] + "\n" + rest)
        assert _check_file(p) is not None


def test_gzip_and_zlib_and_members(tmp_path):
    text = _text(**TINY).encode()
    (tmp_path / "a.pms.gz").write_bytes(gzip.compress(text))
    (tmp_path / "b.pms").write_bytes(zlib.compress(text))
    half = len(text) // 2
    (tmp_path / "c.pms.gz").write_bytes(gzip.compress(text[:half]) + gzip.compress(text[half:]))
    plain = ra.parse_mixture_set(text)
    for name in ["a.pms.gz", "b.pms", "c.pms.gz"]:
        ms = ra.read_mixture_set(str(tmp_path / name))
        _same(ms, {f: getattr(plain, f) for f in FIELDS})
    _check_file(tmp_path / "a.pms.gz")
    _check_file(tmp_path / "c.pms.gz")
    with pytest.raises(ra.GmmError):
        ra.parse_mixture_set(gzip.compress(text)[:-20])  # truncated member


@pytest.mark.parametrize("case", [
    "no_trailing_newline", "truncated", "version_2.1", "covariance_type", "short_header", "float_overflow",
    "inf_token", "bare_exponent", "empty", "negative_count_wraps", "index_out_of_range", "mean_length",
    "u32_overflow", "crlf_header",
])
def test_error_behaviour(tmp_path, case):
    text = _text(**TINY)
    t = dict(TINY)
    if case == "no_trailing_newline":
        text = text.rstrip("\n")
    elif case == "truncated":
        text = text[: len(text) // 2]
    elif case == "version_2.1":
        text = _text(version="2.1", **TINY)
    elif case == "covariance_type":
        text = _text(covtype="FullCovariance", **TINY)
    elif case == "short_header":
        text = "#Version:\n" + text.split("\n", 1)[1]
    elif case == "float_overflow":
        t["means"] = [(3, 0.25, "1e39", 2)] + TINY["means"][1:]
        text = _text(**t)
    elif case == "inf_token":
        t["means"] = [(3, 0.25, "inf", 2)] + TINY["means"][1:]
        text = _text(**t)
    elif case == "bare_exponent":
        t["means"] = [(3, 0.25, "1e", 2)] + TINY["means"][1:]
        text = _text(**t)
    elif case == "empty":
        text = ""
    elif case == "negative_count_wraps":
        t["header"] = (3, 2, 3, 3, "-1")
        text = _text(**t)
    elif case == "index_out_of_range":
        t["densities"] = [(0, 0), (1, 1), (2, 0)]
        text = _text(**t)
    elif case == "mean_length":
        t["means"] = [(2, 0.25, -1.5)] + TINY["means"][1:]
        text = _text(**t)
    elif case == "u32_overflow":
        t["mixtures"] = [(2, 4294967296, -0.5, 1, -0.9), (1, 2, 0)]
        text = _text(**t)
    elif case == "crlf_header":
        text = text.replace("\n", "\r\n")
    p = tmp_path / "e.pms"
    p.write_text(text)
    assert _check_file(p) is None  # both refuse (or the product refuses what the scorers cannot index)
    with pytest.raises(ra.GmmError):
        ra.read_mixture_set(str(p))


def test_missing_file():
    with pytest.raises(ra.GmmError, match="cannot open"):
        ra.read_mixture_set("/nonexistent/model.pms")


@pytest.mark.parametrize("precision", [6, 9, 17])
def test_writer_matches_reference_format(tmp_path, precision):
    ms = ra.synthetic_mixture_set(7, [3, 1, 0, 2, 5, 1, 4], 5, seed=7, n_covariances=3, weights="random")
    p = tmp_path / f"w{precision}.pms"
    ra.write_mixture_set(str(p), ms, precision)
    lines = p.read_text().split("\n")
    assert lines[0] == "#Version: 2.0" and lines[1] == "#CovarianceType: DiagonalCovariance"
    assert lines[2] == f"5 7 {ms.n_densities} {ms.n_densities} 3"
    assert lines[3 + 2] == "0"  # empty mixture
    m0 = ms.means[0]
    assert lines[3 + 7 + ms.n_densities] == "5 " + " ".join(f"{float(v):.{precision}g}" for v in m0)
    assert lines[3 + 7 + 2 * ms.n_densities].startswith(" 5 ")
    back = _check_file(p)
    if precision >= 9:  # f32 tables round-trip from 9 significant digits
        np.testing.assert_array_equal(back.means, ms.means)
        np.testing.assert_array_equal(back.variances, ms.variances)
    if precision == 17:
        np.testing.assert_array_equal(back.mixture_log_weights, ms.mixture_log_weights)
    gz = tmp_path / f"w{precision}.pms.gz"
    ra.write_mixture_set(str(gz), ms, precision)
    assert gz.read_bytes()[:2] == b"\x1f\x8b"
    _same(ra.read_mixture_set(str(gz)), {f: getattr(back, f) for f in FIELDS})


def test_fuzzed_files_agree_with_istream(tmp_path):
    """Random edits of a valid file: the product accepts exactly what std::istream accepts,
    with identical tables."""
    rng = random.Random(1234)
    base = _text(**TINY)
    alphabet = "0123456789 .-+eE\n\tx"
    for i in range(400):
        s = list(base)
        for _ in range(rng.randint(1, 3)):
            pos = rng.randrange(len(s))
            op = rng.random()
            if op < 0.4:
                del s[pos]
            elif op < 0.8:
                s.insert(pos, rng.choice(alphabet))
            else:
                s[pos] = rng.choice(alphabet)
        p = tmp_path / f"f{i}.pms"
        p.write_text("".join(s))
        _check_file(p)


def test_larger_model_round_trip(tmp_path):
    ms = ra.synthetic_mixture_set(200, 16, 39, seed=3, weights="random")
    p = tmp_path / "m.pms.gz"
    ra.write_mixture_set(str(p), ms, 9)
    back = _check_file(p)
    np.testing.assert_array_equal(back.means, ms.means)
    np.testing.assert_array_equal(back.variances, ms.variances)


def test_capi_errors():
    import ctypes
    lib = ra.load_library()
    d = _capi.MixtureSetDesc()
    assert lib.gmm_mixture_set_read(None, 0, 0, ctypes.byref(d)) == -1
    assert lib.gmm_mixture_set_write(b"/tmp/x.pms", None, 6) == -1
    assert lib.gmm_mixture_set_free(None) == -1


@pytest.mark.gpu
def test_scorer_on_model_read_from_file(tmp_path, gpu):
    """Read a model from a .pms.gz file and score it: SIMD bit-exact against the oracle."""
    import torch

    import oracle
    src = ra.synthetic_mixture_set(50, 12, 39, seed=11, weights="random", n_covariances=2)
    p = tmp_path / "m.pms.gz"
    ra.write_mixture_set(str(p), src, 6)  # lossy precision: the file, not src, is the model
    ms = ra.read_mixture_set(str(p))
    frames = ra.synthetic_frames(96, 39, seed=5)
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=96, device=0)
    scores, best = sc.score_host(frames)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    np.testing.assert_array_equal(scores, ref_s)
    np.testing.assert_array_equal(best, ref_b)
    del sc
    torch.cuda.synchronize()
