"""The density clustering's cache archive: "density-clustering.cache-archive" (src/Mm/DensityClustering.cc:27-28,
59-95; DensityClustering.tcc:25-55) in RASR's cache-archive file format (src/Core/MappedArchive.{hh,cc}).

The archive layout is restated here in Python, independently of the library's C++ reader/writer:
  file  = u32 version 0x17231 (MappedArchive.cc:52, 116-119), then items
  item  = u32 name length, u64 data size, name, data (MappedArchive.cc:185-195, 228-233); the LAST item of a
          name wins (getItem, cc:298-303)
  value = raw POD; vector = u64 count + elements; string = vector<char> with the NUL (MappedArchive.hh:401-466)
  "density-clustering" = "SPRINT-DC", u32 2, feature type name, distance type name ("f32" "f32" /
          "u8" "s32"), u32 dimension (padded), u32 clusters, u32 densities, vector<u8> cluster of every
          density, vector<feature type> cluster means (DensityClustering.cc:82-95, .tcc:25-45)
Tolerances: the clustering read back is bit-exact; scores of a scorer that loaded a clustering compare with the
oracle over that same clustering -- int bit-exact, float within 1e-4 relative (the preselection tests' bar).
Parity status: unpinned (the reference ships no archive fixture); the format follows the reference's source.
"""
import os
import struct

import numpy as np
import pytest

import oracle
import rasr_amd as ra
from rasr_amd.scorer import cache_archive_read, cache_archive_write

VERSION = 0x17231
ITEM = "density-clustering"


# ---------------------------------------------------------------------------
# the format restated
# ---------------------------------------------------------------------------
def parse_archive(path):
    with open(path, "rb") as f:
        b = f.read()
    assert struct.unpack_from("<I", b, 0)[0] == VERSION
    o, items = 4, []
    while o + 12 <= len(b):
        nl, ds = struct.unpack_from("<IQ", b, o)
        o += 12
        items.append((b[o:o + nl].decode(), b[o + nl:o + nl + ds]))
        o += nl + ds
    assert o == len(b)
    return items


def build_archive(path, items):
    with open(path, "wb") as f:
        f.write(struct.pack("<I", VERSION))
        for name, data in items:
            f.write(struct.pack("<IQ", len(name), len(data)) + name.encode() + data)


def _vec(a):
    a = np.ascontiguousarray(a)
    return struct.pack("<Q", a.size) + a.tobytes()


def _str(s):
    return _vec(np.frombuffer(s.encode() + b"\0", np.uint8))


def encode_clustering(kind, dp, coe, means):
    ft, dt = ("f32", "f32") if kind == "float" else ("u8", "s32")
    return (_str("SPRINT-DC") + struct.pack("<I", 2) + _str(ft) + _str(dt) +
            struct.pack("<III", dp, means.shape[0], coe.size) + _vec(coe.astype(np.uint8)) + _vec(means.ravel()))


def decode_clustering(b):
    o = 0

    def take(fmt):
        nonlocal o
        v = struct.unpack_from(fmt, b, o)
        o += struct.calcsize(fmt)
        return v[0]

    def vec(dtype):
        nonlocal o
        n = take("<Q")
        a = np.frombuffer(b, dtype, n, o)
        o += a.nbytes
        return a

    def string():
        return vec(np.uint8).tobytes().split(b"\0")[0].decode()

    magic, ver, ft, dt = string(), take("<I"), string(), string()
    dp, nc, nd = take("<I"), take("<I"), take("<I")
    coe = vec(np.uint8)
    means = vec(np.float32 if ft == "f32" else np.uint8).reshape(nc, dp)
    assert o == len(b)
    return dict(magic=magic, version=ver, types=(ft, dt), dp=dp, clusters=nc, densities=nd, coe=coe, means=means)


# ---------------------------------------------------------------------------
# CPU: the library's archive reader / writer (host only)
# ---------------------------------------------------------------------------
def test_archive_items_round_trip(built, tmp_path):
    p = str(tmp_path / "global.cache")
    cache_archive_write(p, "alpha", b"first")
    cache_archive_write(p, "beta", bytes(range(256)) * 3)
    assert cache_archive_read(p, "alpha") == b"first"
    assert cache_archive_read(p, "beta") == bytes(range(256)) * 3
    cache_archive_write(p, "alpha", b"")  # rewriting one item keeps the others
    assert cache_archive_read(p, "alpha") == b""
    assert dict(parse_archive(p)) == {"alpha": b"", "beta": bytes(range(256)) * 3}
    assert not [f for f in os.listdir(tmp_path) if ".temp." in f]  # temp file renamed over the archive


def test_archive_reads_reference_layout(built, tmp_path):
    # an archive laid out by the restatement above, with a repeated name: the last item of a name wins
    p = str(tmp_path / "a.cache")
    build_archive(p, [("x", b"old"), ("density-clustering", b"\1\2\3"), ("x", b"new")])
    assert cache_archive_read(p, "x") == b"new"
    assert cache_archive_read(p, ITEM) == b"\1\2\3"
    cache_archive_write(p, "y", b"z")
    assert dict(parse_archive(p)) == {"x": b"new", ITEM: b"\1\2\3", "y": b"z"}


def test_archive_errors(built, tmp_path):
    p = str(tmp_path / "missing.cache")
    with pytest.raises(ra._capi.GmmError):
        cache_archive_read(p, "x")
    with open(p, "wb") as f:
        f.write(struct.pack("<I", VERSION + 1) + b"junk")  # not this archive version
    with pytest.raises(ra._capi.GmmError):
        cache_archive_read(p, "x")
    build_archive(p, [("x", b"1")])
    with pytest.raises(ra._capi.GmmError):
        cache_archive_read(p, "y")
    with open(p, "ab") as f:  # a truncated item ends the list (MappedArchive::loadData)
        f.write(struct.pack("<IQ", 1, 99) + b"t")
    assert cache_archive_read(p, "x") == b"1"
    with pytest.raises(ra._capi.GmmError):  # an archive that cannot be written (missing directory)
        cache_archive_write(str(tmp_path / "no-such-dir" / "a.cache"), "x", b"1")
    with pytest.raises(ra._capi.GmmError):  # an empty item name (MappedArchive::loadData rejects name length 0)
        cache_archive_write(p, "", b"1")


def test_cache_archive_config_field(built):
    cfg = ra.default_config()
    assert cfg.cache_archive is None  # no cache by default: the clustering is built
    assert ra._capi.GMM_FLAG_CACHE_ARCHIVE_READ_ONLY == 64


# ---------------------------------------------------------------------------
# GPU: preselection scorers write, reuse and rebuild the item
# ---------------------------------------------------------------------------
def _model(seed=21):
    return ra.synthetic_mixture_set(60, 10, 33, seed=seed, weights="random")


def _check_scores(sc, ref, frames, kind):
    s, _ = sc.score_host(frames)
    ref_s = ref.score(frames, n_threads=8, selection=ref.select(frames))
    if kind == "int":
        assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
    else:
        assert np.array_equal(s == np.float32(40000.0), ref_s == np.float32(40000.0))
        err = np.abs(s.astype(np.float64) - ref_s) / np.maximum(1.0, np.abs(ref_s.astype(np.float64)))
        assert err.max() <= 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["float", "int"])
def test_clustering_written_then_reused(gpu, tmp_path, kind):
    ms = _model()
    frames = ra.synthetic_frames(200, 33, seed=3)
    p = str(tmp_path / "global.cache")
    build_archive(p, [("lexicon-cache", b"keep me")])
    t = f"preselection-batch-{kind}"
    sc = ra.Scorer(ms, t, max_frames=200, clusters=64, select_clusters=8, cache_archive=p)
    assert sc.clustering_source() == "written"
    coe, means = sc.density_clustering()
    items = dict(parse_archive(p))
    assert items["lexicon-cache"] == b"keep me"
    item = decode_clustering(items[ITEM])
    assert item["magic"] == "SPRINT-DC" and item["version"] == 2
    assert item["types"] == (("f32", "f32") if kind == "float" else ("u8", "s32"))
    assert (item["dp"], item["clusters"], item["densities"]) == (means.shape[1], 64, coe.size)
    assert np.array_equal(item["coe"], coe)
    assert np.array_equal(item["means"].view(np.uint8), means.view(np.uint8))
    sc.close()

    # a different valid clustering of the same model (one k-means iteration instead of five) in the archive:
    # a scorer created on it reads it (DensityClusteringBase::load; the iterations are not part of the item)
    # and scores with it
    ref = oracle.OraclePresel(ms, kind, clusters=64, select=8, iterations=1)
    assert not np.array_equal(ref.cluster_of_entry, coe)
    cache_archive_write(p, ITEM, encode_clustering(kind, ref.dp, ref.cluster_of_entry, ref.cluster_means))
    sc = ra.Scorer(ms, t, max_frames=200, clusters=64, select_clusters=8, cache_archive=p)
    assert sc.clustering_source() == "cached"
    coe2, means2 = sc.density_clustering()
    assert np.array_equal(coe2, ref.cluster_of_entry)
    assert np.array_equal(means2.view(np.uint8), ref.cluster_means.view(np.uint8))
    _check_scores(sc, ref, frames, kind)
    assert dict(parse_archive(p))["lexicon-cache"] == b"keep me"


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["float", "int"])
def test_clustering_mismatch_rebuilds(gpu, tmp_path, kind):
    ms = _model(seed=5)
    p = str(tmp_path / "global.cache")
    t = f"preselection-batch-{kind}"
    ra.Scorer(ms, t, max_frames=64, clusters=32, select_clusters=4, cache_archive=p).close()
    assert decode_clustering(dict(parse_archive(p))[ITEM])["clusters"] == 32
    # another cluster count: the item does not match (DensityClustering.cc:73-76) -> built and rewritten
    sc = ra.Scorer(ms, t, max_frames=64, clusters=48, select_clusters=4, cache_archive=p)
    assert sc.clustering_source() == "written"
    ref = oracle.OraclePresel(ms, kind, clusters=48, select=4)
    coe, means = sc.density_clustering()
    assert np.array_equal(coe, ref.cluster_of_entry)
    assert np.array_equal(means.view(np.uint8), ref.cluster_means.view(np.uint8))
    assert decode_clustering(dict(parse_archive(p))[ITEM])["clusters"] == 48
    sc.close()
    # the other kind's item (other type names), a corrupt cluster index, a truncated item: rebuilt too
    other = "int" if kind == "float" else "float"
    oref = oracle.OraclePresel(ms, other, clusters=48, select=4)
    bad = ref.cluster_of_entry.copy()
    bad[0] = 48
    for blob in (encode_clustering(other, oref.dp, oref.cluster_of_entry, oref.cluster_means),
                 encode_clustering(kind, ref.dp, bad, ref.cluster_means),
                 encode_clustering(kind, ref.dp, ref.cluster_of_entry, ref.cluster_means)[:-5]):
        cache_archive_write(p, ITEM, blob)
        sc = ra.Scorer(ms, t, max_frames=64, clusters=48, select_clusters=4, cache_archive=p)
        assert sc.clustering_source() == "written"
        coe, _ = sc.density_clustering()
        assert np.array_equal(coe, ref.cluster_of_entry)
        sc.close()
        item = decode_clustering(dict(parse_archive(p))[ITEM])
        assert item["types"] == (("f32", "f32") if kind == "float" else ("u8", "s32"))
        assert np.array_equal(item["coe"], ref.cluster_of_entry)


@pytest.mark.gpu
def test_clustering_read_only_archive(gpu, tmp_path):
    ms = _model(seed=7)
    p = str(tmp_path / "ro.cache")
    sc = ra.Scorer(ms, "preselection-batch-int", max_frames=64, clusters=16, select_clusters=4, cache_archive=p,
                   cache_archive_read_only=True)
    assert sc.clustering_source() == "built"
    sc.close()
    assert not os.path.exists(p)  # built, not written
    ref = oracle.OraclePresel(ms, "int", clusters=16, select=4, iterations=2)
    build_archive(p, [(ITEM, encode_clustering("int", ref.dp, ref.cluster_of_entry, ref.cluster_means))])
    sc = ra.Scorer(ms, "preselection-batch-int", max_frames=64, clusters=16, select_clusters=4, cache_archive=p,
                   cache_archive_read_only=True)
    assert sc.clustering_source() == "cached"
    assert np.array_equal(sc.density_clustering()[0], ref.cluster_of_entry)  # read
    sc.close()
    # no archive: built; a type without preselection has no clustering
    assert ra.Scorer(ms, "preselection-batch-int", max_frames=64, clusters=16,
                     select_clusters=4).clustering_source() == "built"
    with pytest.raises(ra._capi.GmmError):
        ra.Scorer(ms, "batch-diagonal-maximum-int", max_frames=64).clustering_source()
