"""GPU: the build's locality launch order changes no output.

build_slots (vector-store-text_amd/csrc/vsg_index.cpp) launches the nodes of each
insert batch grouped by locality cell (nearest of up to 1,024 pivot rows, found on the
bf16 matrix cores by csrc/cells.hip, or by the f32 MFMA exact kernel with
VSG_BUILD_CELLS_F32=1), dealt XCD-contiguously, so that co-resident waves insert
neighbouring vectors and share rows in cache.  Nodes of one batch descend from the same
graph snapshot, write only their own rows and their own pair range, and the pairs are
sorted by (level, v, u) before the reverse-link kernel -- so the graph must be the same
bit for bit with and without the reordering (VSG_BUILD_LOCALITY=0), for every metric,
row width, f32 and f16 storage (f16 rows widened chunk by chunk for the MFMA kernel)
and for appends to a non-empty graph.  The reference's add() is
usearch's sequential insert (/root/reference/src/index/usearch.rs:221); parity of the
batched build with it is covered by test_gpu_parity / test_gpu_c2_parity.
"""
import numpy as np
import pytest

import vsg
from vsg import datagen as G

pytestmark = pytest.mark.gpu


def _build(monkeypatch, locality, metric, quant, x, parts):
    monkeypatch.setenv("VSG_BUILD_LOCALITY", locality)
    monkeypatch.setenv("VSG_BUILD_LOCALITY_MIN", "256")  # small batches reorder too
    idx = vsg.Index(x.shape[1], metric, quant, 16, 96, 64, seed=7)
    lo = 0
    for n in parts:
        idx.add(np.arange(lo, lo + n), x[lo:lo + n])
        lo += n
    return idx


@pytest.mark.parametrize("metric,quant,dim,data", [
    ("cos", "f32", 768, "clustered"),
    ("l2sq", "f32", 128, "sift"),
    ("l2sq", "f16", 128, "sift"),
    ("ip", "f32", 96, "clustered"),
])
def test_locality_order_same_graph(metric, quant, dim, data, monkeypatch):
    n = 40_000
    gen = G.sift_like if data == "sift" else G.clustered
    x = gen(n, dim, 21, 22)
    parts = (30_000, 10_000)  # a bulk build, then an append to the non-empty graph
    a = _build(monkeypatch, "0", metric, quant, x, parts)
    b = _build(monkeypatch, "1", metric, quant, x, parts)
    monkeypatch.setenv("VSG_BUILD_CELLS_F32", "1")
    c = _build(monkeypatch, "1", metric, quant, x, parts)
    monkeypatch.delenv("VSG_BUILD_CELLS_F32")
    ga, gb = a.export(), b.export()
    assert (ga["entry"], ga["max_level"]) == (gb["entry"], gb["max_level"])
    for f in ("levels", "adj0", "upper_off", "upper", "keys"):
        np.testing.assert_array_equal(ga[f], gb[f], err_msg=f)
        np.testing.assert_array_equal(ga[f], c.export()[f], err_msg=f + " (f32 cells)")
    sa, sb = a.stats(), b.stats()
    for f in ("build_distances", "build_adjacency", "build_batches"):
        assert sa[f] == sb[f], f
    q = gen(200, dim, 23, 22)
    ma, mb = a.search(q, 10, 64), b.search(q, 10, 64)
    np.testing.assert_array_equal(ma.keys, mb.keys)
    np.testing.assert_array_equal(ma.distances, mb.distances)


@pytest.mark.parametrize("metric,quant,dim,M,efc", [
    ("cos", "f32", 768, 16, 128),
    ("l2sq", "f16", 128, 16, 192),
    ("ip", "f32", 96, 48, 64),
])
def test_split_insert_same_graph(metric, quant, dim, M, efc, monkeypatch):
    """The insert as two launches (beam kernel -> lists in HBM -> selection kernel,
    csrc/hnsw.hip hnsw_insert_beam_kernel / hnsw_insert_select_kernel) builds the
    graph of the fused hnsw_insert_kernel bit for bit (VSG_BUILD_SPLIT=0)."""
    n = 30_000
    x = (G.sift_like if quant == "f16" else G.clustered)(n, dim, 61, 62)

    def build(split):
        monkeypatch.setenv("VSG_BUILD_SPLIT", split)
        idx = vsg.Index(dim, metric, quant, M, efc, 64, seed=8)
        idx.add(np.arange(20_000), x[:20_000])
        idx.add(np.arange(20_000, n), x[20_000:])
        return idx

    a, b = build("0"), build("1")
    ga, gb = a.export(), b.export()
    assert (ga["entry"], ga["max_level"]) == (gb["entry"], gb["max_level"])
    for f in ("levels", "adj0", "upper_off", "upper"):
        np.testing.assert_array_equal(ga[f], gb[f], err_msg=f)
    sa, sb = a.stats(), b.stats()
    for f in ("build_distances", "build_adjacency", "build_select_distances"):
        assert sa[f] == sb[f], f


def test_staging_and_rejected_call_leave_the_same_graph(monkeypatch):
    """add() enqueues the rows and the locality cells before it maps the keys (their
    slots lie beyond the index's size), and stages its uploads in pinned memory up to
    VSG_PIN_MAX: a call rejected for a duplicate key changes nothing -- the next add
    builds the graph of an index that never saw it -- and pageable staging
    (VSG_PIN_MAX=0) builds the same graph as pinned."""
    n, dim = 30_000, 96
    x = G.clustered(n + 5_000, dim, 71, 72)
    monkeypatch.setenv("VSG_BUILD_LOCALITY_MIN", "256")

    def build(pin, reject):
        monkeypatch.setenv("VSG_PIN_MAX", pin)
        idx = vsg.Index(dim, "l2sq", "f32", 16, 96, 64, seed=9)
        idx.add(np.arange(20_000), x[:20_000])
        if reject:
            keys = np.arange(20_000, 25_000)
            keys[-1] = 5  # already in the index
            with pytest.raises(vsg.VsgError):
                idx.add(keys, x[20_000:25_000] + 1.0)
            assert idx.size() == 20_000
        idx.add(np.arange(20_000, n), x[20_000:n])
        return idx

    ref = build(str(512 << 20), False).export()
    for pin, reject in (("0", False), (str(512 << 20), True), ("0", True)):
        g = build(pin, reject).export()
        assert (g["entry"], g["max_level"]) == (ref["entry"], ref["max_level"])
        for f in ("levels", "adj0", "upper_off", "upper", "keys"):
            np.testing.assert_array_equal(g[f], ref[f], err_msg=f"{f} pin={pin} reject={reject}")
