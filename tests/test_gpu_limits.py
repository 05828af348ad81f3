"""GPU: the reference's parameter space at the boundary (VERDICT r1 missing #2).

The reference passes any Connectivity / ExpansionAdd / ExpansionSearch to usearch
(/root/reference/src/index/usearch.rs:89-96) and any Limit: NonZeroUsize
(/root/reference/src/lib.rs:234-256).  This library supports connectivity up to 64
(level-0 rows of 128 entries, read as two wave-wide pieces), search ef and build efC up
to 4096 (sorted LDS list above the register set's 1024), exact k up to 8192; anything
beyond is VSG_EUNSUPPORTED with a message -- never a silent clamp.  Each lifted limit is
checked bit-exactly against the oracle on integer data.
"""
import numpy as np
import pytest

import oracle as O
import vsg
from vsg import datagen as G
from vsg._lib import VSG_EUNSUPPORTED

pytestmark = pytest.mark.gpu


def recall(found, truth, k):
    return float(np.mean([len(set(found[i][:k].tolist()) & set(truth[i][:k].tolist())) / k
                          for i in range(truth.shape[0])]))


@pytest.mark.parametrize("reg", ["1", "0"])
@pytest.mark.parametrize("M,dim", [(48, 32), (64, 64)])
def test_wide_connectivity_same_graph_bitexact(M, dim, reg, monkeypatch):
    """M = 48 / 64 (level-0 rows of 96 / 128 entries): GPU traversal of the
    oracle-built graph == oracle traversal, every ef class."""
    monkeypatch.setenv("VSG_SEARCH_REG", reg)
    n = 8000
    x = G.uint8_valued(n, dim, 11)
    q = G.uint8_valued(80, dim, 12)
    h = O.HnswOracle(dim, "l2sq", M, 96, 48, seed=3)
    h.add(np.arange(n), x, threads=0)
    h.remove(np.arange(0, n, 19))
    idx = vsg.Index(dim, "l2sq", "f32", M, 96, 48, seed=3)
    idx.import_graph(h.export())
    for ef, k in ((10, 10), (64, 10), (300, 30), (1500, 10)):
        ok, od, oc = h.search(q, k, ef)
        m = idx.search(q, k, ef)
        np.testing.assert_array_equal(m.counts, oc)
        np.testing.assert_array_equal(m.keys, ok)
        np.testing.assert_array_equal(m.distances, od)


@pytest.mark.parametrize("M,efc", [(64, 128), (40, 256)])
def test_wide_connectivity_build_equals_oracle_one_node_batches(M, efc, monkeypatch):
    n, dim = 1200, 24
    x = G.uint8_valued(n, dim, 13)
    monkeypatch.setenv("VSG_BUILD_PERMUTE", "0")
    monkeypatch.setenv("VSG_BUILD_BATCH_MAX", "1")
    gpu = vsg.Index(dim, "l2sq", "f32", M, efc, 64, seed=4)
    gpu.add(np.arange(n), x)
    h = O.HnswOracle(dim, "l2sq", M, efc, 64, seed=4)
    h.add(np.arange(n), x, threads=1)
    a, b = gpu.export(), h.export()
    assert (a["entry"], a["max_level"]) == (b["entry"], b["max_level"])
    for key in ("levels", "adj0", "upper"):
        np.testing.assert_array_equal(a[key], b[key], err_msg=key)


def test_wide_connectivity_build_recall():
    n, dim, nq = 20000, 96, 300
    bs, qs, ms = G.config_seeds(2)
    x = G.clustered(n, dim, bs, ms)
    q = G.clustered(nq, dim, qs, ms)
    gk, _, _ = O.exact_search("l2sq", x, q, 10)
    h = O.HnswOracle(dim, "l2sq", 64, 128, 64, seed=9)
    h.add(np.arange(n), x, threads=0)
    idx = vsg.Index(dim, "l2sq", "f32", 64, 128, 64, seed=9)
    idx.add(np.arange(n), x)
    for ef in (16, 64):
        rc = recall(h.search(q, 10, ef)[0], gk, 10)
        rg = recall(idx.search(q, 10, ef).keys, gk, 10)
        assert rg >= rc - 0.005, (ef, rg, rc)


@pytest.mark.parametrize("ef,k", [(2000, 10), (4096, 4096), (1025, 1025), (3000, 1500)])
def test_large_ef_and_k_bitexact(ef, k):
    """ef / k above the register set's 1024: the sorted LDS-list kernel, bit-exact."""
    n, dim = 9000, 16
    x = G.uint8_valued(n, dim, 21)
    q = G.uint8_valued(24, dim, 22)
    h = O.HnswOracle(dim, "l2sq", 16, 64, 48, seed=5)
    h.add(np.arange(n), x, threads=0)
    h.remove(np.arange(0, n, 31))
    idx = vsg.Index(dim, "l2sq", "f32", 16, 64, 48, seed=5)
    idx.import_graph(h.export())
    ok, od, oc = h.search(q, k, ef)
    m = idx.search(q, k, ef)
    np.testing.assert_array_equal(m.counts, oc)
    np.testing.assert_array_equal(m.keys, ok)
    np.testing.assert_array_equal(m.distances, od)


@pytest.mark.parametrize("k", [1500, 8192])
def test_exact_large_k_bitexact(k):
    n, dim = 20000, 24
    x = G.uint8_valued(n, dim, 23)
    q = G.uint8_valued(40, dim, 24)
    idx = vsg.Index(dim, "l2sq")
    idx.add(np.arange(n), x)
    idx.remove(np.arange(0, n, 7))
    removed = np.zeros(n, np.uint8)
    removed[::7] = 1
    ok, od, oc = O.exact_search("l2sq", x, q, k, removed=removed)
    m = idx.exact_search(q, k)
    np.testing.assert_array_equal(m.counts, oc)
    np.testing.assert_array_equal(m.keys, ok)
    np.testing.assert_array_equal(m.distances, od)


def test_large_expansion_add_build():
    """efC above the register beam's 192 and the old 1024 cap: the LDS-list insert beam."""
    n, dim, nq = 6000, 32, 100
    x = G.uint8_valued(n, dim, 25)
    q = G.uint8_valued(nq, dim, 26)
    gk, _, _ = O.exact_search("l2sq", x, q, 10)
    idx = vsg.Index(dim, "l2sq", "f32", 16, 2048, 64, seed=6)
    idx.add(np.arange(n), x)
    assert recall(idx.search(q, 10, 64).keys, gk, 10) >= 0.97


def test_limits_are_errors_not_clamps():
    x = G.uint8_valued(500, 8, 27)
    idx = vsg.Index(8, "l2sq", "f32", 16, 64, 64)
    idx.add(np.arange(500), x)
    for call in (lambda: idx.search(x[:2], 10, 4097), lambda: idx.search(x[:2], 5000),
                 lambda: idx.exact_search(x[:2], 8193)):
        with pytest.raises(vsg.VsgError) as e:
            call()
        assert e.value.code == VSG_EUNSUPPORTED
    with pytest.raises(vsg.VsgError) as e:
        vsg.Index(8, "l2sq", "f32", 16, 5000, 64)
    assert e.value.code == VSG_EUNSUPPORTED and "expansion_add" in str(e.value)
    with pytest.raises(vsg.VsgError) as e:
        vsg.Index(8, "l2sq", "f32", 65)
    assert e.value.code == VSG_EUNSUPPORTED
    idx.set_f16_traversal(True)
    with pytest.raises(vsg.VsgError) as e:
        idx.search(x[:2], 10, 2000)
    assert e.value.code == VSG_EUNSUPPORTED
    idx.set_f16_traversal(False)
    m = idx.search(x[:2], 10, 4096)  # the largest supported ef works
    assert (m.counts == 10).all()
