"""GPU: opt-in f16 traversal + exact f32 re-rank (csrc/rerank.hip).

No usearch equivalent (the reference searches the f32 rows,
src/index/usearch.rs:275-277), so the bar is stated against this repo's own f32
path on the same graph:
  * integer-valued rows (0..255) are exact in f16 and every partial sum is an
    integer < 2^24, so the f16 walk evaluates the same distances as the f32 walk
    and the re-ranked top-k must equal the f32 search bit for bit (keys and
    distances), including after tombstones, appends and compaction;
  * float data: every returned distance is the f32 metric value of that key
    (checked against numpy f64 within 1e-5 absolute, cos/ip are in [0, 2]),
    and recall@10 stays within 1 % of the f32 walk at matched ef.
"""
import numpy as np
import pytest

import oracle as O
import vsg
from vsg import datagen as G

pytestmark = pytest.mark.gpu


def recall(found, truth, k):
    return float(np.mean([len(set(found[i][:k].tolist()) & set(truth[i][:k].tolist())) / k
                          for i in range(truth.shape[0])]))


def _same(a, b):
    np.testing.assert_array_equal(a.keys, b.keys)
    np.testing.assert_array_equal(a.distances, b.distances)
    np.testing.assert_array_equal(a.counts, b.counts)


@pytest.mark.parametrize("metric,dim", [("l2sq", 128), ("ip", 64), ("l2sq", 100)])
def test_rerank_equals_f32_walk_on_integer_data(metric, dim):
    n, nq = 12000, 200
    x = G.uint8_valued(n, dim, 71)
    q = G.uint8_valued(nq, dim, 72)
    if metric == "ip":  # keep |dot| < 2^24 and 1 - dot exact
        x = np.floor(x / 16).astype(np.float32)
        q = np.floor(q / 16).astype(np.float32)
    idx = vsg.Index(dim, metric, "f32", 16, 96, 64, seed=3)
    idx.add(np.arange(n), x)
    for ef, k in ((10, 10), (48, 10), (200, 32)):
        ref = idx.search(q, k, ef)
        idx.set_f16_traversal(True)
        got = idx.search(q, k, ef)
        idx.set_f16_traversal(False)
        _same(got, ref)


def test_rerank_tracks_appends_removals_and_compaction():
    dim, nq = 64, 150
    x = G.uint8_valued(10000, dim, 81)
    q = G.uint8_valued(nq, dim, 82)
    a = vsg.Index(dim, "l2sq", "f32", 16, 64, 40, seed=5)
    b = vsg.Index(dim, "l2sq", "f32", 16, 64, 40, seed=5, f16_traversal=True)
    for s in range(0, 6000, 2000):  # shadow extended after each append (and capacity growth)
        a.add(np.arange(s, s + 2000), x[s:s + 2000])
        b.add(np.arange(s, s + 2000), x[s:s + 2000])
        _same(b.search(q, 10), a.search(q, 10))
    assert a.remove(np.arange(0, 3000, 2)) == b.remove(np.arange(0, 3000, 2)) == 1500
    _same(b.search(q, 10, 64), a.search(q, 10, 64))
    assert not np.isin(b.search(q, 10).keys, np.arange(0, 3000, 2)).any()
    assert a.compact() == b.compact() == 1500  # rows move: shadow rebuilt
    _same(b.search(q, 10, 64), a.search(q, 10, 64))
    a.add(np.arange(6000, 10000), x[6000:])
    b.add(np.arange(6000, 10000), x[6000:])
    _same(b.search(q, 16, 80), a.search(q, 16, 80))


def test_rerank_tracks_replaced_rows():
    """Replaces re-link freed slots in place (vsg_index_replace): the f16 copy gets exactly
    the rewritten rows re-converted (not the whole copy), and the f16 walk + re-rank still
    equals the f32 walk bit for bit on integer data -- after replace calls of one key and of
    many, with the copy built before them."""
    dim, nq, n = 64, 150, 8000
    x = G.uint8_valued(n + 3000, dim, 91)
    q = G.uint8_valued(nq, dim, 92)
    a = vsg.Index(dim, "l2sq", "f32", 16, 64, 40, seed=6)
    b = vsg.Index(dim, "l2sq", "f32", 16, 64, 40, seed=6, f16_traversal=True)
    a.add(np.arange(n), x[:n])
    b.add(np.arange(n), x[:n])
    _same(b.search(q, 10, 48), a.search(q, 10, 48))  # the copy exists before the replaces
    rng = np.random.default_rng(4)
    row = n
    for batch in (1, 40, 700):
        keys = rng.choice(n, batch, replace=False).astype(np.uint64)
        assert (a.replace(keys, x[row:row + batch]) == 0).all()
        assert (b.replace(keys, x[row:row + batch]) == 0).all()
        row += batch
        _same(b.search(q, 10, 48), a.search(q, 10, 48))
    assert b.graph_info()["slots"] <= n + 1


def test_rerank_after_compacting_everything():
    """Every row removed, compaction drops all of them (slots -> 0), different rows
    re-added: the f16 copy must be rebuilt, not reused."""
    dim, nq = 32, 100
    x = G.uint8_valued(8000, dim, 91)
    q = G.uint8_valued(nq, dim, 92)
    a = vsg.Index(dim, "l2sq", "f32", 16, 64, 40, seed=2)
    b = vsg.Index(dim, "l2sq", "f32", 16, 64, 40, seed=2, f16_traversal=True)
    for idx in (a, b):
        idx.add(np.arange(4000), x[:4000])
    _same(b.search(q, 10), a.search(q, 10))
    for idx in (a, b):
        assert idx.remove(np.arange(4000)) == 4000
        assert idx.compact() == 4000
        idx.add(np.arange(4000, 8000), x[4000:])
    _same(b.search(q, 10, 64), a.search(q, 10, 64))
    assert np.isin(b.search(q, 10).keys, np.arange(4000, 8000)).all()


def test_rerank_requires_f32_storage():
    idx = vsg.Index(32, "l2sq", "f16")
    with pytest.raises(vsg.VsgError):
        idx.set_f16_traversal(True)
    with pytest.raises(vsg.VsgError):
        vsg.Index(32, "l2sq", "f16", f16_traversal=True)


@pytest.mark.parametrize("metric,dim", [("cos", 768), ("ip", 256), ("l2sq", 128)])
def test_rerank_float_data_exact_distances_and_recall(metric, dim):
    n, nq, k = 20000, 300, 10
    bs, qs, ms = G.config_seeds(1)
    x = G.clustered(n, dim, bs, ms)
    q = G.clustered(nq, dim, qs, ms)
    if metric == "ip":
        x /= np.linalg.norm(x, axis=1, keepdims=True)
        q /= np.linalg.norm(q, axis=1, keepdims=True)
    gk, _, _ = O.exact_search(metric, x, q, k)
    idx = vsg.Index(dim, metric, "f32", 16, 128, 64, seed=9)
    idx.add(np.arange(n), x)
    for ef in (16, 64):
        ref = idx.search(q, k, ef)
        idx.set_f16_traversal(True)
        got = idx.search(q, k, ef)
        idx.set_f16_traversal(False)
        assert (got.counts == k).all()
        # distances: the f32 metric value of the returned key, ascending
        xs = x[got.keys.astype(np.int64)].astype(np.float64)
        qq = q.astype(np.float64)[:, None, :]
        if metric == "l2sq":
            want = ((xs - qq) ** 2).sum(-1)
            tol = 1e-5 * np.maximum(1.0, want)
        else:
            if metric == "cos":
                xs = xs / np.linalg.norm(xs, axis=-1, keepdims=True)
                qq = qq / np.linalg.norm(qq, axis=-1, keepdims=True)
            want = 1.0 - (xs * qq).sum(-1)
            tol = 1e-5
        assert (np.abs(got.distances - want) <= tol).all()
        assert (np.diff(got.distances, axis=1) >= 0).all()
        rg, rf = recall(got.keys, gk, k), recall(ref.keys, gk, k)
        assert rg >= rf - 0.01, (ef, rg, rf)
