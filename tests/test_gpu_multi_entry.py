"""GPU: opt-in multi-entry descent (vsg_index_set_upper_ef; hnsw_search_reg.hip).

Not a usearch mode (usearch descends greedily, src/index/usearch.rs:275-277 ->
usearch search), so it is parity-unpinned against the reference and checked by
properties instead:
  * upper_ef 0/1 is the default path, bit for bit;
  * an index with no upper levels (max_level 0) gives identical results;
  * results are well-formed: ascending, no duplicates, no tombstones, every
    distance the exact metric value of its key (integer data: bit-exact vs the
    oracle's exact distances);
  * recall@10 at matched ef is no worse than the greedy descent's - 0.5 %.
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


def test_upper_ef_default_and_one_are_greedy():
    dim = 64
    x = G.uint8_valued(8000, dim, 51)
    q = G.uint8_valued(100, dim, 52)
    idx = vsg.Index(dim, "l2sq", "f32", 16, 64, 48, seed=2)
    idx.add(np.arange(len(x)), x)
    ref = idx.search(q, 10, 48)
    idx.set_upper_ef(1)
    _same(idx.search(q, 10, 48), ref)
    idx.set_upper_ef(0)
    _same(idx.search(q, 10, 48), ref)


def test_upper_ef_without_upper_levels_is_identity():
    dim = 32
    x = G.uint8_valued(40, dim, 53)  # tiny: check max_level
    q = G.uint8_valued(20, dim, 54)
    idx = vsg.Index(dim, "l2sq", "f32", 16, 64, 48, seed=3)
    idx.add(np.arange(len(x)), x)
    if idx.graph_info()["max_level"] != 0:
        pytest.skip("level sample put a node above level 0")
    ref = idx.search(q, 5, 16)
    idx.set_upper_ef(16)
    _same(idx.search(q, 5, 16), ref)


@pytest.mark.parametrize("metric,dim,quant", [("l2sq", 64, "f32"), ("ip", 48, "f32"), ("l2sq", 128, "f16")])
def test_upper_ef_results_well_formed_and_exact(metric, dim, quant):
    n, nq, k = 12000, 150, 10
    x = np.floor(G.uint8_valued(n, dim, 55) / (16.0 if metric == "ip" else 1.0))
    q = np.floor(G.uint8_valued(nq, dim, 56) / (16.0 if metric == "ip" else 1.0))
    idx = vsg.Index(dim, metric, quant, 16, 64, 48, seed=4)
    idx.add(np.arange(n), x)
    dead = np.arange(0, n, 9)
    idx.remove(dead)
    for ue, ef in ((4, 10), (16, 48), (64, 200), (300, 300)):
        idx.set_upper_ef(ue)
        m = idx.search(q, k, ef)
        # tombstones stay in the beam (usearch semantics), so a beam of ef == k
        # may hold fewer than k live nodes; wider beams fill k
        assert (m.counts <= k).all() and (ef == k or (m.counts == k).all())
        for i in range(nq):
            c = int(m.counts[i])
            keys = m.keys[i, :c].astype(np.int64)
            assert len(set(keys.tolist())) == c
            assert not np.isin(keys, dead).any()
            assert (m.keys[i, c:] == np.uint64(2**64 - 1)).all()
            d = m.distances[i, :c]
            assert (np.diff(d) >= 0).all()
            xs = x[keys].astype(np.float64)
            if metric == "l2sq":
                want = ((xs - q[i]) ** 2).sum(-1)
            else:
                want = 1.0 - (xs * q[i]).sum(-1)
            np.testing.assert_array_equal(d, want.astype(np.float32))


@pytest.mark.parametrize("metric,dim", [("cos", 128), ("l2sq", 64)])
def test_upper_ef_recall_not_worse(metric, dim):
    n, nq = 30000, 300
    bs, qs, ms = G.config_seeds(1)
    x = G.clustered(n, dim, bs, ms)
    q = G.clustered(nq, dim, qs, ms)
    gk, _, _ = O.exact_search(metric, x, q, 10)
    idx = vsg.Index(dim, metric, "f32", 16, 128, 64, seed=9)
    idx.add(np.arange(n), x)
    for ef in (10, 16, 32, 64):
        idx.set_upper_ef(0)
        r0 = recall(idx.search(q, 10, ef).keys, gk, 10)
        idx.set_upper_ef(16)
        r1 = recall(idx.search(q, 10, ef).keys, gk, 10)
        assert r1 >= r0 - 0.005, (ef, r0, r1)
