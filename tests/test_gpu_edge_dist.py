"""Per-edge distances stored beside the adjacency.

The reverse-link prune (hnsw_reverse_kernel) used to re-fetch every existing neighbour
row of the node it re-selects, to recompute distances the build had already computed.
The build now stores each edge's distance with the row (DevGraph.adjd0 / upperd) and the
prune reads them.  The stored value is the one the insert computed -- dist(v, x) when v
selected x, dist(x, v) when x's insert appended the reverse link -- and rows_dist is
operand-symmetric bit for bit ((a-b)^2 and a.b, same lane order, same shuffle tree), so
the graph must not change at all: these tests build the same rows with the stored
distances and with the recompute path (VSG_BUILD_EDGE_DIST=0) and compare every row.
An imported or loaded graph carries no distances; the next add fills them
(edge_dist_fill_kernel) -- checked the same way.
"""
import numpy as np
import pytest

import oracle as O
import vsg
from vsg import datagen as G

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _graph(g):
    return {k: g[k] for k in ("levels", "upper_off", "adj0", "upper")}, (g["entry"], g["max_level"])


def _same(a, b):
    ga, ea = _graph(a)
    gb, eb = _graph(b)
    assert ea == eb
    for k in ga:
        np.testing.assert_array_equal(ga[k], gb[k], err_msg=k)


@pytest.mark.parametrize("metric,dim,quant,M", [("cos", 768, "f32", 16), ("l2sq", 128, "f16", 16),
                                                ("ip", 96, "f32", 8), ("l2sq", 64, "f32", 40)])
def test_stored_edge_distances_build_the_same_graph(metric, dim, quant, M, monkeypatch):
    n = 40000
    bs, _, ms = G.config_seeds(1)
    x = G.sift_like(n, dim, bs, ms) if quant == "f16" else G.clustered(n, dim, bs, ms)
    out = []
    for flag in ("0", "1"):
        monkeypatch.setenv("VSG_BUILD_EDGE_DIST", flag)
        idx = vsg.Index(dim, metric, quant, M, 128, 64, seed=7)
        idx.add(np.arange(n // 2), x[: n // 2])  # two calls: the second prunes rows of the first
        idx.add(np.arange(n // 2, n), x[n // 2:])
        out.append(idx.export())
        if flag == "1":
            st = idx.stats()
            assert st["reverse_prunes"] > 0 and st["reverse_recompute_distances"] == 0
    _same(out[0], out[1])


def test_import_and_load_then_add_fill_the_distances(tmp_path, monkeypatch):
    n, extra, dim = 6000, 3000, 32
    x = G.uint8_valued(n + extra, dim, 91)
    h = O.HnswOracle(dim, "l2sq", 8, 64, 48, seed=5)
    h.add(np.arange(n), x[:n])
    g = h.export()
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("VSG_BUILD_EDGE_DIST", flag)
        a = vsg.Index(dim, "l2sq", "f32", 8, 64, 48, seed=5)
        a.import_graph(g)
        a.add(np.arange(n, n + extra), x[n:])
        res.append(a.export())
        if flag == "1":  # the same through save / load
            p = tmp_path / "g.vsg"
            b = vsg.Index(dim, "l2sq", "f32", 8, 64, 48, seed=5)
            b.import_graph(g)
            b.save(p)
            c = vsg.Index.load(p)
            c.add(np.arange(n, n + extra), x[n:])
            res.append(c.export())
    _same(res[0], res[1])
    _same(res[0], res[2])


def test_add_to_imported_graph_without_upper_rows(tmp_path, monkeypatch):
    """a loaded / imported graph with no level > 0 node has no upper
    distance table; adding a level-0 vector must fill the level-0 distances only and
    build the oracle's graph (the 6-node ring case), through import and through load."""
    dim = 16
    x = G.uint8_valued(8, dim, 93)
    for seed in range(1, 200):
        h = O.HnswOracle(dim, "l2sq", 16, 64, 48, seed=seed)
        h.add(np.arange(6), x[:6], threads=1)
        g = h.export()
        if g["max_level"] != 0:
            continue
        h.add([6], x[6:7], threads=1)
        want = h.export()
        if want["max_level"] != 0:
            continue  # the new node would bring upper rows: not the case under test
        res = []
        for flag in ("0", "1"):
            monkeypatch.setenv("VSG_BUILD_EDGE_DIST", flag)
            a = vsg.Index(dim, "l2sq", "f32", 16, 64, 48, seed=seed)
            a.import_graph(g)
            a.add([6], x[6:7])
            res.append(a.export())
        p = tmp_path / "ring.vsg"
        b = vsg.Index(dim, "l2sq", "f32", 16, 64, 48, seed=seed)
        b.import_graph(g)
        b.save(p)
        c = vsg.Index.load(p)
        c.add([6], x[6:7])
        res.append(c.export())
        for r in res:
            _same(r, want)
        return
    pytest.fail("no seed in 1..199 gave a level-0 graph")
