"""CPU: pin the oracle (oracle/vsg_oracle.c) against the golden fixtures and
the reference's own known-answer tests, and check its HNSW semantics.

Parity status: exact path pinned by numpy-f64 goldens + the
reference KATs; the HNSW restatement is "parity unpinned" vs upstream usearch
(not buildable/importable here) and is checked for recall and API semantics.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, golden_inputs, load_golden
from vsg import datagen as G


@pytest.mark.parametrize("name", ["g1_u8_l2sq.npz", "g1_u8_ip.npz"])
def test_oracle_exact_bitexact_integer(name):
    g = load_golden(name)
    x, q = golden_inputs(g)
    k = int(g["k"])
    ok, od, oc = O.exact_search(str(g["metric"]), x, q, k)
    assert (oc == k).all()
    np.testing.assert_array_equal(ok.astype(np.int64), g["ids"])
    np.testing.assert_array_equal(od.astype(np.float64), g["dist"])


@pytest.mark.parametrize("name", ["g2_cl_ip.npz", "g2_cl_cos.npz", "g2_cl_l2sq.npz", "g3_cl768_cos.npz"])
def test_oracle_exact_float(name):
    g = load_golden(name)
    x, q = golden_inputs(g)
    k = int(g["k"])
    ok, od, _ = O.exact_search(str(g["metric"]), x, q, k)
    # distances within f32 accumulation tolerance of the f64 truth
    scale = np.maximum(1.0, np.abs(g["dist"]))
    assert np.max(np.abs(od - g["dist"]) / scale) < 1e-4
    # ids equal except where the f64 gap to the neighbouring rank is a near-tie
    for i in range(ok.shape[0]):
        if set(ok[i].tolist()) != set(g["ids"][i].tolist()):
            assert g["gap"][i] < 1e-4, (i, ok[i], g["ids"][i])


def _kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


class KeyedOracle:
    """Host key map over the oracle, as the reference actor does
    (src/index/usearch.rs:174-233: monotonic u64 keys, replace = remove + add)."""

    def __init__(self, dim, metric):
        self.idx = O.HnswOracle(dim, metric)
        self.pk2key = {}
        self.key2pk = {}
        self.next = 0

    def add_or_replace(self, pk, emb):
        pk = tuple(pk)
        if pk in self.pk2key:
            key = self.pk2key[pk]
            self.idx.remove([key])
        else:
            key = self.next
            self.next += 1
            self.pk2key[pk] = key
            self.key2pk[key] = pk
        # usearch add of a removed key is allowed
        self.idx.add([key], np.array([emb], np.float32))

    def remove(self, pk):
        pk = tuple(pk)
        key = self.pk2key.pop(pk, None)
        if key is not None:
            self.key2pk.pop(key)
            self.idx.remove([key])

    def ann(self, emb, limit):
        k, d, c = self.idx.search(np.array([emb], np.float32), limit)
        return [self.key2pk[int(x)] for x in k[0][: int(c[0])]], d[0][: int(c[0])]

    def count(self):
        return self.idx.size()


@pytest.mark.parametrize("metric", ["l2sq", "ip"])
def test_oracle_reference_unit_kat(metric):
    """/root/reference/src/index/usearch.rs:322-425 re-expressed."""
    kat = _kats()["unit_actor"]
    a = KeyedOracle(kat["dimensions"], metric)
    for st in kat["steps"]:
        if st["op"] == "add_or_replace":
            a.add_or_replace(st["pk"], st["embedding"])
        elif st["op"] == "remove":
            a.remove(st["pk"])
        elif st["op"] == "count":
            assert a.count() == st["expect"]
        elif st["op"] == "ann":
            pks, dists = a.ann(st["embedding"], st["limit"])
            assert len(pks) == 1 and len(dists) == 1
            assert list(pks[0]) == st["expect_pk"]


@pytest.mark.parametrize("metric", ["l2sq", "ip"])
def test_oracle_reference_integration_kat(metric):
    """/root/reference/tests/integration/usearch.rs:74-123 re-expressed."""
    kat = _kats()["integration"]
    a = KeyedOracle(kat["dimensions"], metric)
    for pk, emb in kat["rows"]:
        a.add_or_replace(pk, emb)
    assert a.count() == kat["count"]
    pks, _ = a.ann(kat["ann"]["embedding"], kat["ann"]["limit"])
    assert list(pks[0]) == kat["ann"]["expect_pk"]


def test_oracle_hnsw_recall_and_determinism():
    bs, qs, ms = G.config_seeds(1)
    x = G.clustered(5000, 64, bs, ms)
    q = G.clustered(100, 64, qs, ms)
    gk, _, _ = O.exact_search("l2sq", x, q, 10)
    h1 = O.HnswOracle(64, "l2sq", 16, 64, 64, seed=7)
    h1.add(np.arange(5000), x, threads=1)
    h2 = O.HnswOracle(64, "l2sq", 16, 64, 64, seed=7)
    h2.add(np.arange(5000), x, threads=1)
    k1, d1, _ = h1.search(q, 10)
    k2, d2, _ = h2.search(q, 10)
    np.testing.assert_array_equal(k1, k2)  # sequential build is deterministic
    rec = np.mean([len(set(k1[i]) & set(gk[i])) / 10 for i in range(100)])
    assert rec >= 0.97
    # results ascending
    assert (np.diff(d1, axis=1) >= 0).all()


def test_oracle_remove_and_duplicates():
    x = G.uint8_valued(300, 16, 3)
    h = O.HnswOracle(16, "l2sq", 8, 32, 32)
    h.add(np.arange(300), x)
    assert h.size() == 300
    with pytest.raises(KeyError):
        h.add([5], x[:1])
    assert h.remove([5, 6, 999]) == 2
    assert h.size() == 298
    k, _, c = h.search(x[5:7], 5)
    assert 5 not in k[0][: int(c[0])] and 6 not in k[1][: int(c[1])]
    h.add([5], x[5:6])  # re-add after removal is allowed
    k, d, _ = h.search(x[5:6], 1)
    assert int(k[0][0]) == 5 and d[0][0] == 0.0


def test_oracle_export_import_roundtrip():
    x = G.uint8_valued(2000, 32, 11)
    q = G.uint8_valued(50, 32, 12)
    h = O.HnswOracle(32, "l2sq", 8, 64, 32, seed=3)
    h.add(np.arange(2000), x)
    h.remove([1, 2, 3])
    g = h.export()
    h2 = O.HnswOracle(32, "l2sq", 8, 64, 32, seed=3)
    h2.import_graph(g)
    assert h2.size() == h.size()
    a = h.search(q, 10)
    b = h2.search(q, 10)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def test_oracle_empty_and_padding():
    h = O.HnswOracle(8, "l2sq")
    k, d, c = h.search(np.zeros((2, 8), np.float32), 3)
    assert (c == 0).all() and (k == np.uint64(2**64 - 1)).all() and np.isinf(d).all()
    h.add([1, 2], np.eye(2, 8, dtype=np.float32))
    k, d, c = h.search(np.zeros((1, 8), np.float32), 5)
    assert int(c[0]) == 2 and k[0][2] == np.uint64(2**64 - 1)


def test_level_sampling_distribution():
    lv = np.array([O.sample_level(123, s, 16) for s in range(20000)])
    # P(level >= 1) = 1/M for the 1/ln(M) multiplier
    assert abs((lv >= 1).mean() - 1 / 16) < 0.01
    assert lv.max() <= 30


# ------------------------------------------- usearch v2 semantics (round 4) --

def test_oracle_new_node_keeps_at_most_M_forward_links():
    """usearch connect_new_node_ refines with config_.connectivity (M) on every
    level: a node's own level-0 row holds <= M entries until other nodes' reverse
    links land (reconnect_neighbor_nodes_ fills it up to M0 = 2M)."""
    M, n = 8, 1200
    x = G.uint8_valued(n + 10, 24, 101).astype(np.float32)
    h = O.HnswOracle(24, "l2sq", M, 64, 32, seed=13)
    h.add(np.arange(n), x[:n], threads=1)
    for i in range(10):  # the newest node has only its forward links
        h.add([n + i], x[n + i:n + i + 1], threads=1)
        g = h.export()
        row = g["adj0"][n + i]
        assert (row != 0xFFFFFFFF).sum() <= M
        for l in range(1, int(g["levels"][n + i]) + 1):
            up = g["upper"][int(g["upper_off"][n + i]) + l - 1]
            assert (up != 0xFFFFFFFF).sum() <= M
    fill = (g["adj0"] != 0xFFFFFFFF).sum(1)
    assert fill.max() <= 2 * M and fill.max() > M  # reverse links still fill to M0


def test_oracle_refine_early_return_complete_small_graph():
    """refine_ returns fewer than `needed` candidates unfiltered: while the graph
    holds fewer than M nodes every new node links to all of them, and the reverse
    links (rows below M0) append, so M nodes form a complete graph (the heuristic
    would drop some: clustered data has close pairs)."""
    M = 16
    x = G.clustered(M, 32, 5, 6)
    h = O.HnswOracle(32, "l2sq", M, 64, 32, seed=2)
    h.add(np.arange(M), x, threads=1)
    g = h.export()
    for i in range(M):
        row = g["adj0"][i]
        assert sorted(row[row != 0xFFFFFFFF].tolist()) == [j for j in range(M) if j != i]


@pytest.mark.parametrize("frac", [0.3, 0.7])
def test_oracle_removed_entries_are_traversed_not_returned(frac):
    """index_dense's `allow` predicate: removed nodes never take a result slot,
    so k live results come back at ef = k even with 70 % tombstones (a
    post-filter of the ef-beam would return about (1 - frac) k)."""
    n, dim = 4000, 32
    x = G.uint8_valued(n, dim, 111).astype(np.float32)
    q = G.uint8_valued(100, dim, 112).astype(np.float32)
    h = O.HnswOracle(dim, "l2sq", 16, 64, 10, seed=1)
    h.add(np.arange(n), x)
    rm = np.random.default_rng(3).choice(n, int(frac * n), replace=False)
    h.remove(rm)
    k, d, c = h.search(q, 10, 10)
    assert (c == 10).all()
    assert not np.isin(k.astype(np.int64), rm).any()
    assert (np.diff(d, axis=1) >= 0).all()


@pytest.mark.parametrize("frac", [0.0, 0.4, 0.8])
def test_oracle_matches_literal_usearch_loops(frac):
    """The C restatement (set formulation, (distance, slot) keys) against a
    literal transcription of usearch's heap loops (tests/usearch_literal.py:
    search_to_insert_, refine_, reconnect_neighbor_nodes_, search_for_one_,
    search_to_find_in_base_ with the `allow` predicate) on float data (no
    ties): identical graph, identical results with tombstones."""
    import usearch_literal as UL
    n, dim, M, efc = 400, 12, 6, 24
    x = G.clustered(n, dim, 7, 8)
    q = G.clustered(40, dim, 9, 8)
    h = O.HnswOracle(dim, "l2sq", M, efc, 16, seed=17)
    h.add(np.arange(n), x, threads=1)
    lit = UL.LiteralHnsw(dim, "l2sq", M, efc, seed=17)
    for i in range(n):
        lit.add(i, x[i])
    g = h.export()
    assert (g["entry"], g["max_level"]) == (lit.entry, lit.max_level)
    for s in range(n):
        for l in range(int(g["levels"][s]) + 1):
            if l == 0:
                row = g["adj0"][s]
            else:
                row = g["upper"][int(g["upper_off"][s]) + l - 1]
            assert row[row != 0xFFFFFFFF].tolist() == lit.links[s][l], (s, l)
    rm = np.random.default_rng(5).choice(n, int(frac * n), replace=False)
    h.remove(rm)
    lit.remove(rm)
    for ef in (6, 16, 50):
        k, d, c = h.search(q, 6, ef)
        for i in range(len(q)):
            lk, ld = lit.search(q[i], 6, ef)
            assert k[i][: int(c[i])].tolist() == lk, (ef, i)
            np.testing.assert_array_equal(d[i][: int(c[i])], np.array(ld, np.float32))


def _graph_rows(g, s, l):
    row = g["adj0"][s] if l == 0 else g["upper"][int(g["upper_off"][s]) + l - 1]
    return row[row != 0xFFFFFFFF].tolist()


@pytest.mark.parametrize("metric", ["l2sq", "ip"])
def test_oracle_slot_reuse_matches_literal_usearch_update(metric):
    """Free-slot reuse (usearch index_dense add_ -> index_gt::update, the
    reference's replace = remove + add, /root/reference/src/index/usearch.rs:
    214-221, 245): remove/add churn in calls of 1 and of several keys, the C
    restatement against the literal transcription -- same free ring, same slot
    for every key, identical graph (every row, order included) and identical
    search results with the tombstones left over."""
    import usearch_literal as UL
    n, dim, M, efc = 300, 12, 6, 24
    x = G.clustered(n + 400, dim, 31, 8)
    if metric == "ip":
        x = x / np.linalg.norm(x, axis=1, keepdims=True)
    q = G.clustered(30, dim, 33, 8)
    h = O.HnswOracle(dim, metric, M, efc, 16, seed=23)
    lit = UL.LiteralHnsw(dim, metric, M, efc, seed=23)
    h.add(np.arange(n), x[:n], threads=1)
    for i in range(n):
        lit.add(i, x[i])
    slot_key = {i: i for i in range(n)}
    rng = np.random.default_rng(7)
    nxt = n
    for step in range(12):
        live = [s for s in slot_key if s not in lit.removed]
        rm = rng.choice(live, int(rng.integers(1, 25)), replace=False)
        h.remove(np.array([slot_key[int(s)] for s in rm], np.uint64))
        lit.remove(rm)
        np.testing.assert_array_equal(h.free_list(), np.array(list(lit.free), np.uint32))
        nadd = int(rng.integers(1, 30)) if step % 3 else 1
        keys = np.arange(nxt, nxt + nadd, dtype=np.uint64)
        vecs = x[nxt:nxt + nadd]  # fresh rows: no exact ties (the literal compares distances only)
        h.add(keys, vecs, threads=1)
        slots = lit.add_batch(list(vecs))
        for key, s in zip(keys, slots):
            slot_key[s] = int(key)
        nxt += nadd
        np.testing.assert_array_equal(h.free_list(), np.array(list(lit.free), np.uint32))
    g = h.export()
    assert (g["entry"], g["max_level"]) == (lit.entry, lit.max_level)
    assert len(g["keys"]) == len(lit.vecs)
    for s in range(len(lit.vecs)):
        assert int(g["keys"][s]) == slot_key[s] or s in lit.removed
        assert bool(g["removed"][s]) == (s in lit.removed)
        for l in range(int(g["levels"][s]) + 1):
            assert _graph_rows(g, s, l) == lit.links[s][l], (s, l)
    for ef in (6, 16, 50):
        k, d, c = h.search(q, 6, ef)
        for i in range(len(q)):
            ls, ld = lit.search(q[i], 6, ef)
            assert k[i][: int(c[i])].tolist() == [slot_key[s] for s in ls], (ef, i)
            np.testing.assert_array_equal(d[i][: int(c[i])], np.array(ld, np.float32))


@pytest.mark.parametrize("metric", ["l2sq", "ip"])
def test_oracle_replace_stream_matches_literal_usearch(metric):
    """The reference's upsert stream one message at a time (/root/reference/src/index/
    usearch.rs:214-221: remove the live key, then add; fed per key by
    src/monitor_items.rs:56-80): orc_hnsw_replace against the literal transcription's
    remove + add_one per message -- existing keys, new keys and a key repeated inside
    one call, with net deletes interleaved so the free ring is not empty.  Same slot
    per key, same ring, identical graph and search results."""
    import usearch_literal as UL
    n, dim, M, efc = 250, 12, 6, 24
    x = G.clustered(n + 600, dim, 51, 8)
    if metric == "ip":
        x = x / np.linalg.norm(x, axis=1, keepdims=True)
    q = G.clustered(30, dim, 53, 8)
    h = O.HnswOracle(dim, metric, M, efc, 16, seed=29)
    lit = UL.LiteralHnsw(dim, metric, M, efc, seed=29)
    h.add(np.arange(n), x[:n], threads=1)
    for i in range(n):
        lit.add(i, x[i])
    slot_of = {i: i for i in range(n)}
    rng = np.random.default_rng(11)
    row = n
    for step in range(8):
        if step % 3 == 2:  # a few net deletes: later adds take these slots first
            gone = rng.choice(sorted(slot_of), 5, replace=False)
            h.remove(np.array(gone, np.uint64))
            lit.remove([slot_of.pop(int(k)) for k in gone])
        nrep = int(rng.integers(5, 40))
        keys = rng.integers(0, n + 60, nrep).astype(np.uint64)  # some new, maybe repeated
        keys[-1] = keys[0]
        vecs = x[row:row + nrep]
        row += nrep
        st = h.replace(keys, vecs)
        assert (st == 0).all()
        for key, v in zip(keys.tolist(), vecs):
            lit.replace(slot_of, key, v)
        np.testing.assert_array_equal(h.free_list(), np.array(list(lit.free), np.uint32))
    g = h.export()
    assert (g["entry"], g["max_level"]) == (lit.entry, lit.max_level)
    assert h.size() == len(slot_of)
    key_of = {s: k for k, s in slot_of.items()}
    for s in range(len(lit.vecs)):
        assert bool(g["removed"][s]) == (s in lit.removed)
        if s in key_of:
            assert int(g["keys"][s]) == key_of[s]
        for l in range(int(g["levels"][s]) + 1):
            assert _graph_rows(g, s, l) == lit.links[s][l], (s, l)
    for ef in (6, 16, 50):
        k, d, c = h.search(q, 6, ef)
        for i in range(len(q)):
            ls, ld = lit.search(q[i], 6, ef)
            assert k[i][: int(c[i])].tolist() == [key_of[s] for s in ls], (ef, i)
            np.testing.assert_array_equal(d[i][: int(c[i])], np.array(ld, np.float32))


def test_oracle_slot_reuse_rules():
    """The reuse rules on their own: a replaced key takes the OLDEST free slot
    (FIFO), keeps that slot's level, never links to itself, the entry point's
    slot stays in the ring while it is the entry, rows hold no duplicate ids,
    and with reuse off the add appends (round-4 behaviour)."""
    n, dim = 2000, 16
    x = G.clustered(n + 200, dim, 41, 8)
    h = O.HnswOracle(dim, "l2sq", 8, 48, 32, seed=3)
    h.add(np.arange(n), x[:n], threads=1)
    g0 = h.export()
    e, _ = h.entry()
    rm = np.array([17, int(e), 5, 900], np.uint64)  # slot == key here
    h.remove(rm)
    assert h.free_list().tolist() == [17, e, 5, 900]
    h.add(np.array([n, n + 1], np.uint64), x[n:n + 2], threads=1)
    g = h.export()
    assert h.free_list().tolist() == [e, 900]        # 17 then 5 reused; the entry skipped
    assert int(g["keys"][17]) == n and int(g["keys"][5]) == n + 1
    assert g["levels"][17] == g0["levels"][17] and g["levels"][5] == g0["levels"][5]
    assert h.slots() == n and h.size() == n - 2
    for s in range(h.slots()):
        for l in range(int(g["levels"][s]) + 1):
            row = _graph_rows(g, s, l)
            assert s not in row and len(set(row)) == len(row), (s, l)
    h.set_slot_reuse(False)
    h.add(np.array([n + 2], np.uint64), x[n + 2:n + 3], threads=1)
    assert h.slots() == n + 1 and h.free_list().tolist() == [e, 900]
