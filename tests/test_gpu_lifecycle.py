"""GPU: compaction and persistence of an index.

Compaction keeps the live set and its slot order, so exact search is
bit-identical before and after; the rebuilt graph is checked for recall
against the oracle's exact answers over the live rows.  A saved and reloaded
index answers bit-identically (HNSW and exact), keeps keys / tombstones /
capacity growth working, and a damaged file is refused.
"""
import numpy as np
import pytest

import oracle as O
import vsg
from vsg import datagen as G

pytestmark = pytest.mark.gpu

NOKEY = np.uint64(2**64 - 1)


def recall(found, truth, k):
    return float(np.mean([len(set(found[i][:k].tolist()) & set(truth[i][:k].tolist())) / k
                          for i in range(truth.shape[0])]))


@pytest.mark.parametrize("metric,quant", [("l2sq", "f32"), ("ip", "f16"), ("cos", "f32")])
def test_compact_keeps_exact_answers_and_recall(metric, quant):
    n, dim = 12000, 64
    x = G.uint8_valued(n, dim, 81) if metric == "l2sq" else G.clustered(n, dim, *G.config_seeds(1)[::2])
    q = G.uint8_valued(100, dim, 82) if metric == "l2sq" else G.clustered(100, dim, *G.config_seeds(1)[1:])
    idx = vsg.Index(dim, metric, quant, 16, 128, 64, seed=3)
    idx.add(np.arange(n), x)
    rng = np.random.default_rng(1)
    dead = rng.choice(n, size=5000, replace=False)
    assert idx.remove(dead) == 5000
    before = idx.exact_search(q, 10)
    assert idx.graph_info()["slots"] == n
    assert idx.compact() == 5000
    assert idx.compact() == 0  # nothing left to drop
    assert idx.size() == n - 5000 and idx.graph_info()["slots"] == n - 5000
    after = idx.exact_search(q, 10)
    np.testing.assert_array_equal(before.keys, after.keys)
    np.testing.assert_array_equal(before.distances, after.distances)
    live = np.setdiff1d(np.arange(n), dead)
    assert all(idx.contains(int(k)) for k in live[:50]) and not any(idx.contains(int(k)) for k in dead[:50])
    m = idx.search(q, 10, 64)
    assert not np.isin(m.keys, dead).any()
    # the rebuilt graph is as good as a fresh build over the live rows
    fresh = vsg.Index(dim, metric, quant, 16, 128, 64, seed=3)
    fresh.add(live, x[live])
    r_fresh = recall(fresh.search(q, 10, 64).keys, after.keys, 10)
    assert recall(m.keys, after.keys, 10) >= r_fresh - 0.02
    if metric == "l2sq":  # oracle over the live rows (integer data: exact distances)
        ok, od, _ = O.exact_search("l2sq", x[live], q, 10)
        np.testing.assert_array_equal(after.distances, od)
        np.testing.assert_array_equal(after.keys, live[ok.astype(np.int64)].astype(np.uint64))
    # dropped keys can come back; compacted keys can go
    idx.add(dead[:100], x[dead[:100]])
    assert idx.remove(live[:10]) == 10
    if metric != "ip":  # self is the nearest neighbour under l2sq / cos
        m = idx.search(x[dead[:100]], 1, 64)
        assert (m.keys[:, 0] == dead[:100]).mean() > 0.95


def test_compact_everything_and_exact_only():
    idx = vsg.Index(8, "l2sq")
    idx.add(np.arange(50), np.random.default_rng(0).standard_normal((50, 8)).astype(np.float32))
    idx.remove(np.arange(50))
    assert idx.compact() == 50 and idx.size() == 0
    m = idx.search(np.zeros((2, 8), np.float32), 3)
    assert (m.counts == 0).all() and (m.keys == NOKEY).all()
    idx.add([5], np.ones((1, 8), np.float32))
    assert int(idx.search(np.zeros((1, 8), np.float32), 1).keys[0, 0]) == 5
    e = vsg.Index(16, "ip", exact_only=True)
    xe = G.uint8_valued(500, 16, 3)
    e.add(np.arange(500), xe)
    e.remove(np.arange(0, 500, 2))
    before = e.exact_search(xe[:20], 5)
    assert e.compact() == 250
    after = e.exact_search(xe[:20], 5)
    np.testing.assert_array_equal(before.keys, after.keys)


@pytest.mark.parametrize("metric,quant,dim", [("cos", "f32", 768), ("l2sq", "f16", 128), ("ip", "f32", 40)])
def test_save_load_roundtrip_bitexact(tmp_path, metric, quant, dim):
    n = 20000
    bs, qs, ms = G.config_seeds(1)
    x = G.clustered(n, dim, bs, ms)
    q = G.clustered(200, dim, qs, ms)
    a = vsg.Index(dim, metric, quant, 16, 128, 48, seed=9)
    a.add(np.arange(n) * 3 + 1, x)
    a.remove(np.arange(0, 600) * 3 + 1)
    p = tmp_path / "idx.vsg"
    a.save(p)
    info = vsg.file_info(p)
    assert info["slots"] == n and info["live"] == n - 600 and info["dimensions"] == dim
    assert info["metric"] == metric and info["quantization"] == quant
    b = vsg.Index.load(p, device=0)
    assert b.size() == a.size() and b.graph_info() == a.graph_info()
    for ef in (0, 16, 100):
        ma, mb = a.search(q, 10, ef), b.search(q, 10, ef)
        np.testing.assert_array_equal(ma.keys, mb.keys)
        np.testing.assert_array_equal(ma.distances, mb.distances)
    ea, eb = a.exact_search(q, 10), b.exact_search(q, 10)
    np.testing.assert_array_equal(ea.keys, eb.keys)
    np.testing.assert_array_equal(ea.distances, eb.distances)
    ga, gb = a.export(), b.export()
    for k in ("keys", "removed", "levels", "adj0", "upper_off", "upper", "vectors"):
        np.testing.assert_array_equal(ga[k], gb[k])
    # the loaded index keeps working: duplicate keys, new rows, removes
    with pytest.raises(vsg.DuplicateKeyError):
        b.add([1801], x[1:2])  # key of row 600: live
    b.add([1], x[0:1])  # key 1 was removed: may come back
    b.add(np.arange(500) + 10**9, x[:500])
    assert b.size() == n - 600 + 1 + 500
    assert b.remove([1, 1801, 1804, 4]) == 3  # key 4 was removed before the save


def test_load_rejects_damaged_payload(tmp_path):
    a = vsg.Index(16, "l2sq")
    a.add(np.arange(300), G.uint8_valued(300, 16, 4))
    p = tmp_path / "d.vsg"
    a.save(p)
    raw = bytearray(p.read_bytes())
    raw[200] ^= 0x10  # inside the stored rows
    p.write_bytes(bytes(raw))
    with pytest.raises(vsg.VsgError, match="checksum"):
        vsg.Index.load(p)
    p.write_bytes(bytes(raw[:-8]))
    with pytest.raises(vsg.VsgError):
        vsg.Index.load(p)


def test_load_validates_crafted_graph(tmp_path):
    """A file whose checksums are valid but whose graph is not: adjacency
    ids past the slot count, an entry point off the top level, upper rows outside
    the table, a reserved live key -- each refused before any kernel reads it."""
    from test_persistence_format import write_file
    M, slots, E = 4, 6, 0xFFFFFFFF
    chain = np.full((slots, 2 * M), 0xFFFFFFFF, np.uint32)
    for s in range(slots):  # a ring on level 0
        chain[s, 0], chain[s, 1] = (s + 1) % slots, (s - 1) % slots
    ok = dict(dim=8, M=M, slots=slots, live=slots, upper_rows=0, entry=2, max_level=0, adj0=chain)
    p = tmp_path / "g.vsg"
    write_file(p, **ok)
    b = vsg.Index.load(p)
    assert b.size() == slots and int(b.search(np.zeros((1, 8), np.float32), 3).counts[0]) == 3
    # a valid two-level graph still loads: slot 2 (level 1, the entry) links slot 4 (level 1)
    two = dict(ok, levels=[0, 0, 1, 0, 1, 0], max_level=1, upper_rows=2, upper_off=[E, E, 0, E, 1, E],
               upper=[4, E, E, E, 2, E, E, E])
    write_file(p, **two)
    assert int(vsg.Index.load(p).search(np.zeros((1, 8), np.float32), 3).counts[0]) == 3
    bad = chain.copy()
    bad[3, 2] = slots + 5
    cases = [(dict(ok, adj0=bad), "adjacency"),
             (dict(ok, entry=slots), "entry"),
             (dict(ok, max_level=2), "entry"),
             (dict(ok, levels=[0, 0, 0, 1, 0, 0]), "level"),
             (dict(ok, levels=[0, 0, 1, 0, 0, 0], max_level=1, upper_off=[0xFFFFFFFF, 0xFFFFFFFF, 0] + [0xFFFFFFFF] * 3),
              "upper rows"),
             # an upper row of level 1 naming a level-0 node (its upper_off is EMPTY)
             (dict(ok, levels=[0, 0, 1, 0, 0, 0], max_level=1, upper_rows=1, upper_off=[E, E, 0, E, E, E],
                   upper=[4, E, E, E]), "below that level"),
             (dict(ok, keys=[0, 1, 2, 2**64 - 2, 4, 5]), "reserved"),
             (dict(ok, keys=[0, 1, 2, 3, 3, 5]), "duplicate")]
    for kw, msg in cases:
        write_file(p, **kw)
        with pytest.raises(vsg.VsgError, match=msg):
            vsg.Index.load(p)


def test_import_validates_graph():
    h = vsg.Index(8, "l2sq", connectivity=4)
    n = 10
    g = {"vectors": np.zeros((n, 8), np.float32), "keys": np.arange(n, dtype=np.uint64),
         "removed": np.zeros(n, np.uint8), "levels": np.zeros(n, np.int8),
         "adj0": np.full((n, 8), 0xFFFFFFFF, np.uint32), "upper_off": np.full(n, 0xFFFFFFFF, np.uint32),
         "upper": np.zeros((0, 4), np.uint32), "entry": 0, "max_level": 0}
    g["adj0"][1, 0] = 99
    with pytest.raises(vsg.VsgError, match="adjacency"):
        h.import_graph(g)
    g["adj0"][1, 0] = 2
    g["entry"] = 10
    with pytest.raises(vsg.VsgError, match="entry"):
        h.import_graph(g)
    g["entry"] = 0
    # slot 0 (level 1, the entry) lists slot 5 (level 0) in its level-1 row
    g2 = dict(g, levels=np.zeros(n, np.int8), max_level=1, upper=np.full((1, 4), 0xFFFFFFFF, np.uint32),
              upper_off=np.full(n, 0xFFFFFFFF, np.uint32))
    g2["levels"][0] = 1
    g2["upper_off"][0] = 0
    g2["upper"][0, 0] = 5
    with pytest.raises(vsg.VsgError, match="below that level"):
        h.import_graph(g2)
    h.import_graph(g)
    assert h.size() == n


def test_reserved_keys_never_match():
    """UINT64_MAX-1 is the key map's tombstone: removing or probing it after ordinary
    removals must not hit a tombstone -- size stays right."""
    idx = vsg.Index(4, "l2sq")
    idx.add(np.arange(100), G.uint8_valued(100, 4, 2))
    assert idx.remove(np.arange(0, 100, 3)) == 34
    for _ in range(3):
        assert idx.remove([2**64 - 2]) == 0
        assert idx.remove([2**64 - 1]) == 0
    assert not idx.contains(2**64 - 2) and idx.size() == 66
    with pytest.raises(vsg.VsgError):
        idx.add([2**64 - 2], np.zeros((1, 4), np.float32))
    assert idx.remove([0, 1, 1, 2]) == 2  # 0 was removed before; 1 listed twice counts once
    assert idx.size() == 64
