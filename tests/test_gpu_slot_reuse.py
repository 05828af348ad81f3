"""GPU: usearch index_dense's free-slot reuse on the reference's replace path.

The reference replaces a key by remove + add (/root/reference/src/index/usearch.rs:
214-221; plain removes :245).  usearch v2's index_dense queues a removed entry's slot
in `free_keys_` (a FIFO ring) and the next `add_` pops it and runs `index_gt::update`
on it: the node keeps its slot and level, its own rows are cleared and re-linked,
other nodes' links into it stay.  oracle/vsg_oracle.c restates it (orc_hnsw_add, rules
in vsg_oracle.h; checked against a literal transcription in tests/test_oracle.py);
here the GPU build is checked against the oracle:

  * one-node batches in slot order (VSG_BUILD_BATCH_MAX=1, VSG_BUILD_PERMUTE=0) on
    integer data: after rounds of remove / add churn the GPU graph equals the oracle's
    bit for bit -- every row, levels, entry point, keys, flags -- and so do the free
    ring and the search results (l2sq and ip; the split register-beam insert at
    efC 64 and the fused LDS-list insert at efC 300; an imported graph, whose edge
    distances are filled by the first add, and a built one, whose stored distances of
    links into a reused slot are refreshed);
  * the entry point's slot is not reused while it is the entry point;
  * a rejected add (duplicate key) leaves index and ring unchanged;
  * save / load keep the ring; VSG_FLAG_NO_SLOT_REUSE appends.
"""
import numpy as np
import pytest

import oracle as O
import vsg
from vsg import datagen as G

pytestmark = pytest.mark.gpu

EMPTY = 0xFFFFFFFF


def _same_graph(a, b, what=""):
    for key in ("levels", "upper_off", "adj0", "upper", "removed"):
        np.testing.assert_array_equal(a[key], b[key], err_msg=f"{key} {what}")
    live = a["removed"] == 0
    np.testing.assert_array_equal(a["keys"][live], b["keys"][live], err_msg=f"keys {what}")
    assert (a["entry"], a["max_level"]) == (b["entry"], b["max_level"]), what


def _rows(g, s):
    out = [g["adj0"][s]]
    for l in range(1, int(g["levels"][s]) + 1):
        out.append(g["upper"][int(g["upper_off"][s]) + l - 1])
    return out


@pytest.mark.parametrize("metric,M,efc,start", [("l2sq", 8, 64, "import"), ("ip", 8, 300, "build"),
                                                ("l2sq", 16, 64, "build")])
def test_reuse_one_node_batches_equal_oracle(metric, M, efc, start, monkeypatch):
    n, dim = 1500 if start == "build" else 4000, 24
    x = G.uint8_valued(n + 600, dim, 301).astype(np.float32)
    if metric == "ip":
        x = np.floor(x / 16.0)
    q = G.uint8_valued(64, dim, 302).astype(np.float32)
    monkeypatch.setenv("VSG_BUILD_PERMUTE", "0")
    monkeypatch.setenv("VSG_BUILD_BATCH_MAX", "1")
    h = O.HnswOracle(dim, metric, M, efc, 48, seed=11)
    gpu = vsg.Index(dim, metric, "f32", M, efc, 48, seed=11)
    if start == "import":  # edge distances filled by the first add
        h.add(np.arange(n), x[:n], threads=8)
        gpu.import_graph(h.export())
    else:  # one-node batches from the start: stored distances refreshed on reuse
        h.add(np.arange(n), x[:n], threads=1)
        gpu.add(np.arange(n), x[:n])
        _same_graph(gpu.export(), h.export(), "initial build")
    rng = np.random.default_rng(5)
    live = list(range(n))
    nxt, row = n, n
    for rnd in range(4):
        rm = rng.choice(live, 60, replace=False)
        if rnd == 1:  # the entry point's slot goes too (if its key is still live)
            e = gpu.graph_info()["entry"]
            ek = int(gpu.export()["keys"][e])
            if gpu.contains(ek):
                rm = np.unique(np.append(rm, ek))
        assert gpu.remove(rm) == h.remove(rm) == len(rm)
        live = [k for k in live if k not in set(rm.tolist())]
        np.testing.assert_array_equal(gpu.free_slots(), h.free_list())
        # more keys than free slots in the last round: reuse + append in one call
        nadd = 40 if rnd < 3 else 120
        keys = np.arange(nxt, nxt + nadd, dtype=np.uint64)
        vecs = x[row:row + nadd]
        gpu.add(keys, vecs)
        h.add(keys, vecs, threads=1)
        live += keys.tolist()
        nxt += nadd
        row += nadd
        a, b = gpu.export(), h.export()
        _same_graph(a, b, f"round {rnd}")
        np.testing.assert_array_equal(gpu.free_slots(), h.free_list())
        if rnd == 1:
            assert e in gpu.free_slots().tolist()  # kept while it is the entry point
    assert gpu.size() == h.size() == len(live)
    for ef, k in ((48, 10), (200, 20)):
        ok, od, oc = h.search(q, k, ef)
        m = gpu.search(q, k, ef)
        np.testing.assert_array_equal(m.counts, oc)
        np.testing.assert_array_equal(m.keys, ok)
        np.testing.assert_array_equal(m.distances, od)
    g = gpu.export()
    for s in range(len(g["keys"])):
        for r in _rows(g, s):
            ids = r[r != EMPTY].tolist()
            assert s not in ids and len(set(ids)) == len(ids), s  # no self links, no duplicates
    assert gpu.stats()["slots_reused"] > 0


def test_reuse_batched_build_keeps_quality_and_bookkeeping():
    """Batched (default) GPU adds over freed slots, from the oracle's own graph: slots do
    not grow, each reused slot keeps its level, rows hold no self link or duplicate, and
    recall at matched ef stays within 0.5 % of the oracle run through the same remove/add
    calls -- whose multi-key adds are a sequence of single adds (usearch's add_ pops one
    free slot per call), while the GPU re-links consecutive batches of graph / 4096
    keys, each staged right before it.  (Both start from one graph: a GPU-built start
    graph responds to usearch's update semantics a little differently, which is the
    build's, not the update's; profiles/r05_reuse_variants.jsonl.)"""
    n, dim = 30000, 64
    x = G.clustered(n + 6000, dim, 311, 9)
    q = G.clustered(500, dim, 312, 9)
    gpu = vsg.Index(dim, "cos", "f32", 16, 128, 64, seed=4)
    h = O.HnswOracle(dim, "cos", 16, 128, 64, seed=4)
    h.add(np.arange(n), x[:n], threads=8)
    gpu.import_graph(h.export())
    lv0 = gpu.export()["levels"].copy()
    rng = np.random.default_rng(8)
    cur = x[:n].copy()
    for rnd in range(3):
        keys = np.sort(rng.choice(n, 2000, replace=False)).astype(np.uint64)
        gpu.remove(keys)
        h.remove(keys)
        new = x[n + 2000 * rnd:n + 2000 * (rnd + 1)]
        gpu.add(keys, new)
        h.add(keys, new, threads=8)
        cur[keys.astype(np.int64)] = new
    g = gpu.export()
    assert len(g["keys"]) == n and gpu.size() == n  # every replace reused a slot
    np.testing.assert_array_equal(g["levels"], lv0)
    for s in range(0, n, 7):
        for r in _rows(g, s):
            ids = r[r != EMPTY].tolist()
            assert s not in ids and len(set(ids)) == len(ids)
    gt, _, _ = O.exact_search("cos", cur, q, 10, threads=8)

    def rec(found):
        return np.mean([len(set(found[i].tolist()) & set(gt[i].tolist())) / 10 for i in range(len(q))])
    for ef in (16, 64):
        rg, rc = rec(gpu.search(q, 10, ef).keys), rec(h.search(q, 10, ef)[0])
        print(f"churned 30k cos ef={ef}: GPU {rg:.4f} oracle {rc:.4f}")
        assert abs(rg - rc) <= 0.005, (ef, rg, rc)


def test_reuse_rejected_add_changes_nothing():
    n, dim = 2000, 16
    x = G.uint8_valued(n + 10, dim, 321).astype(np.float32)
    gpu = vsg.Index(dim, "l2sq", "f32", 8, 64, 32, seed=1)
    gpu.add(np.arange(n), x[:n])
    gpu.remove([3, 4, 5])
    before = gpu.export()
    ring = gpu.free_slots().copy()
    with pytest.raises(vsg.DuplicateKeyError):
        gpu.add([n, 7], x[n:n + 2])  # 7 is live: nothing is inserted
    with pytest.raises(vsg.DuplicateKeyError):
        gpu.add([n, n], x[n:n + 2])
    np.testing.assert_array_equal(gpu.free_slots(), ring)
    after = gpu.export()
    for key in ("adj0", "upper", "removed", "keys"):
        np.testing.assert_array_equal(before[key], after[key])
    assert gpu.size() == n - 3 and not gpu.contains(n)
    gpu.add([n], x[n:n + 1])  # then reuses slot 3, the oldest removal
    assert int(gpu.export()["keys"][3]) == n
    np.testing.assert_array_equal(gpu.free_slots(), ring[1:])


def test_reuse_ring_survives_save_load_and_flag_appends(tmp_path):
    n, dim = 3000, 32
    x = G.clustered(n + 50, dim, 331, 3)
    gpu = vsg.Index(dim, "l2sq", "f32", 16, 64, 32, seed=2)
    gpu.add(np.arange(n), x[:n])
    gpu.remove([900, 10, 2500, 11])
    p = tmp_path / "r.vsg"
    gpu.save(p)
    assert vsg.file_info(p)["version"] == 2
    ld = vsg.Index.load(p)
    np.testing.assert_array_equal(ld.free_slots(), [900, 10, 2500, 11])
    ld.add([n], x[n:n + 1])
    gpu.add([n], x[n:n + 1])
    np.testing.assert_array_equal(ld.free_slots(), gpu.free_slots())
    assert int(ld.export()["keys"][900]) == n
    # append-only: removed slots stay tombstones, the add grows the slot count
    ap = vsg.Index(dim, "l2sq", "f32", 16, 64, 32, seed=2, slot_reuse=False)
    ap.add(np.arange(n), x[:n])
    ap.remove([1, 2])
    ap.add([n], x[n:n + 1])
    assert ap.graph_info()["slots"] == n + 1 and ap.free_slots().tolist() == [1, 2]
    assert ap.compact() == 2 and len(ap.free_slots()) == 0
