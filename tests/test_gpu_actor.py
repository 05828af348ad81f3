"""GPU: the coalescing actor (include/vsg.h "Actor") behind the reference's
message API (src/index/usearch.rs:141-311)."""
import ctypes as C
import threading

import numpy as np
import pytest

import oracle as O
import vsg
from vsg import datagen as G
from vsg._lib import check, lib
from vsg.actor import Actor, UsearchIndex, new_usearch

from test_gpu_parity import _kats

pytestmark = pytest.mark.gpu


def _direct_search(actor, q, k, ef):
    h = lib().vsg_actor_index(actor._h)
    nq = q.shape[0]
    keys = np.empty((nq, k), np.uint64)
    dist = np.empty((nq, k), np.float32)
    cnt = np.empty(nq, np.uint64)
    q = np.ascontiguousarray(q, np.float32)
    check(lib().vsg_index_search(h, C.c_void_p(q.ctypes.data), nq, k, ef, C.c_void_p(keys.ctypes.data),
                                 C.c_void_p(dist.ctypes.data), C.c_void_p(cnt.ctypes.data)))
    return keys, dist, cnt


@pytest.mark.parametrize("metric", ["l2sq", "ip"])
def test_actor_reference_unit_kat(metric):
    """src/index/usearch.rs:322-425 through the factory / IndexExt surface."""
    kat = _kats()["unit_actor"]
    idx = new_usearch(metric=metric).create_index("ks.idx", kat["dimensions"])
    for st in kat["steps"]:
        if st["op"] == "add_or_replace":
            idx.add_or_replace(tuple(st["pk"]), st["embedding"])
        elif st["op"] == "remove":
            idx.remove(tuple(st["pk"]))
        elif st["op"] == "count":
            assert idx.count() == st["expect"]
        else:
            pks, dists = idx.ann(st["embedding"], st["limit"])
            assert len(pks) == 1 and len(dists) == 1
            assert list(pks[0]) == st["expect_pk"]
    idx.close()


@pytest.mark.parametrize("metric", ["l2sq", "ip"])
def test_actor_reference_integration_kat(metric):
    """tests/integration/usearch.rs:74-123."""
    kat = _kats()["integration"]
    idx = new_usearch(metric=metric).create_index("ks.idx", kat["dimensions"])
    for pk, emb in kat["rows"]:
        idx.add_or_replace(tuple(pk), emb)
    assert idx.count() == kat["count"]
    pks, _ = idx.ann(kat["ann"]["embedding"], kat["ann"]["limit"])
    assert list(pks[0]) == kat["ann"]["expect_pk"]
    idx.close()


def test_actor_errors_match_reference():
    idx = UsearchIndex(4)
    with pytest.raises(vsg.VsgError, match="ann: embedding dimensions == 0"):
        idx.ann([], 1)
    with pytest.raises(vsg.VsgError, match=r"ann: wrong embedding dimensions: 3 != 4"):
        idx.ann([1, 2, 3], 1)
    with pytest.raises(vsg.VsgError, match="wrong embedding dimensions"):
        idx.actor.add_or_replace(1, [1, 2, 3])
    assert idx.ann([0, 0, 0, 1], 5) == ([], [])  # empty index
    idx.close()


def test_actor_concurrent_anns_batched_and_exact():
    """32 threads of single-query anns: answers equal the index's own batched
    search of the same queries (batching changes nothing) and the worker
    coalesced them."""
    n, dim = 20000, 64
    bs, qs, ms = G.config_seeds(1)
    x = G.clustered(n, dim, bs, ms)
    q = G.clustered(640, dim, qs, ms)
    a = Actor(dim, "cos", connectivity=16, expansion_add=128, expansion_search=32, seed=4)
    for i in range(n):
        a.add_or_replace(i, x[i])
    a.flush()
    assert a.count() == n
    c0 = a.counters()
    assert c0["add_calls"] < n / 16, c0  # single-vector messages became batches
    ks = [1 + (i % 3) * 7 for i in range(len(q))]  # k in {1, 8, 15}: ef = 32 for all
    out = [None] * len(q)

    def worker(t):
        for i in range(t, len(q), 32):
            out[i] = a.ann(q[i], ks[i])

    th = [threading.Thread(target=worker, args=(t,)) for t in range(32)]
    [t.start() for t in th]
    [t.join() for t in th]
    c = a.counters()
    assert c["anns"] == len(q)
    assert c["search_calls"] < len(q) and c["max_search_batch"] > 1, c
    dk, dd, dc = _direct_search(a, q, 15, 32)
    for i in range(len(q)):
        k, d = out[i]
        assert len(k) == ks[i]
        np.testing.assert_array_equal(k, dk[i, :ks[i]])
        np.testing.assert_array_equal(d, dd[i, :ks[i]])
    a.close()


def test_actor_replace_remove_semantics_vs_oracle():
    """A CDC-style upsert stream (replace = remove + add, removes of unknown
    keys ignored) through the actor ends in the same live set as a dict; exact
    answers over it equal the oracle's."""
    dim = 16
    rng = np.random.default_rng(5)
    idx = UsearchIndex(dim, metric="l2sq")
    live = {}
    for it in range(6000):
        pk = ("pk", int(rng.integers(0, 800)))
        if rng.random() < 0.25:
            idx.remove(pk)
            live.pop(pk, None)
        else:
            v = rng.integers(0, 16, dim).astype(np.float32)
            idx.add_or_replace(pk, v)
            live[pk] = v
    assert idx.count() == len(live)
    # exact search on the actor's index == oracle over the live dict
    h = lib().vsg_actor_index(idx.actor._h)
    q = rng.integers(0, 16, (50, dim)).astype(np.float32)
    keys = np.empty((50, 10), np.uint64)
    dist = np.empty((50, 10), np.float32)
    check(lib().vsg_index_exact_search(h, C.c_void_p(q.ctypes.data), 50, 10, C.c_void_p(keys.ctypes.data),
                                       C.c_void_p(dist.ctypes.data), None))
    pks = list(live)
    mat = np.stack([live[p] for p in pks])
    # oracle ties break by row order; compare distances exactly and the key
    # sets up to ties
    _, od, _ = O.exact_search("l2sq", mat, q, 10)
    np.testing.assert_array_equal(dist, od)
    for r in range(50):
        got = {idx._key2pk[int(k)] for k in keys[r]}
        for pk in got:
            assert pk in live
    idx.close()


def test_actor_capacity_growth_rule():
    """reserve(capacity + increment) whenever free < threshold (usearch.rs:200-212)."""
    a = Actor(8, reserve_increment=1000, reserve_threshold=333)
    assert a.capacity() == 1000
    x = np.random.default_rng(1).standard_normal((5000, 8)).astype(np.float32)
    for i in range(5000):
        a.add_or_replace(i, x[i])
    a.flush()
    assert a.count() == 5000
    cap = a.capacity()
    assert cap % 1000 == 0 and cap - 5000 >= 333 - 1
    assert a.counters()["reserve_calls"] >= 4
    a.close()


def _upsert_stream(dim, nkeys, rounds, seed=9):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 32, (nkeys, dim)).astype(np.float32) for _ in range(rounds)]


def test_actor_upsert_stream_reuses_slots(monkeypatch):
    """A CDC-style upsert stream (every write a replace = remove + add,
    /root/reference/src/index/usearch.rs:214-221, fed per key by src/monitor_items.rs:
    56-80) through the actor, whose runs go to vsg_index_replace: each replace's freed
    slot is re-linked in place, so the index does not grow and never needs a
    compaction; answers are those of the live rows; self-recall within +-0.5 % of the
    reference's one-replace-at-a-time sequence run on the oracle; and the same graph on
    two runs -- the chunks follow the stream, not the worker's drain timing (below
    8,192 live rows every replace is its own chunk; the tail of a drained run waits
    for the next messages or a barrier)."""
    # a chunk tail is applied by the next messages or the flush barrier, not by the
    # liveness timeout (a Python producer can pause for milliseconds)
    monkeypatch.setenv("VSG_ACTOR_HOLD_US", "5000000")
    dim, nkeys = 32, 3000
    vals = _upsert_stream(dim, nkeys, 4)
    graphs = []
    for run in range(2):
        a = Actor(dim, "l2sq", connectivity=16, expansion_add=64, expansion_search=64, seed=2)
        for rnd in range(4):
            for k in range(nkeys):
                a.add_or_replace(k, vals[rnd][k])
        a.flush()
        c = a.counters()
        assert c["compactions"] == 0 and c["add_errors"] == 0, c
        assert a.count() == nkeys
        h = lib().vsg_actor_index(a._h)
        graphs.append(vsg.Index._borrowed(h, dim, "l2sq", "f32", 0, owner=a).export())
        if run == 0:
            s = C.c_size_t()
            check(lib().vsg_index_graph_info(h, C.byref(s), None, None, None, None))
            assert s.value <= nkeys + 1  # the entry point's slot may wait in the ring
            q = np.random.default_rng(10).integers(0, 32, (40, dim)).astype(np.float32)
            keys = np.empty((40, 10), np.uint64)
            dist = np.empty((40, 10), np.float32)
            check(lib().vsg_index_exact_search(h, C.c_void_p(q.ctypes.data), 40, 10,
                                               C.c_void_p(keys.ctypes.data), C.c_void_p(dist.ctypes.data), None))
            mat = vals[3]
            _, od, _ = O.exact_search("l2sq", mat, q, 10)
            np.testing.assert_array_equal(dist, od)
            # the reference's sequence on the oracle: each replace's remove + add before
            # the next message
            h_o = O.HnswOracle(dim, "l2sq", 16, 64, 64, seed=2)
            for rnd in range(4):
                assert (h_o.replace(np.arange(nkeys, dtype=np.uint64), vals[rnd]) == 0).all()
            _, d_o, _ = h_o.search(mat, 1, 64, threads=8)
            ref = float(np.mean(d_o[:, 0] == 0.0))
            print(f"oracle, one replace at a time: self-hit {ref:.4f}")
            _self_hits(a, mat, ref - 0.005, ref + 0.005)
        a.close()
    for key in ("levels", "upper_off", "adj0", "upper", "removed", "keys"):
        np.testing.assert_array_equal(graphs[0][key], graphs[1][key], err_msg=key)
    assert (graphs[0]["entry"], graphs[0]["max_level"]) == (graphs[1]["entry"], graphs[1]["max_level"])


def _self_hits(a, mat, bar, top=1.0):
    """Each key's latest vector, searched at k 1 / ef 64, finds itself for a share of
    the keys in [bar, top]; Ann through the actor answers as the direct batched search
    does.  (Removing a large part of the index before its re-adds costs self-recall
    under usearch's update semantics -- 0.87 for 3,000-key remove-then-add segments of
    this stream against 0.999 one replace at a time, oracle -- so replace runs are
    applied in chunks of live / 4096 keys: vsg_index_replace.)"""
    kk, dd, _ = _direct_search(a, mat, 1, 64)
    hit = float(np.mean(dd[:, 0] == 0.0))
    print(f"self-hit {hit:.4f}")
    assert bar <= hit <= top, (hit, bar, top)
    for k in range(0, len(mat), 97):
        ak, ad = a.ann(mat[k], 1)
        assert ad[0] == dd[k, 0] and (ak[0] == kk[k, 0] or ad[0] != 0.0)


def test_actor_upsert_stream_compacts_append_only():
    """The same stream on an append-only index (VSG_FLAG_NO_SLOT_REUSE) leaves a
    tombstone per replace; the actor compacts once they reach compact_percent, and
    answers stay those of the live rows."""
    dim, nkeys = 32, 3000
    rng = np.random.default_rng(9)
    a = Actor(dim, "l2sq", connectivity=16, expansion_add=64, expansion_search=64, seed=2,
              compact_percent=40, compact_min_dead=1000, slot_reuse=False)
    cur = {}
    for rnd in range(4):
        vals = rng.integers(0, 32, (nkeys, dim)).astype(np.float32)
        for k in range(nkeys):
            a.add_or_replace(k, vals[k])
            cur[k] = vals[k]
    a.flush()
    c = a.counters()
    assert c["compactions"] >= 1 and c["compact_errors"] == 0, c
    assert a.count() == nkeys
    h = lib().vsg_actor_index(a._h)
    s = C.c_size_t()
    check(lib().vsg_index_graph_info(h, C.byref(s), None, None, None, None))
    assert s.value < 4 * nkeys  # tombstones were dropped
    q = rng.integers(0, 32, (40, dim)).astype(np.float32)
    keys = np.empty((40, 10), np.uint64)
    dist = np.empty((40, 10), np.float32)
    check(lib().vsg_index_exact_search(h, C.c_void_p(q.ctypes.data), 40, 10, C.c_void_p(keys.ctypes.data),
                                       C.c_void_p(dist.ctypes.data), None))
    mat = np.stack([cur[k] for k in range(nkeys)])
    _, od, _ = O.exact_search("l2sq", mat, q, 10)
    np.testing.assert_array_equal(dist, od)
    _self_hits(a, mat, 0.99)
    a.close()


def test_actor_f16_traversal_answers_exact_distances():
    """Actor built with the opt-in f16 walk + f32 re-rank (VSG_FLAG_F16_TRAVERSAL):
    single-query answers carry the exact f32 distance of each returned key
    (integer rows: bit-exact vs numpy), ascending, and find the true top-10
    (recall vs the oracle's brute force; the coalesced batches make the graph
    timing-dependent, so no bit-exact comparison with a second actor)."""
    n, dim = 6000, 64
    x = G.uint8_valued(n, dim, 97)
    q = G.uint8_valued(64, dim, 98)
    ok, _, _ = O.exact_search("l2sq", x, q, 10)
    b = Actor(dim, "l2sq", connectivity=16, expansion_add=64, expansion_search=128, seed=8, f16_traversal=True)
    for i in range(n):
        b.add_or_replace(i, x[i])
    b.flush()
    hits = 0
    for i in range(len(q)):
        kb, db = b.ann(q[i], 10)
        assert len(kb) == 10 and (np.diff(db) >= 0).all()
        want = ((x[kb.astype(np.int64)].astype(np.float64) - q[i]) ** 2).sum(-1).astype(np.float32)
        np.testing.assert_array_equal(db, want)
        hits += len(set(kb.tolist()) & set(ok[i].tolist()))
    assert hits / (10 * len(q)) >= 0.9  # iid uniform 64-d rows: low contrast (0.91 measured at ef 64)
    b.close()
