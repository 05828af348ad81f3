"""The row-sharded index behind the C ABI (include/vsg.h "Sharded index"; SURVEY §8b
`create(opts{..., n_gpus, seed})`, §8e; VERDICT r2 missing #1).

The GPU box has one MI355X, so the shards share device 0: the same code path as one
shard per GPU except that the gather is a device-local copy instead of a peer DMA.
Checks:
  * exact search over 2 and 3 shards == one index over all rows, bit for bit (integer
    data; ties by (distance, key) = insertion order), and == the oracle;
  * HNSW: the C-ABI result is exactly the merge of its shards' own top-k (plumbing
    bit-exact), and its recall@10 >= the single-graph recall - 0.5 % at matched ef;
  * key routing, all-or-nothing adds (duplicates and reserved keys anywhere insert
    nothing), remove / replace / compaction, the device-resident call, the actor.
Reference call sites: usearch::Index::new/add/search/remove/size,
/root/reference/src/index/usearch.rs:89-99, 215, 221, 245, 276, 309.
"""
import numpy as np
import pytest

import oracle as O
import vsg
from vsg import datagen as G

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def recall(found, truth, k=10):
    return float(np.mean([len(set(found[i][:k].tolist()) & set(truth[i][:k].tolist())) / k
                          for i in range(truth.shape[0])]))


@pytest.mark.parametrize("shards", [2, 3])
def test_sharded_exact_equals_one_index(shards):
    n, d = 30000, 64
    x = G.uint8_valued(n, d, 51)
    q = G.uint8_valued(200, d, 52)
    one = vsg.Index(d, "l2sq", "f32", 16, 64, 64, seed=3)
    one.add(np.arange(n), x)
    sh = vsg.ShardedIndex(d, "l2sq", "f32", 16, 64, 64, devices=[0] * shards, seed=3)
    sh.reserve(n)
    sh.add(np.arange(n), x)
    assert sh.size() == n and sh.capacity() >= n
    sizes = [sh.shard(g).size() for g in range(shards)]
    assert sum(sizes) == n and min(sizes) > 0.9 * n / shards, sizes  # hash routing balances
    for key in (0, 17, 29999):
        assert sh.contains(key) and sh.shard(sh.route(key)).contains(key)
    for k in (1, 10, 100):
        a, b = sh.exact_search(q, k), one.exact_search(q, k)
        np.testing.assert_array_equal(a.keys, b.keys)
        np.testing.assert_array_equal(a.distances, b.distances)
        np.testing.assert_array_equal(a.counts, b.counts)
    ok, od, _ = O.exact_search("l2sq", x, q, 10)
    m = sh.exact_search(q, 10)
    np.testing.assert_array_equal(m.keys, ok)
    np.testing.assert_array_equal(m.distances, od)


def _merge_host(parts_k, parts_d, k):
    """(distance, key) ascending over every shard's rows (the merge kernel's order)."""
    keys = np.concatenate(parts_k, 1)
    dist = np.concatenate(parts_d, 1)
    out_k = np.full((keys.shape[0], k), vsg.NO_KEY, np.uint64)
    out_d = np.full((keys.shape[0], k), np.inf, np.float32)
    for i in range(keys.shape[0]):
        live = keys[i] != vsg.NO_KEY
        kk, dd = keys[i][live], dist[i][live]
        o = np.lexsort((kk, dd))[:k]
        out_k[i, :len(o)], out_d[i, :len(o)] = kk[o], dd[o]
    return out_k, out_d


def test_sharded_hnsw_is_the_merge_of_its_shards_and_keeps_recall():
    n, d, nq = 60000, 128, 500
    bs, qs, ms = G.config_seeds(1)
    x = G.clustered(n, d, bs, ms)
    q = G.clustered(nq, d, qs, ms)
    one = vsg.Index(d, "cos", "f32", 16, 128, 64, seed=5)
    one.add(np.arange(n), x)
    gt = one.exact_search(q, 10).keys
    sh = vsg.ShardedIndex(d, "cos", "f32", 16, 128, 64, devices=[0, 0], seed=5)
    sh.add(np.arange(n), x)
    for ef in (16, 32, 64):
        m = sh.search(q, 10, ef)
        per = [sh.shard(g).search(q, 10, ef) for g in range(2)]
        mk, md = _merge_host([p.keys for p in per], [p.distances for p in per], 10)
        np.testing.assert_array_equal(m.keys, mk)
        np.testing.assert_array_equal(m.distances, md)
        r_sh, r_one = recall(m.keys, gt), recall(one.search(q, 10, ef).keys, gt)
        print(f"ef {ef}: 2 shards {r_sh:.4f}, one graph {r_one:.4f}")
        assert r_sh >= r_one - 0.005, (ef, r_sh, r_one)


def test_sharded_adds_are_all_or_nothing():
    d = 16
    x = G.uint8_valued(3000, d, 61)
    sh = vsg.ShardedIndex(d, "l2sq", devices=[0, 0, 0], seed=1)
    sh.add(np.arange(1000), x[:1000])
    keys = np.arange(5000, 5100, dtype=np.uint64)
    for bad in (np.concatenate([keys, [7]]),            # 7 is live on its shard
                np.concatenate([keys, [5003]])):        # duplicate inside the batch
        with pytest.raises(vsg.DuplicateKeyError):
            sh.add(bad, x[1000:1000 + len(bad)])
        assert sh.size() == 1000 and not any(sh.contains(int(k)) for k in keys)
    with pytest.raises(vsg.VsgError):
        sh.add(np.concatenate([keys, [2**64 - 1]]), x[1000:1101])
    assert sh.size() == 1000
    sh.add(keys, x[1000:1100])
    assert sh.size() == 1100


def test_sharded_remove_replace_compact_and_device_search():
    import torch
    n, d = 20000, 32
    x = G.uint8_valued(n, d, 71)
    q = G.uint8_valued(100, d, 72)
    sh = vsg.ShardedIndex(d, "l2sq", "f32", 16, 64, 64, devices=[0, 0], seed=2)
    sh.add(np.arange(n), x)
    gone = np.arange(0, n, 3)
    assert sh.remove(np.concatenate([gone, [n + 5]])) == len(gone)
    assert sh.size() == n - len(gone)
    live = np.setdiff1d(np.arange(n), gone)
    ok, od, _ = O.exact_search("l2sq", x[live], q, 10, keys=live)
    m = sh.exact_search(q, 10)
    np.testing.assert_array_equal(m.keys, ok)
    np.testing.assert_array_equal(m.distances, od)
    h = sh.search(q, 10, 64)
    assert not np.isin(h.keys, gone).any()
    # replace = remove + add of the same keys with new rows (usearch.rs:214-221)
    sh.remove(live[:50])
    sh.add(live[:50], x[:50] + 1)
    assert sh.size() == n - len(gone)
    assert sh.compact() >= len(gone)
    assert sh.size() == n - len(gone)
    x2 = x.copy()
    x2[live[:50]] = x[:50] + 1
    ok2, od2, _ = O.exact_search("l2sq", x2[live], q, 11, keys=live)
    m2 = sh.exact_search(q, 10)
    # replaced rows sit in new slots, so equal distances may come out in another key
    # order within a shard: distances bit-exact, key sets equal unless tied at the 10th
    np.testing.assert_array_equal(m2.distances, od2[:, :10])
    for i in range(len(q)):
        assert od2[i, 9] == od2[i, 10] or set(m2.keys[i].tolist()) == set(ok2[i, :10].tolist()), i
    # device-resident call (queries and outputs on the answering device) == host call
    qt = torch.from_numpy(q).cuda()
    s = torch.cuda.current_stream()
    for exact in (False, True):
        kt, dt = sh.search_device(qt, 10, 64, exact=exact, stream=s)
        torch.cuda.synchronize()
        ref = sh.exact_search(q, 10) if exact else sh.search(q, 10, 64)
        np.testing.assert_array_equal(kt.cpu().numpy().view(np.uint64), ref.keys)
        np.testing.assert_array_equal(dt.cpu().numpy(), ref.distances)
    st = sh.stats()
    assert st["search_queries"] > 0 and st["build_vectors"] >= n


def test_sharded_actor_matches_sharded_index():
    from vsg.actor import Actor
    n, d = 3000, 24
    x = G.uint8_valued(n, d, 81)
    q = G.uint8_valued(20, d, 82)
    a = Actor(d, "l2sq", devices=[0, 0], seed=4, reserve_increment=10000)
    for i in range(n):
        a.add_or_replace(i, x[i])
    a.flush()
    assert a.count() == n and a.size_now() == n and a.capacity() >= n
    ok, od, _ = O.exact_search("l2sq", x, q, 5)
    rec = np.mean([len(set(a.ann(q[i], 5)[0].tolist()) & set(ok[i].tolist())) / 5 for i in range(len(q))])
    assert rec >= 0.9
    assert a.counters()["add_errors"] == 0
    a.close()
