"""GPU: searches beside a running insert (VERDICT r1 missing #1).

The reference runs `add` and `search` concurrently: both take its RwLock's read side
and rely on usearch's internal thread safety (/root/reference/src/index/usearch.rs:
201-221 add on rayon, :274-277 search on rayon).  vsg_index holds its exclusive lock
only to stage an add's slots and to publish them; the batched GPU build runs with no
lock, so a search issued during a 900k-row build answers at once.  Its results come from
a prefix of the writes: every returned key is a key already added or being added, with
its exact distance (rows are written before any link to them), ascending.
"""
import threading
import time

import numpy as np
import pytest

import vsg
from vsg import datagen as G

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _true_dist(x, q, keys):
    xs = x[keys.astype(np.int64)].astype(np.float64)
    xs /= np.linalg.norm(xs, axis=-1, keepdims=True)
    qq = q.astype(np.float64)
    qq /= np.linalg.norm(qq, axis=-1, keepdims=True)
    return 1.0 - np.einsum("ikd,id->ik", xs, qq)


def test_search_during_a_large_add():
    import torch
    n0, n, dim, nq = 100_000, 1_000_000, 768, 64
    bs, qs, ms = G.config_seeds(1)
    xt = vsg.datagen_device("clustered", n, dim, bs, ms)
    q = G.clustered(nq, dim, qs, ms)
    idx = vsg.Index(dim, "cos", "f32", 16, 128, 64, seed=3)
    idx.reserve(n)  # no reallocation during the add (that one needs the exclusive lock)
    idx.add_device(np.arange(n0, dtype=np.uint64), xt[:n0].contiguous())
    torch.cuda.synchronize()
    before = idx.search(q, 10, 64)
    rest = xt[n0:].contiguous()
    torch.cuda.synchronize()
    done = threading.Event()
    t_add = {}
    # An index of an earlier test freed by a garbage collection in this loop no longer
    # stalls it: vsg_index_free returns its buffers to the device pool in stream order
    # (round 5 held collections off here: a hipFree waited for this build, a 361 ms search)

    def writer():
        t0 = time.perf_counter()
        idx.add_device(np.arange(n0, n, dtype=np.uint64), rest)
        t_add["s"] = time.perf_counter() - t0
        done.set()

    th = threading.Thread(target=writer)
    t_start = time.perf_counter()
    th.start()
    time.sleep(0.05)
    lat, results, slow = [], [], []
    while not done.is_set():
        t0 = time.perf_counter()
        m = idx.search(q, 10, 64)
        dt = time.perf_counter() - t0
        if not done.is_set():
            lat.append(dt)
            results.append(m)
            if dt > 0.02:
                slow.append((round(t0 - t_start, 3), round(dt, 3)))
    th.join()
    print("slow searches (start s, latency s):", slow)
    xh = xt.cpu().numpy()
    print(f"add {t_add['s']:.3f} s; {len(lat)} searches during it, max latency {max(lat or [0]) * 1e3:.1f} ms")
    assert len(lat) >= 3, "searches must not wait for the whole build"
    assert max(lat) < 0.25 * t_add["s"]
    for m in results:
        assert (m.counts == 10).all()
        assert (m.keys < n).all()
        assert np.all(np.diff(m.distances, axis=1) >= 0)
        np.testing.assert_allclose(m.distances, _true_dist(xh, q, m.keys), atol=2e-5)
    after = idx.search(q, 10, 64)
    assert idx.size() == n and idx.graph_info()["slots"] == n
    # 10x the rows: the nearest neighbour found is at least as close for almost every query
    assert np.mean(after.distances[:, 0] <= before.distances[:, 0] + 1e-6) >= 0.95


def test_exact_search_sees_only_published_rows_during_add():
    import torch
    n0, n, dim = 50_000, 600_000, 256
    bs, qs, ms = G.config_seeds(2)
    xt = vsg.datagen_device("clustered", n, dim, bs, ms)
    q = G.clustered(40, dim, qs, ms)
    idx = vsg.Index(dim, "l2sq", "f32", 16, 128, 64, seed=5)
    idx.reserve(n)
    idx.add_device(np.arange(n0, dtype=np.uint64), xt[:n0].contiguous())
    torch.cuda.synchronize()
    ref = idx.exact_search(q, 10)
    rest = xt[n0:].contiguous()
    torch.cuda.synchronize()
    th = threading.Thread(target=lambda: idx.add_device(np.arange(n0, n, dtype=np.uint64), rest))
    th.start()
    time.sleep(0.03)
    during = idx.exact_search(q, 10)
    running = th.is_alive()
    th.join()
    if running:  # answered from the published rows [0, n0)
        np.testing.assert_array_equal(during.keys, ref.keys)
        np.testing.assert_array_equal(during.distances, ref.distances)
    full = idx.exact_search(q, 10)
    assert (full.distances[:, 0] <= ref.distances[:, 0]).all()


def test_actor_concurrent_reads_mode():
    """vsg.Actor(concurrent_reads=True): Anns on their own worker beside a write run."""
    dim = 64
    x = G.uint8_valued(300_000, dim, 77)
    from vsg.actor import Actor
    a = Actor(dim, "l2sq", "f32", 16, 128, 64, reserve_increment=400_000, concurrent_reads=True,
                  max_batch=400_000)
    for i in range(1000):
        a.add_or_replace(i, x[i])
    a.flush()
    for i in range(1000, 300_000):
        a.add_or_replace(i, x[i])
    t0 = time.perf_counter()
    keys, dist = a.ann(x[5], 3)
    lat = time.perf_counter() - t0
    t1 = time.perf_counter()
    a.flush()
    rest = time.perf_counter() - t1
    print(f"ann latency {lat * 1e3:.1f} ms while the writes took {rest * 1e3:.1f} ms more")
    assert int(keys[0]) == 5 and float(dist[0]) == 0.0
    assert a.count() == 300_000
    k2, _ = a.ann(x[250_000], 1)
    assert int(k2[0]) == 250_000
    a.close()


def test_index_free_and_growth_do_not_wait_for_other_indexes():
    """VERDICT r5 next #4 (the reference drops an index on Engine::DelIndex and grows one
    by reserve without stopping the others, /root/reference/src/engine.rs:113-115,
    src/index/usearch.rs:200-212): while index A builds 1M rows, freeing a 1M-row index B
    returns in < 5 ms, growing a third index's capacity does not wait for A either, and
    single searches on a small index C stay < 5 ms throughout -- every buffer comes
    from a per-device pool and goes back in stream order (no device-wide hipFree)."""
    import torch
    bs, qs, ms = G.config_seeds(1)
    a_rows = vsg.datagen_device("clustered", 1_000_000, 768, bs, ms)
    b = vsg.Index(128, "l2sq", "f32", 16, 64, 64, seed=7)
    b.add_device(np.arange(1_000_000, dtype=np.uint64), vsg.datagen_device("gaussian", 1_000_000, 128, 5, 0))
    c = vsg.Index(128, "l2sq", "f32", 16, 64, 64, seed=8)
    c.add(np.arange(20_000), G.uint8_valued(20_000, 128, 9))
    grow = vsg.Index(128, "l2sq", "f32", 16, 64, 64, seed=9)
    grow.add(np.arange(1000), G.uint8_valued(1000, 128, 10))
    q = G.uint8_valued(8, 128, 11)
    c.search(q, 10, 64)
    a = vsg.Index(768, "cos", "f32", 16, 128, 64, seed=6)
    a.reserve(1_000_000)
    torch.cuda.synchronize()
    done = threading.Event()
    t = {}

    def build():
        t0 = time.perf_counter()
        a.add_device(np.arange(1_000_000, dtype=np.uint64), a_rows)
        t["build"] = time.perf_counter() - t0
        done.set()

    def free_and_grow():
        time.sleep(0.08)
        t0 = time.perf_counter()
        b.close()
        t["free"] = time.perf_counter() - t0
        t["free_during_build"] = not done.is_set()
        time.sleep(0.02)
        t0 = time.perf_counter()
        grow.reserve(400_000)
        t["reserve"] = time.perf_counter() - t0
        t["reserve_during_build"] = not done.is_set()

    tb = threading.Thread(target=build)
    tf = threading.Thread(target=free_and_grow)
    tb.start()
    tf.start()
    lat = []
    while not done.is_set():
        t0 = time.perf_counter()
        m = c.search(q, 10, 64)
        lat.append(time.perf_counter() - t0)
        assert (m.counts == 10).all()
    tb.join()
    tf.join()
    print(f"build {t['build']:.3f} s; free {t['free'] * 1e3:.2f} ms (during build: {t['free_during_build']}); "
          f"reserve {t['reserve'] * 1e3:.2f} ms (during build: {t['reserve_during_build']}); "
          f"{len(lat)} searches, max {max(lat) * 1e3:.2f} ms")
    assert t["free_during_build"] and t["free"] < 0.005
    assert t["reserve_during_build"] and t["reserve"] < 0.05  # 400k rows: its own copies only
    assert max(lat) < 0.005
    assert grow.capacity() >= 400_000 and grow.size() == 1000
    assert a.size() == 1_000_000
