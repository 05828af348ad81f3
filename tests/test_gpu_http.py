"""GPU end-to-end: HTTP -> engine -> GPU actor -> libvsg.

Mirrors tests/integration/usearch.rs:21-143 (simple_create_search_delete_index)
with the reference's KAT rows, under the two metrics for which that KAT is
deterministic (tests/golden/kats.json), then checks that concurrent HTTP anns
return what one batched search of the same queries returns.
"""
import threading

import numpy as np
import pytest

from vsg.actor import new_usearch
from vsg.httproutes import HttpClient, IndexMetadata, run

from test_gpu_parity import _kats

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("metric", ["l2sq", "ip"])
def test_http_simple_create_search_delete_index(metric):
    kat = _kats()["integration"]
    meta = IndexMetadata("vector", "items", "ann", "embedding", kat["dimensions"], primary_key_columns=("pk", "ck"))
    srv, addr = run(("127.0.0.1", 0), new_usearch(metric=metric))
    try:
        client = HttpClient(addr)
        srv.engine.add_index(meta)
        idx = srv.engine.get_index(meta.id)
        for pk, emb in kat["rows"]:
            idx.add_or_replace(tuple(pk), emb)
        idx.flush()
        assert client.count(meta) == kat["count"]
        assert client.indexes() == ["vector.ann"]
        pks, dists = client.ann(meta, kat["ann"]["embedding"], kat["ann"]["limit"])
        assert len(dists) == 1 and len(pks["pk"]) == 1 and len(pks["ck"]) == 1
        assert [pks["pk"][0], pks["ck"][0]] == kat["ann"]["expect_pk"]
        srv.engine.del_index(meta.id)
        assert client.indexes() == []
    finally:
        srv.close()


def test_http_concurrent_anns_match_batched_search():
    from vsg import datagen as G
    n, dim = 5000, 32
    bs, qs, ms = G.config_seeds(1)
    x = G.clustered(n, dim, bs, ms)
    q = G.clustered(128, dim, qs, ms)
    meta = IndexMetadata("ks", "t", "i", "v", dim, 16, 64, 48)
    srv, addr = run(("127.0.0.1", 0), new_usearch(metric="cos", seed=3))
    try:
        srv.engine.add_index(meta)
        idx = srv.engine.get_index(meta.id)
        for i in range(n):
            idx.add_or_replace(i, x[i])
        idx.flush()
        client = HttpClient(addr)
        out = [None] * len(q)

        def worker(t):
            for i in range(t, len(q), 16):
                out[i] = client.ann(meta, q[i].tolist(), 10)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
        [t.start() for t in th]
        [t.join() for t in th]
        for i in range(len(q)):
            pks, dists = out[i]
            kk, dd = idx.ann(q[i], 10)
            assert pks["pk"] == list(kk) and np.allclose(dists, dd, rtol=0, atol=0)
    finally:
        srv.close()
