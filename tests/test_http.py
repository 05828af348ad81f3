"""HTTP layer on CPU: routing, status codes, request defaults and
the response shape of tests/integration/httpclient.rs:35-80.  The index behind
the engine here is a test double with the IndexExt surface (host logic only;
the GPU-backed end-to-end case is tests/test_gpu_http.py)."""
import json

import pytest

from vsg.httproutes import Engine, HttpClient, IndexMetadata, ann_response, parse_ann_request, run


class FakeIndex:
    """Exact L2 over a dict; stands in for vsg.actor.UsearchIndex."""

    def __init__(self, dimensions):
        self.dimensions = dimensions
        self.rows = {}
        self.closed = False

    def add_or_replace(self, pk, emb):
        self.rows[pk] = list(emb)

    def remove(self, pk):
        self.rows.pop(pk, None)

    def ann(self, emb, limit):
        if len(emb) != self.dimensions:
            raise RuntimeError(f"ann: wrong embedding dimensions: {len(emb)} != {self.dimensions}")
        d = sorted((sum((a - b) ** 2 for a, b in zip(v, emb)), pk) for pk, v in self.rows.items())[:limit]
        return [p for _, p in d], [x for x, _ in d]

    def count(self):
        return len(self.rows)

    def close(self):
        self.closed = True


class FakeFactory:
    def __init__(self):
        self.created = []

    def create_index(self, id, dimensions, connectivity=0, expansion_add=0, expansion_search=0):
        if dimensions <= 0:
            raise ValueError("dimensions")
        self.created.append(id)
        return FakeIndex(dimensions)


META = IndexMetadata("vector", "items", "ann", "embedding", 3, primary_key_columns=("pk", "ck"))


@pytest.fixture()
def server():
    srv, addr = run(("127.0.0.1", 0), FakeFactory())
    yield srv, HttpClient(addr)
    srv.close()


def test_parse_ann_request_defaults_and_errors():
    assert parse_ann_request(b'{"embedding": [1, 2.5]}') == ([1.0, 2.5], 1)
    assert parse_ann_request(b'{"embedding": [], "limit": 7}') == ([], 7)
    for bad in (b'{"limit": 1}', b'{"embedding": [1], "limit": 0}', b'{"embedding": [1], "limit": -2}',
                b'{"embedding": ["a"]}', b'{"embedding": [1], "limit": 1.5}', b'not json', b'[1,2]',
                b'{"embedding": [true]}'):
        with pytest.raises(Exception):
            parse_ann_request(bad)


def test_ann_response_is_column_major():
    r = ann_response(("pk", "ck"), [(2, "two"), (1, "one")], [0.5, 1.25])
    assert r == {"primary_keys": {"pk": [2, 1], "ck": ["two", "one"]}, "distances": [0.5, 1.25]}
    assert ann_response(("pk",), [7], [0.0]) == {"primary_keys": {"pk": [7]}, "distances": [0.0]}
    assert ann_response(("pk", "ck"), [], []) == {"primary_keys": {"pk": [], "ck": []}, "distances": []}


def test_engine_add_is_not_replace_and_del_closes():
    f = FakeFactory()
    e = Engine(f)
    e.add_index(META)
    first = e.get_index(META.id)
    e.add_index(META)  # engine.rs:101-105
    assert e.get_index(META.id) is first and f.created == ["vector.ann"]
    e.add_index(IndexMetadata("vector", "items", "bad", "embedding", 0))  # factory error: not added
    assert e.get_index_ids() == ["vector.ann"]
    e.del_index(META.id)
    assert first.closed and e.get_index_ids() == [] and e.get_index(META.id) is None


def test_http_create_search_count_delete(server):
    """tests/integration/usearch.rs:21-143 with the engine fed directly."""
    srv, client = server
    assert client.indexes() == []
    assert client.count(META) is None  # unknown index -> 404
    srv.engine.add_index(META)
    idx = srv.engine.get_index(META.id)
    for pk, emb in [((1, "one"), [1, 1, 1]), ((2, "two"), [2, -2, 2]), ((3, "three"), [3, 3, 3])]:
        idx.add_or_replace(pk, emb)
    assert client.count(META) == 3
    assert client.indexes() == ["vector.ann"]
    pks, dists = client.ann(META, [2.1, -2.0, 2.0], 1)
    assert len(dists) == 1 and pks["pk"] == [2] and pks["ck"] == ["two"]
    pks, dists = client.ann(META, [2.1, -2.0, 2.0], None)  # limit defaults to 1
    assert len(dists) == 1
    pks, dists = client.ann(META, [0, 0, 0], 10)  # fewer rows than limit
    assert pks["pk"] == [1, 2, 3] and dists == sorted(dists)
    srv.engine.del_index(META.id)
    assert client.indexes() == []


def test_http_status_codes(server):
    srv, client = server
    st, _ = client.ann(META, [1, 2, 3], 1)
    assert st == 404
    srv.engine.add_index(META)
    st, body = client.ann(META, [1, 2], 1)  # index error -> 500 + message
    assert st == 500 and b"wrong embedding dimensions" in body
    url = f"{client.url_api}/indexes/vector/ann/ann"
    assert client._req("POST", url, {"embedding": [1, 2, 3], "limit": 0})[0] == 422
    assert client._req("POST", url, {"limit": 1})[0] == 422
    assert client._req("GET", url)[0] == 405
    assert client._req("GET", f"{client.url_api}/nope")[0] == 404
    st, body = client._req("GET", f"{client.url_api}/indexes/vector/ann/count")
    assert st == 200 and json.loads(body) == 0


def test_http_burst_of_concurrent_clients(server):
    """64 simultaneous connections (the listen backlog must not reset them)."""
    import threading
    srv, client = server
    srv.engine.add_index(META)
    idx = srv.engine.get_index(META.id)
    for i in range(20):
        idx.add_or_replace((i, str(i)), [i, 0, 0])
    out = [None] * 256

    def worker(t):
        for i in range(t, 256, 64):
            out[i] = client.ann(META, [i % 20, 0, 0], 1)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(64)]
    [t.start() for t in th]
    [t.join() for t in th]
    for i in range(256):
        pks, dists = out[i]
        assert pks["pk"] == [i % 20] and dists == [0.0]
