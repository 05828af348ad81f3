"""Vector-index HTTP endpoints and the engine registry.

The reference's compiled server only routes the text backend
(src/httproutes.rs:37-150); its vector endpoints exist as the client shape the
integration tests call (tests/integration/httpclient.rs:35-80):

    GET  /api/v1/indexes                    -> [IndexId]            (:35-44)
    POST /api/v1/indexes/{ks}/{index}/ann   {embedding, limit}
                                            -> {primary_keys: {column: [value]},
                                                distances: [f32]}   (:46-67)
    GET  /api/v1/indexes/{ks}/{index}/count -> usize                (:69-80)

This module serves exactly that shape over the GPU actor (vsg.actor), with
the reference's status behaviour (src/httproutes.rs:117-149): unknown index
-> 404 with an empty body, an index error -> 500 with the error text, a body
that does not deserialize (wrong types, ``limit`` 0 — ``Limit`` is a
``NonZeroUsize``, src/lib.rs:240-256) -> 422, missing ``limit`` -> 1.

``Engine`` mirrors src/engine.rs:22-139: ``add_index`` on a known id is
ignored (:101-105), ``del_index`` drops the index, ``get_index_ids`` lists ids.
``IndexId`` is ``"{keyspace}.{index}"`` (tests/integration/usearch.rs:113).

Threading: one handler thread per connection (``ThreadingHTTPServer``).
Concurrent ``ann`` calls meet in the native actor's queue, which coalesces
them into one GPU search launch (csrc/actor.hpp) — the GPU analogue of the
reference's rayon fan-out (src/index/usearch.rs:115-131).
"""
from __future__ import annotations

import json
import threading
from dataclasses import dataclass
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, List, Optional, Sequence, Tuple

API = "/api/v1"


@dataclass(frozen=True)
class IndexMetadata:
    """src/lib.rs IndexMetadata (fields used by tests/integration/usearch.rs:24-36),
    plus the table's primary-key column names (db_basic Table.primary_keys)."""

    keyspace_name: str
    table_name: str
    index_name: str
    target_column: str
    dimensions: int
    connectivity: int = 0
    expansion_add: int = 0
    expansion_search: int = 0
    primary_key_columns: Tuple[str, ...] = ("pk",)
    version: str = ""

    @property
    def id(self) -> str:
        return f"{self.keyspace_name}.{self.index_name}"


class Engine:
    """src/engine.rs: registry IndexId -> index actor (anything with IndexExt
    methods ``add_or_replace / remove / ann / count``)."""

    def __init__(self, index_factory):
        self._factory = index_factory
        self._lock = threading.Lock()
        self._indexes: Dict[str, Tuple[IndexMetadata, object]] = {}

    def get_index_ids(self) -> List[str]:
        with self._lock:
            return list(self._indexes)

    def add_index(self, meta: IndexMetadata) -> None:
        with self._lock:
            if meta.id in self._indexes:  # engine.rs:101-105: never replaced
                return
            try:
                index = self._factory.create_index(meta.id, meta.dimensions, meta.connectivity,
                                                   meta.expansion_add, meta.expansion_search)
            except Exception:  # engine.rs:107-113: logged, index not added
                return
            self._indexes[meta.id] = (meta, index)

    def del_index(self, index_id: str) -> None:
        with self._lock:
            entry = self._indexes.pop(index_id, None)
        if entry is not None and hasattr(entry[1], "close"):
            entry[1].close()

    def get_index(self, index_id: str):
        with self._lock:
            entry = self._indexes.get(index_id)
        return None if entry is None else entry[1]

    def get_metadata(self, index_id: str) -> Optional[IndexMetadata]:
        with self._lock:
            entry = self._indexes.get(index_id)
        return None if entry is None else entry[0]

    def close(self) -> None:
        for i in self.get_index_ids():
            self.del_index(i)


class _Unprocessable(Exception):
    pass


def parse_ann_request(body: bytes) -> Tuple[List[float], int]:
    """PostIndexAnnRequest {embedding: Embedding(Vec<f32>), limit: Limit (default 1)}."""
    try:
        req = json.loads(body)
    except (ValueError, UnicodeDecodeError) as e:
        raise _Unprocessable(f"Failed to parse the request body as JSON: {e}")
    if not isinstance(req, dict) or "embedding" not in req:
        raise _Unprocessable("Failed to deserialize the JSON body: missing field `embedding`")
    emb = req["embedding"]
    if not isinstance(emb, list) or not all(
            isinstance(x, (int, float)) and not isinstance(x, bool) for x in emb):
        raise _Unprocessable("Failed to deserialize the JSON body: embedding: invalid type, expected f32")
    limit = req.get("limit", 1)
    if isinstance(limit, bool) or not isinstance(limit, int) or limit < 1:
        raise _Unprocessable("Failed to deserialize the JSON body: limit: expected a nonzero usize")
    return [float(x) for x in emb], limit


def ann_response(pk_columns: Sequence[str], primary_keys: Sequence, distances: Sequence[float]) -> dict:
    """PostIndexAnnResponse: primary keys column-major, one list per PK column."""
    cols: Dict[str, list] = {c: [] for c in pk_columns}
    for pk in primary_keys:
        vals = pk if isinstance(pk, (tuple, list)) else (pk,)
        if len(vals) != len(pk_columns):
            raise ValueError(f"primary key {pk!r} does not match columns {list(pk_columns)}")
        for c, v in zip(pk_columns, vals):
            cols[c].append(v)
    return {"primary_keys": cols, "distances": [float(d) for d in distances]}


def _handler(engine: Engine) -> Callable:
    class Handler(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, fmt, *args):  # TraceLayer is debug-level in the reference
            pass

        def _send(self, status: int, body: bytes = b"", ctype: str = "application/json"):
            self.send_response(status)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            if body:
                self.wfile.write(body)

        def _json(self, obj, status: int = 200):
            self._send(status, json.dumps(obj, allow_nan=True).encode())

        def _route(self) -> Optional[Tuple[str, Optional[str]]]:
            path = self.path.split("?", 1)[0].rstrip("/")
            if not path.startswith(API + "/indexes"):
                return None
            rest = path[len(API + "/indexes"):]
            if rest == "":
                return ("indexes", None)
            parts = rest.strip("/").split("/")
            if len(parts) == 3 and parts[2] in ("ann", "count"):
                return (parts[2], f"{parts[0]}.{parts[1]}")
            return None

        def do_GET(self):
            r = self._route()
            if r is None or r[0] == "ann":
                return self._send(404 if r is None else 405)
            if r[0] == "indexes":
                return self._json(engine.get_index_ids())
            index = engine.get_index(r[1])
            if index is None:
                return self._send(404)
            try:
                return self._json(int(index.count()))
            except Exception as e:
                return self._send(500, f"index.count request error: {e}".encode(), "text/plain")

        def do_POST(self):
            r = self._route()
            n = int(self.headers.get("Content-Length") or 0)
            body = self.rfile.read(n) if n else b""
            if r is None or r[0] != "ann":
                return self._send(404 if r is None else 405)
            index = engine.get_index(r[1])
            meta = engine.get_metadata(r[1])
            if index is None or meta is None:
                return self._send(404)
            try:
                embedding, limit = parse_ann_request(body)
            except _Unprocessable as e:
                return self._send(422, str(e).encode(), "text/plain")
            try:
                pks, dists = index.ann(embedding, limit)
                resp = ann_response(meta.primary_key_columns, pks, dists)
            except Exception as e:
                return self._send(500, f"index.ann request error: {e}".encode(), "text/plain")
            return self._json(resp)

    return Handler


class _Server(ThreadingHTTPServer):
    request_queue_size = 1024  # listen backlog: the default 5 resets bursts of clients
    daemon_threads = True


class HttpServer:
    """src/httpserver.rs: the router served on a background thread."""

    def __init__(self, engine: Engine, addr: Tuple[str, int] = ("127.0.0.1", 0)):
        self.engine = engine
        self._srv = _Server(addr, _handler(engine))
        self._thread = threading.Thread(target=self._srv.serve_forever, name="vsg-http", daemon=True)
        self._thread.start()

    @property
    def addr(self) -> Tuple[str, int]:
        return self._srv.server_address[:2]

    def close(self) -> None:
        self._srv.shutdown()
        self._srv.server_close()
        self._thread.join()


def run(addr: Tuple[str, int], index_factory) -> Tuple[HttpServer, Tuple[str, int]]:
    """src/lib.rs:265-271 ``run``: engine actor + HTTP server -> (server, bound addr)."""
    srv = HttpServer(Engine(index_factory), addr)
    return srv, srv.addr


class HttpClient:
    """tests/integration/httpclient.rs, over urllib (for tests and tools)."""

    def __init__(self, addr: Tuple[str, int]):
        self.url_api = f"http://{addr[0]}:{addr[1]}{API}"

    def _req(self, method: str, url: str, body: Optional[dict] = None):
        import urllib.error
        import urllib.request
        data = None if body is None else json.dumps(body).encode()
        req = urllib.request.Request(url, data=data, method=method,
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=30) as r:
                return r.status, r.read()
        except urllib.error.HTTPError as e:
            return e.code, e.read()

    def indexes(self) -> List[str]:
        st, body = self._req("GET", f"{self.url_api}/indexes")
        assert st == 200, (st, body)
        return json.loads(body)

    def ann(self, meta: IndexMetadata, embedding: Sequence[float], limit: Optional[int] = 1):
        body = {"embedding": [float(x) for x in embedding]}
        if limit is not None:
            body["limit"] = int(limit)
        st, resp = self._req("POST", f"{self.url_api}/indexes/{meta.keyspace_name}/{meta.index_name}/ann", body)
        if st != 200:
            return st, resp
        r = json.loads(resp)
        return r["primary_keys"], r["distances"]

    def count(self, meta: IndexMetadata) -> Optional[int]:
        st, body = self._req("GET", f"{self.url_api}/indexes/{meta.keyspace_name}/{meta.index_name}/count")
        if st != 200:
            return None
        return json.loads(body)


__all__ = ["IndexMetadata", "Engine", "HttpServer", "HttpClient", "run", "parse_ann_request", "ann_response"]
