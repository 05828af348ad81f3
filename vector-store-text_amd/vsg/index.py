"""`Index` — Python surface of one MI355X index shard over libvsg.so.

Mirrors the usearch::Index calls the reference makes
(/root/reference/src/index/usearch.rs): ``Index(options)`` (:89-98),
``reserve`` (:99, :206), ``capacity``/``size`` (:201-202, :309), ``add`` (:221,
batched), ``remove`` (:215, :245), ``search`` (:276) returning keys and
distances ascending.  Extra: ``exact_search`` (brute force), device-resident
variants taking torch tensors, graph export/import, kernel counters.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import os

from ._lib import METRICS, NO_KEY, SCALARS, VSG_REPLACE_HOLD_TAIL, FileInfo, Options, Stats, check, lib

_METRIC_NAMES = {v: k for k, v in METRICS.items()}
_SCALAR_NAMES = {v: k for k, v in SCALARS.items()}


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def _tp(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream_ptr(stream):
    if stream is None:
        return None
    return C.c_void_p(getattr(stream, "cuda_stream", stream))


class Matches:
    """usearch::Matches analogue: keys / distances rows, ascending."""

    def __init__(self, keys, distances, counts):
        self.keys = keys
        self.distances = distances
        self.counts = counts

    def __iter__(self):
        return iter((self.keys, self.distances, self.counts))


class Index:
    def __init__(self, dimensions: int, metric: str = "l2sq", quantization: str = "f32",
                 connectivity: int = 0, expansion_add: int = 0, expansion_search: int = 0,
                 device: int = 0, seed: int = 0, exact_only: bool = False,
                 f16_traversal: bool = False, slot_reuse: bool = True):
        self.dimensions = int(dimensions)
        self.metric = metric
        self.quantization = quantization
        opt = Options(self.dimensions, METRICS[metric], SCALARS[quantization], connectivity,
                      expansion_add, expansion_search, device,
                      (1 if exact_only else 0) | (2 if f16_traversal else 0) | (0 if slot_reuse else 4), seed)
        h = C.c_void_p()
        check(lib().vsg_index_new(C.byref(opt), C.byref(h)))
        self._h = h
        self.device = device

    @classmethod
    def _borrowed(cls, handle, dimensions, metric, quantization, device, owner=None) -> "Index":
        """Non-owning view of a shard handle (ShardedIndex.shard); `owner` is kept alive."""
        self = cls.__new__(cls)
        self._h = C.c_void_p(handle)
        self._owner = owner
        self.dimensions, self.metric, self.quantization, self.device = int(dimensions), metric, quantization, device
        return self

    def close(self):
        h = getattr(self, "_h", None)
        if h and getattr(self, "_owner", None) is None:
            lib().vsg_index_free(h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- usearch::Index surface ---------------------------------------------
    def reserve(self, capacity: int) -> None:
        check(lib().vsg_index_reserve(self._h, capacity))

    def capacity(self) -> int:
        return lib().vsg_index_capacity(self._h)

    def size(self) -> int:
        return lib().vsg_index_size(self._h)

    def __len__(self):
        return self.size()

    def contains(self, key: int) -> bool:
        return bool(lib().vsg_index_contains(self._h, key))

    def add(self, keys, vectors) -> None:
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        vectors = np.ascontiguousarray(vectors, np.float32).reshape(len(keys), self.dimensions)
        check(lib().vsg_index_add(self._h, _p(keys), _p(vectors), len(keys)))

    def remove(self, keys) -> int:
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        n = C.c_size_t()
        check(lib().vsg_index_remove(self._h, _p(keys), len(keys), C.byref(n)))
        return n.value

    def replace(self, keys, vectors, batch: int = 0, hold_tail: bool = False) -> np.ndarray:
        """The reference's AddOrReplace stream (usearch.rs:214-221): per key in order,
        remove it if live, then add it -- one-message-at-a-time results, applied by the
        GPU in chunks (batch 0: max(1, size / 4096) keys re-linked, max(1, size / 8)
        appended).  Returns the per-key status (0 = ok, VSG_HELD = left for the next
        call under hold_tail); raises on the first error after the whole call ran."""
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        vectors = np.ascontiguousarray(vectors, np.float32).reshape(len(keys), self.dimensions)
        st = np.zeros(len(keys), np.int32)
        na = C.c_size_t()
        check(lib().vsg_index_replace(self._h, _p(keys), _p(vectors), len(keys), int(batch),
                                      VSG_REPLACE_HOLD_TAIL if hold_tail else 0, _p(st), C.byref(na)))
        return st

    def replace_device(self, keys, vectors_t, batch: int = 0, stream=None) -> np.ndarray:
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        assert vectors_t.is_cuda and vectors_t.is_contiguous()
        assert vectors_t.shape == (len(keys), self.dimensions)
        st = np.zeros(len(keys), np.int32)
        check(lib().vsg_index_replace_device(self._h, _p(keys), _tp(vectors_t), len(keys), int(batch), _p(st),
                                             _stream_ptr(stream)))
        return st

    def free_slots(self) -> np.ndarray:
        """The free ring (usearch index_dense free_keys_): removed slots, oldest removal
        first; the next adds re-link them in this order."""
        n = lib().vsg_index_free_slots(self._h, None, 0)
        out = np.empty(n, np.uint32)
        n2 = lib().vsg_index_free_slots(self._h, _p(out), n)
        return out[:min(n, n2)]

    def _search(self, queries, k, ef, exact):
        q = np.ascontiguousarray(queries, np.float32).reshape(-1, self.dimensions)
        nq = q.shape[0]
        ok = np.empty((nq, k), np.uint64)
        od = np.empty((nq, k), np.float32)
        oc = np.empty(nq, np.uint64)
        if exact:
            check(lib().vsg_index_exact_search(self._h, _p(q), nq, k, _p(ok), _p(od), _p(oc)))
        else:
            check(lib().vsg_index_search(self._h, _p(q), nq, k, ef, _p(ok), _p(od), _p(oc)))
        return Matches(ok, od, oc)

    def search(self, queries, k: int, ef: int = 0) -> Matches:
        return self._search(queries, k, ef, False)

    def exact_search(self, queries, k: int) -> Matches:
        return self._search(queries, k, 0, True)

    # -- device-resident variants (torch tensors on this index's GPU) ----------
    def add_device(self, keys, vectors_t, stream=None) -> None:
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        assert vectors_t.is_cuda and vectors_t.is_contiguous()
        assert vectors_t.shape == (len(keys), self.dimensions)
        check(lib().vsg_index_add_device(self._h, _p(keys), _tp(vectors_t), len(keys),
                                         _stream_ptr(stream)))

    def search_device(self, queries_t, k, ef=0, out_keys=None, out_dist=None, out_counts=None,
                      stream=None, exact=False):
        import torch
        nq = queries_t.shape[0]
        assert queries_t.is_cuda and queries_t.is_contiguous() and queries_t.dtype == torch.float32
        dev = queries_t.device
        if out_keys is None:
            out_keys = torch.empty((nq, k), dtype=torch.int64, device=dev)
        if out_dist is None:
            out_dist = torch.empty((nq, k), dtype=torch.float32, device=dev)
        if exact:
            check(lib().vsg_index_exact_search_device(self._h, _tp(queries_t), nq, k, _tp(out_keys),
                                                      _tp(out_dist), _tp(out_counts),
                                                      _stream_ptr(stream)))
        else:
            check(lib().vsg_index_search_device(self._h, _tp(queries_t), nq, k, ef, _tp(out_keys),
                                                _tp(out_dist), _tp(out_counts), _stream_ptr(stream)))
        return out_keys, out_dist

    # -- introspection ---------------------------------------------------------
    def stats(self) -> dict:
        s = Stats()
        check(lib().vsg_index_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in Stats._fields_}

    def set_f16_traversal(self, enable: bool) -> None:
        """Opt-in: HNSW search walks an f16 copy of the rows and re-ranks its ef-beam
        with exact f32 distances (csrc/rerank.hip; no usearch equivalent)."""
        check(lib().vsg_index_set_f16_traversal(self._h, 1 if enable else 0))

    def set_upper_ef(self, upper_ef: int) -> None:
        """Opt-in multi-entry descent: a level-1 beam of this width seeds level 0
        (0/1 = usearch greedy descent, the default)."""
        check(lib().vsg_index_set_upper_ef(self._h, int(upper_ef)))

    def reset_stats(self) -> None:
        check(lib().vsg_index_reset_stats(self._h))

    def graph_info(self) -> dict:
        slots, urows, m = C.c_size_t(), C.c_size_t(), C.c_size_t()
        entry, maxl = C.c_uint32(), C.c_int()
        check(lib().vsg_index_graph_info(self._h, C.byref(slots), C.byref(urows), C.byref(m),
                                         C.byref(entry), C.byref(maxl)))
        return {"slots": slots.value, "upper_rows": urows.value, "connectivity": m.value,
                "entry": entry.value, "max_level": maxl.value}

    def export(self) -> dict:
        gi = self.graph_info()
        s, ur, M = gi["slots"], gi["upper_rows"], gi["connectivity"]
        g = {
            "vectors": np.empty((s, self.dimensions), np.float32),
            "keys": np.empty(s, np.uint64),
            "removed": np.empty(s, np.uint8),
            "levels": np.empty(s, np.int8),
            "adj0": np.empty((s, 2 * M), np.uint32),
            "upper_off": np.empty(s, np.uint32),
            "upper": np.empty((ur, M), np.uint32),
        }
        check(lib().vsg_index_export(self._h, *[_p(g[x]) for x in (
            "vectors", "keys", "removed", "levels", "adj0", "upper_off", "upper")]))
        g["entry"], g["max_level"] = gi["entry"], gi["max_level"]
        return g

    def import_graph(self, g) -> None:
        dt = {"vectors": np.float32, "keys": np.uint64, "removed": np.uint8, "levels": np.int8,
              "adj0": np.uint32, "upper_off": np.uint32, "upper": np.uint32}
        a = {k: np.ascontiguousarray(g[k], t) for k, t in dt.items()}
        s = a["keys"].shape[0]
        check(lib().vsg_index_import(self._h, s, _p(a["vectors"]), _p(a["keys"]), _p(a["removed"]),
                                     _p(a["levels"]), _p(a["adj0"]), _p(a["upper_off"]),
                                     _p(a["upper"]), a["upper"].shape[0], int(g["entry"]),
                                     int(g["max_level"])))


    # -- compaction / persistence -------------------------
    def compact(self) -> int:
        """Drop tombstoned rows and rebuild the graph over the live ones; returns
        the number of slots freed."""
        n = C.c_size_t()
        check(lib().vsg_index_compact(self._h, C.byref(n)))
        return n.value

    def save(self, path) -> None:
        check(lib().vsg_index_save(self._h, os.fsencode(path)))

    @classmethod
    def load(cls, path, device: int = 0) -> "Index":
        info = file_info(path)
        h = C.c_void_p()
        check(lib().vsg_index_load(os.fsencode(path), int(device), C.byref(h)))
        self = cls.__new__(cls)
        self._h = h
        self.device = device
        self.dimensions = info["dimensions"]
        self.metric = info["metric"]
        self.quantization = info["quantization"]
        return self


def file_info(path) -> dict:
    """Header of a saved index (no device needed)."""
    fi = FileInfo()
    check(lib().vsg_index_file_info(os.fsencode(path), C.byref(fi)))
    o = fi.options
    return {"dimensions": o.dimensions, "metric": _METRIC_NAMES[o.metric],
            "quantization": _SCALAR_NAMES[o.quantization], "connectivity": o.connectivity,
            "expansion_add": o.expansion_add, "expansion_search": o.expansion_search,
            "flags": o.flags, "seed": o.seed, "version": fi.version, "max_level": fi.max_level,
            "slots": fi.slots, "live": fi.live, "upper_rows": fi.upper_rows, "file_bytes": fi.file_bytes}


def merge_topk_device(keys_t, dist_t, k, stream=None):
    """k-way merge of gathered per-shard results: (parts, nq, k_in) -> (nq, k)."""
    import torch
    parts, nq, kin = keys_t.shape
    ok = torch.empty((nq, k), dtype=torch.int64, device=keys_t.device)
    od = torch.empty((nq, k), dtype=torch.float32, device=keys_t.device)
    check(lib().vsg_merge_topk_device(_tp(keys_t), _tp(dist_t), parts, nq, kin, k, _tp(ok), _tp(od),
                                      _stream_ptr(stream)))
    return ok, od


def datagen_device(kind: str, n: int, dim: int, seed: int, model_seed: int = 0, start: int = 0,
                   out=None, stream=None):
    import torch
    kinds = {"clustered": 0, "gaussian": 1, "uint8": 2, "sift": 3}
    if out is None:
        out = torch.empty((n, dim), dtype=torch.float32, device="cuda")
    check(lib().vsg_datagen_device(kinds[kind], n, dim, seed, model_seed, start, _tp(out),
                                   _stream_ptr(stream)))
    return out


def sample_level(seed: int, slot: int, connectivity: int) -> int:
    return lib().vsg_sample_level(seed, slot, connectivity)


NO_KEY = NO_KEY
