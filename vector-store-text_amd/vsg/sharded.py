"""`ShardedIndex` — one logical index row-sharded over GPUs (include/vsg.h "Sharded index").

The in-process counterpart of vsg/distributed.py (one process per GPU): one
`vsg_sharded_t` owns a `vsg_index_t` per shard, routes each key to shard
splitmix64(key) mod n, builds the shards concurrently and answers a search by
searching every shard and merging the per-shard top-k on the answering device
(peer DMA over xGMI, HIP k-way merge).  Same surface as `Index` (usearch::Index
calls of /root/reference/src/index/usearch.rs:98-309); SURVEY §8b
`create(opts{..., n_gpus, seed})`.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import METRICS, SCALARS, Options, ShardedOptions, Stats, check, lib
from .index import Index, Matches, _p, _stream_ptr, _tp


class ShardedIndex:
    def __init__(self, dimensions: int, metric: str = "l2sq", quantization: str = "f32",
                 connectivity: int = 0, expansion_add: int = 0, expansion_search: int = 0,
                 devices=None, n_shards: int = 0, answer_device: int = -1, seed: int = 0,
                 exact_only: bool = False):
        if devices is not None:
            devices = [int(d) for d in devices]
            n_shards = n_shards or len(devices)
            if len(devices) != n_shards:
                raise ValueError("len(devices) != n_shards")
        if n_shards < 1:
            raise ValueError("n_shards >= 1 (or a device list) required")
        self.dimensions = int(dimensions)
        self.metric, self.quantization = metric, quantization
        self._devs = (C.c_int32 * n_shards)(*devices) if devices is not None else None
        opt = ShardedOptions(Options(self.dimensions, METRICS[metric], SCALARS[quantization], connectivity,
                                     expansion_add, expansion_search, 0, 1 if exact_only else 0, seed),
                             n_shards, answer_device,
                             C.cast(self._devs, C.POINTER(C.c_int32)) if self._devs is not None else None)
        h = C.c_void_p()
        check(lib().vsg_sharded_new(C.byref(opt), C.byref(h)))
        self._h = h
        self.devices = devices if devices is not None else [None] * n_shards
        self.n_shards = n_shards

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            lib().vsg_sharded_free(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- usearch::Index surface ---------------------------------------------
    def reserve(self, capacity: int) -> None:
        check(lib().vsg_sharded_reserve(self._h, capacity))

    def capacity(self) -> int:
        return lib().vsg_sharded_capacity(self._h)

    def size(self) -> int:
        return lib().vsg_sharded_size(self._h)

    def __len__(self):
        return self.size()

    def contains(self, key: int) -> bool:
        return bool(lib().vsg_sharded_contains(self._h, key))

    def route(self, key: int) -> int:
        return lib().vsg_sharded_route(self._h, key)

    def add(self, keys, vectors) -> None:
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        vectors = np.ascontiguousarray(vectors, np.float32).reshape(len(keys), self.dimensions)
        check(lib().vsg_sharded_add(self._h, _p(keys), _p(vectors), len(keys)))

    def remove(self, keys) -> int:
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        n = C.c_size_t()
        check(lib().vsg_sharded_remove(self._h, _p(keys), len(keys), C.byref(n)))
        return n.value

    def replace(self, keys, vectors, batch: int = 0) -> np.ndarray:
        """vsg_index_replace on every shard (each key's messages meet on its shard)."""
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        vectors = np.ascontiguousarray(vectors, np.float32).reshape(len(keys), self.dimensions)
        st = np.zeros(len(keys), np.int32)
        na = C.c_size_t()
        check(lib().vsg_sharded_replace(self._h, _p(keys), _p(vectors), len(keys), int(batch), 0, _p(st),
                                        C.byref(na)))
        return st

    def _search(self, queries, k, ef, exact):
        q = np.ascontiguousarray(queries, np.float32).reshape(-1, self.dimensions)
        nq = q.shape[0]
        ok = np.empty((nq, k), np.uint64)
        od = np.empty((nq, k), np.float32)
        oc = np.empty(nq, np.uint64)
        if exact:
            check(lib().vsg_sharded_exact_search(self._h, _p(q), nq, k, _p(ok), _p(od), _p(oc)))
        else:
            check(lib().vsg_sharded_search(self._h, _p(q), nq, k, ef, _p(ok), _p(od), _p(oc)))
        return Matches(ok, od, oc)

    def search(self, queries, k: int, ef: int = 0) -> Matches:
        return self._search(queries, k, ef, False)

    def exact_search(self, queries, k: int) -> Matches:
        return self._search(queries, k, 0, True)

    def search_device(self, queries_t, k, ef=0, exact=False, out_keys=None, out_dist=None, stream=None):
        """queries and outputs on the answering device; enqueued on `stream`."""
        import torch
        nq = queries_t.shape[0]
        assert queries_t.is_cuda and queries_t.is_contiguous() and queries_t.dtype == torch.float32
        dev = queries_t.device
        if out_keys is None:
            out_keys = torch.empty((nq, k), dtype=torch.int64, device=dev)
        if out_dist is None:
            out_dist = torch.empty((nq, k), dtype=torch.float32, device=dev)
        check(lib().vsg_sharded_search_device(self._h, _tp(queries_t), nq, k, ef, 1 if exact else 0,
                                              _tp(out_keys), _tp(out_dist), _stream_ptr(stream)))
        return out_keys, out_dist

    def compact(self) -> int:
        n = C.c_size_t()
        check(lib().vsg_sharded_compact(self._h, C.byref(n)))
        return n.value

    # -- shards / counters ------------------------------------------------------
    def shard(self, g: int) -> Index:
        """Borrowed view of shard g (valid while this index lives)."""
        h = lib().vsg_sharded_shard(self._h, g)
        if not h:
            raise IndexError(g)
        return Index._borrowed(h, self.dimensions, self.metric, self.quantization, self.devices[g], owner=self)

    def stats(self) -> dict:
        s = Stats()
        check(lib().vsg_sharded_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in Stats._fields_}

    def reset_stats(self) -> None:
        check(lib().vsg_sharded_reset_stats(self._h))
