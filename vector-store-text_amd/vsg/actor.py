"""The reference's index actor over the GPU index (host-side mirror).

``Actor`` wraps the native coalescing actor of libvsg (include/vsg.h "Actor",
csrc/actor.hpp): thread-safe single-vector / single-query calls that the
worker thread turns into batched GPU calls.  ``UsearchIndex`` adds what the
reference keeps in Rust around it — the ``BiMap<PrimaryKey, Key>`` and the
``AtomicU64`` key counter (src/index/usearch.rs:109-113, :181-196) — and exposes
the ``IndexExt`` methods (``add_or_replace``, ``remove``, ``ann``, ``count``) with
the reference's argument meaning and error texts (:251-311).
``UsearchIndexFactory.create_index`` mirrors ``IndexFactory::create_index``
(:37-54).
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Hashable, Sequence

import numpy as np

from ._lib import (ADD_DONE_FN, METRICS, NO_KEY, SCALARS, ActorCounters, ActorOptions, Options, Stats, VsgError,
                   check, lib)


class Actor:
    """Native actor: one GPU index + one worker thread (csrc/actor.hpp)."""

    def __init__(self, dimensions: int, metric: str = "l2sq", quantization: str = "f32",
                 connectivity: int = 0, expansion_add: int = 0, expansion_search: int = 0,
                 device: int = 0, seed: int = 0, reserve_increment: int = 0, reserve_threshold: int = 0,
                 max_batch: int = 0, max_wait_us: int = 0, compact_percent: int = 0, compact_min_dead: int = 0,
                 f16_traversal: bool = False, concurrent_reads: int = 0, devices=None,
                 slot_reuse: bool = True):
        """devices: a list of device ordinals => one shard per entry (vsg_actor_new_sharded,
        include/vsg.h "Sharded index"); None => one index on `device`.
        concurrent_reads: 0 (or False) = submission order; n (or True = 1) = n read workers
        beside the writes (n >= 2: n search batches in flight).
        slot_reuse: False => VSG_FLAG_NO_SLOT_REUSE (append-only adds; compaction reclaims)."""
        self.dimensions = int(dimensions)
        # f16_traversal: opt-in VSG_FLAG_F16_TRAVERSAL (f16 walk + exact f32 re-rank)
        opt = ActorOptions(Options(self.dimensions, METRICS[metric], SCALARS[quantization], connectivity,
                                   expansion_add, expansion_search, device,
                                   (2 if f16_traversal else 0) | (0 if slot_reuse else 4), seed),
                           reserve_increment, reserve_threshold, max_batch, max_wait_us, compact_percent,
                           int(concurrent_reads), compact_min_dead)
        h = C.c_void_p()
        if devices is None:
            check(lib().vsg_actor_new(C.byref(opt), C.byref(h)))
        else:
            devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
            check(lib().vsg_actor_new_sharded(C.byref(opt), len(devices), C.cast(devs, C.c_void_p), C.byref(h)))
        self._h = h
        self.sharded = devices is not None

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h:
            lib().vsg_actor_free(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_or_replace(self, key: int, embedding, done=None) -> None:
        """done: optional ADD_DONE_FN(ctx, key, status), called on the worker thread when
        the batched add carrying this message finished (keep it referenced until then)."""
        v = np.ascontiguousarray(embedding, dtype=np.float32).reshape(-1)
        if done is None:
            check(lib().vsg_actor_add_or_replace(self._h, int(key), C.c_void_p(v.ctypes.data), v.size))
        else:
            check(lib().vsg_actor_add_or_replace_cb(self._h, int(key), C.c_void_p(v.ctypes.data), v.size, done,
                                                    None))

    def size_now(self) -> int:
        """Live size without waiting for queued writes (the reference's count, usearch.rs:308-311)."""
        return lib().vsg_actor_size(self._h)

    def remove(self, key: int) -> None:
        check(lib().vsg_actor_remove(self._h, int(key)))

    def ann(self, embedding, limit: int):
        """-> (keys u64[n], distances f32[n]), n <= limit, ascending."""
        v = np.ascontiguousarray(embedding, dtype=np.float32).reshape(-1)
        k = np.empty(max(int(limit), 1), np.uint64)
        d = np.empty(max(int(limit), 1), np.float32)
        n = C.c_size_t()
        check(lib().vsg_actor_ann(self._h, C.c_void_p(v.ctypes.data) if v.size else None, v.size, int(limit),
                                  C.c_void_p(k.ctypes.data), C.c_void_p(d.ctypes.data), C.byref(n)))
        return k[:n.value], d[:n.value]

    def count(self) -> int:
        n = C.c_size_t()
        check(lib().vsg_actor_count(self._h, C.byref(n)))
        return n.value

    def flush(self) -> None:
        check(lib().vsg_actor_flush(self._h))

    def counters(self) -> dict:
        c = ActorCounters()
        check(lib().vsg_actor_counters(self._h, C.byref(c)))
        return {f: getattr(c, f) for f, _ in ActorCounters._fields_}

    def capacity(self) -> int:
        if self.sharded:
            return lib().vsg_sharded_capacity(lib().vsg_actor_sharded(self._h))
        return lib().vsg_index_capacity(lib().vsg_actor_index(self._h))

    def index_stats(self) -> dict:
        s = Stats()
        if self.sharded:
            check(lib().vsg_sharded_stats(lib().vsg_actor_sharded(self._h), C.byref(s)))
        else:
            check(lib().vsg_index_stats(lib().vsg_actor_index(self._h), C.byref(s)))
        return {f: getattr(s, f) for f, _ in Stats._fields_}


class UsearchIndex:
    """src/index/usearch.rs's per-index actor, as seen through ``IndexExt``.

    Primary keys are any hashable values (the reference's ``PrimaryKey`` is a
    ``Vec<CqlValue>`` newtype); the GPU sees u64 keys only.
    """

    def __init__(self, dimensions: int, connectivity: int = 0, expansion_add: int = 0,
                 expansion_search: int = 0, metric: str = "l2sq", **kw):
        self.actor = Actor(dimensions, metric, "f32", connectivity, expansion_add, expansion_search, **kw)
        self.dimensions = int(dimensions)
        self._lock = threading.Lock()
        self._pk2key: dict = {}
        self._key2pk: dict = {}
        self._next = 0  # usearch_key AtomicU64, usearch.rs:113
        # a failed add drops the PK <-> key mapping again (usearch.rs:230-232)
        self._done = ADD_DONE_FN(self._add_done)
        self.failed_adds = 0

    def _add_done(self, _ctx, key, status):
        if status == 0:
            return
        with self._lock:
            self.failed_adds += 1
            pk = self._key2pk.pop(key, None)
            if pk is not None and self._pk2key.get(pk) == key:
                del self._pk2key[pk]

    # usearch.rs:174-233
    def add_or_replace(self, primary_key: Hashable, embedding: Sequence[float]) -> None:
        with self._lock:
            key = self._pk2key.get(primary_key)
            if key is None:  # insert_no_overwrite succeeded (:183-188)
                key = self._next
                self._next += 1
                self._pk2key[primary_key] = key
                self._key2pk[key] = primary_key
        # replace: the actor removes the live key first
        self.actor.add_or_replace(key, embedding, done=self._done)

    # usearch.rs:235-249
    def remove(self, primary_key: Hashable) -> None:
        with self._lock:
            key = self._pk2key.pop(primary_key, None)
            if key is None:
                return
            del self._key2pk[key]
        self.actor.remove(key)

    # usearch.rs:251-306
    def ann(self, embedding: Sequence[float], limit: int):
        emb = np.asarray(embedding, dtype=np.float32).reshape(-1)
        if emb.size == 0:
            raise VsgError(1, "ann: embedding dimensions == 0")
        if emb.size != self.dimensions:
            raise VsgError(1, f"ann: wrong embedding dimensions: {emb.size} != {self.dimensions}")
        if int(limit) < 1:
            raise ValueError("limit must be >= 1 (Limit is NonZeroUsize)")
        keys, dist = self.actor.ann(emb, int(limit))
        with self._lock:
            pks = []
            for k in keys.tolist():
                if k not in self._key2pk:
                    raise VsgError(1, f"not defined primary key column {k}")
                pks.append(self._key2pk[k])
        return pks, [float(x) for x in dist]

    # usearch.rs:308-311
    def count(self) -> int:
        return self.actor.count()

    def flush(self) -> None:
        self.actor.flush()

    def close(self) -> None:
        self.actor.close()


class UsearchIndexFactory:
    """``IndexFactory`` (src/index/usearch.rs:37-54) over the GPU actor."""

    def __init__(self, metric: str = "l2sq", device: int = 0, **actor_kw):
        self.metric = metric
        self.device = device
        self.actor_kw = actor_kw

    def create_index(self, id, dimensions: int, connectivity: int = 0, expansion_add: int = 0,
                     expansion_search: int = 0) -> UsearchIndex:
        return UsearchIndex(dimensions, connectivity, expansion_add, expansion_search, metric=self.metric,
                            device=self.device, **self.actor_kw)


def new_usearch(**kw) -> UsearchIndexFactory:
    """usearch.rs:56-58."""
    return UsearchIndexFactory(**kw)


__all__ = ["Actor", "UsearchIndex", "UsearchIndexFactory", "new_usearch", "NO_KEY"]
