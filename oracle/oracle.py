"""ctypes wrapper over oracle/build/libvsg_oracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, as the parity checker / CPU baseline.  The product path
(vector-store-text_amd/vsg, libvsg.so) never imports it.

It restates the usearch-backed index path of the reference
(/root/reference/src/index/usearch.rs:82-311; algorithm of the unvendored,
unpinned unum-cloud/usearch library).  See vsg_oracle.h for parity status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libvsg_oracle.so")

METRICS = {"l2sq": 0, "ip": 1, "cos": 2}

_lib = None


def build() -> str:
    subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        sz = C.c_size_t
        L.orc_splitmix64.restype = C.c_uint64
        L.orc_splitmix64.argtypes = [C.c_uint64]
        L.orc_sample_level.restype = C.c_int
        L.orc_sample_level.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
        L.orc_distance.restype = C.c_float
        L.orc_distance.argtypes = [C.c_int, P, P, sz]
        L.orc_set_fast_metric.argtypes = [C.c_int]
        L.orc_fast_isa.restype = C.c_char_p
        L.orc_exact_search.argtypes = [C.c_int, P, P, P, sz, sz, P, sz, sz, P, P, P, C.c_int]
        L.orc_hnsw_new.restype = P
        L.orc_hnsw_new.argtypes = [sz, C.c_int, sz, sz, sz, C.c_uint64]
        L.orc_hnsw_free.argtypes = [P]
        L.orc_hnsw_reserve.argtypes = [P, sz]
        for f in ("orc_hnsw_size", "orc_hnsw_slots", "orc_hnsw_capacity", "orc_hnsw_upper_rows"):
            getattr(L, f).restype = sz
            getattr(L, f).argtypes = [P]
        L.orc_hnsw_params.argtypes = [P, P, P, P, P]
        L.orc_hnsw_add.argtypes = [P, P, P, sz, C.c_int]
        L.orc_hnsw_remove.restype = sz
        L.orc_hnsw_remove.argtypes = [P, P, sz]
        L.orc_hnsw_replace.argtypes = [P, P, P, sz, P]
        L.orc_hnsw_free_list.restype = sz
        L.orc_hnsw_free_list.argtypes = [P, P, sz]
        L.orc_hnsw_set_slot_reuse.argtypes = [P, C.c_int]
        L.orc_hnsw_search.argtypes = [P, P, sz, sz, sz, P, P, P, C.c_int, P]
        L.orc_hnsw_entry.argtypes = [P, P, P]
        L.orc_hnsw_export.argtypes = [P] * 8
        L.orc_hnsw_import.argtypes = [P, sz, P, P, P, P, P, P, P, sz, C.c_uint32, C.c_int]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def sample_level(seed: int, slot: int, connectivity: int) -> int:
    return lib().orc_sample_level(seed, slot, connectivity)


def set_fast_metric(on: bool) -> None:
    lib().orc_set_fast_metric(1 if on else 0)


def fast_isa() -> str:
    return lib().orc_fast_isa().decode()


def distance(metric: str, a, b) -> float:
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return lib().orc_distance(METRICS[metric], _p(a), _p(b), a.size)


def exact_search(metric, base, queries, k, keys=None, removed=None, threads=0):
    base = np.ascontiguousarray(base, np.float32)
    queries = np.ascontiguousarray(queries, np.float32)
    n, d = base.shape
    nq = queries.shape[0]
    ok = np.empty((nq, k), np.uint64)
    od = np.empty((nq, k), np.float32)
    oc = np.empty(nq, np.uint64)
    keys = None if keys is None else np.ascontiguousarray(keys, np.uint64)
    removed = None if removed is None else np.ascontiguousarray(removed, np.uint8)
    rc = lib().orc_exact_search(METRICS[metric], _p(base), _p(keys), _p(removed), n, d,
                                _p(queries), nq, k, _p(ok), _p(od), _p(oc), threads)
    if rc:
        raise ValueError(f"orc_exact_search rc={rc}")
    return ok, od, oc


class HnswOracle:
    """CPU restatement of usearch::Index (reference call sites usearch.rs:98-309)."""

    def __init__(self, dimensions, metric="l2sq", connectivity=0, expansion_add=0,
                 expansion_search=0, seed=0):
        self.dim = dimensions
        self.metric = metric
        self.h = lib().orc_hnsw_new(dimensions, METRICS[metric], connectivity, expansion_add,
                                    expansion_search, seed)
        if not self.h:
            raise ValueError("orc_hnsw_new failed")

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            lib().orc_hnsw_free(h)
            self.h = None

    def params(self):
        v = [C.c_size_t() for _ in range(4)]
        lib().orc_hnsw_params(self.h, *[C.byref(x) for x in v])
        return tuple(x.value for x in v)

    def reserve(self, n):
        if lib().orc_hnsw_reserve(self.h, n):
            raise MemoryError("reserve")

    def size(self):
        return lib().orc_hnsw_size(self.h)

    def slots(self):
        return lib().orc_hnsw_slots(self.h)

    def capacity(self):
        return lib().orc_hnsw_capacity(self.h)

    def add(self, keys, vecs, threads=1):
        keys = np.ascontiguousarray(keys, np.uint64)
        vecs = np.ascontiguousarray(vecs, np.float32).reshape(len(keys), self.dim)
        rc = lib().orc_hnsw_add(self.h, _p(keys), _p(vecs), len(keys), threads)
        if rc == 3:
            raise KeyError("duplicate key")
        if rc:
            raise RuntimeError(f"orc_hnsw_add rc={rc}")

    def remove(self, keys):
        keys = np.ascontiguousarray(keys, np.uint64)
        return lib().orc_hnsw_remove(self.h, _p(keys), len(keys))

    def replace(self, keys, vecs):
        """The reference's AddOrReplace stream one message at a time (usearch.rs:
        214-221): per key, remove if live, then add.  Returns per-key status."""
        keys = np.ascontiguousarray(keys, np.uint64)
        vecs = np.ascontiguousarray(vecs, np.float32).reshape(len(keys), self.dim)
        st = np.zeros(len(keys), np.int32)
        lib().orc_hnsw_replace(self.h, _p(keys), _p(vecs), len(keys), _p(st))
        return st

    def free_list(self):
        """The free ring (usearch index_dense free_keys_), oldest removal first."""
        n = lib().orc_hnsw_free_list(self.h, None, 0)
        out = np.empty(n, np.uint32)
        lib().orc_hnsw_free_list(self.h, _p(out), n)
        return out

    def set_slot_reuse(self, on: bool) -> None:
        lib().orc_hnsw_set_slot_reuse(self.h, 1 if on else 0)

    def search(self, queries, k, ef=0, threads=0, return_ndist=False):
        queries = np.ascontiguousarray(queries, np.float32).reshape(-1, self.dim)
        nq = queries.shape[0]
        ok = np.empty((nq, k), np.uint64)
        od = np.empty((nq, k), np.float32)
        oc = np.empty(nq, np.uint64)
        nd = C.c_uint64()
        rc = lib().orc_hnsw_search(self.h, _p(queries), nq, k, ef, _p(ok), _p(od), _p(oc),
                                   threads, C.byref(nd))
        if rc:
            raise RuntimeError(f"orc_hnsw_search rc={rc}")
        if return_ndist:
            return ok, od, oc, nd.value
        return ok, od, oc

    def entry(self):
        e = C.c_uint32()
        m = C.c_int()
        lib().orc_hnsw_entry(self.h, C.byref(e), C.byref(m))
        return e.value, m.value

    def export(self):
        M, M0, _, _ = self.params()
        s = self.slots()
        ur = lib().orc_hnsw_upper_rows(self.h)
        g = {
            "vectors": np.empty((s, self.dim), np.float32),
            "keys": np.empty(s, np.uint64),
            "removed": np.empty(s, np.uint8),
            "levels": np.empty(s, np.int8),
            "adj0": np.empty((s, M0), np.uint32),
            "upper_off": np.empty(s, np.uint32),
            "upper": np.empty((max(ur, 0), M), np.uint32),
        }
        lib().orc_hnsw_export(self.h, *[_p(g[x]) for x in
                                        ("vectors", "keys", "removed", "levels", "adj0",
                                         "upper_off", "upper")])
        g["entry"], g["max_level"] = self.entry()
        return g

    def import_graph(self, g):
        dt = {"vectors": np.float32, "keys": np.uint64, "removed": np.uint8, "levels": np.int8,
              "adj0": np.uint32, "upper_off": np.uint32, "upper": np.uint32}
        # keep every converted array referenced until the call returns
        arrs = {k: np.ascontiguousarray(g[k], t) for k, t in dt.items()}
        s = arrs["keys"].shape[0]
        rc = lib().orc_hnsw_import(self.h, s, _p(arrs["vectors"]), _p(arrs["keys"]),
                                   _p(arrs["removed"]), _p(arrs["levels"]), _p(arrs["adj0"]),
                                   _p(arrs["upper_off"]), _p(arrs["upper"]),
                                   arrs["upper"].shape[0], int(g["entry"]), int(g["max_level"]))
        if rc:
            raise RuntimeError(f"orc_hnsw_import rc={rc}")
