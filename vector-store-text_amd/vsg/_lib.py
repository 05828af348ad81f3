"""ctypes binding of libvsg.so (include/vsg.h).

The product path: every call goes to the gfx950 HIP library.  There is no CPU
fallback — if the shared library is missing or no GPU is visible, calls fail
loudly (the oracle under /root/repo/oracle is test infrastructure only).
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("VSG_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libvsg.so")
HEADER = os.path.join(REPO_ROOT, "include", "vsg.h")

VSG_OK = 0
VSG_EINVAL = 1
VSG_ENOMEM = 2
VSG_EDUPKEY = 3
VSG_EDEVICE = 4
VSG_EUNSUPPORTED = 5
VSG_HELD = 6  # vsg_index_replace status: left unapplied under VSG_REPLACE_HOLD_TAIL
VSG_REPLACE_HOLD_TAIL = 1

METRICS = {"l2sq": 0, "ip": 1, "cos": 2}
SCALARS = {"f32": 0, "f16": 1}
NO_KEY = (1 << 64) - 1


class VsgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"vsg error {code}: {msg}")
        self.code = code


class DuplicateKeyError(VsgError, KeyError):
    pass


class Options(C.Structure):
    _fields_ = [
        ("dimensions", C.c_uint32),
        ("metric", C.c_uint32),
        ("quantization", C.c_uint32),
        ("connectivity", C.c_uint32),
        ("expansion_add", C.c_uint32),
        ("expansion_search", C.c_uint32),
        ("device", C.c_int32),
        ("flags", C.c_uint32),
        ("seed", C.c_uint64),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("search_queries", C.c_uint64),
        ("search_distances", C.c_uint64),
        ("search_adjacency", C.c_uint64),
        ("build_vectors", C.c_uint64),
        ("build_distances", C.c_uint64),
        ("build_adjacency", C.c_uint64),
        ("build_batches", C.c_uint64),
        ("build_select_distances", C.c_uint64),
        ("reverse_recompute_distances", C.c_uint64),
        ("reverse_select_distances", C.c_uint64),
        ("reverse_prunes", C.c_uint64),
        ("reverse_appends", C.c_uint64),
        ("build_insert_ns", C.c_uint64),
        ("build_sort_ns", C.c_uint64),
        ("build_reverse_ns", C.c_uint64),
        ("build_select_ns", C.c_uint64),
        ("search_filter_overflow", C.c_uint64),
        ("search_filter_reruns", C.c_uint64),
        ("slots_reused", C.c_uint64),
        ("ktile_copy_failures", C.c_uint64),
        ("host_searches", C.c_uint64),
        ("host_search_ns", C.c_uint64),
        ("host_h2d_ns", C.c_uint64),
        ("host_device_ns", C.c_uint64),
        ("host_d2h_ns", C.c_uint64),
    ]


class FileInfo(C.Structure):
    _fields_ = [
        ("options", Options),
        ("version", C.c_uint32),
        ("max_level", C.c_int32),
        ("slots", C.c_uint64),
        ("live", C.c_uint64),
        ("upper_rows", C.c_uint64),
        ("file_bytes", C.c_uint64),
    ]


class ActorOptions(C.Structure):
    _fields_ = [
        ("index", Options),
        ("reserve_increment", C.c_uint64),
        ("reserve_threshold", C.c_uint64),
        ("max_batch", C.c_uint32),
        ("max_wait_us", C.c_uint32),
        ("compact_percent", C.c_uint32),
        ("concurrent_reads", C.c_uint32),
        ("compact_min_dead", C.c_uint64),
    ]


class ShardedOptions(C.Structure):
    _fields_ = [
        ("index", Options),
        ("n_shards", C.c_uint32),
        ("answer_device", C.c_int32),
        ("devices", C.POINTER(C.c_int32)),
    ]


# void (*)(void* ctx, uint64_t key, int status): vsg_actor_add_or_replace_cb completion
ADD_DONE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64, C.c_int)
# void (*)(void* ctx, int status, size_t count): vsg_actor_ann_cb completion
ANN_DONE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_size_t)


class ActorCounters(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in (
        "messages", "writes", "anns", "counts", "add_calls", "remove_calls", "search_calls",
        "reserve_calls", "add_errors", "remove_errors", "search_errors", "max_search_batch",
        "max_add_batch", "compactions", "compacted_rows", "compact_errors",
        "ann_queue_ns", "ann_wake_ns", "batch_search_ns", "batch_notify_ns")]


_lib = None


def declared_symbols() -> list[str]:
    """Every function declared in include/vsg.h."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(vsg_\w+)\s*\(", txt, re.M)))


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libvsg.so not built at {LIB_PATH}: run `make -C vector-store-text_amd` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same
    # soname as /opt/rocm's).  Loading torch first makes libvsg bind to that copy,
    # so device pointers and hipStream_t handles are shared with torch.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P, sz, u64, u32 = C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint32
    sigs = {
        "vsg_index_new": (C.c_int, [C.POINTER(Options), C.POINTER(P)]),
        "vsg_index_free": (None, [P]),
        "vsg_index_reserve": (C.c_int, [P, sz]),
        "vsg_index_capacity": (sz, [P]),
        "vsg_index_size": (sz, [P]),
        "vsg_index_dimensions": (sz, [P]),
        "vsg_index_contains": (C.c_int, [P, u64]),
        "vsg_index_add": (C.c_int, [P, P, P, sz]),
        "vsg_index_add_device": (C.c_int, [P, P, P, sz, P]),
        "vsg_index_remove": (C.c_int, [P, P, sz, C.POINTER(sz)]),
        "vsg_index_replace": (C.c_int, [P, P, P, sz, sz, u32, P, C.POINTER(sz)]),
        "vsg_index_replace_device": (C.c_int, [P, P, P, sz, sz, P, P]),
        "vsg_index_free_slots": (sz, [P, P, sz]),
        "vsg_index_search": (C.c_int, [P, P, sz, sz, sz, P, P, P]),
        "vsg_index_exact_search": (C.c_int, [P, P, sz, sz, P, P, P]),
        "vsg_index_search_device": (C.c_int, [P, P, sz, sz, sz, P, P, P, P]),
        "vsg_index_exact_search_device": (C.c_int, [P, P, sz, sz, P, P, P, P]),
        "vsg_merge_topk_device": (C.c_int, [P, P, sz, sz, sz, sz, P, P, P]),
        "vsg_index_stats": (C.c_int, [P, C.POINTER(Stats)]),
        "vsg_index_reset_stats": (C.c_int, [P]),
        "vsg_index_set_f16_traversal": (C.c_int, [P, C.c_int]),
        "vsg_index_set_upper_ef": (C.c_int, [P, sz]),
        "vsg_index_graph_info": (C.c_int, [P, C.POINTER(sz), C.POINTER(sz), C.POINTER(sz),
                                           C.POINTER(u32), C.POINTER(C.c_int)]),
        "vsg_index_export": (C.c_int, [P] * 8),
        "vsg_index_import": (C.c_int, [P, sz, P, P, P, P, P, P, P, sz, u32, C.c_int]),
        "vsg_index_compact": (C.c_int, [P, C.POINTER(sz)]),
        "vsg_index_save": (C.c_int, [P, C.c_char_p]),
        "vsg_index_load": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(P)]),
        "vsg_index_file_info": (C.c_int, [C.c_char_p, C.POINTER(FileInfo)]),
        "vsg_datagen_device": (C.c_int, [C.c_int, sz, sz, u64, u64, sz, P, P]),
        "vsg_sample_level": (C.c_int, [u64, u64, u32]),
        "vsg_actor_new": (C.c_int, [C.POINTER(ActorOptions), C.POINTER(P)]),
        "vsg_actor_free": (None, [P]),
        "vsg_actor_add_or_replace": (C.c_int, [P, u64, P, sz]),
        "vsg_actor_remove": (C.c_int, [P, u64]),
        "vsg_actor_ann": (C.c_int, [P, P, sz, sz, P, P, C.POINTER(sz)]),
        "vsg_actor_count": (C.c_int, [P, C.POINTER(sz)]),
        "vsg_actor_flush": (C.c_int, [P]),
        "vsg_actor_counters": (C.c_int, [P, C.POINTER(ActorCounters)]),
        "vsg_actor_index": (P, [P]),
        "vsg_actor_sharded": (P, [P]),
        "vsg_actor_new_sharded": (C.c_int, [C.POINTER(ActorOptions), u32, P, C.POINTER(P)]),
        "vsg_actor_add_or_replace_cb": (C.c_int, [P, u64, P, sz, ADD_DONE_FN, P]),
        "vsg_actor_ann_cb": (C.c_int, [P, P, sz, sz, P, P, ANN_DONE_FN, P]),
        "vsg_actor_size": (sz, [P]),
        "vsg_sharded_new": (C.c_int, [C.POINTER(ShardedOptions), C.POINTER(P)]),
        "vsg_sharded_free": (None, [P]),
        "vsg_sharded_reserve": (C.c_int, [P, sz]),
        "vsg_sharded_capacity": (sz, [P]),
        "vsg_sharded_size": (sz, [P]),
        "vsg_sharded_dimensions": (sz, [P]),
        "vsg_sharded_contains": (C.c_int, [P, u64]),
        "vsg_sharded_shard_count": (sz, [P]),
        "vsg_sharded_route": (u32, [P, u64]),
        "vsg_sharded_shard": (P, [P, sz]),
        "vsg_sharded_add": (C.c_int, [P, P, P, sz]),
        "vsg_sharded_remove": (C.c_int, [P, P, sz, C.POINTER(sz)]),
        "vsg_sharded_replace": (C.c_int, [P, P, P, sz, sz, u32, P, C.POINTER(sz)]),
        "vsg_sharded_search": (C.c_int, [P, P, sz, sz, sz, P, P, P]),
        "vsg_sharded_exact_search": (C.c_int, [P, P, sz, sz, P, P, P]),
        "vsg_sharded_search_device": (C.c_int, [P, P, sz, sz, sz, C.c_int, P, P, P]),
        "vsg_sharded_compact": (C.c_int, [P, C.POINTER(sz)]),
        "vsg_sharded_stats": (C.c_int, [P, C.POINTER(Stats)]),
        "vsg_sharded_reset_stats": (C.c_int, [P]),
        "vsg_last_error": (C.c_char_p, []),
        "vsg_version": (C.c_char_p, []),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc: int) -> None:
    if rc == VSG_OK:
        return
    msg = lib().vsg_last_error().decode(errors="replace")
    if rc == VSG_EDUPKEY:
        raise DuplicateKeyError(rc, msg)
    raise VsgError(rc, msg)
