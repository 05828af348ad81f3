"""vsg — MI355X-native ANN index (HNSW build/search + exact search) for the
usearch-backed index path of swasik/vector-store-text.

Product path: libvsg.so (gfx950 HIP kernels behind include/vsg.h), reached
through ctypes.  No CPU fallback.
"""
from ._lib import (DuplicateKeyError, VsgError, LIB_PATH, NO_KEY, declared_symbols, lib)  # noqa: F401
from .index import Index, Matches, datagen_device, file_info, merge_topk_device, sample_level  # noqa: F401
from .sharded import ShardedIndex  # noqa: F401

__all__ = ["Index", "ShardedIndex", "Matches", "DuplicateKeyError", "VsgError", "datagen_device",
           "merge_topk_device", "sample_level", "file_info", "declared_symbols", "lib", "LIB_PATH", "NO_KEY"]
