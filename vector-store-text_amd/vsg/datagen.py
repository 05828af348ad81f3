"""Portable synthetic embeddings.

Counter-based generator: every element is a pure function of (seed, index),
so any prefix, shard or row range can be regenerated independently, on the
host (numpy, here) or on the GPU (vsg_datagen_* in libvsg.so, same formulas).

* splitmix64 counter stream -> uniform in (0, 1] -> Box-Muller (cos branch).
* ``clustered``: 1024 centres in a 64-d latent space (sigma 1), point =
  centre + 0.5*N(0,1) in latent, projected by W in R^{64 x D} (N(0,1)/8), plus
  0.05*N(0,1) per output dim.  Relative contrast ~2.4 at 768-d (vs ~1.09 for
  iid Gaussian, reported as a stress row).
* ``uint8``: integer-valued 0..255 (SIFT-shape), exact in f32 and f16, so L2sq
  and IP sums are exact and brute-force top-k IDs are bit-exact on any
  summation order.
Seeds: base 0x5EED0000+config, queries 0x5EED1000+config, model 0x5EED2000+config.
"""
from __future__ import annotations

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)

# stream tags (xor-ed into the seed) — identical constants in csrc/datagen.hip
TAG_CLUSTER = 0x436C7573
TAG_LATENT = 0x4C6174
TAG_NOISE = 0x4E6F6973
TAG_CENTRE = 0x43656E74
TAG_PROJ = 0x50726F6A
TAG_U8 = 0x55380000

N_CENTRES = 1024
LATENT = 64


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
    return z ^ (z >> np.uint64(31))


def _stream(seed: int, tag: int) -> np.uint64:
    return splitmix64(np.uint64((seed ^ tag) & 0xFFFFFFFFFFFFFFFF))


def uniform(seed: int, tag: int, idx) -> np.ndarray:
    """uniform in (0, 1], f64."""
    base = _stream(seed, tag)
    with np.errstate(over="ignore"):
        r = splitmix64(base + np.asarray(idx, dtype=np.uint64))
    return ((r >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)


def normal(seed: int, tag: int, idx) -> np.ndarray:
    idx = np.asarray(idx, dtype=np.uint64)
    u1 = uniform(seed, tag, idx * np.uint64(2))
    u2 = uniform(seed, tag, idx * np.uint64(2) + np.uint64(1))
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)).astype(np.float32)


def model(dim: int, model_seed: int):
    """Cluster centres (1024 x 64) and projection W (64 x dim)."""
    centres = normal(model_seed, TAG_CENTRE, np.arange(N_CENTRES * LATENT)).reshape(N_CENTRES, LATENT)
    w = (normal(model_seed, TAG_PROJ, np.arange(LATENT * dim)).reshape(LATENT, dim) / 8.0).astype(np.float32)
    return centres, w


def clustered(n: int, dim: int, seed: int, model_seed: int, start: int = 0) -> np.ndarray:
    centres, w = model(dim, model_seed)
    rows = np.arange(start, start + n, dtype=np.uint64)
    cl = (splitmix64(_stream(seed, TAG_CLUSTER) + rows) % np.uint64(N_CENTRES)).astype(np.int64)
    lat_idx = rows[:, None] * np.uint64(LATENT) + np.arange(LATENT, dtype=np.uint64)[None, :]
    lat = centres[cl] + 0.5 * normal(seed, TAG_LATENT, lat_idx)
    out = lat.astype(np.float32) @ w
    noise_idx = rows[:, None] * np.uint64(dim) + np.arange(dim, dtype=np.uint64)[None, :]
    out += 0.05 * normal(seed, TAG_NOISE, noise_idx)
    return np.ascontiguousarray(out, dtype=np.float32)


def gaussian(n: int, dim: int, seed: int, start: int = 0) -> np.ndarray:
    rows = np.arange(start, start + n, dtype=np.uint64)
    idx = rows[:, None] * np.uint64(dim) + np.arange(dim, dtype=np.uint64)[None, :]
    return normal(seed, TAG_NOISE, idx)


def uint8_valued(n: int, dim: int, seed: int, start: int = 0) -> np.ndarray:
    rows = np.arange(start, start + n, dtype=np.uint64)
    idx = rows[:, None] * np.uint64(dim) + np.arange(dim, dtype=np.uint64)[None, :]
    r = splitmix64(_stream(seed, TAG_U8) + idx)
    return (r % np.uint64(256)).astype(np.float32)


SIFT_SCALE = 48.0


def sift_like(n: int, dim: int, seed: int, model_seed: int, start: int = 0) -> np.ndarray:
    """Clustered-latent rows, ReLU, scaled by 48 and rounded into 0..255 (SIFT
    shape): integer-valued, so exact in f16 and in f32 sums."""
    y = clustered(n, dim, seed, model_seed, start)
    return np.clip(np.rint(np.maximum(y, 0.0) * SIFT_SCALE), 0, 255).astype(np.float32)


def config_seeds(config: int):
    return 0x5EED0000 + config, 0x5EED1000 + config, 0x5EED2000 + config
