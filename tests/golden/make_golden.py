"""Generate the committed golden fixtures (run from repo root: python tests/golden/make_golden.py).

Inputs are NOT committed: they are regenerated from the seeds below by the
portable counter-based generator (vector-store-text_amd/vsg/datagen.py).  Only
seeds, shapes and expected outputs are stored.  Expected top-k comes from a
numpy float64 brute force with ties broken by ascending key (SURVEY.md §8c,
G1-G5).  The reference's own known-answer tests are re-expressed in kats.json.

Fixtures:
  G1 g1_u8_l2sq.npz   10k x 128 integer 0..255, 100 queries, k=10, L2sq (exact)
  G1b g1_u8_ip.npz    same inputs, IP (exact: integer sums < 2^24)
  G2 g2_cl_ip.npz / g2_cl_cos.npz   10k x 128 clustered float, IP / cos, with d_k+1 - d_k gaps
  G3 g3_cl768_cos.npz 2k x 768 clustered cos, 50 queries
  G4 kats.json        /root/reference/src/index/usearch.rs:322-425 and
                      /root/reference/tests/integration/usearch.rs:74-123
  G5 (f16 storage) reuses G1: integers <= 255 are exact in f16.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))
from vsg import datagen as G  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def exact_f64(metric, base, queries, k):
    b = base.astype(np.float64)
    q = queries.astype(np.float64)
    if metric == "l2sq":
        d = (q * q).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2.0 * q @ b.T
        # recompute exactly for integer inputs to avoid cancellation noise
        d = np.stack([((b - qi) ** 2).sum(1) for qi in q])
    elif metric == "ip":
        d = 1.0 - q @ b.T
    else:
        nb = np.sqrt((b * b).sum(1))
        nq = np.sqrt((q * q).sum(1))
        d = 1.0 - (q @ b.T) / (nq[:, None] * nb[None, :])
    keys = np.arange(base.shape[0])
    ids = np.empty((q.shape[0], k + 1), np.int64)
    dist = np.empty((q.shape[0], k + 1), np.float64)
    for i in range(q.shape[0]):
        order = np.lexsort((keys, d[i]))[: k + 1]
        ids[i] = order
        dist[i] = d[i][order]
    return ids, dist


def save(name, **kw):
    np.savez(os.path.join(OUT, name), **kw)
    print("wrote", name, {k: getattr(v, "shape", v) for k, v in kw.items()})


def main():
    # G1: integer-valued SIFT-shape, config 0 (BASELINE.json configs[0]: 10k x 128 L2)
    bs, qs, _ = G.config_seeds(0)
    n, d, nq, k = 10_000, 128, 100, 10
    x = G.uint8_valued(n, d, bs)
    q = G.uint8_valued(nq, d, qs)
    for metric, fname in (("l2sq", "g1_u8_l2sq.npz"), ("ip", "g1_u8_ip.npz")):
        ids, dist = exact_f64(metric, x, q, k)
        save(fname, gen=np.array("uint8"), n=n, dim=d, nq=nq, k=k, base_seed=bs, query_seed=qs,
             metric=np.array(metric), ids=ids[:, :k], dist=dist[:, :k], gap=dist[:, k] - dist[:, k - 1])
    # G2: clustered float, same shape
    bs, qs, ms = G.config_seeds(0)
    x = G.clustered(n, d, bs, ms)
    q = G.clustered(nq, d, qs, ms)
    for metric, fname in (("ip", "g2_cl_ip.npz"), ("cos", "g2_cl_cos.npz"), ("l2sq", "g2_cl_l2sq.npz")):
        ids, dist = exact_f64(metric, x, q, k)
        save(fname, gen=np.array("clustered"), n=n, dim=d, nq=nq, k=k, base_seed=bs, query_seed=qs,
             model_seed=ms, metric=np.array(metric), ids=ids[:, :k], dist=dist[:, :k],
             gap=dist[:, k] - dist[:, k - 1])
    # G3: 768-d cosine (BASELINE.json configs[1] shape, reduced rows)
    bs, qs, ms = G.config_seeds(1)
    n3, d3, nq3 = 2_000, 768, 50
    x = G.clustered(n3, d3, bs, ms)
    q = G.clustered(nq3, d3, qs, ms)
    ids, dist = exact_f64("cos", x, q, k)
    save("g3_cl768_cos.npz", gen=np.array("clustered"), n=n3, dim=d3, nq=nq3, k=k, base_seed=bs,
         query_seed=qs, model_seed=ms, metric=np.array("cos"), ids=ids[:, :k], dist=dist[:, :k],
         gap=dist[:, k] - dist[:, k - 1])
    # G4: the reference's known-answer tests, as data.
    kats = {
        "source": [
            "/root/reference/src/index/usearch.rs:322-425 (add_or_replace_size_ann)",
            "/root/reference/tests/integration/usearch.rs:74-123 (simple_create_search_delete_index)",
        ],
        "note": "metric unset in the reference (usearch.rs:89-96); deterministic under l2sq and ip, "
                "a rounding tie under cos (SURVEY.md §0.5), so cos is excluded",
        "metrics": ["l2sq", "ip"],
        "unit_actor": {
            "dimensions": 3,
            "steps": [
                {"op": "add_or_replace", "pk": [1, "one"], "embedding": [1.0, 1.0, 1.0]},
                {"op": "add_or_replace", "pk": [2, "two"], "embedding": [2.0, -2.0, 2.0]},
                {"op": "add_or_replace", "pk": [3, "three"], "embedding": [3.0, 3.0, 3.0]},
                {"op": "count", "expect": 3},
                {"op": "ann", "embedding": [2.2, -2.2, 2.2], "limit": 1, "expect_pk": [2, "two"]},
                {"op": "add_or_replace", "pk": [3, "three"], "embedding": [2.1, -2.1, 2.1]},
                {"op": "ann", "embedding": [2.2, -2.2, 2.2], "limit": 1, "expect_pk": [3, "three"]},
                {"op": "remove", "pk": [3, "three"]},
                {"op": "count", "expect": 2},
                {"op": "ann", "embedding": [2.2, -2.2, 2.2], "limit": 1, "expect_pk": [2, "two"]},
            ],
        },
        "integration": {
            "dimensions": 3,
            "rows": [[[1, "one"], [1.0, 1.0, 1.0]], [[2, "two"], [2.0, -2.0, 2.0]],
                     [[3, "three"], [3.0, 3.0, 3.0]]],
            "count": 3,
            "ann": {"embedding": [2.1, -2.0, 2.0], "limit": 1, "expect_pk": [2, "two"]},
        },
    }
    with open(os.path.join(OUT, "kats.json"), "w") as f:
        json.dump(kats, f, indent=1)
    print("wrote kats.json")


if __name__ == "__main__":
    main()
