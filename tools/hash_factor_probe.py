"""Search QPS vs visited-table size (VSG_SEARCH_HASH_FACTOR), one build.

usage (GPU box): python tools/hash_factor_probe.py rows dim metric quant data ef [factors...]
prints one JSON line per factor: QPS over 10,000 queries, distance evals/query,
recall@10 (200 queries vs exact) -- recall must not depend on the factor.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))


def main():
    rows, dim, metric, quant, data, ef = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4],
                                         sys.argv[5], int(sys.argv[6]))
    factors = [int(f) for f in sys.argv[7:]] or [12, 16, 24, 32]
    import torch
    import vsg
    from vsg import datagen as G

    bs, qs, ms = G.config_seeds(3 if data == "sift" else 2)
    x = vsg.datagen_device(data, rows, dim, bs, ms)
    q = vsg.datagen_device(data, 10000, dim, qs, ms)
    idx = vsg.Index(dim, metric, quant, 16, 128, 64, seed=1)
    t0 = time.time()
    idx.add_device(np.arange(rows, dtype=np.uint64), x)
    torch.cuda.synchronize()
    bt = time.time() - t0
    del x
    gt = idx.search_device(q[:200], 10, exact=True)[0].cpu().numpy()
    for f in factors:
        os.environ["VSG_SEARCH_HASH_FACTOR"] = str(f)
        k = idx.search_device(q[:200], 10, ef)[0].cpu().numpy()
        rec = float(np.mean([len(set(a) & set(b)) / 10 for a, b in zip(k, gt)]))
        idx.search_device(q, 10, ef)
        torch.cuda.synchronize()
        idx.reset_stats()
        t0 = time.time()
        for _ in range(3):
            idx.search_device(q, 10, ef)
        torch.cuda.synchronize()
        dt = (time.time() - t0) / 3
        st = idx.stats()
        print(json.dumps({"rows": rows, "dim": dim, "metric": metric, "quant": quant, "ef": ef, "factor": f,
                          "build_s": round(bt, 2), "qps": round(10000 / dt, 1), "recall": round(rec, 4),
                          "dist_per_query": round(st["search_distances"] / st["search_queries"], 1)}),
              flush=True)


if __name__ == "__main__":
    main()
