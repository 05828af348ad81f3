"""Recall with distance ties: key-set recall vs distance-threshold recall.

usage (GPU box): python tools/tie_recall_probe.py rows dim metric quant data config efs
Integer-valued data (sift_like) has integer distances, so many rows can sit at
the k-th neighbour's distance; exact search breaks those ties by slot, HNSW
returns whichever tied rows it reached.  Prints, per ef: key-set recall@10,
distance-threshold recall@10 (a result counts if its distance <= the exact
10th distance, ann-benchmarks style), and the share of queries whose exact
10th and 11th distances tie.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))


def main():
    rows, dim, metric, quant, data, config = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4],
                                              sys.argv[5], int(sys.argv[6]))
    efs = [int(e) for e in sys.argv[7].split(",")]
    seed = int(sys.argv[8], 0) if len(sys.argv) > 8 else 1
    import torch
    import vsg
    from vsg import datagen as G

    bs, qs, ms = G.config_seeds(config)
    idx = vsg.Index(dim, metric, quant, 16, 128, 64, seed=seed)
    idx.reserve(rows)
    step = rows  # one add call, as bench.py
    t0 = time.time()
    for lo in range(0, rows, step):
        n = min(step, rows - lo)
        x = vsg.datagen_device(data, n, dim, bs, ms, start=lo)
        idx.add_device(np.arange(lo, lo + n, dtype=np.uint64), x)
        del x
    torch.cuda.synchronize()
    st = idx.stats()
    print(json.dumps({"build_s": round(time.time() - t0, 1), "seed": seed, "batches": st["build_batches"],
                      "batch_max": os.environ.get("VSG_BUILD_BATCH_MAX", "32768"),
                      "graph": idx.graph_info()}), flush=True)
    q = vsg.datagen_device(data, 200, dim, qs, ms)
    gk, gd = [t.cpu().numpy() for t in idx.search_device(q, 11, exact=True)[:2]]
    ties = float(np.mean(gd[:, 9] == gd[:, 10]))
    for ef in efs:
        k, d = [t.cpu().numpy() for t in idx.search_device(q, 10, ef)[:2]]
        key_rec = float(np.mean([len(set(a) & set(b[:10])) / 10 for a, b in zip(k, gk)]))
        dist_rec = float(np.mean([(d[i] <= gd[i, 9]).sum() / 10 for i in range(len(q))]))
        print(json.dumps({"rows": rows, "seed": seed, "ef": ef, "recall_keys": round(key_rec, 4), "recall_dist": round(dist_rec, 4),
                          "queries_with_10th_11th_tie": round(ties, 3)}), flush=True)


if __name__ == "__main__":
    main()
