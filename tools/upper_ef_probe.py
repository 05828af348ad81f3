"""Opt-in multi-entry descent probe (VSG_SEARCH_UPPER_EF): one graph, recall@10
and QPS per (upper_ef, ef) against exact GPU ground truth.  usage (GPU box):
  python tools/upper_ef_probe.py ROWS DIM METRIC QUANT DATA CONFIG EFS UPPER_EFS [SEED]
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
    ues = [int(e) for e in sys.argv[8].split(",")]
    seed = int(sys.argv[9], 0) if len(sys.argv) > 9 else 0x5EED
    import torch
    import vsg
    from vsg import datagen as G

    bs, qs, ms = G.config_seeds(config)
    idx = vsg.Index(dim, metric, quant, 16, 128, 64, seed=seed)
    idx.reserve(rows)
    t0 = time.time()
    x = vsg.datagen_device(data, rows, dim, bs, ms)
    idx.add_device(np.arange(rows, dtype=np.uint64), x)
    torch.cuda.synchronize()
    del x
    print(json.dumps({"rows": rows, "build_s": round(time.time() - t0, 1), "graph": idx.graph_info()}), flush=True)
    qg = vsg.datagen_device(data, 500, dim, qs, ms)
    q = vsg.datagen_device(data, 10000, dim, qs, ms)
    gk = idx.search_device(qg, 10, exact=True)[0].cpu().numpy()
    for ue in ues:
        os.environ["VSG_SEARCH_UPPER_EF"] = str(ue)
        for ef in efs:
            k = idx.search_device(qg, 10, ef)[0].cpu().numpy()
            rec = float(np.mean([len(set(a) & set(b)) / 10 for a, b in zip(k, gk)]))
            idx.search_device(q, 10, ef)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                idx.search_device(q, 10, ef)
            torch.cuda.synchronize()
            qps = 3 * len(q) / (time.perf_counter() - t0)
            print(json.dumps({"rows": rows, "upper_ef": ue, "ef": ef, "recall_at_10": round(rec, 4),
                              "qps": round(qps, 1)}), flush=True)


if __name__ == "__main__":
    main()
