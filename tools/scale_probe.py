"""Probe recall / build behaviour at scale (GPU box).

usage: python tools/scale_probe.py rows dim metric quant data [batch_max] [efs...]
prints one JSON line: build time, build distance evals/vector, recall@10 per ef
against exact ground truth (200 queries).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))


def main():
    rows, dim, metric, quant, data = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    bmax = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    efs = [int(e) for e in sys.argv[7:]] or [32, 64, 128]
    if bmax:
        os.environ["VSG_BUILD_BATCH_MAX"] = str(bmax)
    import torch
    import vsg
    from vsg import datagen as G

    bs, qs, ms = G.config_seeds(3 if data == "sift" else 2)
    x = vsg.datagen_device(data, rows, dim, bs, ms)
    q = vsg.datagen_device(data, 200, dim, qs, ms)
    xs = x[:: max(1, rows // 5)].cpu().numpy()
    idx = vsg.Index(dim, metric, quant, 16, 128, 64, seed=1)
    t0 = time.time()
    idx.add_device(np.arange(rows, dtype=np.uint64), x)
    torch.cuda.synchronize()
    bt = time.time() - t0
    st = idx.stats()
    gt = idx.search_device(q, 10, exact=True)[0].cpu().numpy()
    ex = idx.export() if rows <= 2_000_000 else None
    out = {"rows": rows, "dim": dim, "metric": metric, "quant": quant, "data": data, "batch_max": bmax,
           "build_s": round(bt, 2), "build_dist_per_vec": round(st["build_distances"] / rows, 1),
           "batches": st["build_batches"], "sample_rows_nonzero": float(np.mean(np.abs(xs).sum(1) > 0)),
           "gt_valid": float(np.mean(gt >= 0)), "recall": {},
           "build_breakdown_per_vec": {f: round(st[f] / rows, 2) for f in (
               "build_select_distances", "reverse_recompute_distances", "reverse_select_distances",
               "reverse_prunes", "reverse_appends", "build_adjacency")}}
    out["build_breakdown_per_vec"]["beam_distances"] = round(
        (st["build_distances"] - st["build_select_distances"] - st["reverse_recompute_distances"]
         - st["reverse_select_distances"]) / rows, 1)
    info = idx.graph_info()
    out["max_level"] = info["max_level"]
    if ex is not None:
        deg = (ex["adj0"] != 0xFFFFFFFF).sum(1)
        out["deg0_mean"] = float(deg.mean())
        out["deg0_min"] = int(deg.min())
    for ef in efs:
        k = idx.search_device(q, 10, ef)[0].cpu().numpy()
        out["recall"][ef] = round(float(np.mean([len(set(a) & set(b)) / 10 for a, b in zip(k, gt)])), 4)
    st = idx.stats()
    out["search_dist_per_query"] = round(st["search_distances"] / max(1, st["search_queries"]), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
