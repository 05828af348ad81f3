"""Graph quality: GPU batched build vs the oracle's concurrent CPU build.

Both graphs are searched by the SAME search (the oracle's C restatement on
the host, and the GPU kernel), against exact GPU ground truth, so recall
differences come from the graphs alone.  usage (GPU box):
  python tools/graph_quality.py --rows 1000000 --dim 768 --metric cos
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--metric", default="cos")
    ap.add_argument("--queries", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--data", default="clustered")
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--efs", default="16,24,32,36,48,64,128")
    a = ap.parse_args()
    import torch
    import oracle as O
    import vsg
    from vsg import datagen as G

    bs, qs, ms = G.config_seeds(a.config)
    x = vsg.datagen_device(a.data, a.rows, a.dim, bs, ms)
    q = vsg.datagen_device(a.data, a.queries, a.dim, qs, ms)
    idx = vsg.Index(a.dim, a.metric, "f32", 16, 128, 64, seed=1)
    t0 = time.time()
    idx.add_device(np.arange(a.rows, dtype=np.uint64), x)
    gpu_build = time.time() - t0
    gt = idx.search_device(q, 10, exact=True)[0].cpu().numpy().astype(np.uint64)
    O.set_fast_metric(True)
    hg = O.HnswOracle(a.dim, a.metric, 16, 128, 64)
    hg.import_graph(idx.export())
    xh = x.cpu().numpy()
    qh = q.cpu().numpy()
    hc = O.HnswOracle(a.dim, a.metric, 16, 128, 64, seed=1)
    t0 = time.time()
    hc.add(np.arange(a.rows), xh, threads=a.threads)
    cpu_build = time.time() - t0
    res = {"rows": a.rows, "dim": a.dim, "data": a.data, "metric": a.metric,
           "gpu_build_s": round(gpu_build, 2), "cpu_build_s": round(cpu_build, 2),
           "cpu_threads": a.threads, "recall": {}}
    # the CPU-built graph searched by the GPU kernel too
    ic = vsg.Index(a.dim, a.metric, "f32", 16, 128, 64, seed=1)
    ic.import_graph(hc.export())
    for ef in [int(e) for e in a.efs.split(",")]:
        rg = np.mean([len(set(r) & set(t)) / 10 for r, t in zip(hg.search(qh, 10, ef)[0], gt)])
        rc = np.mean([len(set(r) & set(t)) / 10 for r, t in zip(hc.search(qh, 10, ef)[0], gt)])
        kg = idx.search(qh, 10, ef).keys
        rk = np.mean([len(set(r) & set(t)) / 10 for r, t in zip(kg, gt)])
        kc = ic.search(qh, 10, ef).keys
        rkc = np.mean([len(set(r) & set(t)) / 10 for r, t in zip(kc, gt)])
        res["recall"][ef] = {"gpu_graph_cpu_search": round(rg, 4), "cpu_graph_cpu_search": round(rc, 4),
                             "gpu_graph_gpu_search": round(rk, 4), "cpu_graph_gpu_search": round(rkc, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
