#!/usr/bin/env python3
"""Build-quality probe: GPU HNSW build of the C2 workload under several batch
settings (VSG_BUILD_* env knobs), recall@10 at fixed ef against exact ground
truth, build wall time.  One JSON line per setting.

  python tools/build_quality_probe.py --rows 1000000 --dim 768 \
      --set frac=0.0625,max=32768 --set frac=0.015625,max=32768
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))

KNOBS = {"frac": "VSG_BUILD_BATCH_FRAC", "max": "VSG_BUILD_BATCH_MAX", "refine": "VSG_BUILD_REFINE",
         "frac2": "VSG_BUILD_BATCH_FRAC2", "switch": "VSG_BUILD_BATCH_SWITCH"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--metric", default="cos")
    ap.add_argument("--data", default="clustered")
    ap.add_argument("--quant", default="f32")
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--queries", type=int, default=1000)
    ap.add_argument("--ef", default="36,128")
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    import torch

    import vsg
    from vsg import datagen as G
    bs, qs, ms = G.config_seeds(a.config)
    x = vsg.datagen_device(a.data, a.rows, a.dim, bs, ms)
    q = vsg.datagen_device(a.data, a.queries, a.dim, qs, ms)
    gt = None
    for st in a.set or [""]:
        env = dict(kv.split("=") for kv in st.split(",") if kv)
        for k, v in env.items():
            os.environ[KNOBS.get(k, k)] = v
        idx = vsg.Index(a.dim, a.metric, a.quant, 16, 128, 64, seed=0x5EED)
        idx.reserve(a.rows)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        idx.add_device(np.arange(a.rows, dtype=np.uint64), x)
        torch.cuda.synchronize()
        bt = time.perf_counter() - t0
        if gt is None:
            gt = idx.search_device(q, 10, exact=True)[0].cpu().numpy()
        out = {"set": st, "build_s": round(bt, 3), "build_vps": round(a.rows / bt, 1),
               "batches": idx.stats()["build_batches"]}
        for ef in map(int, a.ef.split(",")):
            f = idx.search_device(q, 10, ef)[0].cpu().numpy()
            out[f"recall_ef{ef}"] = round(float(np.mean([len(set(f[i]) & set(gt[i])) / 10
                                                         for i in range(len(f))])), 4)
        print(json.dumps(out), flush=True)
        for k in env:
            os.environ.pop(KNOBS.get(k, k), None)
        del idx


if __name__ == "__main__":
    main()
