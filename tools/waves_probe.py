"""Search QPS vs waves per query (VSG_SEARCH_WAVES), one build.

usage (GPU box): python tools/waves_probe.py rows dim metric quant data efs waves
  efs, waves: comma lists, e.g. 36,128,321 1,2,4
prints one JSON line per (ef, waves): QPS over 10,000 queries, recall@10 (200
queries vs exact) and whether keys/distances equal the 1-wave kernel's.
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))


def main():
    rows, dim, metric, quant, data = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    efs = [int(e) for e in sys.argv[6].split(",")]
    waves = sys.argv[7].split(",")  # "1", "2", "4": LDS-list kernels; "r": register kernel; "s": + runner-up; "v": + bucketed visited; "w": both
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
    for ef in efs:
        base = None
        for w in waves:
            os.environ["VSG_SEARCH_REG"] = "1" if w in "rsvw" else "0"
            os.environ["VSG_SEARCH_SPEC"] = "1" if w in "sw" else "0"
            os.environ["VSG_SEARCH_VIS8"] = "1" if w in "vw" else "0"
            os.environ["VSG_SEARCH_WAVES"] = "1" if w in "rsvw" else w
            kk, dd = idx.search_device(q, 10, ef)[:2]
            kk, dd = kk.cpu().numpy(), dd.cpu().numpy()
            if base is None:
                base = (kk, dd)
            same = bool((kk == base[0]).all() and (dd == base[1]).all())
            rec = float(np.mean([len(set(a) & set(b)) / 10 for a, b in zip(kk[:200], gt)]))
            torch.cuda.synchronize()
            idx.reset_stats()
            t0 = time.time()
            for _ in range(3):
                idx.search_device(q, 10, ef)
            torch.cuda.synchronize()
            dt = (time.time() - t0) / 3
            st = idx.stats()
            raw = (C.c_uint64 * 16)()
            vsg.lib().vsg_debug_counters(idx._h, raw)
            nq = max(1, st["search_queries"])
            extra = {"dist_per_query": round(st["search_distances"] / nq, 1),
                     "expansions_per_query": round(st["search_adjacency"] / nq, 1)}
            if raw[10] or raw[11]:  # profiling build: wave-microseconds per query per phase
                extra.update({f"us_{k}": round(raw[i] / 100.0 / nq, 2) for k, i in (("adj", 10), ("dist", 11), ("merge", 12))})
            print(json.dumps({"rows": rows, "dim": dim, "metric": metric, "quant": quant, "ef": ef, "kernel": {"r": "reg", "s": "reg+spec", "v": "reg+vis8", "w": "reg+vis8+spec"}.get(w, f"list{w}"),
                              "build_s": round(bt, 2), "qps": round(10000 / dt, 1), "recall": round(rec, 4),
                              "same_as_1wave": same, **extra}), flush=True)


if __name__ == "__main__":
    main()
