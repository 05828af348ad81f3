"""Build-schedule probe: one process, several GPU builds of the same rows under
different VSG_BUILD_* knob settings (read per add call), each reported with wall
time, kernel device times, batch count and recall@10 at a few ef against the
exact ground truth.  Used for the small-shard build work.

usage: python tools/build_probe.py --rows 125000 --settings 'base;VSG_BUILD_BATCH_FRAC=1'
  --settings: ';'-separated, each a ','-separated list of KEY=VALUE ('base' = none)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=125_000)
    ap.add_argument("--start", type=int, default=0, help="first row (shard r of G: r * N / G)")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--metric", default="cos")
    ap.add_argument("--quant", default="f32")
    ap.add_argument("--data", default="clustered")
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--queries", type=int, default=5000)
    ap.add_argument("--efs", default="10,16,24,32")
    ap.add_argument("--reps", type=int, default=2, help="builds per setting (the first warms up)")
    ap.add_argument("--settings", default="base")
    ap.add_argument("--out", default="gpurun_out/build_probe.jsonl")
    a = ap.parse_args()

    import torch

    import vsg
    from vsg import datagen as G

    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    bs, qs, ms = G.config_seeds(a.config)
    x = vsg.datagen_device(a.data, a.rows, a.dim, bs, ms, start=a.start)
    q = vsg.datagen_device(a.data, a.queries, a.dim, qs, ms)
    keys = np.arange(a.start, a.start + a.rows, dtype=np.uint64)
    gt = None
    for setting in a.settings.split(";"):
        kv = {} if setting.strip() in ("", "base") else dict(p.split("=", 1) for p in setting.split(","))
        for k, v in kv.items():
            os.environ[k] = v
        walls, st, idx = [], None, None
        for _ in range(a.reps):
            idx = vsg.Index(a.dim, a.metric, a.quant, 16, 128, 64, seed=0x5EED)
            idx.reserve(a.rows)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            idx.add_device(keys, x)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
            st = idx.stats()
        if gt is None:
            gt = idx.search_device(q, 10, exact=True)[0].cpu().numpy()
        rec = {}
        for ef in (int(e) for e in a.efs.split(",")):
            f = idx.search_device(q, 10, ef)[0].cpu().numpy()
            rec[ef] = round(float((f[:, :, None] == gt[:, None, :]).any(axis=1).sum(axis=1).mean() / 10), 4)
        line = {"rows": a.rows, "dim": a.dim, "setting": kv or "base",
                "lib": os.environ.get("VSG_LIB_PATH", "lib/libvsg.so").split("/")[-2], "wall_s": [round(w, 4) for w in walls],
                "insert_s": round(st["build_insert_ns"] * 1e-9, 4), "sort_s": round(st["build_sort_ns"] * 1e-9, 4),
                "reverse_s": round(st["build_reverse_ns"] * 1e-9, 4),
                "select_s": round(st["build_select_ns"] * 1e-9, 4), "batches": st["build_batches"],
                "select_dist_per_vec": round(st["build_select_distances"] / a.rows, 1),
                "reverse_dist_per_vec": round((st["reverse_select_distances"] + st["reverse_recompute_distances"]) / a.rows, 1),
                "recall": rec, "vec_per_s": round(a.rows / min(walls), 1)}
        print(json.dumps(line), flush=True)
        with open(a.out, "a") as fo:
            fo.write(json.dumps(line) + "\n")
        for k in kv:
            os.environ.pop(k, None)
        del idx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
