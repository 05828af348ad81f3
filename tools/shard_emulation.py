"""Row-sharded index of C3/C4 emulated on ONE GPU.

All G shards live in this GPU's HBM (C4: 8 x 12.5M x 128 f16 ~ 40 GB of 288 GB);
each is built and searched exactly as one rank of bench.py's shard leg would
(same seeds, rows [r N/G, (r+1) N/G), seed 0x5EED + r), and the per-shard top-k
lists are merged by the same HIP merge kernel the RCCL all-gather feeds.  What
is NOT emulated: the all-gather itself (B x k x 12 B per rank, latency-bound).

Reports per ef: merged recall@10 vs exact ground truth (exact per shard +
merge), per-shard search time for the whole query batch, the projected G-GPU
QPS = B / max shard time, and the measured 1-GPU QPS = B / sum of shard times.
Hybrid layouts (round 4): on --gpus-total T GPUs, T / G replica groups of these
G row shards each serve their own batch -> projected T-GPU QPS = (T / G) x the
G-shard QPS; the build of each group is the G-shard build (every group holds the
whole index).

usage: python tools/shard_emulation.py --rows 100000000 --dim 128 --quant f16 --metric l2sq --data sift --config 3
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
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--quant", default="f16")
    ap.add_argument("--metric", default="l2sq")
    ap.add_argument("--data", default="sift")
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--gt-queries", type=int, default=1_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--efs", default="16,32,64,96,128,192,256")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/shard_emulation.jsonl")
    ap.add_argument("--gpus-total", type=int, default=8, help="hybrid projection: GPUs of the node")
    a = ap.parse_args()

    import torch

    import vsg
    from vsg import datagen as G
    from vsg.distributed import merge_topk

    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    bs, qs, ms = G.config_seeds(a.config)
    G_ = a.shards
    shards, build_s = [], []
    for r in range(G_):
        lo, hi = r * a.rows // G_, (r + 1) * a.rows // G_
        x = vsg.datagen_device(a.data, hi - lo, a.dim, bs, ms, start=lo)
        idx = vsg.Index(a.dim, a.metric, a.quant, 16, 128, 128, seed=0x5EED + r)
        idx.reserve(hi - lo)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        idx.add_device(np.arange(lo, hi, dtype=np.uint64), x)
        torch.cuda.synchronize()
        build_s.append(time.perf_counter() - t0)
        del x
        torch.cuda.empty_cache()
        shards.append(idx)
        print(f"shard {r}: {hi - lo} rows built in {build_s[-1]:.2f} s", flush=True)
    q = vsg.datagen_device(a.data, a.queries, a.dim, qs, ms)
    qgt = vsg.datagen_device(a.data, a.gt_queries, a.dim, qs, ms)

    def merged(qt, ef, exact=False):
        outs = [s.search_device(qt, a.k, ef, exact=exact) for s in shards]
        gk = torch.stack([o[0] for o in outs])
        gd = torch.stack([o[1] for o in outs])
        return merge_topk(gk, gd, a.k)

    t0 = time.perf_counter()
    gt = merged(qgt, 0, exact=True)[0].cpu().numpy()
    print(f"ground truth: {time.perf_counter() - t0:.1f} s", flush=True)
    head = {"rows": a.rows, "shards": G_, "dim": a.dim, "quant": a.quant, "metric": a.metric, "data": a.data,
            "queries": a.queries, "build_s_per_shard": [round(b, 2) for b in build_s],
            "build_vectors_per_s_1gpu": round(a.rows / sum(build_s), 1),
            "build_vectors_per_s_projected": round(a.rows / max(build_s), 1)}
    with open(a.out, "a") as f:
        f.write(json.dumps(head) + "\n")
    print(json.dumps(head), flush=True)
    for ef in [int(e) for e in a.efs.split(",")]:
        f_ = merged(qgt, ef)[0].cpu().numpy()
        rec = float(np.mean([len(set(f_[i]) & set(gt[i])) / a.k for i in range(gt.shape[0])]))
        per, dpq, gbs = [], [], []
        per16 = 4 if a.quant == "f32" else 8
        row_bytes = (a.dim + per16 - 1) // per16 * 16
        for s in shards:
            s.search_device(q, a.k, ef)  # warm
            s.reset_stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                s.search_device(q, a.k, ef)
            torch.cuda.synchronize()
            per.append((time.perf_counter() - t0) / a.steps)
            st = s.stats()
            nq = max(1, st["search_queries"])
            # per-shard algorithmic bytes (rows evaluated + adjacency rows read)
            alg = (st["search_distances"] * row_bytes + st["search_adjacency"] * 32 * 4) / a.steps
            dpq.append(round(st["search_distances"] / nq, 1))
            gbs.append(round(alg / per[-1] / 1e9, 1))
        tm = time.perf_counter()
        for _ in range(a.steps):
            merged(q, ef)
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - tm) / a.steps
        line = {"ef": ef, "recall_at_10": round(rec, 4), "shard_ms": [round(1000 * p, 3) for p in per],
                "dist_evals_per_query_per_shard": dpq, "alg_gbs_per_shard": gbs,
                "qps_projected_gpus": round(a.queries / max(per), 1),
                "qps_1gpu_all_shards": round(a.queries / t_all, 1)}
        if a.gpus_total % G_ == 0:
            grp = a.gpus_total // G_
            line["hybrid_projection"] = {"gpus": a.gpus_total, "shards_per_group": G_, "groups": grp,
                                         "qps": round(grp * a.queries / max(per), 1),
                                         "build_vectors_per_s": round(a.rows / max(build_s), 1)}
        with open(a.out, "a") as f:
            f.write(json.dumps(line) + "\n")
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
