#!/usr/bin/env python3
"""bench.py — kNN QPS @ recall@10 >= 0.95 (+ build vectors/s) on synthetic 1M x 768 f32 cosine.

Workload = BASELINE.json configs[1]: 1M x 768 f32, cosine, HNSW M=16, efC=128,
k=10, clustered-latent synthetic data generated in HBM (vsg/datagen.py formulas).
One step = one HNSW search pass of the query batch (10,000 queries, inputs
resident in HBM) at the smallest ef whose recall@10 against exact ground truth is
>= 0.95 (ef swept on a 1,000-query subset).  N > 1: the index is
row-range sharded (rank r owns rows [r N/G, (r+1) N/G)), every rank searches its
shard, per-shard top-k is all-gathered over RCCL and k-way merged on every rank
(SURVEY.md §8e).  Total work is fixed as N grows => "scaling": "strong".

Also reported: build vectors/s (GPU batched HNSW build of the whole index, max over
ranks), the HBM roofline of the search kernel (algorithmic bytes counted by the
kernel: distance evaluations x row bytes + adjacency rows x 128 B, per launch, /
HIP-event time on the launching stream), and the CPU baseline (oracle/ C
restatement of usearch, SIMD metrics, all host cores or
SCYLLA_USEARCH_BACKGROUND_THREADS) timed on a bounded sample on rank 0 at N=1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--metric", default="cos")
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--gt-queries", type=int, default=1_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--efc", type=int, default=128)
    ap.add_argument("--ef", type=int, default=0, help="fixed ef (0 = sweep for recall >= target)")
    ap.add_argument("--target-recall", type=float, default=0.95)
    ap.add_argument("--config", type=int, default=1, help="seed set (BASELINE.json configs index)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget per CPU-baseline leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--mode", default="hnsw", choices=("hnsw", "exact"),
                    help="exact: brute-force MFMA path (C5: --rows 1000000 --dim 1536 --metric ip)")
    ap.add_argument("--batch", type=int, default=1024, help="exact mode: queries per step")
    ap.add_argument("--quant", default="f32", choices=("f32", "f16"), help="HBM storage type")
    ap.add_argument("--sort-queries", default="none", choices=("none", "cluster"),
                    help="experiment: order the query batch by synthetic cluster id")
    ap.add_argument("--sort-base", default="none", choices=("none", "cluster"),
                    help="experiment: insert base rows in synthetic-cluster order (spatial slot ids)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearse several ranks on one GPU (collectives via host)")
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import vsg
    from vsg import datagen as G

    from vsg.distributed import gather_topk, merge_topk

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())  # >1 rank per GPU only for gloo rehearsal
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.dist_backend)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    bs, qs, ms = G.config_seeds(a.config)
    lo, hi = rank * a.rows // world, (rank + 1) * a.rows // world
    nloc = hi - lo
    stream = torch.cuda.current_stream()

    # ---- inputs in HBM
    x = vsg.datagen_device("clustered", nloc, a.dim, bs, ms, start=lo)
    q = vsg.datagen_device("clustered", a.queries, a.dim, qs, ms)
    if a.sort_queries == "cluster":
        cl = (G.splitmix64(G._stream(qs, G.TAG_CLUSTER) + np.arange(a.queries, dtype=np.uint64))
              % np.uint64(G.N_CENTRES)).astype(np.int64)
        q = q[torch.from_numpy(np.argsort(cl, kind="stable")).to(dev)].contiguous()
    torch.cuda.synchronize()

    if a.mode == "exact":
        return run_exact(a, x, q, lo, hi, world, rank, local, dev, stream, barrier, max_over_ranks)

    # ---- build (timed; not part of the QPS step)
    index = vsg.Index(a.dim, a.metric, a.quant, a.M, a.efc, 128, device=local, seed=0x5EED + rank)
    index.reserve(nloc)
    keys_np = np.arange(lo, hi, dtype=np.uint64)
    if a.sort_base == "cluster":
        cl = (G.splitmix64(G._stream(bs, G.TAG_CLUSTER) + keys_np) % np.uint64(G.N_CENTRES)).astype(np.int64)
        order = np.argsort(cl, kind="stable")
        x = x[torch.from_numpy(order).to(dev)].contiguous()
        keys_np = keys_np[order]
    barrier()
    t0 = time.perf_counter()
    index.add_device(keys_np, x, stream=stream)
    torch.cuda.synchronize()
    build_s = max_over_ranks(time.perf_counter() - t0)
    build_vps = a.rows / build_s
    bstats = index.stats()

    def sharded(qt, ef, exact=False):
        keys, dists = index.search_device(qt, a.k, ef, stream=stream, exact=exact)
        if world == 1:
            return keys, dists
        gk, gd = gather_topk(keys, dists)
        return merge_topk(gk, gd, a.k, stream=stream)

    # ---- ground truth (exact, GPU brute force, same sharded merge path)
    qgt = q[: a.gt_queries].contiguous()
    gt_keys, _ = sharded(qgt, 0, exact=True)
    gt = gt_keys.cpu().numpy()

    def recall_of(keys_t):
        f = keys_t.cpu().numpy()
        return float(np.mean([len(set(f[i]) & set(gt[i])) / a.k for i in range(gt.shape[0])]))

    # ---- ef selection
    sweep = []
    if a.ef:
        ef = a.ef
        sweep.append((ef, recall_of(sharded(qgt, ef)[0])))
    else:
        ef, lo_fail = None, None
        for cand in (16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512):
            r = recall_of(sharded(qgt, cand)[0])
            sweep.append((cand, r))
            if r >= a.target_recall:
                ef = cand
                break
            lo_fail = cand
        if ef is None:
            ef = sweep[-1][0]
        elif lo_fail is not None:
            # smallest ef in (lo_fail, ef] that still meets the target
            e_lo, e_hi = lo_fail, ef
            while e_hi - e_lo > 2:
                mid = (e_lo + e_hi) // 2
                r = recall_of(sharded(qgt, mid)[0])
                sweep.append((mid, r))
                if r >= a.target_recall:
                    e_hi = mid
                else:
                    e_lo = mid
            ef = e_hi
    recall = dict(sweep)[ef]

    # ---- timed QPS steps
    for _ in range(a.warmup):
        sharded(q, ef)
    index.reset_stats()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    kern_ms = 0.0
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ev0.record(stream)
        keys, dists = index.search_device(q, a.k, ef, stream=stream)
        ev1.record(stream)
        if world > 1:
            gk, gd = gather_topk(keys, dists)
            keys, dists = merge_topk(gk, gd, a.k, stream=stream)
        torch.cuda.synchronize()
        kern_ms += ev0.elapsed_time(ev1)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    ms_per_step = 1000.0 * elapsed / a.steps
    qps = a.queries * a.steps / elapsed
    st = index.stats()
    per16 = 4 if a.quant == "f32" else 8
    row_bytes = ((a.dim + per16 - 1) // per16) * 16
    alg_bytes = (st["search_distances"] * row_bytes + st["search_adjacency"] * 2 * a.M * 4) / a.steps
    kern_ms_avg = kern_ms / a.steps
    achieved = alg_bytes / (kern_ms_avg * 1e-3) / 1e9

    out = {
        "metric": "kNN QPS @ recall@10>=0.95 (HNSW, 1M x 768 f32 cos)",
        "value": round(qps, 1),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": a.quant,
        "data": "synthetic clustered-latent embeddings generated in HBM (vsg/datagen.py), 10k queries/step",
        "config": {"workload": f"C2: {a.rows} x {a.dim} f32 {a.metric} HNSW M={a.M} efC={a.efc} k={a.k}",
                   "index_rows": a.rows, "dim": a.dim, "queries_per_step": a.queries,
                   "ef": ef, "recall_at_10": round(recall, 4), "ef_sweep": sweep,
                   "parallelism": f"row-shard x{world}" + (" + RCCL all-gather top-k" if world > 1 else "")},
        "build_vectors_per_s": round(build_vps, 1),
        "build_seconds": round(build_s, 3),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": pmc_traffic(a, ef),
                     "kernel": "hnsw_search_kernel<64,3,4,float,1>", "kernel_ms": round(kern_ms_avg, 3),
                     "alg_bytes_per_launch": int(alg_bytes),
                     "dist_evals_per_query": round(st["search_distances"] / max(1, st["search_queries"]), 1)},
        "build_stats": {"distance_evals_per_vector": round(bstats["build_distances"] / max(1, nloc), 1),
                        "batches": bstats["build_batches"]},
    }

    # ---- CPU baseline (rank 0, N=1 only): oracle/ restatement of usearch
    if world == 1 and rank == 0 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(a, index, q, ef, x)
        if out["cpu_baseline"].get("qps"):
            out["gpu_over_cpu_qps"] = round(qps / out["cpu_baseline"]["qps"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense


def run_exact(a, x, q, lo, hi, world, rank, local, dev, stream, barrier, max_over_ranks):
    """Brute-force mode: one step = exact top-k of a batch of
    queries over the whole index on the f32 matrix cores; roofline bound = MFMA."""
    import torch

    import vsg
    from vsg.distributed import gather_topk, merge_topk

    nloc = hi - lo
    index = vsg.Index(a.dim, a.metric, a.quant, device=local, exact_only=True)
    index.add_device(np.arange(lo, hi, dtype=np.uint64), x, stream=stream)
    qb = q[: a.batch].contiguous()

    def step():
        keys, dists = index.search_device(qb, a.k, stream=stream, exact=True)
        if world > 1:
            gk, gd = gather_topk(keys, dists)
            keys, dists = merge_topk(gk, gd, a.k, stream=stream)
        return keys, dists

    for _ in range(a.warmup):
        step()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kern_ms = 0.0
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ev0.record(stream)
        keys, dists = index.search_device(qb, a.k, stream=stream, exact=True)
        ev1.record(stream)
        if world > 1:
            gk, gd = gather_topk(keys, dists)
            keys, dists = merge_topk(gk, gd, a.k, stream=stream)
        torch.cuda.synchronize()
        kern_ms += ev0.elapsed_time(ev1)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    qps = a.batch * a.steps / elapsed
    kms = kern_ms / a.steps
    flops = 2.0 * a.batch * nloc * a.dim
    tflops = flops / (kms * 1e-3) / 1e12
    out = {
        "metric": f"brute-force kNN QPS (exact, f32 MFMA), {a.rows} x {a.dim} f32 {a.metric}, batch {a.batch}",
        "value": round(qps, 1), "unit": "queries/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(1000 * elapsed / a.steps, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic clustered-latent embeddings generated in HBM (vsg/datagen.py)",
        "config": {"workload": f"C5: {a.rows} x {a.dim} f32 {a.metric} brute force, k={a.k}",
                   "batch": a.batch, "parallelism": f"row-shard x{world}"},
        "roofline": {"bound": "mfma", "achieved": round(tflops, 2), "peak": MFMA_F32_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(tflops / MFMA_F32_PEAK_TFLOPS, 4), "traffic": None,
                     "kernel": "mfma_exact_kernel<16,MET> (+prepare, merge)", "kernel_ms": round(kms, 3),
                     "flops_per_launch": flops},
    }
    if world == 1 and rank == 0 and not a.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        O.set_fast_metric(True)
        threads = host_cores()
        xh = x.cpu().numpy()
        qh = qb.cpu().numpy()
        n = 4
        t0 = time.perf_counter()
        ok, od, _ = O.exact_search(a.metric, xh, qh[:n], a.k, threads=threads)
        dt = time.perf_counter() - t0
        n2 = int(min(a.batch, max(n, n * a.cpu_seconds / max(dt, 1e-6))))
        t0 = time.perf_counter()
        ok, od, _ = O.exact_search(a.metric, xh, qh[:n2], a.k, threads=threads)
        dt = time.perf_counter() - t0
        gk = keys[:n2].cpu().numpy().view(np.uint64)
        agree = float(np.mean([len(set(gk[i]) & set(ok[i])) / a.k for i in range(n2)]))
        out["cpu_baseline"] = {"value": round(n2 / dt, 2), "unit": "queries/s", "cores": threads, "kind": "port",
                               "cpu": cpu_model(),
                               "sample": f"{n2} queries, exact scan of {a.rows} rows, SIMD f32, {threads} threads"}
        out["parity_sample_recall_vs_oracle"] = round(agree, 5)
    if rank == 0:
        print(json.dumps(out), flush=True)


def pmc_traffic(a, ef):
    """HBM bytes per search launch from the committed rocprofv3 PMC summary
    (profiles/search_pmc.json, written by tools/pmc_summary.py from separate
    --pmc FETCH_SIZE / WRITE_SIZE passes of this same workload, gfx950 x2
    FETCH_SIZE correction applied there), or None when it does not match."""
    p = os.path.join(ROOT, "profiles", "search_pmc.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None
    w = d.get("workload", {})
    if (w.get("n"), w.get("dim"), w.get("queries"), w.get("ef"), w.get("metric")) != (
            a.rows, a.dim, a.queries, ef, a.metric):
        return None
    return d.get("hbm_bytes_per_launch")


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """SCYLLA_USEARCH_BACKGROUND_THREADS (README.md:14-15), else this process's
    real CPU share: cgroup cpu.max quota, then affinity (os.cpu_count() reports
    the whole machine on the GPU box, not our share)."""
    env = int(os.environ.get("SCYLLA_USEARCH_BACKGROUND_THREADS", "0") or 0)
    if env > 0:
        return env
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        n = min(n, omp)
    return max(1, n)


def cpu_baseline(a, index, q_t, ef, x_t):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # the checker / CPU baseline only (never the product path)

    O.set_fast_metric(True)
    threads = host_cores()
    res = {"unit": "queries/s", "cores": threads, "kind": "port", "cpu": cpu_model()}
    # (1) search QPS: the same graph, exported from HBM, searched by the C restatement
    g = index.export()
    h = O.HnswOracle(a.dim, a.metric, a.M, a.efc, ef)
    h.import_graph(g)
    del g
    qh = q_t.cpu().numpy()
    n = 256
    t0 = time.perf_counter()
    h.search(qh[:n], a.k, ef, threads=threads)
    dt = time.perf_counter() - t0
    n2 = int(min(len(qh), max(n, n * a.cpu_seconds / max(dt, 1e-6))))
    t0 = time.perf_counter()
    h.search(qh[:n2], a.k, ef, threads=threads)
    dt = time.perf_counter() - t0
    res["value"] = round(n2 / dt, 1)
    res["qps"] = res["value"]
    del h
    # (2) build vectors/s: concurrent inserts into a fresh index, bounded sample
    xh = x_t[: 200_000].cpu().numpy()
    hb = O.HnswOracle(a.dim, a.metric, a.M, a.efc, ef)
    nb = 20_000
    t0 = time.perf_counter()
    hb.add(np.arange(nb), xh[:nb], threads=threads)
    dt = time.perf_counter() - t0
    nb2 = int(min(len(xh), max(nb, nb * (1 + a.cpu_seconds / max(dt, 1e-6)))))
    hb2 = O.HnswOracle(a.dim, a.metric, a.M, a.efc, ef)
    t0 = time.perf_counter()
    hb2.add(np.arange(nb2), xh[:nb2], threads=threads)
    dt = time.perf_counter() - t0
    res["build_vectors_per_s"] = round(nb2 / dt, 1)
    res["sample"] = (f"search: {n2} queries at ef={ef} over the GPU-built 1M-row graph exported to host; "
                     f"build: {nb2} inserts into a fresh index (efC={a.efc}, M={a.M}); "
                     f"{threads} threads, SIMD f32 metrics")
    return res


if __name__ == "__main__":
    main()
