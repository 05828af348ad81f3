#!/usr/bin/env python3
"""bench.py — kNN QPS @ recall@10 >= 0.95 (+ build vectors/s) on synthetic 1M x 768 f32 cosine.

Workload = BASELINE.json configs[1]: 1M x 768 f32, cosine, HNSW M=16, efC=128,
k=10, clustered-latent synthetic data generated in HBM (vsg/datagen.py formulas).
One step = one HNSW search pass of the query batch (10,000 queries, inputs
resident in HBM) at the smallest ef whose recall@10 against exact ground truth is
>= 0.95 (ef swept on a 1,000-query subset).

N > 1 (--multi all, default) measures up to three layouts in one run:
  * shard: rank r owns rows [r N/G, (r+1) N/G) of the 1M index, every query is
    searched on every shard, the per-shard top-k' is all-gathered over RCCL (xGMI)
    and k-way merged by the HIP merge kernel; (ef, k') re-tuned for merged recall
    >= 0.95; total work fixed => "strong".  The build is sharded too.
  * replica: every rank holds the whole 1M index (3 GB of 288 GB HBM) and serves
    its own 10,000-query batch per step (weak).
  * hybrid (N >= 4, --shards-per-group S=2): N/S groups of S row shards, each
    group serving its own batch, all-gather inside the group only (weak).
`value` is the hybrid leg when it ran (N = 4, 8), else the shard leg (N = 2); the
others are reported beside it.  DESIGN.md §6 explains the trade-off (replicas
maximise QPS when the index fits one GPU, shards win the build and the recall-ef).
With --abi-leg 1 rank 0 also times the one-process sharded C ABI (vsg_sharded_*).

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
    ap.add_argument("--gt-queries", type=int, default=10_000,
                    help="recall@k is measured on this many queries (the first of the batch)")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--efc", type=int, default=128)
    ap.add_argument("--ef", type=int, default=0, help="fixed ef (0 = sweep for recall >= target)")
    ap.add_argument("--target-recall", type=float, default=0.95)
    ap.add_argument("--config-ef", type=int, default=128,
                    help="also time the config's nominal efSearch (BASELINE configs[1]: 128); 0 = skip")
    ap.add_argument("--config", type=int, default=1, help="seed set (BASELINE.json configs index)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU search-baseline sample")
    ap.add_argument("--cpu-build-rows", type=int, default=0,
                    help="rows of the CPU build baseline (0 = all --rows: BASELINE.md's build vectors/s is "
                         "N over the wall-clock insert time of the whole index)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--warm-build", type=int, default=1,
                    help="small throwaway build before the timed one (0: none -- PMC passes count one build)")
    ap.add_argument("--upper-ef", type=int, default=8,
                    help="N=1: also time the opt-in multi-entry descent at this level-1 beam width (0 = off)")
    ap.add_argument("--rerank-leg", type=int, default=1,
                    help="N=1 f32 storage: also time the opt-in f16 traversal + f32 re-rank mode")
    ap.add_argument("--mode", default="hnsw", choices=("hnsw", "exact"),
                    help="exact: brute-force MFMA path (C5: --rows 1000000 --dim 1536 --metric ip)")
    ap.add_argument("--batch", type=int, default=1024, help="exact mode: queries per step")
    ap.add_argument("--quant", default="f32", choices=("f32", "f16"), help="HBM storage type")
    ap.add_argument("--data", default="clustered", choices=("clustered", "sift", "gaussian"),
                    help="synthetic generator (sift: clustered, ReLU, x48, rounded 0..255; C4)")
    ap.add_argument("--sort-queries", default="none", choices=("none", "cluster"),
                    help="experiment: order the query batch by synthetic cluster id")
    ap.add_argument("--sort-base", default="none", choices=("none", "cluster"),
                    help="experiment: insert base rows in synthetic-cluster order (spatial slot ids)")
    ap.add_argument("--multi", default="all", choices=("all", "both", "shard", "replica", "hybrid"),
                    help="N>1 legs: shard = row-range shards over all N GPUs + all-gather merge (strong); "
                         "replica = full replicas, query split (weak); hybrid = S-GPU row-shard groups x "
                         "N/S replica groups, each group serving its own batch (weak in groups); "
                         "all = every leg, the hybrid one as value; both = shard (value) + replica")
    ap.add_argument("--shards-per-group", type=int, default=2,
                    help="hybrid leg: GPUs (row shards) per replica group")
    ap.add_argument("--streams-leg", type=int, default=2,
                    help="N=1: also time the K steps round-robin over this many streams (0/1: off)")
    ap.add_argument("--abi-leg", type=int, default=1,
                    help="N>1: also time the drop-in's own multi-GPU path -- one vsg_sharded_t over all N "
                         "devices in rank 0's process (include/vsg.h vsg_sharded_*), peer-DMA gather + HIP merge")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearse several ranks on one GPU (collectives via host)")
    ap.add_argument("--actor-leg", type=int, default=1,
                    help="N=1: closed-loop single-query anns through the actor (tools/actor_load child "
                         "process) at 512 and 2,048 clients on the headline index and ef")
    ap.add_argument("--host-abi-leg", type=int, default=1,
                    help="N=1: also time the drop-in's host-buffer ABI -- build via vsg_index_add from host f32 "
                         "rows, QPS via vsg_index_search from host queries (PCIe included) -- beside `value`")
    return ap.parse_args()


class Ctx:
    """Per-process run context (rank, device, collectives)."""

    def __init__(self, a):
        import torch
        import torch.distributed as dist

        self.a = a
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        self.local = local % max(1, torch.cuda.device_count())  # >1 rank per GPU only for gloo rehearsal
        torch.cuda.set_device(self.local)
        self.dev = torch.device("cuda", self.local)
        if self.world > 1:
            if a.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group(a.dist_backend)
        self.stream = torch.cuda.current_stream()
        self._groups = {}

    def group_of(self, S):
        """Process group of this rank's row-shard group (ranks [g S, (g+1) S));
        every rank creates every group, in the same order."""
        if S not in self._groups:
            self._groups[S] = [self.dist.new_group(list(range(g * S, (g + 1) * S))) for g in range(self.world // S)]
        return self._groups[S][self.rank // S]

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def rank_devices(self) -> dict:
        """Which device every rank ran on: each rank's ordinal,
        PCI address and uuid, all-gathered; the communicator's size, and under RCCL an
        all-reduce of ones over it (the number of ranks the collective really joined).
        A duplicated or missing device under RCCL fails the run before any value is
        printed; the gloo rehearsal on one GPU is flagged as such."""
        torch, dist = self.torch, self.dist
        p = torch.cuda.get_device_properties(self.dev)
        me = {"rank": self.rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": self.local,
              "pci_bus": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
              "uuid": str(getattr(p, "uuid", "")), "name": p.name}
        if self.world == 1:
            return {"ranks": [me], "distinct_devices": 1, "comm_world": 1, "rccl_world": None, "backend": None}
        ranks = [None] * self.world
        dist.all_gather_object(ranks, me)
        backend = str(dist.get_backend())
        comm = dist.get_world_size()
        rccl = None
        if backend == "nccl":
            t = torch.ones(1, device=self.dev)
            dist.all_reduce(t)
            rccl = int(t.item())
        distinct = len({(r["pci_bus"], r["uuid"]) for r in ranks})
        out = {"ranks": ranks, "distinct_devices": distinct, "comm_world": comm, "rccl_world": rccl,
               "backend": backend}
        if comm != self.world or [r["rank"] for r in ranks] != list(range(self.world)):
            raise SystemExit(f"bench.py: communicator of {comm} ranks for WORLD_SIZE={self.world}: {ranks}")
        if backend == "nccl" and (distinct != self.world or rccl != self.world):
            raise SystemExit(f"bench.py: {self.world} ranks but {distinct} distinct devices / RCCL all-reduce "
                             f"over {rccl}: {ranks}")
        if backend != "nccl":
            out["rehearsal"] = f"{backend} collectives, {distinct} device(s) for {self.world} ranks"
        return out

    def max_over_ranks(self, x: float) -> float:
        if self.world == 1:
            return x
        dev = self.dev if self.a.dist_backend == "nccl" else "cpu"
        t = self.torch.tensor([x], dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


def hnsw_leg(c, mode):
    """One HNSW measurement.  mode: "single" (N=1), "shard" (row-range shards,
    every query on every shard, RCCL all-gather + HIP merge; strong scaling) or
    "replica" (every rank holds the whole index and serves its own query batch;
    weak scaling).  Returns the measured fields and the index."""
    import numpy as np
    import torch

    import vsg
    from vsg import datagen as G
    from vsg.distributed import gather_topk, merge_topk

    a, world, rank = c.a, c.world, c.rank
    # shard topology: (position in the row-shard group, its size, its process group)
    # and the replica group this rank belongs to (each group serves its own batch)
    if mode == "shard":
        srank, sworld, pg, grp, ngrp = rank, world, None, 0, 1
    elif mode == "hybrid":
        S = max(1, min(a.shards_per_group, world))
        if world % S:
            raise SystemExit(f"bench.py: --shards-per-group {S} does not divide {world} ranks")
        pg = c.group_of(S)
        srank, sworld, grp, ngrp = rank % S, S, rank // S, world // S
    elif mode == "replica":
        srank, sworld, pg, grp, ngrp = 0, 1, None, rank, world
    else:
        srank, sworld, pg, grp, ngrp = 0, 1, None, 0, 1
    sharded = sworld > 1
    replica = ngrp > 1
    bs, qs, ms = G.config_seeds(a.config)
    lo, hi = (srank * a.rows // sworld, (srank + 1) * a.rows // sworld) if sharded else (0, a.rows)
    nloc = hi - lo

    # inputs in HBM
    x = vsg.datagen_device(a.data, nloc, a.dim, bs, ms, start=lo)
    q = vsg.datagen_device(a.data, a.queries, a.dim, qs, ms, start=grp * a.queries)
    qgt = vsg.datagen_device(a.data, a.gt_queries, a.dim, qs, ms, start=0)  # same on every rank
    if a.sort_queries == "cluster":
        cl = (G.splitmix64(G._stream(qs, G.TAG_CLUSTER) + np.arange(a.queries, dtype=np.uint64))
              % np.uint64(G.N_CENTRES)).astype(np.int64)
        q = q[torch.from_numpy(np.argsort(cl, kind="stable")).to(c.dev)].contiguous()
    keys_np = np.arange(lo, hi, dtype=np.uint64)
    if a.sort_base == "cluster":
        cl = (G.splitmix64(G._stream(bs, G.TAG_CLUSTER) + keys_np) % np.uint64(G.N_CENTRES)).astype(np.int64)
        order = np.argsort(cl, kind="stable")
        x = x[torch.from_numpy(order).to(c.dev)].contiguous()
        keys_np = keys_np[order]
    torch.cuda.synchronize()

    per16 = 4 if a.quant == "f32" else 8
    row_bytes = ((a.dim + per16 - 1) // per16) * 16

    # warm-up: a small throwaway build of the same row shape loads the build kernels'
    # code objects and warms the runtime's allocator, as a serving process has
    # done before its first large add (round 2 timed these one-time costs inside
    # the build: ~0.05 s of a 0.6 s build)
    if a.warm_build:
        warm = vsg.Index(a.dim, a.metric, a.quant, a.M, a.efc, 128, device=c.local, seed=1)
        nw = min(nloc, 32768)
        warm.add_device(keys_np[:nw], x[:nw].contiguous(), stream=c.stream)
        torch.cuda.synchronize()
        del warm

    # build (timed; not part of the QPS step)
    seed = 0x5EED + (srank if sharded else 0)
    index = vsg.Index(a.dim, a.metric, a.quant, a.M, a.efc, 128, device=c.local, seed=seed)
    index.reserve(nloc)
    c.barrier()
    t0 = time.perf_counter()
    index.add_device(keys_np, x, stream=c.stream)
    torch.cuda.synchronize()
    build_s = c.max_over_ranks(time.perf_counter() - t0)
    rows_built = a.rows  # sharded: S shards of rows/S concurrently (every group builds the whole index)
    bstats = index.stats()

    def search(qt, ef, ks, exact=False):
        keys, dists = index.search_device(qt, ks, ef, stream=c.stream, exact=exact)
        if not sharded:
            return keys, dists
        gk, gd = gather_topk(keys, dists, pg)
        return merge_topk(gk, gd, a.k, stream=c.stream)

    # ground truth: exact GPU brute force (f32 MFMA), same merge path
    gt = search(qgt, 0, a.k, exact=True)[0].cpu().numpy()

    def recall_of(keys_t):
        # |found & truth| / k per query (truth keys are distinct), averaged
        f = keys_t.cpu().numpy()
        return float((f[:, :, None] == gt[:, None, :]).any(axis=1).sum(axis=1).mean() / a.k)

    # (ef, k_shard): smallest ef whose merged recall@k >= target.  A shard returns
    # k_shard = min(k, ef) candidates (shards x k_shard >= k); one index returns k.
    def kshard(ef):
        return min(a.k, ef) if sharded else a.k

    def sweep_ef(fixed):
        sweep = []
        if fixed:
            sweep.append((fixed, recall_of(search(qgt, fixed, kshard(fixed))[0])))
            return fixed, sweep
        grid = (4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512, 768, 1024)
        if not sharded:
            grid = tuple(e for e in grid if e >= max(16, a.k))
        ef, lo_fail = None, None
        for cand in grid:
            if sharded and cand * sworld < a.k:
                continue
            r = recall_of(search(qgt, cand, kshard(cand))[0])
            sweep.append((cand, r))
            if r >= a.target_recall:
                ef = cand
                break
            lo_fail = cand
        if ef is None:
            ef = sweep[-1][0]
        elif lo_fail is not None:
            e_lo, e_hi = lo_fail, ef
            while e_hi - e_lo > 1:
                mid = (e_lo + e_hi) // 2
                r = recall_of(search(qgt, mid, kshard(mid))[0])
                sweep.append((mid, r))
                if r >= a.target_recall:
                    e_hi = mid
                else:
                    e_lo = mid
            ef = e_hi
        return ef, sweep

    ef, sweep = sweep_ef(a.ef)
    recall = dict(sweep)[ef]
    ks = kshard(ef)

    # timed QPS steps: W warmup, then exactly K steps between barriers
    for _ in range(a.warmup):
        search(q, ef, ks)
    index.reset_stats()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    # Steps are enqueued back to back (no host round trip between them); the
    # shard leg alternates two streams so one step's all-gather + merge (latency-
    # bound) runs under the next step's search, while the searches
    # themselves stay one after another (each waits for the previous one's end
    # event), so the HIP events time one launch each.  Every step's search,
    # gather and merge run inside the timed region; barrier + synchronize on both
    # sides.
    streams = [c.stream, torch.cuda.Stream(device=c.dev)] if sharded else [c.stream]
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    c.barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        s = streams[i % len(streams)]
        with torch.cuda.stream(s):
            if i and s is not streams[(i - 1) % len(streams)]:
                s.wait_event(evs[i - 1][1])
            evs[i][0].record(s)
            keys, dists = index.search_device(q, ks, ef, stream=s)
            evs[i][1].record(s)
            if sharded:
                gk, gd = gather_topk(keys, dists, pg)
                keys, dists = merge_topk(gk, gd, a.k, stream=s)
    c.barrier()
    elapsed = c.max_over_ranks(time.perf_counter() - t0)
    kern_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs)
    queries_done = ngrp * a.queries * a.steps
    st = index.stats()
    alg_bytes = (st["search_distances"] * row_bytes + st["search_adjacency"] * 2 * a.M * 4) / a.steps
    kern_ms_avg = kern_ms / a.steps

    # the same K steps spread over --streams-leg streams (beside the headline, never
    # `value`): a step may start while the previous one's last partial round of
    # resident waves drains, as concurrent clients of one index would run them
    # (each search takes its own scratch set, csrc/vsg_index.cpp ws_acquire)
    conc = None
    if a.streams_leg > 1 and not sharded and world == 1:
        ss = [c.stream] + [torch.cuda.Stream(device=c.dev) for _ in range(a.streams_leg - 1)]
        outs = [(torch.empty((a.queries, ks), dtype=torch.int64, device=c.dev),
                 torch.empty((a.queries, ks), dtype=torch.float32, device=c.dev)) for _ in ss]
        for j, sj in enumerate(ss):  # warm-up: one scratch set per stream
            sj.wait_stream(c.stream)
            index.search_device(q, ks, ef, out_keys=outs[j][0], out_dist=outs[j][1], stream=sj)
        c.barrier()
        t0 = time.perf_counter()
        for i in range(a.steps):
            j = i % len(ss)
            index.search_device(q, ks, ef, out_keys=outs[j][0], out_dist=outs[j][1], stream=ss[j])
        c.barrier()
        el_c = c.max_over_ranks(time.perf_counter() - t0)
        same = all(torch.equal(o[0], keys) and torch.equal(o[1], dists) for o in outs)
        conc = {"streams": len(ss), "qps": round(queries_done / el_c, 1), "ms_per_step": round(1000.0 * el_c / a.steps, 3),
                "results_equal_single_stream": bool(same),
                "note": "same K steps and ef, round-robin over the streams: a step's search may start while the "
                        "previous one drains its last partial round of waves (serving with concurrent clients)"}
    # the config's nominal efSearch, timed the same way (reported beside the headline)
    at_cfg = None
    if a.config_ef and a.config_ef != ef:
        e2 = a.config_ef
        r2 = recall_of(search(qgt, e2, kshard(e2))[0])
        for _ in range(max(1, a.warmup)):
            search(q, e2, kshard(e2))
        c.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            search(q, e2, kshard(e2))
            torch.cuda.synchronize()
        c.barrier()
        el2 = c.max_over_ranks(time.perf_counter() - t0)
        at_cfg = {"ef": e2, "k_shard": kshard(e2), "qps": round(queries_done / el2, 1),
                  "ms_per_step": round(1000.0 * el2 / a.steps, 3), "recall_at_10": round(r2, 4)}
    # opt-in f16 traversal + exact f32 re-rank on the same graph (csrc/rerank.hip):
    # reported beside the headline, never as `value` (the walk reads f16 rows)
    rerank = None
    if a.rerank_leg and not sharded and a.quant == "f32" and world == 1:
        index.set_f16_traversal(True)
        search(qgt[:1], 16, a.k)  # builds the f16 copy (untimed, once per index state)
        ef_r, sw_r = sweep_ef(0)
        for _ in range(max(1, a.warmup)):
            search(q, ef_r, a.k)
        index.reset_stats()
        km = 0.0
        c.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ev0.record(c.stream)
            index.search_device(q, a.k, ef_r, stream=c.stream)
            ev1.record(c.stream)
            torch.cuda.synchronize()
            km += ev0.elapsed_time(ev1)
        c.barrier()
        el_r = c.max_over_ranks(time.perf_counter() - t0)
        st_r = index.stats()
        rb16 = ((a.dim + 7) // 8) * 16
        ab_r = (st_r["search_distances"] * rb16 + st_r["search_adjacency"] * 2 * a.M * 4) / a.steps \
            + a.queries * ef_r * row_bytes  # re-rank reads the beam's f32 rows
        index.set_f16_traversal(False)
        rerank = {"qps": round(queries_done / el_r, 1), "ms_per_step": round(1000.0 * el_r / a.steps, 3),
                  "ef": ef_r, "recall_at_10": round(dict(sw_r)[ef_r], 4), "ef_sweep": sw_r,
                  "kernels_ms": round(km / a.steps, 3),
                  "alg_bytes_per_step": int(ab_r),
                  "achieved_gbs": round(ab_r / (km / a.steps * 1e-3) / 1e9, 1),
                  "dist_evals_per_query": round(st_r["search_distances"] / max(1, st_r["search_queries"]), 1),
                  "note": "opt-in mode (no usearch equivalent): HNSW walk over an f16 copy of the rows, "
                          "ef-beam re-ranked with exact f32 distances; same graph as the headline"}
    # opt-in multi-entry descent (level-1 beam of width upper_ef seeds level 0):
    # same graph, f32 walk, then also with the f16 walk + re-rank; beside the headline
    multi = None
    if a.upper_ef > 1 and not sharded and world == 1:
        multi = {"upper_ef": a.upper_ef,
                 "note": "opt-in mode (not usearch's greedy descent): level-1 beam seeds the level-0 beam"}
        index.set_upper_ef(a.upper_ef)
        for tag, f16 in (("f32_walk", False), ("f16_walk_f32_rerank", True)):
            if f16 and a.quant != "f32":
                continue
            index.set_f16_traversal(f16)
            ef_m, sw_m = sweep_ef(0)
            for _ in range(max(1, a.warmup)):
                search(q, ef_m, a.k)
            c.barrier()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                search(q, ef_m, a.k)
                torch.cuda.synchronize()
            c.barrier()
            el_m = c.max_over_ranks(time.perf_counter() - t0)
            multi[tag] = {"qps": round(queries_done / el_m, 1), "ms_per_step": round(1000.0 * el_m / a.steps, 3),
                          "ef": ef_m, "recall_at_10": round(dict(sw_m)[ef_m], 4)}
        index.set_f16_traversal(False)
        index.set_upper_ef(0)
    return {
        "concurrent": conc,
        "multi_entry": multi,
        "f16_rerank": rerank,
        "mode": mode, "index": index, "q": q, "x": x, "nloc": nloc, "shards": sworld, "groups": ngrp,
        "qps": queries_done / elapsed, "ms_per_step": 1000.0 * elapsed / a.steps,
        "ef": ef, "k_shard": ks, "recall": recall, "sweep": sweep,
        "build_s": build_s, "build_vps": rows_built / build_s,
        "kern_ms": kern_ms_avg, "alg_bytes": alg_bytes,
        "achieved_gbs": alg_bytes / (kern_ms_avg * 1e-3) / 1e9,
        "dist_per_query": st["search_distances"] / max(1, st["search_queries"]),
        "build_dist_per_vector": bstats["build_distances"] / max(1, nloc),
        # algorithmic bytes of the whole build: every distance evaluation reads one
        # row, every adjacency visit one 2M-entry level-0 row (upper rows are shorter)
        "bstats": bstats, "row_bytes": row_bytes, "gt": gt,
        "build_batches": bstats["build_batches"],
        "at_config_ef": at_cfg,
    }


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_workers(a):
    """`--gpus N` with no launcher around us: start N ranks (one per GPU) under
    torch.distributed.run as a CHILD process -- never an exec: nothing here has
    touched the GPU yet, and the parent only waits -- and return its exit code.
    Under a launcher (WORLD_SIZE set) the world size must equal --gpus, so a
    run asked for N GPUs can never silently measure one."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != a.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {a.gpus}")
        return None
    if a.gpus <= 1:
        return None
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    a = parse()
    rc = launch_workers(a)
    if rc is not None:
        sys.exit(rc)
    c = Ctx(a)
    world, rank = c.world, c.rank
    devices = c.rank_devices()  # before any measurement: a wrong layout never prints a value
    if a.mode == "exact":
        import vsg
        from vsg import datagen as G
        bs, qs, ms = G.config_seeds(a.config)
        lo, hi = rank * a.rows // world, (rank + 1) * a.rows // world
        x = vsg.datagen_device("clustered", hi - lo, a.dim, bs, ms, start=lo)
        q = vsg.datagen_device("clustered", a.batch, a.dim, qs, ms)
        run_exact(a, x, q, lo, hi, world, rank, c.local, c.dev, c.stream, c.barrier, c.max_over_ranks, devices)
        if world > 1:
            c.dist.destroy_process_group()
        return

    S = max(1, min(a.shards_per_group, world))
    hybrid_ok = world > 1 and 1 < S < world and world % S == 0
    if world == 1:
        legs = ["single"]
    elif a.multi == "all":
        legs = ["replica", "shard"] + (["hybrid"] if hybrid_ok else [])
    elif a.multi == "both":
        legs = ["replica", "shard"]
    else:
        legs = [a.multi]
    res = {}
    for m in legs:
        if res:  # free the previous leg's HBM before the next build
            res[list(res)[-1]].pop("index", None)
        res[m] = hnsw_leg(c, m)
    # headline: the hybrid layout (row-shard groups of S GPUs, one replica group per S
    # GPUs) when it was run, else the pure row-shard leg, else the only leg
    head = res.get("hybrid") or res.get("shard") or res[legs[0]]
    replica = head["groups"] > 1
    parallelism = {"single": "1 GPU",
                   "shard": f"row-shard x{world} + RCCL all-gather top-k + HIP merge",
                   "replica": f"replica x{world}, query split ({a.queries} queries/GPU/step)",
                   "hybrid": f"row-shard x{head['shards']} per group x {head['groups']} replica groups "
                             f"(RCCL all-gather top-k within a group + HIP merge; {a.queries} queries/group/step)"}
    out = {
        "metric": f"kNN QPS @ recall@10>={a.target_recall} (HNSW, {a.rows} x {a.dim} {a.quant} {a.metric})",
        "value": round(head["qps"], 1),
        "unit": "queries/s",
        "n_gpus": world,
        "devices": devices,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(head["ms_per_step"], 3),
        "higher_is_better": True,
        # N=1 is the first point of the row-shard series the default N>1 run reports
        "scaling": "weak" if (replica or (world == 1 and a.multi == "replica")) else "strong",
        "layout": {"shards_per_group": head["shards"], "groups": head["groups"]},
        "vs_baseline": None,
        "dtype": a.quant,
        "data": f"synthetic clustered-latent embeddings generated in HBM (vsg/datagen.py), "
                f"{a.queries} queries/step" + ("/group" if replica else ""),
        "config": {"workload": f"C{a.config + 1}: {a.rows} x {a.dim} {a.data} f32 input, {a.quant} storage, "
                               f"{a.metric} HNSW M={a.M} efC={a.efc} k={a.k}",
                   "index_rows": a.rows, "dim": a.dim, "queries_per_step": a.queries * head["groups"],
                   "ef": head["ef"], "k_shard": head["k_shard"], "recall_at_10": round(head["recall"], 4),
                   "ef_sweep": head["sweep"],
                   "parallelism": parallelism[head["mode"]]},
        "build_vectors_per_s": round(head["build_vps"], 1),
        "build_seconds": round(head["build_s"], 3),
        "roofline": {"bound": "hbm", "achieved": round(head["achieved_gbs"], 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(head["achieved_gbs"] / HBM_PEAK_GBS, 4),
                     "traffic": pmc_traffic(a, head["ef"]) if head["mode"] != "shard" else None,
                     "traffic_frac": (round(pmc_traffic(a, head["ef"]) / (head["kern_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                      if head["mode"] != "shard" and pmc_traffic(a, head["ef"]) else None),
                     "kernel": "hnsw_search_reg_kernel", "kernel_ms": round(head["kern_ms"], 3),
                     "alg_bytes_per_launch": int(head["alg_bytes"]),
                     "dist_evals_per_query": round(head["dist_per_query"], 1)},
        "build_stats": {"distance_evals_per_vector": round(head["build_dist_per_vector"], 1),
                        "batches": head["build_batches"]},
        "build_roofline": build_roofline(a, head),
        "at_config_ef": head["at_config_ef"],
        "f16_traversal_rerank": head.get("f16_rerank"),
        "multi_entry": head.get("multi_entry"),
        "concurrent_streams": head.get("concurrent"),
    }
    notes = {"replica": "every rank holds the whole index and serves its own query batch",
             "shard": "every query searched on all N row shards, all-gather + merge (the north star's layout)",
             "hybrid": "row-shard groups of S GPUs, each group serving its own query batch"}
    for m, s in res.items():
        if s is head:
            continue
        out[f"{m}_mode"] = {"qps": round(s["qps"], 1), "ms_per_step": round(s["ms_per_step"], 3),
                            "ef": s["ef"], "k_shard": s["k_shard"], "recall_at_10": round(s["recall"], 4),
                            "build_vectors_per_s": round(s["build_vps"], 1),
                            "build_seconds": round(s["build_s"], 3),
                            "kernel_ms": round(s["kern_ms"], 3),
                            "dist_evals_per_query": round(s["dist_per_query"], 1),
                            "queries_per_step": a.queries * s["groups"],
                            "shards_per_group": s["shards"], "groups": s["groups"],
                            "parallelism": parallelism[m],
                            "scaling": "weak" if s["groups"] > 1 else "strong",
                            "note": notes.get(m, ""),
                            "at_config_ef": s["at_config_ef"]}
    # the drop-in's own multi-GPU path (one vsg_sharded_t over all N devices in one
    # process, as the reference's single process would bind it): rank 0 runs it while
    # the other ranks wait at a barrier with their HBM freed
    if world > 1 and a.abi_leg:
        res[list(res)[-1]].pop("index", None)
        c.barrier()
        if rank == 0:
            # a failure here is reported in the line, never loses the measured legs
            try:
                out["sharded_abi"] = abi_leg(c)
            except Exception as e:  # noqa: BLE001
                out["sharded_abi"] = {"error": f"{type(e).__name__}: {e}"[:400]}
        c.barrier()
    # the host-buffer drop-in ABI at N=1 (vsg_index_add / vsg_index_search take host
    # memory, as usearch's add(key, &[f32]) and search(&[f32], k) do, usearch.rs:221, 276)
    if world == 1 and a.host_abi_leg and a.mode == "hnsw":
        out["host_abi"] = host_abi_leg(c, head)
    # the drop-in's serving path through the actor (single-query messages, N=1)
    if world == 1 and a.actor_leg and a.mode == "hnsw":
        out["actor_serving"] = actor_serving_leg(a, head["ef"])
    # CPU baseline (rank 0, N=1 only): oracle/ restatement of usearch
    if world == 1 and rank == 0 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(a, head["index"], head["q"], head["ef"], head["x"], head["gt"])
        out["config"]["cpu_build_sample_rows"] = out["cpu_baseline"]["build_sample_rows"]
        if out["cpu_baseline"].get("qps"):
            out["gpu_over_cpu_qps"] = round(head["qps"] / out["cpu_baseline"]["qps"], 1)
            out["gpu_over_cpu_build"] = round(head["build_vps"] / out["cpu_baseline"]["build_vectors_per_s"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        c.dist.destroy_process_group()


MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense


def run_exact(a, x, q, lo, hi, world, rank, local, dev, stream, barrier, max_over_ranks, devices=None):
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
    # batches below the MFMA tile threshold run the VALU kernel (vsg_index.cpp
    # VSG_EXACT_MFMA_MIN = 32): HBM-bound, the whole base read once per launch
    mfma = a.batch >= 32 and a.quant == "f32"
    hbm_bytes = nloc * a.dim * (4 if a.quant == "f32" else 2) + a.batch * a.dim * 4
    hbm_gbs = hbm_bytes / (kms * 1e-3) / 1e9
    out = {
        "metric": f"brute-force kNN QPS (exact, {'f32 MFMA' if mfma else 'VALU'}), {a.rows} x {a.dim} {a.quant} "
                  f"{a.metric}, batch {a.batch}",
        "value": round(qps, 1), "unit": "queries/s", "n_gpus": world, "devices": devices, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(1000 * elapsed / a.steps, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic clustered-latent embeddings generated in HBM (vsg/datagen.py)",
        "config": {"workload": f"C5: {a.rows} x {a.dim} f32 {a.metric} brute force, k={a.k}",
                   "batch": a.batch, "parallelism": f"row-shard x{world}"},
        "roofline": ({"bound": "mfma", "achieved": round(tflops, 2), "peak": MFMA_F32_PEAK_TFLOPS,
                      "unit": "TFLOP/s", "frac": round(tflops / MFMA_F32_PEAK_TFLOPS, 4), "traffic": None,
                      "kernel": "mfma_exact_kernel<16,MET> (+prepare, merge)", "kernel_ms": round(kms, 3),
                      "flops_per_launch": flops} if mfma else
                     {"bound": "hbm", "achieved": round(hbm_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(hbm_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                      "kernel": "exact_kernel (VALU, + prepare, merge)", "kernel_ms": round(kms, 3),
                      "alg_bytes_per_launch": hbm_bytes, "tflops": round(tflops, 3)}),
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


def abi_leg(c):
    """One `vsg_sharded_t` over the node's N devices (include/vsg.h vsg_sharded_*,
    csrc/vsg_sharded.cpp): keys routed by splitmix64(key) mod N, shards built
    concurrently (one host thread + stream each), every query searched on every
    shard, per-shard top-k copied to the answering device by peer DMA (xGMI) and
    merged there by the HIP merge kernel.  Same data, ef procedure and recall
    target as the other legs; timed with vsg_sharded_search_device."""
    import torch

    import vsg
    from vsg import datagen as G

    a, world = c.a, c.world
    ndev = max(1, torch.cuda.device_count())
    devices = [r % ndev for r in range(world)]  # 1 GPU (gloo rehearsal): every shard on device 0
    bs, qs, ms = G.config_seeds(a.config)
    idx = vsg.ShardedIndex(a.dim, a.metric, a.quant, a.M, a.efc, 128, devices=devices,
                           answer_device=c.local, seed=0x5EED)
    keys = np.arange(a.rows, dtype=np.uint64)
    CH = 250_000  # host staging in pieces (rows generated in HBM, copied out)
    xs = [vsg.datagen_device(a.data, min(CH, a.rows - s), a.dim, bs, ms, start=s).cpu().numpy()
          for s in range(0, a.rows, CH)]
    x = np.concatenate(xs)
    del xs
    idx.reserve(a.rows)
    t0 = time.perf_counter()
    idx.add(keys, x)
    build_s = time.perf_counter() - t0
    del x
    q = vsg.datagen_device(a.data, a.queries, a.dim, qs, ms, start=0)
    qgt = vsg.datagen_device(a.data, a.gt_queries, a.dim, qs, ms, start=0)
    torch.cuda.synchronize()
    gt = idx.search_device(qgt, a.k, exact=True, stream=c.stream)[0].cpu().numpy()

    def recall_at(ef):
        f = idx.search_device(qgt, a.k, ef, stream=c.stream)[0].cpu().numpy()
        return float((f[:, :, None] == gt[:, None, :]).any(axis=1).sum(axis=1).mean() / a.k)

    sweep, ef, lo_fail = [], None, None
    for cand in (10, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512):
        r = recall_at(cand)
        sweep.append((cand, r))
        if r >= a.target_recall:
            ef = cand
            break
        lo_fail = cand
    if ef is None:
        ef = sweep[-1][0]
    elif lo_fail is not None:
        e_lo, e_hi = lo_fail, ef
        while e_hi - e_lo > 1:
            mid = (e_lo + e_hi) // 2
            r = recall_at(mid)
            sweep.append((mid, r))
            e_lo, e_hi = (e_lo, mid) if r >= a.target_recall else (mid, e_hi)
        ef = e_hi
    for _ in range(max(1, a.warmup)):
        idx.search_device(q, a.k, ef, stream=c.stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        idx.search_device(q, a.k, ef, stream=c.stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = idx.stats()
    res = {"qps": round(a.queries * a.steps / el, 1), "ms_per_step": round(1000.0 * el / a.steps, 3),
           "ef": ef, "recall_at_10": round(dict(sweep)[ef], 4), "ef_sweep": sweep,
           "build_vectors_per_s": round(a.rows / build_s, 1), "build_seconds": round(build_s, 3),
           "build_device_s_max_shard": round((st["build_insert_ns"] + st["build_sort_ns"] +
                                              st["build_reverse_ns"]) * 1e-9, 4),
           "shards": world, "devices": devices, "answer_device": c.local,
           # hipDeviceCanAccessPeer of every (shard device -> answering device) gather
           # this leg used (the copies take the peer path where it is 1, else staged)
           "peer_access": [[d, c.local, bool(torch.cuda.can_device_access_peer(d, c.local))]
                           for d in sorted(set(devices)) if d != c.local],
           "shard_rows": [idx.shard(g).size() for g in range(world)],
           "note": "one process, vsg_sharded_* C ABI over all N devices: host-buffer add (PCIe included in "
                   "build_seconds), device-resident queries, peer-DMA gather + HIP merge"}
    idx.close()
    return res


def actor_serving_leg(a, ef, clients_list=(512, 2048), total=51200):
    """The drop-in's own serving path: the reference answers one Ann
    per message through a oneshot (/root/reference/src/index/usearch.rs:251-306), so
    closed-loop clients each keep one single-query vsg_actor_ann_cb in flight on an actor
    over the headline index (same rows, parameters and level seed, built in the child)
    at the headline ef; the actor coalesces them into batched GPU searches.  Runs
    tools/actor_load as a child process (no exec): QPS, latency p50 / p99 and whether
    every answer equals the batched search's."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "actor_load")
    if not os.path.exists(exe):
        return {"error": "tools/actor_load not built (__graft_entry__.build)"}
    out = {"note": "closed-loop clients of single-query vsg_actor_ann_cb (completion = the reference's "
                   "oneshot), one read worker beside the write FIFO (concurrent_reads = 1, the Rust drop-in's "
                   "setting, rust/src/index/gpu.rs); index rebuilt in the child with the headline rows/seed",
           "read_workers": 1,
           "ef": ef}
    for cl in clients_list:
        cmd = [exe, str(a.rows), str(a.dim), str({"l2sq": 0, "ip": 1, "cos": 2}[a.metric]), str(cl),
               str(max(1, total // cl)), str(a.k), str(ef), "0", "1", "1", str(0x5EED)]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or not line:
                out[f"clients_{cl}"] = {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
                continue
            j = json.loads(line[-1])
            out[f"clients_{cl}"] = {"qps": j["actor_qps"], "lat_us_p50": j["lat_us_p50"],
                                    "lat_us_p99": j["lat_us_p99"], "mean_batch": j["mean_batch"],
                                    "mismatch_vs_batched": j["mismatch_vs_batched"], "errors": j["errors"],
                                    "batched_qps_same_queries": j["batched_qps"]}
        except subprocess.TimeoutExpired:
            out[f"clients_{cl}"] = {"error": "timeout"}
    return out


def host_abi_leg(c, head):
    """N=1, beside `value`: the reference's own call shapes through the C ABI with host
    buffers (PCIe included).  Build: a fresh index filled by vsg_index_add from host f32
    rows (the rows `value`'s index was built from, copied out of HBM first, untimed).
    Search: vsg_index_search with host queries / host outputs over the headline index at
    the headline ef, K steps; results compared with the device-resident search."""
    import torch

    import vsg

    a = c.a
    xh = head["x"].cpu().numpy()
    qh = head["q"].cpu().numpy()
    idx = vsg.Index(a.dim, a.metric, a.quant, a.M, a.efc, 128, device=c.local, seed=0x5EED)
    idx.reserve(a.rows)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx.add(np.arange(a.rows, dtype=np.uint64), xh)
    build_s = time.perf_counter() - t0
    del xh
    ef, index = head["ef"], head["index"]
    ng = head["gt"].shape[0]
    rb = recall_np(idx.search(qh[:ng], a.k, ef).keys, head["gt"], a.k)
    idx.close()
    for _ in range(max(1, a.warmup)):
        m = index.search(qh, a.k, ef)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        m = index.search(qh, a.k, ef)
    el = time.perf_counter() - t0
    dk, dd = index.search_device(head["q"], a.k, ef)
    same = bool(np.array_equal(dk.cpu().numpy().view(np.uint64), m.keys) and np.array_equal(dd.cpu().numpy(), m.distances))
    return {"build_vectors_per_s": round(a.rows / build_s, 1), "build_seconds": round(build_s, 3),
            "build_recall_at_10": round(rb, 4),
            "qps": round(a.queries * a.steps / el, 1), "ms_per_step": round(1000.0 * el / a.steps, 3), "ef": ef,
            "over_device_value": round(a.queries * a.steps / el / head["qps"], 3),
            "pieces": int(os.environ.get("VSG_HOST_SEARCH_PIECES", "1")),
            "results_equal_device_search": same,
            "note": "vsg_index_add from host f32 rows (a fresh index of the same rows, PCIe included) and "
                    "vsg_index_search with host queries and outputs over the headline index (PCIe both ways; "
                    "queries staged through pinned memory by 8 host threads, 4-MiB DMA pieces): the reference's "
                    "add(key, &[f32]) / search(&[f32], k) call shapes, batched"}


def recall_np(found, gt, k):
    f = np.asarray(found).astype(np.int64)
    g = np.asarray(gt).astype(np.int64)
    n = min(len(f), len(g))
    return float((f[:n, :k, None] == g[:n, None, :k]).any(axis=1).sum(axis=1).mean() / k)


def kernel_src_sha() -> str:
    """sha256 over the library sources (vector-store-text_amd/csrc): a PMC summary
    is used only while the kernels it profiled are the ones in this tree."""
    import hashlib
    d = os.path.join(ROOT, "vector-store-text_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".hpp", ".cpp")):
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def build_roofline(a, head):
    """The build against the HBM roofline on DEVICE time (HIP events around every
    batch's launches on the build stream, vsg_stats_t.build_*_ns).  Dominant kernel:
    hnsw_insert_beam_kernel (descent + efC beam; build_insert_ns - build_select_ns),
    beside it hnsw_insert_select_kernel (heuristic neighbour selection) and
    hnsw_reverse_kernel (reverse links), each with its own line.

    `frac` = measured HBM bytes / device time / 8 TB/s: the PMC bytes of the kernel
    over the whole build (profiles/build_pmc.json -- FETCH_SIZE x2 + WRITE_SIZE,
    separate rocprofv3 --pmc passes of this workload) over the same kernel's device
    time; None when no PMC summary of this workload is committed.  It can not
    exceed 1.  The kernel-counted figure -- one row per distance evaluation, one
    adjacency row per expansion -- counts rows that co-resident waves share through
    L2 / MALL once per evaluation, so over the device time it is a cache-credited
    rate that can exceed the HBM peak (round 3 reported it as `frac`: 1.03 / 2.23 /
    1.37); it is kept as `alg_gbs_cache_credited` with `alg_over_traffic`."""
    st, rb = head["bstats"], head["row_bytes"]
    sel_ins = st["build_select_distances"]
    sel_rev = st["reverse_select_distances"] + st["reverse_recompute_distances"]
    beam = st["build_distances"] - sel_ins - sel_rev
    beam_bytes = beam * rb + st["build_adjacency"] * 2 * a.M * 4
    sel_bytes = sel_ins * rb
    rev_bytes = sel_rev * rb
    ns = {k: max(1, st[f"build_{k}_ns"]) * 1e-9 for k in ("insert", "sort", "reverse", "select")}
    t_beam = max(1e-9, ns["insert"] - (ns["select"] if st["build_select_ns"] else 0.0))
    pmc = {}
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "build_pmc.json")))
        w = d.get("workload", {})
        if (w.get("n"), w.get("dim"), w.get("metric"), w.get("M"), w.get("efc"), w.get("forward_links")) == (
                head["nloc"], a.dim, a.metric, a.M, a.efc, "M") and d.get("kernel_src_sha") == kernel_src_sha():
            pmc = d
    except (OSError, ValueError):
        pass

    def line(kernel, alg, t, traffic):
        g = alg / t / 1e9
        return {"kernel": kernel, "kernel_s": round(t, 4),
                "achieved": round(traffic / t / 1e9, 1) if traffic else None,
                "frac": round(traffic / t / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                "traffic": traffic, "alg_bytes": int(alg), "alg_gbs_cache_credited": round(g, 1),
                "alg_over_traffic": round(alg / traffic, 3) if traffic and alg else None}

    out = line("hnsw_insert_beam_kernel", beam_bytes, t_beam, pmc.get("beam_hbm_bytes"))
    out.update({"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "traffic_unit": "HBM bytes over all launches of the kernel in the build (PMC)",
                "kernel_s_all": {"beam": round(t_beam, 4), "select": round(ns["select"], 4),
                                 "sort": round(ns["sort"], 4), "reverse": round(ns["reverse"], 4)},
                "select": line("hnsw_insert_select_kernel", sel_bytes, ns["select"], pmc.get("select_hbm_bytes")),
                "reverse": line("hnsw_reverse_kernel", rev_bytes, ns["reverse"], pmc.get("reverse_hbm_bytes")),
                "wall_s": round(head["build_s"], 4),
                "beam_distance_evals_per_vector": round(beam / max(1, head["nloc"]), 1),
                "selection_distance_evals_per_vector": round(sel_ins / max(1, head["nloc"]), 1),
                "reverse_distance_evals_per_vector": round(sel_rev / max(1, head["nloc"]), 1),
                "reverse_prunes": st["reverse_prunes"], "reverse_appends": st["reverse_appends"]})
    return out


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
    # forward_links "M": a graph built with usearch's <= M forward links per level
    # (round 4); earlier summaries profiled the M0-forward graph
    if (w.get("n"), w.get("dim"), w.get("queries"), w.get("ef"), w.get("metric"), w.get("forward_links")) != (
            a.rows, a.dim, a.queries, ef, a.metric, "M"):
        return None
    # profiled kernels must be this tree's (the summary records the source hash it ran)
    if d.get("kernel_src_sha") != kernel_src_sha():
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


def cpu_baseline(a, index, q_t, ef, x_t, gt):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # the checker / CPU baseline only (never the product path)

    O.set_fast_metric(True)
    threads = host_cores()
    res = {"unit": "queries/s", "cores": threads, "kind": "port", "cpu": cpu_model(), "isa": O.fast_isa()}
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
    ck = h.search(qh[:n2], a.k, ef, threads=threads)[0]
    dt = time.perf_counter() - t0
    res["value"] = round(n2 / dt, 1)
    res["qps"] = res["value"]
    # the CPU's recall at the matched ef (the bench queries' first rows are the
    # ground-truth queries): equal to the GPU's up to near-ties on the same graph
    ng = min(n2, gt.shape[0])
    res["recall_at_10"] = round(float(np.mean([len(set(ck[i].astype(np.int64)) & set(gt[i])) / a.k for i in range(ng)])), 4)
    res["ef"] = ef
    del h
    # (2) build vectors/s: the whole index (N / wall-clock insert time;
    # the insert rate falls as the graph grows, so a prefix sample flatters it),
    # concurrent one-vector inserts into a fresh index as the reference's rayon adds
    nb = a.cpu_build_rows or a.rows
    xh = x_t[:nb].cpu().numpy()
    hb = O.HnswOracle(a.dim, a.metric, a.M, a.efc, ef)
    hb.reserve(nb)
    t0 = time.perf_counter()
    hb.add(np.arange(nb), xh, threads=threads)
    dt = time.perf_counter() - t0
    del hb, xh
    res["build_vectors_per_s"] = round(nb / dt, 1)
    res["build_seconds"] = round(dt, 2)
    res["build_sample_rows"] = nb
    res["sample"] = (f"search: {n2} queries at ef={ef} over the GPU-built {a.rows}-row graph exported to host "
                     f"(recall on the first {ng}); build: all {nb} rows inserted into a fresh index "
                     f"(efC={a.efc}, M={a.M}) in {dt:.1f} s; {threads} threads, {O.fast_isa()} f32 metrics")
    return res


if __name__ == "__main__":
    main()
