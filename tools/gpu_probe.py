#!/usr/bin/env python3
"""One parameterised GPU probe (replaces round 1's ~45 one-off gpu_*.sh scripts).

  search  build one index (optionally shard s of S row shards), then for every ef and
          every knob setting (--set KEY=V,KEY=V; VSG_* env knobs) time the device
          search of the query batch with HIP events on the launching stream and
          report kernel ms, QPS, distance evaluations / query, algorithmic GB/s
          (n_dist x row bytes + n_adj x M0 x 4 per launch, no cache credit), fraction
          of the 8 TB/s HBM roofline, recall@10 against exact ground truth, and
          whether keys/distances equal the first setting's (same traversal).
  build   build the index under every knob setting; report build seconds, batches,
          device time per build kernel and recall at --efs.

Runs unchanged under rocprofv3 (one program, no launcher hops), e.g.
  rocprofv3 --kernel-trace --stats -d gpurun_out/p -- python3 tools/gpu_probe.py search ...
  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/f -- python3 tools/gpu_probe.py search ...

C4 per-shard example (one of 8 row shards of 100M x 128 f16 sift-like):
  python3 tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 --dim 128 \
      --quant f16 --metric l2sq --data sift --config 3 --efs 64,128,192
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))

KNOBS = {"frac": "VSG_BUILD_BATCH_FRAC", "max": "VSG_BUILD_BATCH_MAX", "frac2": "VSG_BUILD_BATCH_FRAC2",
         "switch": "VSG_BUILD_BATCH_SWITCH", "reg": "VSG_SEARCH_REG", "waves": "VSG_SEARCH_WAVES",
         "hash": "VSG_SEARCH_HASH_FACTOR", "xcd": "VSG_SEARCH_XCD_MAP", "upper": "VSG_SEARCH_UPPER_EF",
         "loc": "VSG_BUILD_LOCALITY", "locmin": "VSG_BUILD_LOCALITY_MIN",
         "piv": "VSG_BUILD_LOCALITY_PIVOTS",
         "split": "VSG_BUILD_SPLIT", "bhash": "VSG_BUILD_HASH_FACTOR", "hmin": "VSG_SEARCH_HASH_MIN"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("search", "build"))
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--shards", type=int, default=1)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--metric", default="cos")
    ap.add_argument("--quant", default="f32")
    ap.add_argument("--data", default="clustered")
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--efc", type=int, default=128)
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--gt-queries", type=int, default=1000)
    ap.add_argument("--efs", default="36,128")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--sort-base", action="store_true",
                    help="build: rows inserted in synthetic-cluster order (slot ids spatial; probe of "
                         "VSG_BUILD_LOCALITY=2)")
    ap.add_argument("--streams", type=int, default=1,
                    help="search: also time the steps round-robin over this many streams (wall clock; "
                         "sustained algorithmic bytes / wall)")
    ap.add_argument("--seeds", default="0", help="index seeds (offsets from the default; search mode: the first)")
    ap.add_argument("--phases", action="store_true",
                    help="with VSG_LIB_PATH=lib_prof/libvsg.so (make prof): build mode, insert-wave "
                         "clock split into beam / heuristic selection; search mode, the register beam's "
                         "cycles per expansion (select, adjacency wait, visited, row wait, row VALU, "
                         "admission, compaction)")
    return ap.parse_args()


def apply(setting):
    env = dict(kv.split("=") for kv in setting.split(",") if kv)
    for k, v in env.items():
        os.environ[KNOBS.get(k, k)] = v
    return env


def clear(env):
    for k in env:
        os.environ.pop(KNOBS.get(k, k), None)


def build(a, x, seed=0):
    import torch
    import vsg
    lo = a.shard * a.rows // a.shards
    idx = vsg.Index(a.dim, a.metric, a.quant, a.M, a.efc, 64, seed=0x5EED + a.shard + seed)
    idx.reserve(x.shape[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx.add_device(np.arange(lo, lo + x.shape[0], dtype=np.uint64), x)
    torch.cuda.synchronize()
    return idx, time.perf_counter() - t0


def recall(f, gt, k):
    return round(float(np.mean([len(set(f[i]) & set(gt[i])) / k for i in range(gt.shape[0])])), 4)


def main():
    a = parse()
    import torch

    import vsg
    from vsg import datagen as G
    bs, qs, ms = G.config_seeds(a.config)
    lo, hi = a.shard * a.rows // a.shards, (a.shard + 1) * a.rows // a.shards
    x = vsg.datagen_device(a.data, hi - lo, a.dim, bs, ms, start=lo)
    if a.sort_base:
        cl = (G.splitmix64(G._stream(bs, G.TAG_CLUSTER) + np.arange(lo, hi, dtype=np.uint64))
              % np.uint64(G.N_CENTRES)).astype(np.int64)
        x = x[torch.from_numpy(np.argsort(cl, kind="stable")).to(x.device)].contiguous()
    q = vsg.datagen_device(a.data, a.queries, a.dim, qs, ms)
    qg = q[: a.gt_queries].contiguous()
    per16 = 4 if a.quant == "f32" else 8
    row_bytes = (a.dim + per16 - 1) // per16 * 16
    efs = [int(e) for e in a.efs.split(",")]
    stream = torch.cuda.current_stream()
    head = {"rows": hi - lo, "of_rows": a.rows, "dim": a.dim, "metric": a.metric, "quant": a.quant,
            "data": a.data, "queries": a.queries}
    if a.mode == "build":
        gt = None
        for st, seed in [(st, int(sd)) for st in a.set or [""] for sd in a.seeds.split(",")]:
            env = apply(st)
            idx, bt = build(a, x, seed)
            if gt is None:
                gt = idx.search_device(qg, a.k, exact=True)[0].cpu().numpy()
            s = idx.stats()
            out = dict(head, set=st, seed=seed, build_s=round(bt, 3), build_vps=round((hi - lo) / bt, 1),
                       batches=s["build_batches"],
                       kernel_s={k: round(s[f"build_{k}_ns"] * 1e-9, 4) for k in ("insert", "sort", "reverse")},
                       per_vector={k: round(s[k] / max(1, hi - lo), 2) for k in (
                           "build_distances", "build_select_distances", "reverse_recompute_distances",
                           "reverse_select_distances", "build_adjacency", "reverse_prunes", "reverse_appends")})
            if a.phases:
                import ctypes as C
                from vsg._lib import lib
                raw = (C.c_uint64 * 16)()
                lib().vsg_debug_counters(idx._h, raw)
                tot = max(1, raw[10])
                out["insert_wave_clock_share"] = {"beam": round(raw[15] / tot, 3), "select": round(raw[14] / tot, 3),
                                                  "other": round(1 - (raw[14] + raw[15]) / tot, 3)}
            for ef in efs:
                out[f"recall_ef{ef}"] = recall(idx.search_device(qg, a.k, ef)[0].cpu().numpy(), gt, a.k)
            print(json.dumps(out), flush=True)
            clear(env)
            del idx
        return
    idx, bt = build(a, x, int(a.seeds.split(",")[0]))
    del x
    gt = idx.search_device(qg, a.k, exact=True)[0].cpu().numpy()
    print(json.dumps(dict(head, build_s=round(bt, 3))), flush=True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for ef in efs:
        base = None
        for st in a.set or [""]:
            env = apply(st)
            kk, dd = idx.search_device(q, a.k, ef, stream=stream)
            torch.cuda.synchronize()
            kk, dd = kk.cpu().numpy(), dd.cpu().numpy()
            if base is None:
                base = (kk, dd)
            same = bool((kk == base[0]).all() and (dd == base[1]).all())
            idx.reset_stats()
            ms_k = 0.0
            for _ in range(a.steps):
                ev0.record(stream)
                idx.search_device(q, a.k, ef, stream=stream)
                ev1.record(stream)
                torch.cuda.synchronize()
                ms_k += ev0.elapsed_time(ev1)
            ms_k /= a.steps
            s = idx.stats()
            nq = max(1, s["search_queries"])
            alg = (s["search_distances"] * row_bytes + s["search_adjacency"] * 2 * a.M * 4) / a.steps
            gbs = alg / (ms_k * 1e-3) / 1e9
            phases = {}
            if a.phases:  # VSG_LIB_PATH=lib_prof/libvsg.so: per-expansion cycles of the register beam
                import ctypes as C
                from vsg._lib import lib
                raw = (C.c_uint64 * 32)()
                lib().vsg_debug_counters_n(idx._h, raw, C.c_size_t(32))
                nexp = max(1, raw[28] & ((1 << 40) - 1))
                names = ("select", "adj_wait", "visited", "row_wait", "row_valu", "admit", "compact")
                phases = {"expansions_per_query": round(nexp / nq, 1),
                          "compactions_per_query": round((raw[28] >> 40) / nq, 2),
                          "row_passes_per_expansion": round(raw[29] / nexp, 2),
                          "cycles_per_expansion": {k: round(raw[20 + i] / nexp, 1) for i, k in enumerate(names)},
                          "descent_cycles_per_query": round(raw[27] / nq, 1),
                          "query_cycles": round(raw[30] / nq, 1),
                          "query_us": round(raw[31] / nq / 100.0, 2),
                          "clock_ghz": round(raw[30] / max(1, raw[31]) / 10.0, 3)}
            multi = {}
            if a.streams > 1:
                ss = [torch.cuda.Stream() for _ in range(a.streams)]
                for sj in ss:  # one scratch set per stream
                    idx.search_device(q, a.k, ef, stream=sj)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(a.steps):
                    idx.search_device(q, a.k, ef, stream=ss[i % a.streams])
                torch.cuda.synchronize()
                wall = (time.perf_counter() - t0) / a.steps
                multi = {"streams": a.streams, "streams_ms_per_step": round(wall * 1e3, 3),
                         "streams_qps": round(a.queries / wall, 1),
                         "streams_sustained_frac": round(alg / wall / 1e9 / 8000.0, 4)}
            print(json.dumps(dict(head, **multi, **phases, ef=ef, set=st, kernel_ms=round(ms_k, 3),
                                  qps=round(a.queries / ms_k * 1e3, 1),
                                  dist_per_query=round(s["search_distances"] / nq, 1),
                                  adj_per_query=round(s["search_adjacency"] / nq, 1),
                                  alg_bytes_per_launch=int(alg), achieved_gbs=round(gbs, 1),
                                  hbm_frac=round(gbs / 8000.0, 4),
                                  recall_at_10=recall(kk[: a.gt_queries], gt, a.k), same_as_first=same)),
                  flush=True)
            clear(env)


if __name__ == "__main__":
    main()
