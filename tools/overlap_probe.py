#!/usr/bin/env python3
"""Probe: how much of a 10k-query search step is the tail of its last partial round of
resident waves?  C2 index (1M x 768 cos); K steps timed (a) on one stream, (b) alternating
over 2 / 3 streams (step i+1 may start while step i drains), (c) one stream with 4x larger
batches.  Results of (b) checked equal to (a).  One JSON line per setting."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))
import vsg  # noqa: E402
from vsg import datagen as G  # noqa: E402

rows, dim, nq, ef, K = 1_000_000, 768, 10_000, int(os.environ.get("EF", "36")), 30
bs, qs, ms = G.config_seeds(1)
x = vsg.datagen_device("clustered", rows, dim, bs, ms)
q = vsg.datagen_device("clustered", 4 * nq, dim, qs, ms)
idx = vsg.Index(dim, "cos", "f32", 16, 128, 64, seed=1)
t = time.time()
idx.add_device(np.arange(rows, dtype=np.uint64), x)
torch.cuda.synchronize()
print(json.dumps({"build_s": round(time.time() - t, 3)}), flush=True)
qb = [q[i * nq:(i + 1) * nq].contiguous() for i in range(4)]


def run(nstreams, batch):
    ss = [torch.cuda.Stream() for _ in range(nstreams)]
    outs = []
    for s in ss:
        with torch.cuda.stream(s):
            outs.append((torch.empty((batch, 10), dtype=torch.int64, device="cuda"),
                         torch.empty((batch, 10), dtype=torch.float32, device="cuda")))
    src = [qb[i % 4] for i in range(4)] if batch == nq else [q]
    for w in range(3):  # warmup
        for i, s in enumerate(ss):
            idx.search_device(src[i % len(src)], 10, ef, out_keys=outs[i][0], out_dist=outs[i][1], stream=s.cuda_stream)
    torch.cuda.synchronize()
    steps = K if batch == nq else K // 4
    t0 = time.perf_counter()
    for i in range(steps):
        j = i % nstreams
        with torch.cuda.stream(ss[j]):
            idx.search_device(src[i % len(src)], 10, ef, out_keys=outs[j][0], out_dist=outs[j][1],
                              stream=ss[j].cuda_stream)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return steps * batch / dt, outs


for ns, batch in ((1, nq), (2, nq), (3, nq), (1, 4 * nq), (1, nq), (2, nq), (4, nq)):
    qps, _ = run(ns, batch)
    print(json.dumps({"streams": ns, "batch": batch, "ef": ef, "qps": round(qps, 1)}), flush=True)
# equality: the same batch on a side stream while another runs gives the same keys
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
ka, da = idx.search_device(qb[0], 10, ef)
torch.cuda.synchronize()
kb, db = idx.search_device(qb[0], 10, ef, stream=s1.cuda_stream)
kc, dc = idx.search_device(qb[1], 10, ef, stream=s2.cuda_stream)
torch.cuda.synchronize()
print(json.dumps({"overlap_results_equal": bool(torch.equal(ka, kb) and torch.equal(da, db))}), flush=True)
