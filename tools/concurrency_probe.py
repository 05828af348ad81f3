"""Probe (round 5): host-timeline of searches issued beside a large add
(tests/test_gpu_concurrency.py::test_search_during_a_large_add), with the add's
phase clock (VSG_DEBUG_TIMING=1, stderr) -- which phase a slow search waited on.

  python tools/concurrency_probe.py [n0] [n]
One JSON line on stdout: add wall, every search's (start, latency) in ms from the add's start.
"""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))


def main():
    import torch

    import vsg
    from vsg import datagen as G
    n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    dim, nq = 768, 64
    bs, qs, ms = G.config_seeds(1)
    xt = vsg.datagen_device("clustered", n, dim, bs, ms)
    q = G.clustered(nq, dim, qs, ms)
    idx = vsg.Index(dim, "cos", "f32", 16, 128, 64, seed=3)
    idx.reserve(n)
    idx.add_device(np.arange(n0, dtype=np.uint64), xt[:n0].contiguous())
    torch.cuda.synchronize()
    idx.search(q, 10, 64)
    rest = xt[n0:].contiguous()
    torch.cuda.synchronize()
    done = threading.Event()
    t = {}

    def writer():
        t["a0"] = time.perf_counter()
        idx.add_device(np.arange(n0, n, dtype=np.uint64), rest)
        t["a1"] = time.perf_counter()
        done.set()

    th = threading.Thread(target=writer)
    th.start()
    time.sleep(0.02)
    lat = []
    while not done.is_set():
        s0 = time.perf_counter()
        idx.search(q, 10, 64)
        lat.append((s0, time.perf_counter() - s0))
    th.join()
    a0 = t["a0"]
    print(json.dumps({"n0": n0, "n": n, "persist": os.environ.get("VSG_SEARCH_PERSIST", "1"),
                      "add_ms": round((t["a1"] - a0) * 1e3, 2),
                      "searches": [(round((s - a0) * 1e3, 2), round(d * 1e3, 3)) for s, d in lat[:40]],
                      "max_ms": round(max(d for _, d in lat) * 1e3, 3) if lat else None}), flush=True)


if __name__ == "__main__":
    main()
