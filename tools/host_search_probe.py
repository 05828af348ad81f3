"""Probe (round 5): where a host-buffer search's time goes (vsg_index_search with host
queries / outputs, the reference's search(&[f32], k) shape) at C2: Python wall, library
wall, and the device-timeline split (VSG_PROFILE_HOST_SEARCH=1: upload, kernels,
download), beside the device-resident search of the same batch.

  VSG_PROFILE_HOST_SEARCH=1 python tools/host_search_probe.py [rows] [queries] [ef] [steps]
One JSON line on stdout (per-call means, ms).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))


def main():
    import torch

    import vsg
    from vsg import datagen as G
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    nq = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000
    ef = int(sys.argv[3]) if len(sys.argv) > 3 else 36
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    bs, qs, ms = G.config_seeds(1)
    x = vsg.datagen_device("clustered", rows, 768, bs, ms)
    q = vsg.datagen_device("clustered", nq, 768, qs, ms)
    idx = vsg.Index(768, "cos", "f32", 16, 128, 64, seed=0x5EED)
    idx.reserve(rows)
    idx.add_device(np.arange(rows, dtype=np.uint64), x)
    qh = q.cpu().numpy()
    for _ in range(3):
        idx.search(qh, 10, ef)
        idx.search_device(q, 10, ef)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        idx.search_device(q, 10, ef)
    torch.cuda.synchronize()
    dev_ms = (time.perf_counter() - t0) * 1e3 / steps
    s0 = idx.stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        idx.search(qh, 10, ef)
    host_ms = (time.perf_counter() - t0) * 1e3 / steps
    s1 = idx.stats()

    def d(f):
        return round((s1[f] - s0[f]) * 1e-6 / steps, 3)
    print(json.dumps({"rows": rows, "queries": nq, "ef": ef, "device_search_ms": round(dev_ms, 3),
                      "host_search_python_ms": round(host_ms, 3), "library_wall_ms": d("host_search_ns"),
                      "h2d_ms": d("host_h2d_ns"), "kernels_ms": d("host_device_ns"), "d2h_ms": d("host_d2h_ns"),
                      "profiled": os.environ.get("VSG_PROFILE_HOST_SEARCH", "0")}), flush=True)


if __name__ == "__main__":
    main()
