"""Build time vs pure-performance build knobs (results must be bit-identical).

usage (GPU box): python tools/build_probe.py rows dim metric quant data CFG [CFG...]
CFG = comma list of ENV=value (e.g. VSG_BUILD_HASH_FACTOR=16,VSG_REVERSE_GRID=8192), or "-".
One JSON line per config: build seconds, kernel-counter breakdown, and a
checksum of the exported graph (must match across configs).
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))


def main():
    rows, dim, metric, quant, data = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    import torch
    import vsg
    from vsg import datagen as G

    bs, qs, ms = G.config_seeds(3 if data == "sift" else 2)
    x = vsg.datagen_device(data, rows, dim, bs, ms)
    keys = np.arange(rows, dtype=np.uint64)
    for cfg in sys.argv[6:]:
        env = {}
        if cfg != "-":
            env = dict(kv.split("=") for kv in cfg.split(","))
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        idx = vsg.Index(dim, metric, quant, 16, 128, 64, seed=1)
        torch.cuda.synchronize()
        t0 = time.time()
        idx.add_device(keys, x)
        torch.cuda.synchronize()
        bt = time.time() - t0
        st = idx.stats()
        ex = idx.export()
        import ctypes as C
        raw = (C.c_uint64 * 16)()
        vsg.lib().vsg_debug_counters(idx._h, raw)
        wall = {"insert_wave_us_avg": round(raw[10] / rows / 100, 1), "insert_wave_us_max": round(raw[11] / 100, 1),
                "reverse_wave_us_sum_ms": round(raw[12] / 1e5, 1), "reverse_wave_us_max": round(raw[13] / 100, 1),
                "batches": st["build_batches"]}
        if raw[14] or raw[15]:  # profiling build: insert-wave beam phases per vector
            wall.update({"insert_beam_adj_dist_us": round(raw[15] / rows / 100, 1),
                         "insert_beam_merge_us": round(raw[14] / rows / 100, 1)})
        h = hashlib.sha1(ex["adj0"].tobytes())
        h.update(ex["upper"].tobytes())
        print(json.dumps({"rows": rows, "dim": dim, "cfg": cfg, "build_s": round(bt, 3),
                          "vec_per_s": round(rows / bt), "graph_sha1": h.hexdigest()[:16],
                          "dist_per_vec": round(st["build_distances"] / rows, 1), **wall}), flush=True)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        del idx, ex


if __name__ == "__main__":
    main()
