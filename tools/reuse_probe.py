"""Probe (round 5): recall of GPU vs oracle builds before and after remove/add churn
with free-slot reuse, on a small clustered cos index -- which part of a gap is the
batched build itself and which the re-linking of reused slots.

  python tools/reuse_probe.py [n] [dim] [rep_per_round] [rounds] [churn_batch_max] [oracle_threads]
churn_batch_max > 0: VSG_BUILD_BATCH_MAX for the churn adds only (1 = one-node batches,
the oracle's sequential semantics); oracle_threads: threads of the oracle's adds.
One JSON line per measurement on stdout.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
import vsg  # noqa: E402
from vsg import datagen as G  # noqa: E402


def rec(found, gt):
    return float(np.mean([len(set(found[i].tolist()) & set(gt[i].tolist())) / 10 for i in range(len(gt))]))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
    dim = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    rep = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    cbm = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    oth = int(sys.argv[6]) if len(sys.argv) > 6 else 16
    # start: "own" (each side builds), "oracle" (the GPU indexes import the oracle's graph),
    # "gpu" (the oracle imports the GPU's graph) -- separates update semantics from the
    # starting graph
    start = sys.argv[7] if len(sys.argv) > 7 else "own"
    x = G.clustered(n + rep * rounds, dim, 311, 9)
    q = G.clustered(2000, dim, 312, 9)
    gpu = vsg.Index(dim, "cos", "f32", 16, 128, 64, seed=4)
    app = vsg.Index(dim, "cos", "f32", 16, 128, 64, seed=4, slot_reuse=False)
    h = O.HnswOracle(dim, "cos", 16, 128, 64, seed=4)
    if start == "oracle":
        h.add(np.arange(n), x[:n], threads=oth)
        gpu.import_graph(h.export())
        app.import_graph(h.export())
    elif start == "gpu":
        gpu.add(np.arange(n), x[:n])
        app.import_graph(gpu.export())
        h.import_graph(gpu.export())
    else:
        gpu.add(np.arange(n), x[:n])
        app.add(np.arange(n), x[:n])
        h.add(np.arange(n), x[:n], threads=oth)
    cur = x[:n].copy()
    rng = np.random.default_rng(8)

    def report(tag):
        gt, _, _ = O.exact_search("cos", cur, q, 10, threads=16)
        for ef in (16, 32, 64):
            print(json.dumps({"tag": tag, "n": n, "ef": ef, "churn_batch_max": cbm, "oracle_threads": oth, "start": start, "gpu_reuse": rec(gpu.search(q, 10, ef).keys, gt),
                              "gpu_append": rec(app.search(q, 10, ef).keys, gt),
                              "oracle": rec(h.search(q, 10, ef, threads=16)[0], gt)}), flush=True)

    report("built")
    for rnd in range(rounds):
        keys = np.sort(rng.choice(n, rep, replace=False)).astype(np.uint64)
        new = x[n + rep * rnd:n + rep * (rnd + 1)]
        if cbm:
            os.environ["VSG_BUILD_BATCH_MAX"] = str(cbm)
        for ix in (gpu, app):
            ix.remove(keys)
            ix.add(keys, new)
        os.environ.pop("VSG_BUILD_BATCH_MAX", None)
        h.remove(keys)
        h.add(keys, new, threads=oth)
        cur[keys.astype(np.int64)] = new
        report(f"churn{rnd + 1}")


if __name__ == "__main__":
    main()
