"""Probe (round 5): self-recall under a whole-index replace stream (the actor upsert
test's workload: every key replaced each round, remove + add per segment of keys) --
GPU build settings against the oracle's sequential build run through the same calls.

  python tools/upsert_probe.py [nkeys] [dim] [rounds] [segment] [settings]
settings: ';'-separated, each a ','-separated list of KEY=VALUE env knobs ('base' = none)
One JSON line per (setting, round) on stdout: fraction of keys whose latest vector,
searched at k 1 / ef 64, finds itself.
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


def self_hit(search, mat):
    _, d = search(mat)
    return round(float(np.mean(d[:, 0] == 0.0)), 4)


def stream(nkeys, dim, rounds, seg):
    rng = np.random.default_rng(9)
    for rnd in range(rounds):
        vals = rng.integers(0, 32, (nkeys, dim)).astype(np.float32)
        yield rnd, [(np.arange(s, min(nkeys, s + seg), dtype=np.uint64), vals[s:s + seg]) for s in range(0, nkeys, seg)], vals


def main():
    nkeys = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    dim = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    seg = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    settings = sys.argv[5] if len(sys.argv) > 5 else "base"
    h = O.HnswOracle(dim, "l2sq", 16, 64, 64, seed=2)
    orc = []
    for rnd, segs, vals in stream(nkeys, dim, rounds, seg):
        for keys, v in segs:
            if rnd:
                h.remove(keys)
            h.add(keys, v, threads=1)
        orc.append(self_hit(lambda m: h.search(m, 1, 64, threads=8)[:2], vals))
    for setting in settings.split(";"):
        kv = {} if setting.strip() in ("", "base") else dict(p.split("=", 1) for p in setting.split(","))
        for k, v in kv.items():
            os.environ[k] = v
        g = vsg.Index(dim, "l2sq", "f32", 16, 64, 64, seed=2)
        for rnd, segs, vals in stream(nkeys, dim, rounds, seg):
            for keys, v in segs:
                if rnd:
                    g.remove(keys)
                g.add(keys, v)
            gh = self_hit(lambda m: (lambda r: (r.keys, r.distances))(g.search(m, 1, 64)), vals)
            print(json.dumps({"nkeys": nkeys, "dim": dim, "segment": seg, "setting": kv or "base", "round": rnd,
                              "gpu": gh, "oracle_sequential": orc[rnd], "slots": int(g.graph_info()["slots"])}),
                  flush=True)
        for k in kv:
            os.environ.pop(k, None)


if __name__ == "__main__":
    main()
