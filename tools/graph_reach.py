"""Level-0 reachability of a GPU-built graph (diagnostic for a recall ceiling).

usage (GPU box): python tools/graph_reach.py rows dim metric quant data config seed ef
Builds the index as bench.py does (one add call), exports the graph, runs a BFS
over level-0 adjacency from the entry point on the GPU (torch), and reports the
reachable share of slots, the share of the 200 queries' exact top-10 that is
reachable, and the per-query recall spread at `ef`.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vector-store-text_amd"))


def main():
    rows, dim, metric, quant, data, config = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4],
                                              sys.argv[5], int(sys.argv[6]))
    seed, ef = int(sys.argv[7], 0), int(sys.argv[8])
    import torch
    import vsg
    from vsg import datagen as G

    bs, qs, ms = G.config_seeds(config)
    idx = vsg.Index(dim, metric, quant, 16, 128, 64, seed=seed)
    idx.reserve(rows)
    x = vsg.datagen_device(data, rows, dim, bs, ms)
    idx.add_device(np.arange(rows, dtype=np.uint64), x)
    del x
    torch.cuda.synchronize()
    q = vsg.datagen_device(data, 200, dim, qs, ms)
    gk = idx.search_device(q, 10, exact=True)[0].cpu().numpy()
    k = idx.search_device(q, 10, ef)[0].cpu().numpy()
    per_q = np.array([len(set(a) & set(b)) / 10 for a, b in zip(k, gk)])
    gi = idx.graph_info()
    t0 = time.time()
    g = idx.export()
    adj_np = g["adj0"]
    levels = g["levels"]
    del g
    adj = torch.from_numpy(adj_np.view(np.int32)).cuda()
    n = adj.shape[0]
    vis = torch.zeros(n, dtype=torch.bool, device="cuda")
    front = torch.tensor([gi["entry"]], dtype=torch.int64, device="cuda")
    vis[front] = True
    depth = 0
    while front.numel():
        nb = adj[front].reshape(-1)
        nb = nb[nb >= 0].long()
        nb = nb[~vis[nb]]
        nb = torch.unique(nb)
        vis[nb] = True
        front = nb
        depth += 1
    reach = float(vis.float().mean())
    visn = vis.cpu().numpy()
    gt_reach = float(visn[gk.astype(np.int64)].mean())
    indeg = torch.zeros(n, dtype=torch.int32, device="cuda")
    for c0 in range(0, n, 4_000_000):
        flat = adj[c0:c0 + 4_000_000].reshape(-1)
        flat = flat[flat >= 0].long()
        indeg.index_add_(0, flat, torch.ones_like(flat, dtype=torch.int32))
    out = {"rows": rows, "seed": seed, "ef": ef, "reachable_level0": round(reach, 6), "bfs_depth": depth,
           "gt_top10_reachable": round(gt_reach, 4), "recall_mean": round(float(per_q.mean()), 4),
           "queries_recall_below_0.5": int((per_q < 0.5).sum()), "queries_recall_1.0": int((per_q == 1.0).sum()),
           "zero_indegree_slots": int((indeg == 0).sum()),
           "out_degree_mean": round(float(sum(int((adj[c0:c0 + 4_000_000] >= 0).sum()) for c0 in range(0, n, 4_000_000)) / n), 2),
           "max_level": gi["max_level"], "entry": gi["entry"], "entry_level": int(levels[gi["entry"]]),
           "bfs_s": round(time.time() - t0, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
