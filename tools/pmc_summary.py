"""HBM traffic of the search kernel from rocprofv3 PMC passes.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> n dim queries ef metric
Each dir is the output of its own pass:
  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir> -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d <dir> -- python3 bench.py ...
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of 16-B/lane
coalesced streaming reads -> x2 (the search kernel's row loads are 16 B/lane,
1 KiB contiguous per wave instruction; the 4-B adjacency loads are a small
share and are doubled too, which over-states them).  WRITE_SIZE is taken as-is.
Writes profiles/search_pmc.json, read by bench.py for roofline.traffic.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = defaultdict(float)
    grid = {}
    for r in csv.DictReader(open(files[0])):
        if r.get("Counter_Name") != counter or "hnsw_search_" not in r.get("Kernel_Name", ""):
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] += float(r["Counter_Value"])
        grid[key] = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
    return vals, grid


def main():
    fdir, wdir, n, dim, nq, ef, metric = sys.argv[1:8]
    nq = int(nq)
    fv, fg = per_dispatch(fdir, "FETCH_SIZE")
    wv, wg = per_dispatch(wdir, "WRITE_SIZE")
    full = [k for k in fv if fg[k] == nq * 64]
    fullw = [k for k in wv if wg[k] == nq * 64]
    if not full:
        raise SystemExit(f"no search dispatch with grid {nq * 64}: {sorted(set(fg.values()))}")
    fetch_kib = sum(fv[k] for k in full) / len(full)
    write_kib = sum(wv[k] for k in fullw) / max(1, len(fullw))
    out = {
        "workload": {"n": int(n), "dim": int(dim), "queries": nq, "ef": int(ef), "metric": metric},
        "kernel": "hnsw_search_reg_kernel",
        "dispatches": len(full),
        "fetch_size_kib_raw": round(fetch_kib, 1),
        "write_size_kib_raw": round(write_kib, 1),
        "hbm_bytes_per_launch": int(2 * fetch_kib * 1024 + write_kib * 1024),
        "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), KiB -> bytes",
    }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    json.dump(out, open(os.path.join(root, "profiles", "search_pmc.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
