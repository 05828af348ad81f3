"""HBM traffic from rocprofv3 PMC passes (one counter per pass, MI355X_MICROARCH.md).

  search: python tools/pmc_summary.py search <fetch_dir> <write_dir> n dim queries ef metric [out.json]
          -> profiles/search_pmc.json: bytes per search launch (the bench workload's grid)
  build:  python tools/pmc_summary.py build <fetch_dir> <write_dir> n dim metric M efc [out.json]
          -> profiles/build_pmc.json: bytes over ALL insert / reverse launches of one build

Each dir is the output of its own pass, e.g.
  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir> -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d <dir> -- python3 bench.py ...
FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md
§HBM): FETCH_SIZE reports half the bytes of 16-B/lane coalesced streaming reads -> x2 (the
row loads are 16 B/lane; the 4-B adjacency loads are a small share and are doubled too,
which over-states them).  WRITE_SIZE is taken as-is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def provenance():
    """Which kernels were profiled: bench.kernel_src_sha() of this tree (bench.py uses
    the summary only while its tree hashes the same) and the git head when known."""
    from bench import kernel_src_sha
    head = None
    try:
        import subprocess
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip() or None
    except Exception:  # noqa: BLE001 -- the GPU box's copy has no .git
        pass
    return {"kernel_src_sha": kernel_src_sha(), "git_head": head}


def per_dispatch(d, counter, kernel):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = defaultdict(float)
    grid = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter or kernel not in r.get("Kernel_Name", ""):
                continue
            key = (f, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            vals[key] += float(r["Counter_Value"])
            grid[key] = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
    return vals, grid


def search(fdir, wdir, n, dim, nq, ef, metric, path=None):
    nq = int(nq)
    fv, fg = per_dispatch(fdir, "FETCH_SIZE", "hnsw_search_")
    wv, wg = per_dispatch(wdir, "WRITE_SIZE", "hnsw_search_")
    full = [k for k in fv if fg[k] == nq * 64]
    fullw = [k for k in wv if wg[k] == nq * 64]
    if not full:
        # persistent grid (round 5): every launch has the resident-wave grid whatever
        # its batch; the bench run's searches are all the headline batch (--ef, nq)
        full, fullw = list(fv), list(wv)
    if not full:
        raise SystemExit(f"no search dispatch: {sorted(set(fg.values()))}")
    fetch_kib = float(np.median([fv[k] for k in full]))
    write_kib = float(np.median([wv[k] for k in fullw])) if fullw else 0.0
    out = {
        # forward_links "M": usearch's <= M forward links per level (round 4 on)
        "workload": {"n": int(n), "dim": int(dim), "queries": nq, "ef": int(ef), "metric": metric,
                     "forward_links": "M"},
        "kernel": "hnsw_search_reg_kernel",
        "dispatches": len(full),
        "grid": sorted(set(fg[k] for k in full)),
        "per_dispatch": "median over the dispatches",
        "fetch_size_kib_raw": round(fetch_kib, 1),
        "write_size_kib_raw": round(write_kib, 1),
        "hbm_bytes_per_launch": int(2 * fetch_kib * 1024 + write_kib * 1024),
        "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), KiB -> bytes",
        **provenance(),
    }
    json.dump(out, open(path or os.path.join(ROOT, "profiles", "search_pmc.json"), "w"), indent=1)
    return out


def build(fdir, wdir, n, dim, metric, M, efc, path=None):
    out = {"workload": {"n": int(n), "dim": int(dim), "metric": metric, "M": int(M), "efc": int(efc),
                        "forward_links": "M"},
           "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), KiB -> bytes; summed over every "
                         "dispatch of the kernel in ONE build (the probe builds once per process)",
           **provenance()}
    # "hnsw_insert_": the fused insert kernel or both launches of the split insert
    # (hnsw_insert_beam_kernel + hnsw_insert_select_kernel), then each on its own
    for tag, kern in (("insert", "hnsw_insert_"), ("beam", "hnsw_insert_beam_kernel"),
                      ("select", "hnsw_insert_select_kernel"), ("reverse", "hnsw_reverse_kernel")):
        fv, _ = per_dispatch(fdir, "FETCH_SIZE", kern)
        wv, _ = per_dispatch(wdir, "WRITE_SIZE", kern)
        out[f"{tag}_dispatches"] = len(fv)
        out[f"{tag}_fetch_kib_raw"] = round(sum(fv.values()), 1)
        out[f"{tag}_write_kib_raw"] = round(sum(wv.values()), 1)
        out[f"{tag}_hbm_bytes"] = int(2 * sum(fv.values()) * 1024 + sum(wv.values()) * 1024)
    json.dump(out, open(path or os.path.join(ROOT, "profiles", "build_pmc.json"), "w"), indent=1)
    return out


if __name__ == "__main__":
    mode = sys.argv[1]
    print(json.dumps(search(*sys.argv[2:10]) if mode == "search" else build(*sys.argv[2:10])))
