"""SQ issue counters per kernel from one rocprofv3 --pmc pass (tools/gpu_sq_r03.sh).

usage: python tools/sq_summary.py <pmc_dir> <out.json>

For every kernel name (template arguments kept) sums the counters over its dispatches and
reports the shares of wave time: SQ_WAIT_ANY (parked on s_waitcnt / barrier: memory
latency), SQ_WAIT_INST_ANY (issue stalls), SQ_ACTIVE_INST_ANY (issuing), and
SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, with instructions per wave.  Only the kernels with
the most wave cycles are kept.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src, out = sys.argv[1], sys.argv[2]
files = glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True)
if not files:
    raise SystemExit(f"no counter_collection.csv under {src}")
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in files:
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        k = k.split("(")[0].replace("void ", "").replace("vsg::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r.get("Dispatch_Id") or r.get("Correlation_Id")))
rows = []
for k, c in tot.items():
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if wc <= 0:
        continue
    waves = None
    rows.append({
        "kernel": k, "dispatches": len(disp[k]), "wave_cycles": wc,
        "wait_any": round(c.get("SQ_WAIT_ANY", 0) / wc, 3),
        "wait_inst_any": round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
        "active_inst_any": round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
        "active_inst_valu": round(c.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3),
        "insts_valu": c.get("SQ_INSTS_VALU", 0), "insts_lds": c.get("SQ_INSTS_LDS", 0),
        "insts_salu": c.get("SQ_INSTS_SALU", 0), "counters": dict(c)})
rows.sort(key=lambda r: -r["wave_cycles"])
json.dump({"source": "rocprofv3 --pmc " + " ".join(sorted({n for c in tot.values() for n in c})),
           "note": "shares of SQ_WAVE_CYCLES summed over the kernel's dispatches; counter units as "
                   "rocprofv3 reports them (gfx950 SQ cycle counters may be scaled; compare shares)",
           "kernels": rows[:12]}, open(out, "w"), indent=1)
for r in rows[:12]:
    print(f'{r["kernel"][:70]:70s} n={r["dispatches"]:4d} wait={r["wait_any"]:.3f} '
          f'stall={r["wait_inst_any"]:.3f} active={r["active_inst_any"]:.3f} valu={r["active_inst_valu"]:.3f}')
