"""Condense a rocprofv3 --kernel-trace --stats CSV output dir into profiles/.

usage: python tools/prof_summary.py gpurun_out/prof <tag>
writes profiles/<tag>_kernel_stats.csv (the tool's own stats file) and
profiles/<tag>_summary.md (top kernels + per-grid averages of the hot kernels,
which is what bench.py's HIP-event kernel time is compared against).
"""
import csv
import glob
import os
import shutil
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)
stats = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)
trace = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
lines = [f"# rocprofv3 kernel summary — {tag}", ""]


def demangle(name):
    """Some rocprofv3 runs report mangled kernel names (_ZN3vsg...): demangle with c++filt."""
    if not name.startswith("_Z"):
        return name
    try:
        import subprocess
        # GNU c++filt does not know DF16_ (_Float16): demangle it as Dh (half), rename after
        out = subprocess.run(["c++filt", name.replace("DF16_", "Dh")], capture_output=True, text=True,
                             timeout=10).stdout.strip()
        return out.replace("half", "_Float16") if out and not out.startswith("_Z") else name
    except Exception:  # noqa: BLE001 -- keep the raw name
        return name


if stats:
    shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats[0])))
    lines += ["| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in rows[:12]:
        lines.append(f"| `{demangle(r['Name'])[:80]}` | {r['Calls']} | {int(r['TotalDurationNs'])/1e6:.2f} | "
                     f"{float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.2f} |")
if trace:
    per = defaultdict(list)
    for r in csv.DictReader(open(trace[0])):
        name = demangle(r["Kernel_Name"])
        if "vsg::" not in name or not any(s in name for s in ("hnsw_", "exact", "mfma", "merge")):
            continue
        short = name.split("(")[0].replace("void ", "")
        build = "insert" in short or "reverse" in short  # many batch shapes: aggregate
        per[(short, "all" if build else r["Grid_Size_X"], "-" if build else r.get("Grid_Size_Y", "1"))].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    lines += ["", "Per-launch-shape averages (kernel trace):", "",
              "| kernel | grid x | grid y | launches | avg ms | min ms |", "|---|---|---|---|---|---|"]
    for (k, gx, gy), v in sorted(per.items()):
        lines.append(f"| `{k}` | {gx} | {gy} | {len(v)} | {sum(v)/len(v)/1e6:.4f} | {min(v)/1e6:.4f} |")
open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
