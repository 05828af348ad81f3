"""Summarise hipcc -Rpass-analysis=kernel-resource-usage for one source file.
usage: python tools/kernel_resources.py vector-store-text_amd/csrc/hnsw.hip"""
import re, subprocess, sys
src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Iinclude",
       "-c", src, "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
for r in rows:
    n = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    n = n.replace("vsg::", "").split("(")[0]
    print(f'{n:60s} vgpr={r.get("VGPRs")} agpr={r.get("AGPRs")} sgpr={r.get("SGPRs")} scratch={r.get("ScratchSize")} occ={r.get("Occupancy")}')
