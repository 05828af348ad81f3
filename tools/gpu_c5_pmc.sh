#!/bin/bash
# GPU: SQ counters of the C5 MFMA brute-force kernel (one pass, SQ block only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_c5
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_c5 -o c5 -- python3 bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --batch 1024 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_c5.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -2 gpurun_out/pmc_c5.log
python3 - <<'EOF'
import csv, glob, collections
fs = glob.glob("gpurun_out/pmc_c5/**/*counter_collection.csv", recursive=True)
tot = collections.defaultdict(float)
for f in fs:
    for r in csv.DictReader(open(f)):
        if "mfma_exact" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    print(f"{k} {v:.4g}")
EOF
find gpurun_out/pmc_c5 -name "*counter_collection.csv" -size +20M -delete
exit $rc
