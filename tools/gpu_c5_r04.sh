#!/bin/bash
# Round 4: C5 (1M x 1536 IP) brute force at batch 64 and 1024 -- bench line, one SQ pass
# (8 SQ counters: wave-cycle shares, MFMA busy) and one FETCH_SIZE pass each, to see what
# bounds the 256 x 64 MFMA tile.  Summaries -> gpurun_out/r04_c5_*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_BUSY_CYCLES"
for b in ${BATCHES:-64 1024}; do
  B="python3 -u bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --config 4 --batch $b --steps 5 --no-cpu"
  timeout -k 10 300 $B > gpurun_out/r04_c5_b$b.log 2>&1 || exit 1
  grep '^{' gpurun_out/r04_c5_b$b.log >> gpurun_out/r04_c5_batches.jsonl
  rm -rf gpurun_out/sq_c5
  timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_c5 -- $B > gpurun_out/sq_c5_b$b.log 2>&1 || exit 1
  python3 tools/sq_summary.py gpurun_out/sq_c5 gpurun_out/r04_c5_sq_b$b.json || exit 1
  rm -rf gpurun_out/pmc_c5
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_c5 -- $B > gpurun_out/pmc_c5_b$b.log 2>&1 || exit 1
  python3 - $b <<'PY'
import csv, glob, json, sys
b = sys.argv[1]
tot, n = 0.0, 0
for f in glob.glob("gpurun_out/pmc_c5/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE" and "mfma_exact" in r["Kernel_Name"]:
            tot += float(r["Counter_Value"]); n += 1
print(json.dumps({"batch": int(b), "mfma_dispatches": n, "hbm_read_bytes_per_dispatch_x2": 2 * tot * 1024 / max(1, n)}))
open(f"gpurun_out/r04_c5_fetch_b{b}.json", "w").write(json.dumps({"batch": int(b), "dispatches": n, "fetch_kib_raw_total": tot, "hbm_read_bytes_per_dispatch": 2 * tot * 1024 / max(1, n)}))
PY
  rm -rf gpurun_out/sq_c5 gpurun_out/pmc_c5
done
echo done
