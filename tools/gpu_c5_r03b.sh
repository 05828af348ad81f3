#!/bin/bash
# Round 3 (b): exact-search tests (oracle bit-exact, MFMA == VALU at C5 size), then the C5
# batch sweep (tools/gpu_c5_sweep_r03.sh) with one summary line per batch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "exact or mfma" tests/test_gpu_configs.py \
  > gpurun_out/r03_mfma_tests.log 2>&1 || { tail -30 gpurun_out/r03_mfma_tests.log; exit 1; }
tail -2 gpurun_out/r03_mfma_tests.log
rm -f gpurun_out/r03_bench_c5_batches.jsonl
bash tools/gpu_c5_sweep_r03.sh || exit 1
python3 - <<'EOF'
import json
for l in open("gpurun_out/r03_bench_c5_batches.jsonl"):
    d = json.loads(l)
    r = d["roofline"]
    print(d["config"].get("batch"), d["value"], d["ms_per_step"], r["frac"], r["kernel_ms"])
EOF
