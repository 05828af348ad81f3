#!/bin/bash
# Round 4: C5 batch 64 -- round-3 two-buffer pipeline vs K-tiled copy on / off, alternating (same box); MFMA
# bit-exact tests first.  JSON lines -> gpurun_out/r04_c5_ktile_ab.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "exact or mfma" -m gpu > gpurun_out/r04_c5b_tests.log 2>&1 || { tail -30 gpurun_out/r04_c5b_tests.log; exit 1; }
tail -1 gpurun_out/r04_c5b_tests.log
for wr in 1 0 1 0; do
  VSG_EXACT_KTILE=$wr timeout -k 10 300 python3 -u bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --config 4 --batch ${B:-64} --steps 10 --no-cpu 2>>gpurun_out/r04_c5b.err | grep '^{' | sed "s/^{/{\"ktile\": $wr, /" >> gpurun_out/r04_c5_ktile_ab.jsonl || exit 1
done
echo done
