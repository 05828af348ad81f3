#!/bin/bash
# Round 5: U=4 search shape only for the 2-register-row kernels -- search parity tests,
# the bench without the CPU leg (ef 36 and the config's ef 128), 512-query batches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_usearch_semantics.py tests/test_gpu_limits.py tests/test_gpu_streams.py \
  > gpurun_out/r05_j_tests.log 2>&1 || { tail -30 gpurun_out/r05_j_tests.log; exit 1; }
tail -1 gpurun_out/r05_j_tests.log
timeout -k 10 400 python3 -u bench.py --no-cpu > gpurun_out/r05_j_bench.log 2>&1 || { tail -20 gpurun_out/r05_j_bench.log; exit 1; }
for nq in 512 2048; do
  timeout -k 10 300 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq --efs 36,128 --steps 10 --set reg=1 \
    >> gpurun_out/r05_j_batches.jsonl 2>> gpurun_out/r05_j_batches.err || exit 1
done
echo done
