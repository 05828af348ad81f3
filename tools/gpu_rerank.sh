#!/bin/bash
# GPU: f16-traversal re-rank tests + full parity, then a bench run (no CPU leg)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rerank.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pytest_rerank.log | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench_rerank.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_rerank.log
exit $rc
