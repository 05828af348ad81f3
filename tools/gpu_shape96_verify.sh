#!/bin/bash
# GPU: full GPU suite with the 96-chunk shape default, then bench (no CPU leg)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s96.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/pytest_s96.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench_s96.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_s96.log
exit $rc
