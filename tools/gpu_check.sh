#!/bin/bash
# GPU: parity tests -> default bench (N=1, as the driver runs it)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
exit $rc2
