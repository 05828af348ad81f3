#!/bin/bash
# GPU: parity tests -> full bench (N=1) -> rocprofv3 kernel-trace of the bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
fi
exit $rc
