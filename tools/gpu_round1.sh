#!/bin/bash
# GPU check: smoke -> parity tests -> reduced bench; stop on any crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --rows 100000 --queries 2000 --gt-queries 500 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_small.log
exit $rc
