#!/bin/bash
# GPU: full GPU test suite + smoke on the tree as committed (round-end rehearsal)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_final.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_final.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_final.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_final.log | cut -c1-400
exit $rc
