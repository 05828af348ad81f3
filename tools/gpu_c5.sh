#!/bin/bash
# GPU: exact-search parity subset, C5 bench (MFMA brute force) and its rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "exact or golden or kat" -p no:cacheprovider > gpurun_out/pytest_c5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_c5.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --batch 1024 --steps 5 --warmup 1 ${C5CPU---no-cpu} > gpurun_out/bench_c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/bench_c5.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof_c5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o c5 -- python3 bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --batch 1024 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_c5.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -h mfma_exact gpurun_out/prof_c5/*/*kernel_stats.csv gpurun_out/prof_c5/*kernel_stats.csv 2>/dev/null | cut -c1-160
exit $rc
