#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python bench.py --rows 10000000 --config 2 --no-cpu --steps 3 --warmup 1 > gpurun_out/bench_c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -1 gpurun_out/bench_c3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --rows 100000000 --dim 128 --metric l2sq --quant f16 --data sift --config 3 --no-cpu --gt-queries 200 --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -2 gpurun_out/bench_c4.log
exit $rc
