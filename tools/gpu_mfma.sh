#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --batch 1024 --steps 5 --warmup 1 > gpurun_out/bench_c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/bench_c5.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof_c5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o c5 -- python3 bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --batch 1024 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_c5.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof_c5.log
exit $rc
