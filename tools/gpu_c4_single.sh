#!/bin/bash
# GPU: C4 on ONE GPU (100M x 128 f16 sift-like, one graph)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py --rows 100000000 --dim 128 --metric l2sq --quant f16 --data sift --config 3 --no-cpu --gt-queries 200 --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -1 gpurun_out/bench_c4.log
exit $rc
