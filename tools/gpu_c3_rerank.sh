#!/bin/bash
# GPU: C3 10M x 768 cos on one GPU (f32 walk headline + opt-in f16 walk / f32 re-rank leg)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --rows 10000000 --config 2 --no-cpu --gt-queries 500 --steps 3 --warmup 1 > gpurun_out/bench_c3_rerank.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -1 gpurun_out/bench_c3_rerank.log
exit $rc
