#!/bin/bash
# GPU: C5 1M x 1536 f32 IP -- HNSW leg (recall >= 0.95) beside the exact MFMA brute force
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --rows 1000000 --dim 1536 --metric ip --config 4 --no-cpu --steps 5 --warmup 2 > gpurun_out/bench_c5_hnsw.log 2>&1
rc=$?; echo "c5 hnsw rc=$rc"; tail -1 gpurun_out/bench_c5_hnsw.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --batch 1024 --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_c5_exact.log 2>&1
rc=$?; echo "c5 exact rc=$rc"; tail -1 gpurun_out/bench_c5_exact.log
exit $rc
