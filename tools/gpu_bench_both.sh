#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/bench_gloo2_both.log 2>&1
rc=$?; tail -1 gpurun_out/bench_gloo2_both.log; exit $rc
