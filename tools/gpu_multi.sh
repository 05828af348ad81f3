#!/bin/bash
# GPU tests + multi-rank rehearsal on ONE GPU over gloo (shard x4, replica x2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 600 $TR --nproc-per-node 4 --master-port 29531 bench.py --gpus 4 --dist-backend gloo --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_gloo4_shard.log 2>&1
rc=$?; echo "shard4 rc=$rc"; tail -1 gpurun_out/bench_gloo4_shard.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 $TR --nproc-per-node 2 --master-port 29532 bench.py --gpus 2 --dist-backend gloo --multi replica --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_gloo2_replica.log 2>&1
rc=$?; echo "replica2 rc=$rc"; tail -1 gpurun_out/bench_gloo2_replica.log
exit $rc
