#!/bin/bash
# GPU: C3 / C4 8-shard emulations (one GPU) and the C3 single-GPU bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/shard_emulation.py --rows 10000000 --shards 8 --dim 768 --quant f32 --metric cos --data clustered --config 2 --efs 16,24,32,48,64,128 --out gpurun_out/shard_emu_c3.jsonl > gpurun_out/shard_emu_c3.log 2>&1
rc=$?; echo "c3 emu rc=$rc"; tail -8 gpurun_out/shard_emu_c3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/shard_emulation.py --rows 100000000 --shards 8 --efs 64,128,160,192,256 --out gpurun_out/shard_emu_c4.jsonl > gpurun_out/shard_emu_c4.log 2>&1
rc=$?; echo "c4 emu rc=$rc"; tail -7 gpurun_out/shard_emu_c4.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --rows 10000000 --config 2 --no-cpu --gt-queries 500 --steps 3 --warmup 1 > gpurun_out/bench_c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -1 gpurun_out/bench_c3.log
exit $rc
