#!/bin/bash
# GPU: C3 10M x 768 cos 8-shard emulation on one GPU (current kernels)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/shard_emulation.py --rows 10000000 --shards 8 --dim 768 --quant f32 --metric cos --data clustered --config 2 --efs 16,24,32,48,64,128 --out gpurun_out/shard_emu_c3_s5.jsonl > gpurun_out/shard_emu_c3_s5.log 2>&1
rc=$?; echo "c3 emu rc=$rc"; tail -8 gpurun_out/shard_emu_c3_s5.log
exit $rc
