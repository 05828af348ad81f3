#!/bin/bash
# Round 5 (final kernels): C2 (1M x 768 f32 cos) row-shard emulations on one GPU for S = 2, 4, 8
# shards, each with its hybrid projection on 8 GPUs (8/S groups of S shards).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C2="--rows 1000000 --dim 768 --quant f32 --metric cos --data clustered --config 1 --queries 10000 --gt-queries 10000 --steps 5"
timeout -k 10 300 python3 -u tools/shard_emulation.py $C2 --shards 2 --efs 16,20,24,28,32,36 --out gpurun_out/r05_shard_emulation_c2.jsonl || exit 1
timeout -k 10 300 python3 -u tools/shard_emulation.py $C2 --shards 4 --efs 10,12,16,20,24,28 --out gpurun_out/r05_shard_emulation_c2.jsonl || exit 1
timeout -k 10 400 python3 -u tools/shard_emulation.py $C2 --shards 8 --efs 10,12,14,16,20 --out gpurun_out/r05_shard_emulation_c2.jsonl || exit 1
echo done
