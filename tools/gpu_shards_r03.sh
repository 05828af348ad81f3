#!/bin/bash
# Round 3: row-sharded layouts emulated on the one GPU (tools/shard_emulation.py): C2 as 8
# shards of 125k, C3 as 8 x 1.25M, C4 as 8 x 12.5M f16; per-shard build times, merged
# recall and per-shard search time / distance evaluations / GB/s -> gpurun_out/r03_shards.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r03_shards.jsonl
timeout -k 10 300 python3 -u tools/shard_emulation.py --rows 1000000 --shards 8 --dim 768 --quant f32 --metric cos \
  --data clustered --config 1 --efs 10,12,16 --out $out > gpurun_out/r03_shards_c2.log 2>&1 || exit 1
tail -3 gpurun_out/r03_shards_c2.log
timeout -k 10 400 python3 -u tools/shard_emulation.py --rows 10000000 --shards 8 --dim 768 --quant f32 --metric cos \
  --data clustered --config 2 --efs 16,24,28,32,48 --out $out > gpurun_out/r03_shards_c3.log 2>&1 || exit 1
tail -3 gpurun_out/r03_shards_c3.log
timeout -k 10 500 python3 -u tools/shard_emulation.py --rows 100000000 --shards 8 --dim 128 --quant f16 --metric l2sq \
  --data sift --config 3 --efs 64,128,192,256 --out $out > gpurun_out/r03_shards_c4.log 2>&1 || exit 1
tail -3 gpurun_out/r03_shards_c4.log
echo done
