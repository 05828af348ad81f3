#!/bin/bash
# Round 4: the other BASELINE configs on the usearch-rule graph -- C3 (10M x 768 cos,
# 8 row shards) and C4 (100M x 128 f16 l2sq, 8 row shards) emulated on one GPU, C5 HNSW
# (1M x 1536 IP).  JSON lines -> gpurun_out/r04_configs_*.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/shard_emulation.py --rows 10000000 --dim 768 --quant f32 --metric cos --data clustered --config 2 --shards 8 --queries 10000 --gt-queries 1000 --efs 16,24,28,32,40 --steps 3 --out gpurun_out/r04_configs_c3.jsonl || exit 1
timeout -k 10 600 python3 -u tools/shard_emulation.py --rows 100000000 --dim 128 --quant f16 --metric l2sq --data sift --config 3 --shards 8 --queries 10000 --gt-queries 1000 --efs 128,160,192,256 --steps 3 --out gpurun_out/r04_configs_c4.jsonl || exit 1
timeout -k 10 300 python3 -u bench.py --rows 1000000 --dim 1536 --metric ip --config 4 --no-cpu --upper-ef 0 --rerank-leg 0 2>>gpurun_out/r04_configs.err | grep '^{' >> gpurun_out/r04_configs_c5.jsonl || exit 1
echo done
