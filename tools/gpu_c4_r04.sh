#!/bin/bash
# Round 4: C4 shard (12.5M x 128 f16 sift-like, shard 0 of 8) search at ef 64 / 192 with a
# 10k-query batch: default library vs 8 waves/SIMD forced on the register search kernel
# (lib_w8), and smaller visited tables (VSG_SEARCH_HASH_MIN).  JSON lines ->
# gpurun_out/r04_c4_probe.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P="tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 --metric l2sq --data sift --config 3 --efs 64,192 --steps 5"
timeout -k 10 400 python3 -u $P --set hmin=1024 --set hmin=512 --set hmin=512,hash=2 >> gpurun_out/r04_c4_probe.jsonl 2> gpurun_out/r04_c4_probe.err || exit 1
VSG_LIB_PATH=vector-store-text_amd/lib_w8/libvsg.so timeout -k 10 400 python3 -u $P --set hmin=1024 --set hmin=512 --set hmin=512,hash=2 | sed 's/^{/{"lib": "w8", /' >> gpurun_out/r04_c4_probe.jsonl 2>> gpurun_out/r04_c4_probe.err || exit 1
echo done
