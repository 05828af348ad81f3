#!/bin/bash
# Round 5: the register search kernels compiled for 6 waves per SIMD (lib_w6:
# -DVSG_SEARCH_ATTR=amdgpu_waves_per_eu(6) on hnsw_search_reg.hip; the C4 shard kernel
# holds 87 VGPRs = 5 waves by default) vs the default, C4 shard at ef 64 / 192.
# gpurun_out/r05_c4_w6.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base w6; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  VSG_LIB_PATH=$lib timeout -k 10 400 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 --dim 128 \
    --quant f16 --metric l2sq --data sift --config 3 --efs 64,192 --steps 5 --streams 2 | sed "s/^{/{\"lib\": \"$v\", /" \
    >> gpurun_out/r05_c4_w6.jsonl 2>> gpurun_out/r05_c4_w6.err || exit 1
done
echo done
