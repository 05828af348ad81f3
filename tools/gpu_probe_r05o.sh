#!/bin/bash
# Round 5: the 2-register-row C2 search kernel (32 x 6 x 4 shape, 175 VGPRs = 2 waves/SIMD)
# compiled for 3 waves per SIMD (lib_w3: -DVSG_SEARCH_ATTR=amdgpu_waves_per_eu(3)) vs the
# default; the bench's search leg with 10k queries and 512-query batches.
# gpurun_out/r05_w3.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base w3; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  for nq in 512 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq --efs 36 --steps 10 \
      --set reg=1 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r05_w3.jsonl 2>> gpurun_out/r05_w3.err || exit 1
  done
done
echo done
