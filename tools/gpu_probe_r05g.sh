#!/bin/bash
# Round 5: the register search kernel with 4 row passes in flight for 768-d f32 rows
# (lib_s4: make variant VSRC=hnsw_search_reg.hip VAR=s4 VFLAGS=-DVSG_SHAPE192=32,6,4)
# against the default (2 passes) and the 4-wave cooperative list kernel, by batch size.
# gpurun_out/r05_shape_u4.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base s4; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  for nq in 512 2048 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq --efs 36 --steps 10 \
      --set reg=1 --set reg=0,waves=4 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r05_shape_u4.jsonl 2>> gpurun_out/r05_shape_u4.err || exit 1
  done
done
echo done
