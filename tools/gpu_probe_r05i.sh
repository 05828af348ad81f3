#!/bin/bash
# Round 5: (1) the build kernels with 4 row passes in flight for 768-d f32 rows (lib_b4:
# -DVSG_SHAPE192=32,6,4 on hnsw.hip) vs the default 2, on the C2 1M build; (2) the search
# shape of 1536-d f32 rows with 4 passes (lib_c5u4: -DVSG_SEARCH_SHAPE384=64,6,4 on
# hnsw_search_reg.hip) vs 2, C5 1M x 1536 IP HNSW at 512 / 10,000 queries.
# gpurun_out/r05_b4_build.jsonl, r05_c5u4.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base b4; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  VSG_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/build_probe.py --rows 1000000 --reps 3 --queries 2000 --efs 16,32 \
    --out gpurun_out/r05_b4_build.jsonl >> gpurun_out/r05_b4_build.log 2>&1 || exit 1
done
for v in base c5u4; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  for nq in 512 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --dim 1536 --metric ip --config 4 --queries $nq \
      --gt-queries $nq --efs 30 --steps 10 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r05_c5u4.jsonl 2>> gpurun_out/r05_c5u4.err || exit 1
  done
done
echo done
