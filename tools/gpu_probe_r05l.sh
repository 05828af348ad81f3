#!/bin/bash
# Round 5: 6 / 8 row passes in flight for 768-d f32 rows in the 2-row register search
# (lib_u6 / lib_u8: -DVSG_SEARCH_SHAPE192=32,6,6 / 32,6,8 on hnsw_search_reg.hip) vs the
# default 4, by batch size; then the actor's serving rate on the default library.
# gpurun_out/r05_u68.jsonl, r05_actor_final_c*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base u6 u8; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  for nq in 512 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq --efs 36 --steps 10 \
      --set reg=1 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r05_u68.jsonl 2>> gpurun_out/r05_u68.err || exit 1
  done
done
for CL in 512 2048; do
  VSG_PROFILE_HOST_SEARCH=1 timeout -k 10 300 tools/actor_load 1000000 768 2 $CL $((51200 / CL)) 10 36 0 0 1 > gpurun_out/r05_actor_final_c$CL.json 2> gpurun_out/r05_actor_final_c$CL.err || { tail -5 gpurun_out/r05_actor_final_c$CL.err; exit 1; }
  cat gpurun_out/r05_actor_final_c$CL.json; grep breakdown gpurun_out/r05_actor_final_c$CL.err
done
echo done
