#!/bin/bash
# Round 5: (1) host-buffer search time split at C2 (10k and 512 queries); (2) the C5 build
# (1M x 1536 IP) with 4 row passes in flight in the build kernels (lib_c5b4:
# -DVSG_BUILD_SHAPE384=64,6,4 on hnsw.hip) vs 2.
# gpurun_out/r05_host_search.jsonl, r05_c5b4_build.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
VSG_PROFILE_HOST_SEARCH=1 timeout -k 10 300 python3 -u tools/host_search_probe.py >> gpurun_out/r05_host_search.jsonl 2>> gpurun_out/r05_host_search.err || exit 1
VSG_PROFILE_HOST_SEARCH=1 timeout -k 10 300 python3 -u tools/host_search_probe.py 1000000 512 36 20 >> gpurun_out/r05_host_search.jsonl 2>> gpurun_out/r05_host_search.err || exit 1
for v in ${VARIANTS:-base c5b4}; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/build_probe.py --rows 1000000 --dim 1536 --metric ip --config 4 \
    --queries 2000 --efs 24,48 --reps 2 --out gpurun_out/r05_c5b4_build.jsonl >> gpurun_out/r05_c5b4_build.log 2>&1 || exit 1
done
echo done
