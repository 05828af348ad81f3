#!/bin/bash
# Round 6: per-expansion cycle breakdown of the register search beam (make prof:
# lib_prof, s_memtime stamps; tools/gpu_probe.py --phases) -- C2 at ef 36 for
# 512 and 10k queries, one C4 shard (12.5M x 128 f16) at ef 64 / 192 for 512 and
# 10k queries; and the same workloads on the plain library for the unprofiled times.
# gpurun_out/r06_phases.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r06_phases.jsonl
for v in prof base ce; do
  lib=vector-store-text_amd/lib/libvsg.so
  ph=""
  [ "$v" = prof ] && lib=vector-store-text_amd/lib_prof/libvsg.so && ph="--phases"
  # ce: the compaction stops at the first prefix range that fits (VSG_COMPACT_EARLY)
  [ "$v" = ce ] && lib=vector-store-text_amd/lib_ce/libvsg.so
  [ -f "$lib" ] || continue
  for nq in 512 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 240 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq \
      --efs 36 --steps 5 $ph \
      | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c2\", /" >> $out 2>> gpurun_out/r06_phases.err || exit 1
  done
  # register rows: 4 (default at ef 192) / 8 / 17 -- same results, fewer compactions
  VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 \
    --dim 128 --quant f16 --metric l2sq --data sift --config 3 --queries 10000 --gt-queries 1000 --efs 64,192 \
    --steps 3 $ph --set "" --set VSG_SEARCH_REG_ROWS=8 --set VSG_SEARCH_REG_ROWS=17 \
    | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c4shard\", /" >> $out 2>> gpurun_out/r06_phases.err || exit 1
done
echo done
