#!/bin/bash
# Round 6: compaction that stops at the first prefix range that fits (VSG_COMPACT_EARLY,
# lib_ce) against the tree's exact ef-th-key cut (lib): C4 shard ef 64 / 192 and C2 512 /
# 10k at ef 36.  Same results expected (B stays a superset of the top ef).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r06n_ce.jsonl
for v in base ce base ce; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" = ce ] && lib=vector-store-text_amd/lib_ce/libvsg.so
  VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 \
    --dim 128 --quant f16 --metric l2sq --data sift --config 3 --queries 10000 --gt-queries 1000 --efs 64,192 \
    --steps 3 | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c4shard\", /" >> $out 2>> gpurun_out/r06n.err || exit 2
  for nq in 512 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 240 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq \
      --efs 36 --steps 5 | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c2\", /" >> $out 2>> gpurun_out/r06n.err || exit 2
  done
done
grep -h kernel_ms $out | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['lib'], d['cfg'], d['queries'], d['ef'], d['kernel_ms'], d.get('recall_at_10'), d.get('same_as_first'))"
