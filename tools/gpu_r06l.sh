#!/bin/bash
# Round 6: C2 search row shape 32 x 6 with U = 6 passes in flight (lib_u6) against the
# tree's U = 4 (lib), at 512 / 2,048 / 10,000 queries, ef 36 (same results expected).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r06l_u6.jsonl
for v in u4 u6 u4 u6; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" = u6 ] && lib=vector-store-text_amd/lib_u6/libvsg.so
  for nq in 512 2048 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 240 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq \
      --efs 36 --steps 5 | sed "s/^{/{\"lib\": \"$v\", /" >> $out 2>> gpurun_out/r06l.err || exit 2
  done
done
grep -h kernel_ms $out | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['lib'], d['queries'], d['ef'], d['kernel_ms'], d.get('recall_at_10'))"
