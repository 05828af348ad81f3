#!/bin/bash
# Round 6: rows_dist skips passes past the listed rows (loads only for rows <= 512 B).  (1) A/B lib_base vs lib on
# C2 and one C4 shard; (2) the whole GPU suite (bit-exact search / build tests among them).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ] || { echo "step failed with $1: stop"; exit "$1"; }; }
out=gpurun_out/r06h_ab.jsonl
for v in base new; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" = base ] && lib=vector-store-text_amd/lib_base/libvsg.so
  for nq in 512 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 240 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq \
      --efs 36 --steps 5 | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c2\", /" >> $out 2>> gpurun_out/r06h_ab.err || exit 2
  done
  VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 \
    --dim 128 --quant f16 --metric l2sq --data sift --config 3 --queries 10000 --gt-queries 1000 --efs 64,192 \
    --steps 3 | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c4shard\", /" >> $out 2>> gpurun_out/r06h_ab.err || exit 2
done
grep -h kernel_ms $out | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['lib'], d['cfg'], d['queries'], d['ef'], d['kernel_ms'], d.get('hbm_frac'), d.get('recall_at_10'))"
timeout -k 10 1000 python3 -u -m pytest -v -s --durations=25 --timeout 600 --timeout-method thread -m gpu \
  tests > gpurun_out/r06h_gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|C2 churn" gpurun_out/r06h_gpu_tests.log | tail -12; ok $rc
