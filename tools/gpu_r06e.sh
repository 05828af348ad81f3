#!/bin/bash
# Round 6: (1) the free / growth test with VSG_DEBUG_TIMING (streams now recycled,
# the pool for every index buffer); (2) the bit-exact search / build tests after the
# early next-expansion load in beam_reg; (3) A/B of the search kernel, round-6 start
# library (lib_base) vs this tree (lib): C2 512 / 10k queries at ef 36, one C4 shard
# (12.5M x 128 f16) at ef 64 / 192; (4) the serving sweep (gpu_r06c.sh).
# A pytest failure (exit 1) goes on to the next step; any other non-zero exit ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ] || { echo "step failed with $1: stop"; exit "$1"; }; }
VSG_DEBUG_TIMING=1 timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_concurrency.py > gpurun_out/r06e_conc.log 2>&1
rc=$?; grep -E "vsg timing\] free|passed|failed|^E " gpurun_out/r06e_conc.log | tail -12; ok $rc
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_usearch_semantics.py > gpurun_out/r06e_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r06e_parity.log; ok $rc
out=gpurun_out/r06e_ab.jsonl
for v in base new; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" = base ] && lib=vector-store-text_amd/lib_base/libvsg.so
  for nq in 512 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 240 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq \
      --efs 36 --steps 5 | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c2\", /" >> $out 2>> gpurun_out/r06e_ab.err || exit 2
  done
  VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 \
    --dim 128 --quant f16 --metric l2sq --data sift --config 3 --queries 10000 --gt-queries 1000 --efs 64,192 \
    --steps 3 | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c4shard\", /" >> $out 2>> gpurun_out/r06e_ab.err || exit 2
done
grep -h kernel_ms $out | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['lib'], d['cfg'], d['queries'], d['ef'], d['kernel_ms'], d.get('hbm_frac'), d.get('recall_at_10'))"
bash tools/gpu_r06c.sh
