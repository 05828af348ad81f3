#!/bin/bash
# Round 6: the early next-expansion load in beam_reg as a global (not flat) load.
# (1) bit-exact search / build tests; (2) A/B lib_base vs lib on C2 and one C4 shard;
# (3) SQ issue counters of the C4-shard search (is the kernel issue-bound?);
# (4) serving at 512 / 2048 clients, one read worker.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ] || { echo "step failed with $1: stop"; exit "$1"; }; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_usearch_semantics.py > gpurun_out/r06f_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r06f_parity.log; ok $rc
out=gpurun_out/r06f_ab.jsonl
for v in base new; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" = base ] && lib=vector-store-text_amd/lib_base/libvsg.so
  for nq in 512 10000; do
    VSG_LIB_PATH=$lib timeout -k 10 240 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq \
      --efs 36 --steps 5 | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c2\", /" >> $out 2>> gpurun_out/r06f_ab.err || exit 2
  done
  VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 \
    --dim 128 --quant f16 --metric l2sq --data sift --config 3 --queries 10000 --gt-queries 1000 --efs 64,192 \
    --steps 3 | sed "s/^{/{\"lib\": \"$v\", \"cfg\": \"c4shard\", /" >> $out 2>> gpurun_out/r06f_ab.err || exit 2
done
grep -h kernel_ms $out | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['lib'], d['cfg'], d['queries'], d['ef'], d['kernel_ms'], d.get('hbm_frac'), d.get('recall_at_10'))"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/r06f_sq -o sq --output-format csv -- \
  python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 --metric l2sq \
  --data sift --config 3 --queries 10000 --gt-queries 1000 --efs 192 --steps 2 > gpurun_out/r06f_sq.log 2>&1 || exit 2
out=gpurun_out/r06f_actor.jsonl
for c in 512 2048; do
  timeout -k 10 240 tools/actor_load 1000000 768 2 $c $((51200 / c)) 10 36 0 1 1 0x5EED 0 \
    > gpurun_out/r06f_actor_run.json 2> gpurun_out/r06f_actor_run.err || exit 2
  cat gpurun_out/r06f_actor_run.json >> $out
done
cat $out | cut -c1-400
