#!/bin/bash
# Round 5: (1) self-recall under a whole-index replace stream, GPU build settings vs the
# oracle's sequential build (tools/upsert_probe.py); (2) the C4 shard's search at persistent
# grid fractions (VSG_SEARCH_PERSIST_FRAC, read once per process) vs the plain grid; (3) the
# call's minimum batch count (VSG_BUILD_MIN_BATCHES) on C5 (1M / 200k x 1536 IP) and C2.
# gpurun_out/r05_upsert_probe.jsonl, r05_c4_pfrac.jsonl, r05_minb.jsonl (+ .log / .err).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
U="base;VSG_BUILD_BATCH_MAX=1;VSG_REUSE_BATCH_DIV=512;VSG_BUILD_MIN_BATCHES=64"
for seg in 256 3000; do
  timeout -k 10 200 python3 -u tools/upsert_probe.py 3000 32 4 $seg "$U" >> gpurun_out/r05_upsert_probe.jsonl \
    2>> gpurun_out/r05_upsert_probe.err || exit 1
done
C4P="tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 --metric l2sq --data sift --config 3 --efs 64,192 --steps 5 --streams 2"
for f in 1.0 0.75; do
  VSG_SEARCH_PERSIST_FRAC=$f timeout -k 10 300 python3 -u $C4P --set VSG_SEARCH_PERSIST=1 --set VSG_SEARCH_PERSIST=0 \
    | sed "s/^{/{\"persist_frac\": $f, /" >> gpurun_out/r05_c4_pfrac.jsonl 2>> gpurun_out/r05_c4_pfrac.err || exit 1
done
timeout -k 10 300 python3 -u tools/build_probe.py --rows 1000000 --dim 1536 --metric ip --config 4 --queries 2000 \
  --efs 24,48 --reps 1 --settings "base;VSG_BUILD_MIN_BATCHES=16;VSG_BUILD_MIN_BATCHES=32" \
  --out gpurun_out/r05_minb.jsonl >> gpurun_out/r05_minb.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/build_probe.py --rows 200000 --dim 1536 --metric ip --config 4 --queries 2000 \
  --efs 24,64 --reps 1 --settings "VSG_BUILD_MIN_BATCHES=16;VSG_BUILD_MIN_BATCHES=24" \
  --out gpurun_out/r05_minb.jsonl >> gpurun_out/r05_minb.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/build_probe.py --rows 1000000 --queries 2000 --efs 16,32 --reps 2 \
  --settings "base;VSG_BUILD_MIN_BATCHES=16;VSG_BUILD_MIN_BATCHES=32" \
  --out gpurun_out/r05_minb.jsonl >> gpurun_out/r05_minb.log 2>&1 || exit 1
echo done
