#!/bin/bash
# Round 5: C5's 200k x 1536 IP build (the test's rows / queries: config 4 seeds) under
# build-schedule settings -- where the GPU build's recall gap to the oracle's sequential
# build comes from; then the concurrency / actor tests on their own.
# gpurun_out/r05_c5_sched.{jsonl,log}, gpurun_out/r05_d_tests.log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${SETTINGS:-"base;VSG_BUILD_BATCH_FRAC2=0.25;VSG_BUILD_MIN_BATCHES=32;VSG_BUILD_BATCH_MAX=4096;VSG_BUILD_SPLIT=0;VSG_BUILD_LOCALITY=0;VSG_BUILD_EDGE_DIST=0"}
timeout -k 10 400 python3 -u tools/build_probe.py --rows 200000 --dim 1536 --metric ip --config 4 --queries 2000 \
  --efs 24,64 --reps 1 --settings "$S" --out gpurun_out/r05_c5_sched.jsonl >> gpurun_out/r05_c5_sched.log 2>&1 || exit 1
if [ -n "$C4" ]; then  # C4 shard (12.5M x 128 f16, shard 0 of 8), persistent search grid on / off
  timeout -k 10 400 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 \
    --metric l2sq --data sift --config 3 --efs 64,192 --steps 5 --streams 2 --set VSG_SEARCH_PERSIST=1 \
    --set VSG_SEARCH_PERSIST=0 >> gpurun_out/r05_c4_persist.jsonl 2>> gpurun_out/r05_c4_persist.err || exit 1
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/r05_d_tests.log 2>&1 || exit 1
fi
echo done
