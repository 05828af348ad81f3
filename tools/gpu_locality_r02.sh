#!/bin/bash
# Build launch-order locality (round 2): same-graph tests, then build time with
# the pivot-cell order off / on at C2 (f32) and on one C4 shard (f16).
# Outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_build_locality.py > gpurun_out/loc_test.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/gpu_probe.py build --set loc=0 --set loc=1 --set loc=0 --set loc=1 --efs 34 > gpurun_out/loc_c2.log 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/gpu_probe.py build --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 --metric l2sq --data sift --config 3 --set loc=0 --set loc=1 --efs 192 > gpurun_out/loc_c4.log 2>&1 || exit 1
echo done-c4
