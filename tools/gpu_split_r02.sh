#!/bin/bash
# Split insert (beam kernel + selection kernel) vs the fused insert kernel (round 2):
# same-graph tests, the one-node-batch oracle identities, then build time at C2 and
# on one C4 shard.  Outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_build_locality.py tests/test_gpu_limits.py tests/test_gpu_parity.py -k "same_graph or one_node" > gpurun_out/split_test.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/gpu_probe.py build --set split=0 --set split=1 --set split=0 --set split=1 --efs 34 > gpurun_out/split_c2.log 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/gpu_probe.py build --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 --metric l2sq --data sift --config 3 --set split=0 --set split=1 --efs 192 > gpurun_out/split_c4.log 2>&1 || exit 1
echo done
