#!/bin/bash
# Launch-order locality (round 2): same-result tests, then build time and search
# kernel time with the path-key order off/on at C2 and on one C4 shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_build_locality.py  > gpurun_out/loc_test.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/gpu_probe.py build --set loc=0 --set loc=1 --set loc=0 --set loc=1 --efs 34 > gpurun_out/loc_c2.log 2>&1 || exit 1
echo done
