#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { timeout -k 10 "$1" "${@:2}" >> gpurun_out/bp.log 2>> gpurun_out/bp_err.log; }
: > gpurun_out/bp.log
run 300 python tools/hash_factor_probe.py 1000000 768 cos f32 clustered 36 4 8 12 16 24 32 48 &&
run 300 python tools/build_probe.py 1000000 768 cos f32 clustered - - VSG_BUILD_HASH_FACTOR=8 &&
run 500 python tools/hash_factor_probe.py 10000000 768 cos f32 clustered 321 3 4 6 8 12 16 &&
run 500 python tools/hash_factor_probe.py 20000000 128 l2sq f16 sift 256 3 4 6 8 12 16 32
rc=$?
cat gpurun_out/bp.log; tail -3 gpurun_out/bp_err.log
exit $rc
