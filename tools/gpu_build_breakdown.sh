#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { timeout -k 10 "$1" "${@:2}" >> gpurun_out/bp.log 2>> gpurun_out/bp_err.log; }
: > gpurun_out/bp.log
run 400 python tools/build_probe.py 1000000 768 cos f32 clustered - VSG_REVERSE_GRID=2048 - VSG_REVERSE_PAIRS_PER_WAVE=64 VSG_REVERSE_PAIRS_PER_WAVE=8 VSG_REVERSE_PAIRS_PER_WAVE=4 \
   VSG_BUILD_HASH_FACTOR=16 VSG_BUILD_HASH_FACTOR=12 VSG_BUILD_HASH_FACTOR=8 &&
run 300 python tools/build_probe.py 1000000 128 l2sq f32 sift - VSG_REVERSE_GRID=2048 VSG_BUILD_HASH_FACTOR=16
rc=$?
cat gpurun_out/bp.log; tail -3 gpurun_out/bp_err.log
exit $rc
