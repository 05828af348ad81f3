#!/bin/bash
# Round 6: C2 10 % churn through vsg_index_replace at smaller re-link chunks
# (VSG_REPLACE_DIV 16384 / 65536: 61 / 15 keys at 1M rows) against the oracle's
# one-at-a-time sequence; the actor upsert test at 16384.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 16384 65536; do
  VSG_REPLACE_DIV=$d timeout -k 10 500 python3 -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_c2_parity.py -k churn > gpurun_out/r06i_c2_div$d.log 2>&1
  rc=$?; grep -E "C2 churn|passed|failed" gpurun_out/r06i_c2_div$d.log | cut -c1-220; [ $rc -le 1 ] || exit $rc
done
VSG_REPLACE_DIV=16384 timeout -k 10 300 python3 -u -m pytest -v -s --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_actor.py -k upsert > gpurun_out/r06i_actor.log 2>&1
rc=$?; grep -E "self|passed|failed" gpurun_out/r06i_actor.log | cut -c1-220; exit $rc
