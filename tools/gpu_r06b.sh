#!/bin/bash
# Round 6: the replace path on the GPU (per-batch staging, vsg_index_replace, the
# actor's held chunk tails) -- slot-reuse, actor, filtered-search and multi-entry
# tests, then the C2 parity module (10 % replaced through the replace call vs the
# oracle one replace at a time); then the per-expansion search profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_slot_reuse.py tests/test_gpu_actor.py tests/test_gpu_usearch_semantics.py tests/test_gpu_multi_entry.py tests/test_gpu_concurrency.py tests/test_gpu_rerank.py \
  > gpurun_out/r06b_tests.log 2>&1 || { tail -30 gpurun_out/r06b_tests.log; exit 1; }
tail -3 gpurun_out/r06b_tests.log
timeout -k 10 1000 python3 -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu tests/test_gpu_c2_parity.py \
  > gpurun_out/r06b_c2.log 2>&1 || { tail -30 gpurun_out/r06b_c2.log; exit 1; }
grep -E "C2|passed|failed" gpurun_out/r06b_c2.log | tail -12
bash tools/gpu_probe_r06a.sh
