#!/bin/bash
# Round 6 combined call (the pool is congested: one queue wait for all of it):
#  1. tools/free_probe: which runtime calls wait for unrelated device work
#  2. the free / growth test with VSG_DEBUG_TIMING (where vsg_index_free spends time)
#  3. per-expansion search profile + register-row variants (gpu_probe_r06a.sh)
#  4. serving through the actor, 1 / 2 / 4 read workers (gpu_r06c.sh)
#  5. rerank + C2 parity (replace path at full size)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 tools/free_probe > gpurun_out/r06_free_probe.json 2>&1 && cat gpurun_out/r06_free_probe.json && \
VSG_DEBUG_TIMING=1 timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_concurrency.py -k "free_and_growth" > gpurun_out/r06d_free.log 2>&1
grep -E "vsg timing\] free|build .* free|passed|failed" gpurun_out/r06d_free.log | tail -8
bash tools/gpu_probe_r06a.sh && bash tools/gpu_r06c.sh && \
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_rerank.py \
  > gpurun_out/r06d_rerank.log 2>&1 && tail -2 gpurun_out/r06d_rerank.log && \
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 800 --timeout-method thread -m gpu tests/test_gpu_c2_parity.py \
  > gpurun_out/r06b_c2.log 2>&1; grep -E "C2|passed|failed" gpurun_out/r06b_c2.log | tail -12
