#!/bin/bash
# Round 5: the short-row register search kernels without the persistent loop (87 VGPRs,
# 5 waves/SIMD, instead of 102 / 4): C4 shard at ef 64 / 192, then the search parity tests.
# gpurun_out/r05_c4_nopersist.jsonl, r05_m_tests.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 \
  --metric l2sq --data sift --config 3 --efs 64,192 --steps 5 --streams 2 >> gpurun_out/r05_c4_nopersist.jsonl 2>> gpurun_out/r05_c4_nopersist.err || exit 1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_usearch_semantics.py tests/test_gpu_c4_parity.py tests/test_gpu_limits.py \
  > gpurun_out/r05_m_tests.log 2>&1 || { tail -30 gpurun_out/r05_m_tests.log; exit 1; }
tail -1 gpurun_out/r05_m_tests.log
echo done
