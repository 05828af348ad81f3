#!/bin/bash
# Round 5: after the U=4 search shape for 768-d f32 rows -- search parity tests, the
# small-batch kernel times, and the actor's serving rate (completions, 512 / 2,048 clients).
# gpurun_out/r05_h_tests.log, r05_u4_batches.jsonl, r05_actor_u4_c*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_usearch_semantics.py tests/test_gpu_c2_parity.py tests/test_gpu_streams.py} \
  > gpurun_out/r05_h_tests.log 2>&1 || { tail -30 gpurun_out/r05_h_tests.log; exit 1; }
tail -2 gpurun_out/r05_h_tests.log
for nq in 512 2048 10000; do
  timeout -k 10 300 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq --efs 36 --steps 10 --set reg=1 \
    >> gpurun_out/r05_u4_batches.jsonl 2>> gpurun_out/r05_u4_batches.err || exit 1
done
for CL in 512 2048; do
  VSG_PROFILE_HOST_SEARCH=1 timeout -k 10 300 tools/actor_load 1000000 768 2 $CL $((51200 / CL)) 10 36 0 0 1 > gpurun_out/r05_actor_u4_c$CL.json 2> gpurun_out/r05_actor_u4_c$CL.err || { tail -5 gpurun_out/r05_actor_u4_c$CL.err; exit 1; }
  cat gpurun_out/r05_actor_u4_c$CL.json; grep breakdown gpurun_out/r05_actor_u4_c$CL.err
done
echo done
