#!/bin/bash
# Round 3 (c): parity tests of the current tree, then A/B of kernel-library variants on
# the same box (LIBS: "base" = lib/, else lib_<v>/): C2 search at the headline ef, the C2
# 1M build, and a C4 shard search (ef 64 / 192).  Outputs in gpurun_out/r03_ab_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_c4_parity.py tests/test_gpu_edge_dist.py tests/test_gpu_build_locality.py \
    tests/test_gpu_configs.py tests/test_gpu_rerank.py tests/test_gpu_c2_parity.py \
    > gpurun_out/r03_c_tests.log 2>&1 || { tail -40 gpurun_out/r03_c_tests.log; exit 1; }
  tail -2 gpurun_out/r03_c_tests.log
fi
libpath() { [ "$1" = base ] && echo vector-store-text_amd/lib/libvsg.so || echo vector-store-text_amd/lib_$1/libvsg.so; }
for rep in 1 2; do
  for v in ${LIBS:-base}; do
    VSG_LIB_PATH=$(libpath $v) timeout -k 10 200 python3 -u tools/gpu_probe.py search --efs 34 --steps 10 \
      > gpurun_out/r03_ab_c2_${v}_$rep.log 2>&1 || exit 1
    echo "C2 $v rep $rep: $(grep '"ef": 34' gpurun_out/r03_ab_c2_${v}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["kernel_ms"], d["recall_at_10"], d["hbm_frac"])')"
  done
done
for v in ${LIBS:-base}; do
  VSG_LIB_PATH=$(libpath $v) timeout -k 10 200 python3 -u tools/build_probe.py --rows 1000000 --reps 2 --queries 2000 --efs 16,32 \
    --out gpurun_out/r03_ab_build.jsonl > gpurun_out/r03_ab_build_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/r03_ab_build.jsonl | cut -c1-330
done
for v in ${LIBS:-base}; do
  VSG_LIB_PATH=$(libpath $v) timeout -k 10 300 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 \
    --dim 128 --quant f16 --metric l2sq --data sift --config 3 --efs 64,192 --steps 5 > gpurun_out/r03_ab_c4_$v.log 2>&1 || exit 1
  echo "C4 $v: $(grep '"ef"' gpurun_out/r03_ab_c4_$v.log | python3 -c 'import json,sys
for l in sys.stdin: d=json.loads(l); print(d["ef"], d["kernel_ms"], d["recall_at_10"], d["hbm_frac"], end="; ")')"
done
echo done
