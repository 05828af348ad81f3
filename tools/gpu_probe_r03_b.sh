#!/bin/bash
# Round 3 (b): graph-identity tests of the build kernels on the current tree, then
#  - build variants (selection shape / occupancy, beam register rows, compaction early
#    exit, reverse appends per lane off) on the C2 1M build  -> gpurun_out/r03_sel_probe.jsonl
#  - small-shard batch schedule on a 125k shard              -> same file
#  - C4 shard search (12.5M x 128 f16, 10k queries, ef 64/192): register rows 4 vs 8 and
#    the compaction early exit                               -> gpurun_out/r03_c4_probe.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_edge_dist.py tests/test_gpu_build_locality.py \
  "tests/test_gpu_parity.py::test_hnsw_gpu_build_one_node_batches_equals_oracle_graph" \
  > gpurun_out/r03_b_tests.log 2>&1 || { tail -30 gpurun_out/r03_b_tests.log; exit 1; }
tail -2 gpurun_out/r03_b_tests.log
out=gpurun_out/r03_sel_probe.jsonl
for v in ${VARIANTS:-base}; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  echo "== variant $v" >> gpurun_out/r03_sel_probe.log
  VSG_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/build_probe.py --rows 1000000 --reps 2 --queries 2000 --efs 16,32 --out $out >> gpurun_out/r03_sel_probe.log 2>&1 || exit 1
done
if [ -n "$SHARD_SETTINGS" ]; then
  timeout -k 10 300 python3 -u tools/build_probe.py --rows 125000 --reps 3 --queries 2000 --efs 10,16,24 --settings "$SHARD_SETTINGS" --out $out >> gpurun_out/r03_sel_probe.log 2>&1 || exit 1
fi
for v in ${C4_VARIANTS:-}; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  VSG_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 \
    --dim 128 --quant f16 --metric l2sq --data sift --config 3 --efs 64,192 --steps 5 \
    --set , --set VSG_SEARCH_REG_ROWS=8 > gpurun_out/r03_c4_probe_$v.log 2>&1 || exit 1
  tail -8 gpurun_out/r03_c4_probe_$v.log
done
echo done
