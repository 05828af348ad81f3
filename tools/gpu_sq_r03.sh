#!/bin/bash
# Round 3: SQ issue counters (one --pmc pass of 8 SQ counters each run) for the build and
# search kernels of the C2 bench workload and of a C4 shard search (ef 192, 10k queries):
# is a kernel waiting on memory (SQ_WAIT_ANY) or issuing (SQ_ACTIVE_INST_ANY / _VALU)?
# Summaries -> gpurun_out/r03_sq_{c2,c4}.json (tools/sq_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CNT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
rm -rf gpurun_out/sq_c2 gpurun_out/sq_c4
timeout -s KILL 300 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d gpurun_out/sq_c2 -- \
  python3 -u bench.py --no-cpu --upper-ef 0 --rerank-leg 0 --config-ef 0 --ef 34 --steps 3 --warmup 1 \
  > gpurun_out/sq_c2.log 2>&1 || exit 1
python3 tools/sq_summary.py gpurun_out/sq_c2 gpurun_out/r03_sq_c2.json || exit 1
timeout -s KILL 300 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d gpurun_out/sq_c4 -- \
  python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 \
  --metric l2sq --data sift --config 3 --efs 192 --steps 3 > gpurun_out/sq_c4.log 2>&1 || exit 1
python3 tools/sq_summary.py gpurun_out/sq_c4 gpurun_out/r03_sq_c4.json || exit 1
rm -rf gpurun_out/sq_c2 gpurun_out/sq_c4
echo done
