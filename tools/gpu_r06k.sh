#!/bin/bash
# Round 6, final tree: GPU tests + smoke (gpu_round_r06.sh tests), then the SQ issue
# counters of the C4-shard search with the pass-skipping rows_dist.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_round_r06.sh tests || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/r06k_sq -o sq --output-format csv -- \
  python3 -u tools/gpu_probe.py search --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 --metric l2sq \
  --data sift --config 3 --queries 10000 --gt-queries 1000 --efs 192 --steps 2 > gpurun_out/r06k_sq.log 2>&1 || exit 2
echo done
