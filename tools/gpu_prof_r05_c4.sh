#!/bin/bash
# Round 5: rocprofv3 kernel-trace stats of the C4 shard search (12.5M x 128 f16, shard 0 of 8,
# 10k queries at ef 64 / 192, plain grid) -- the kernel times behind profiles/r05_c4_nopersist.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/prof_c4_$(date +%s)
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $P -- python3 -u tools/gpu_probe.py search \
  --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 --metric l2sq --data sift --config 3 --efs 64,192 --steps 5 \
  > gpurun_out/r05_prof_c4.log 2>&1 || exit 1
find $P -name '*kernel_trace.csv' -size +20M -delete
echo "rocprof output: $P"
