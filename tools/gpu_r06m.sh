#!/bin/bash
# Round 6, final tree: rocprofv3 kernel-trace stats of one C4 shard search (12.5M x 128
# f16, l2sq, 10k queries, ef 64 / 192) -> profiles/r06_c4_shard_summary.md.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/prof_c4_$(date +%s)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P -- python3 -u tools/gpu_probe.py search \
  --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 --metric l2sq --data sift --config 3 --queries 10000 \
  --gt-queries 1000 --efs 64,192 --steps 5 > gpurun_out/r06m_c4.jsonl 2> gpurun_out/r06m_c4.err || exit 2
find $P -name '*kernel_trace.csv' -size +20M -delete
echo "rocprof output: $P"
cat gpurun_out/r06m_c4.jsonl | cut -c1-300
