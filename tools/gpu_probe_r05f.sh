#!/bin/bash
# Round 5: small-batch search latency at C2 (the serving path's batches: 512 / 2,048 queries):
# register kernel vs the cooperative LDS-list kernel with 1 / 2 / 4 waves per query.
# gpurun_out/r05_small_batch.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for nq in ${NQS:-512 2048}; do
  timeout -k 10 300 python3 -u tools/gpu_probe.py search --queries $nq --gt-queries $nq --efs 36 --steps 10 \
    --set reg=1 --set reg=0,waves=1 --set reg=0,waves=2 --set reg=0,waves=4 \
    >> gpurun_out/r05_small_batch.jsonl 2>> gpurun_out/r05_small_batch.err || exit 1
done
echo done
