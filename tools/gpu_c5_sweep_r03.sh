#!/bin/bash
# Round 3: C5 (1M x 1536 IP) brute force at batch 1 / 64 / 256 / 1024 (VALU below
# 32 queries, f32 MFMA above) and the HNSW path on the same data; one JSON line
# each into gpurun_out/r03_bench_c5_batches.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=gpurun_out/r03_bench_c5_batches.jsonl
for b in 1 64 256 1024; do
  cpu=--no-cpu; [ $b = 1024 ] && cpu=
  timeout -k 10 300 python3 -u bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --config 4 --batch $b --steps 5 $cpu 2>>gpurun_out/r03_c5.err | grep '^{' >> $o || exit 1
done
timeout -k 10 300 python3 -u bench.py --rows 1000000 --dim 1536 --metric ip --config 4 --no-cpu --upper-ef 0 --rerank-leg 0 2>>gpurun_out/r03_c5.err | grep '^{' >> $o || exit 1
