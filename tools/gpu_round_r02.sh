#!/bin/bash
# Round-2 measurement: the default bench (N=1) and its rocprofv3 kernel-trace stats,
# plus the C5 exact (MFMA) bench line.  Outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_n1.log 2>&1 || exit 1
# profiled run at the bench's chosen ef (no sweep): every search launch is the headline's
EF=${1:-34}
rm -rf gpurun_out/prof_bench  # one run per summary (tools/prof_summary.py globs the directory)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -- python3 -u bench.py --no-cpu --upper-ef 0 --rerank-leg 0 --config-ef 0 --ef $EF --steps 10 > gpurun_out/prof_bench.log 2>&1 || exit 1
find gpurun_out/prof_bench -name '*kernel_trace.csv' -size +20M -delete
timeout -k 10 300 python3 -u bench.py --mode exact --rows 1000000 --dim 1536 --metric ip --config 4 --batch 1024 --steps 5 > gpurun_out/bench_c5.log 2>&1 || exit 1
echo done
