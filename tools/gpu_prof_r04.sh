#!/bin/bash
# Round 4: rocprofv3 kernel-trace stats of the bench at the headline ef, then the PMC
# HBM-traffic passes (tools/gpu_pmc_r04.sh).  Outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
EF=${1:-36}
P=gpurun_out/prof_r04_ef$EF
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P -- python3 -u bench.py --no-cpu --upper-ef 0 --rerank-leg 0 --config-ef 0 --ef $EF --steps 10 > gpurun_out/r04_prof_bench_ef$EF.log 2>&1 || exit 1
find $P -name '*kernel_trace.csv' -size +20M -delete
bash tools/gpu_pmc_r04.sh $EF || exit 1
echo done
