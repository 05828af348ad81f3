#!/bin/bash
# PMC HBM traffic of the bench workload (C2), one counter per rocprofv3 pass (round 6: --host-abi-leg 0 --streams-leg 0 --actor-leg 0 so the run builds and searches once;
# beam / select / reverse kernels reported apart):
# the search kernel at the bench's ef and the build kernels of the same run.
# Summaries -> gpurun_out/search_pmc.json, gpurun_out/build_pmc.json (copied to profiles/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
EF=${1:-36}
B="python3 -u bench.py --warm-build 0 --no-cpu --host-abi-leg 0 --streams-leg 0 --actor-leg 0 --upper-ef 0 --rerank-leg 0 --config-ef 0 --ef $EF --steps 3 --warmup 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_f -- $B > gpurun_out/pmc_f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_w -- $B > gpurun_out/pmc_w.log 2>&1 || exit 1
python3 tools/pmc_summary.py search gpurun_out/pmc_f gpurun_out/pmc_w 1000000 768 10000 $EF cos gpurun_out/search_pmc.json || exit 1
python3 tools/pmc_summary.py build gpurun_out/pmc_f gpurun_out/pmc_w 1000000 768 cos 16 128 gpurun_out/build_pmc.json || exit 1
rm -rf gpurun_out/pmc_f gpurun_out/pmc_w
