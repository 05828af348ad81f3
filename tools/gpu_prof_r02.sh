#!/bin/bash
# Round-2 profiles: PMC HBM traffic of the C2 build kernels and of the C4 shard search
# (100k-query batch), one counter per rocprofv3 pass; summaries -> gpurun_out/*.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 tools/gpu_probe.py"
C4="search --rows 100000000 --shards 8 --shard 0 --dim 128 --quant f16 --metric l2sq --data sift --config 3 --efs 192 --queries 100000 --steps 2"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_bf -- $P build --efs 36 > gpurun_out/pmc_bf.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_bw -- $P build --efs 36 > gpurun_out/pmc_bw.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_c4f -- $P $C4 > gpurun_out/pmc_c4f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_c4w -- $P $C4 > gpurun_out/pmc_c4w.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -- $P $C4 > gpurun_out/prof_c4.log 2>&1 || exit 1
python3 tools/pmc_summary.py build gpurun_out/pmc_bf gpurun_out/pmc_bw 1000000 768 cos 16 128 gpurun_out/build_pmc.json
python3 tools/pmc_summary.py search gpurun_out/pmc_c4f gpurun_out/pmc_c4w 12500000 128 100000 192 l2sq gpurun_out/c4_search_pmc.json
find gpurun_out/prof_c4 -name '*kernel_trace.csv' -delete  # keep the small stats CSV
rm -rf gpurun_out/pmc_bf gpurun_out/pmc_bw gpurun_out/pmc_c4f gpurun_out/pmc_c4w  # > 64 MiB of CSV
