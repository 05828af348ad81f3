#!/bin/bash
# GPU: full bench (N=1) -> rocprof kernel trace -> PMC FETCH/WRITE passes -> 2-rank gloo rehearsal.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
EF=$(python -c "import json;print(json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1])['config']['ef'])")
echo "ef=$EF"
ARGS="--no-cpu --ef $EF --config-ef 0 --steps 3 --warmup 1 --rerank-leg 0 --upper-ef 0"
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py $ARGS > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python3 bench.py $ARGS > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; tail -1 gpurun_out/pmc_fetch.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o pmc -- python3 bench.py $ARGS > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; tail -1 gpurun_out/pmc_write.log; [ $rc -ne 0 ] && exit $rc
python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write 1000000 768 10000 $EF cos > gpurun_out/pmc_summary.log 2>&1; cat gpurun_out/pmc_summary.log
# keep only the small summaries (counter CSVs can be large)
find gpurun_out/pmc_fetch gpurun_out/pmc_write -name "*counter_collection.csv" -size +20M -delete
# the opt-in f16 walk + f32 re-rank leg on its own (kernel trace only)
rm -rf gpurun_out/prof_rerank
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rerank -o bench -- python3 bench.py --no-cpu --ef $EF --config-ef 0 --steps 3 --warmup 1 --upper-ef 0 > gpurun_out/prof_rerank.log 2>&1
rc=$?; echo "rocprof rerank rc=$rc"; tail -1 gpurun_out/prof_rerank.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --rows 200000 --queries 2000 --gt-queries 500 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 gpurun_out/bench_gloo2.log
exit $rc
