#!/bin/bash
# Round-6 check of the whole tree: GPU tests, smoke, the default bench (N=1) and its
# rocprofv3 kernel-trace stats at the headline ef.  Outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
# heartbeat: long single tests (multi-rank bench rehearsals) print nothing for minutes
( while sleep 50; do echo "[hb] $(date +%T)" >> gpurun_out/r06_heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 1120 python3 -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/r06_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r06_gpu_tests.log; exit 1; }
  tail -3 gpurun_out/r06_gpu_tests.log
  timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || exit 1
  tail -1 gpurun_out/r06_smoke.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 400 python3 -u bench.py > gpurun_out/r06_bench_n1.log 2>&1 || { tail -20 gpurun_out/r06_bench_n1.log; exit 1; }
  tail -c 600 gpurun_out/r06_bench_n1.log
  EF=${2:-36}
  P=gpurun_out/prof_bench_$(date +%s)  # one directory per run: gpurun merges outputs back
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P -- python3 -u bench.py --no-cpu --upper-ef 0 --rerank-leg 0 --config-ef 0 --streams-leg 0 --actor-leg 0 --host-abi-leg 0 --ef $EF --steps 10 > gpurun_out/r06_prof_bench.log 2>&1 || exit 1
  find $P -name '*kernel_trace.csv' -size +20M -delete
  echo "rocprof output: $P"
fi
echo done
