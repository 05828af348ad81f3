#!/bin/bash
# Round-5 probes: (1) recall before / after reuse churn (tools/reuse_probe.py),
# (2) the C2 parity module with its churn tests, (3) persistent search grid A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 50; do echo "[hb] $(date +%T)" >> gpurun_out/r05_heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python3 -u tools/reuse_probe.py 30000 64 2000 3 > gpurun_out/r05_reuse_probe.jsonl 2> gpurun_out/r05_reuse_probe.err || exit 1
cat gpurun_out/r05_reuse_probe.jsonl
B="python3 -u bench.py --no-cpu --upper-ef 0 --rerank-leg 0 --config-ef 0 --host-abi-leg 0 --ef 36 --steps 20 --warmup 3"
for i in 1 2; do
  for P in 0 1; do
    VSG_SEARCH_PERSIST=$P timeout -k 10 200 $B > gpurun_out/r05_persist_${P}_${i}.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'persist': int(sys.argv[2]), 'qps': d['value'], 'kernel_ms': d['roofline']['kernel_ms'], 'frac': d['roofline']['frac'], 'two_streams': d['concurrent_streams']['qps'], 'recall': d['config']['recall_at_10']}))" gpurun_out/r05_persist_${P}_${i}.log $P | tee -a gpurun_out/r05_persist.jsonl
  done
done
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_c2_parity.py -m gpu -q -rf -s --timeout 900 --timeout-method thread > gpurun_out/r05_c2_parity.log 2>&1 || { tail -40 gpurun_out/r05_c2_parity.log; exit 1; }
grep -E "C2|passed|failed" gpurun_out/r05_c2_parity.log
echo done
