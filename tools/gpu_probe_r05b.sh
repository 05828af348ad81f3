#!/bin/bash
# Round-5 probes (b): (1) reuse re-link batch size (VSG_REUSE_BATCH_DIV) vs oracle
# recall after churn; (2) serving-path breakdown of the actor at C2 (tools/actor_load,
# 512 closed-loop clients, VSG_PROFILE_HOST_SEARCH=1), FIFO worker and 2 read workers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 50; do echo "[hb] $(date +%T)" >> gpurun_out/r05_heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for D in ${DIVS:-}; do
  VSG_REUSE_BATCH_DIV=$D timeout -k 10 300 python3 -u tools/reuse_probe.py 30000 64 2000 3 > gpurun_out/r05_reuse_div$D.jsonl 2>/dev/null || exit 1
  echo "div $D"; grep churn3 gpurun_out/r05_reuse_div$D.jsonl
done
for V in ${VARIANTS:-}; do  # "batchmax:oracle_threads:start"
  IFS=: read BM OT ST <<< "$V"
  timeout -k 10 600 python3 -u tools/reuse_probe.py 30000 64 2000 3 $BM $OT ${ST:-own} > gpurun_out/r05_reuse_bm${BM}_ot${OT}_${ST:-own}.jsonl 2>/dev/null || exit 1
  echo "batch_max $BM oracle_threads $OT start ${ST:-own}"; grep -E "built|churn3" gpurun_out/r05_reuse_bm${BM}_ot${OT}_${ST:-own}.jsonl
done
if [ "${ACTOR:-1}" = 1 ]; then
  for R in ${READERS:-0 2}; do
    for MD in ${MODES:-1}; do  # 0: a thread per client (vsg_actor_ann); 1: completions (vsg_actor_ann_cb)
      for CL in ${CLIENTS:-512}; do
        T=r${R}_m${MD}_c${CL}
        VSG_PROFILE_HOST_SEARCH=1 timeout -k 10 300 tools/actor_load 1000000 768 2 $CL $((51200 / CL)) 10 36 0 $R $MD > gpurun_out/r05_actor_$T.json 2> gpurun_out/r05_actor_$T.err || { tail -5 gpurun_out/r05_actor_$T.err; exit 1; }
        echo "readers $R mode $MD clients $CL"; cat gpurun_out/r05_actor_$T.json; grep breakdown gpurun_out/r05_actor_$T.err
      done
    done
  done
fi
B="python3 -u bench.py --no-cpu --upper-ef 0 --rerank-leg 0 --config-ef 0 --host-abi-leg 0 --ef 36 --steps 20 --warmup 3"
for F in ${FRACS:-}; do
  VSG_SEARCH_PERSIST_FRAC=$F timeout -k 10 200 $B > gpurun_out/r05_pfrac_$F.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'persist_frac': float(sys.argv[2]), 'qps': d['value'], 'kernel_ms': d['roofline']['kernel_ms'], 'two_streams': d['concurrent_streams']['qps']}))" gpurun_out/r05_pfrac_$F.log $F | tee -a gpurun_out/r05_pfrac.jsonl
done
echo done
