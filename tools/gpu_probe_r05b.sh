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
for D in ${DIVS:-1 64 256}; do
  VSG_REUSE_BATCH_DIV=$D timeout -k 10 300 python3 -u tools/reuse_probe.py 30000 64 2000 3 > gpurun_out/r05_reuse_div$D.jsonl 2>/dev/null || exit 1
  echo "div $D"; grep churn3 gpurun_out/r05_reuse_div$D.jsonl
done
if [ "${ACTOR:-1}" = 1 ]; then
  for R in 0 2; do
    VSG_PROFILE_HOST_SEARCH=1 timeout -k 10 300 tools/actor_load 1000000 768 2 512 100 10 36 0 $R > gpurun_out/r05_actor_r$R.json 2> gpurun_out/r05_actor_r$R.err || { tail -5 gpurun_out/r05_actor_r$R.err; exit 1; }
    cat gpurun_out/r05_actor_r$R.json; grep breakdown gpurun_out/r05_actor_r$R.err
  done
fi
echo done
