#!/bin/bash
# Round 6: serving through the actor at C2 (tools/actor_load, closed-loop clients of
# single-query vsg_actor_ann_cb, ef 36): one read worker (round 5's configuration) vs
# two / four read workers splitting the anns in flight evenly (one batch per worker on
# the device at once; coalescing window 300 us, or 150).
# gpurun_out/r06_actor.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r06_actor.jsonl
run() {  # clients wait_us readers max_batch
  timeout -k 10 240 tools/actor_load 1000000 768 2 $1 $((51200 / $1)) 10 36 $2 $3 1 0x5EED $4 \
    > gpurun_out/r06_actor_run.json 2> gpurun_out/r06_actor_run.err || { tail -5 gpurun_out/r06_actor_run.err; exit 1; }
  cat gpurun_out/r06_actor_run.json >> $out
  grep breakdown gpurun_out/r06_actor_run.err | sed "s/^/# c$1 w$2 r$3 b$4 /" >> gpurun_out/r06_actor_breakdown.txt || true
}
run 512 0 1 0
run 512 0 2 0
run 512 0 4 0
run 512 150 2 0
run 2048 0 1 0
run 2048 0 2 0
run 2048 0 4 0
echo done
