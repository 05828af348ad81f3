#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/actor_load.log
for c in ${CLIENTS:-1 16 64 256 1024 4096}; do
  timeout -k 10 300 ./tools/actor_load ${ROWS:-1000000} ${DIM:-768} 2 $c $(( (c < 64 ? 4000 : 40000) / c)) 10 36 >> gpurun_out/actor_load.log 2>&1 || { rc=$?; cat gpurun_out/actor_load.log; exit $rc; }
done
cat gpurun_out/actor_load.log
