#!/bin/bash
# GPU: default bench (with the config-ef leg), then the C4 8-shard emulation
# (small rehearsal first).  Each step under its own limit; stop on failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench_cfgef.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_cfgef.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/shard_emulation.py --rows 400000 --shards 4 --efs 16,64 --queries 2000 --gt-queries 200 --out gpurun_out/shard_emu_small.jsonl > gpurun_out/shard_emu_small.log 2>&1
rc=$?; echo "small rc=$rc"; tail -3 gpurun_out/shard_emu_small.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/shard_emulation.py ${C4ARGS:---rows 100000000 --shards 8} --out gpurun_out/shard_emu_c4.jsonl > gpurun_out/shard_emu_c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -12 gpurun_out/shard_emu_c4.log
exit $rc
