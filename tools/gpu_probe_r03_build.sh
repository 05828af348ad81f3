#!/bin/bash
# Round 3: build-schedule probe at a C2 shard of 125k rows (small-shard efficiency,
# VERDICT r2 next #5) and the stored-edge-distance A/B (next #4); outputs in gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/build_probe.py --rows 125000 --reps 3 --settings "${1:-base}" --out gpurun_out/r03_build_probe_125k.jsonl > gpurun_out/r03_build_probe.log 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/build_probe.py --rows 1000000 --reps 2 --queries 2000 --settings "${2:-base}" --out gpurun_out/r03_build_probe_1m.jsonl > gpurun_out/r03_build_probe_1m.log 2>&1 || exit 1
