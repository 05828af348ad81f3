#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() { tag=$1; shift; timeout -k 10 300 "$@" > gpurun_out/exp3_$tag.log 2>&1; rc=$?; [ $rc -ne 0 ] && { echo "$tag rc=$rc"; tail -3 gpurun_out/exp3_$tag.log; exit $rc; }
  python -c "import json;d=json.loads(open('gpurun_out/exp3_$tag.log').read().strip().splitlines()[-1]);print('$tag', d['value'], d['config']['ef'], d['config']['recall_at_10'], d['roofline']['kernel_ms'], d['build_vectors_per_s'])"; }
run base python bench.py --no-cpu --steps 5
run sortedbase python bench.py --no-cpu --steps 5 --sort-base cluster
run sortedbq python bench.py --no-cpu --steps 5 --sort-base cluster --sort-queries cluster
