#!/bin/bash
# Locality experiments on C2: XCD query mapping, cluster-ordered base, cluster-ordered queries.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 300 env "$@" > gpurun_out/exp2_$tag.log 2>&1; rc=$?; [ $rc -ne 0 ] && { echo "$tag rc=$rc"; tail -3 gpurun_out/exp2_$tag.log; exit $rc; }
  python -c "import json;d=json.loads(open('gpurun_out/exp2_$tag.log').read().strip().splitlines()[-1]);print('$tag', d['value'], d['config']['ef'], d['config']['recall_at_10'], d['roofline']['kernel_ms'], d['build_vectors_per_s'])"; }
B="python bench.py --no-cpu --steps 5"
run base VSG_SEARCH_XCD_MAP=0 $B
run xcd VSG_SEARCH_XCD_MAP=1 $B
run q VSG_SEARCH_XCD_MAP=0 $B --sort-queries cluster
run qxcd VSG_SEARCH_XCD_MAP=1 $B --sort-queries cluster
run bq VSG_SEARCH_XCD_MAP=0 $B --sort-queries cluster --sort-base cluster
run bqxcd VSG_SEARCH_XCD_MAP=1 $B --sort-queries cluster --sort-base cluster
run b VSG_SEARCH_XCD_MAP=0 $B --sort-base cluster
