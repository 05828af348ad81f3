#!/bin/bash
# GPU: default Shape<32,6,2> vs <32,6,3>, <32,6,4>, <16,12,1>, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in lib lib_d lib_e lib_f lib lib_d lib_e lib_f; do
  VSG_LIB_PATH=vector-store-text_amd/$v/libvsg.so timeout -k 10 300 python bench.py --no-cpu --config-ef 0 --ef 36 --rerank-leg 0 --steps 10 > gpurun_out/shape192r_$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && echo "$v rc=$rc" && exit $rc
  python -c "import json,sys;d=json.loads(open('gpurun_out/shape192r_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], d['roofline']['kernel_ms'], d['build_vectors_per_s'])"
done
