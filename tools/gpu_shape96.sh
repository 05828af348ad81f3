#!/bin/bash
# GPU: f16 walk row-shape probe (96-chunk rows): default lib vs Shape<32,3,U> builds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in lib lib_u2 lib_u4; do
  VSG_LIB_PATH=vector-store-text_amd/$v/libvsg.so timeout -k 10 300 python bench.py --no-cpu --config-ef 0 --ef 36 > gpurun_out/shape96_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python -c "import json,sys;d=json.loads(open('gpurun_out/shape96_$v.log').read().strip().splitlines()[-1]);r=d['f16_traversal_rerank'];print('$v', d['value'], r['qps'], r['ef'], r['recall_at_10'], r['kernels_ms'])"
done
