#!/bin/bash
# GPU: f32 768-d row-shape probe (192-chunk rows): default Shape<64,3,4> vs probe builds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in lib lib_a lib_b lib_c; do
  VSG_LIB_PATH=vector-store-text_amd/$v/libvsg.so timeout -k 10 300 python bench.py --no-cpu --config-ef 0 --ef 36 --rerank-leg 0 > gpurun_out/shape192_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python -c "import json,sys;d=json.loads(open('gpurun_out/shape192_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], d['roofline']['kernel_ms'], d['config']['recall_at_10'], d['build_vectors_per_s'])"
done
