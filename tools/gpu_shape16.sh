#!/bin/bash
# GPU: 128-d f16 row-shape probe (16-chunk rows) on sift-like 10M x 128 f16 (integer data:
# every shape gives the same graph and results, only speed differs)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in lib lib_g lib_h lib lib_g lib_h; do
  VSG_LIB_PATH=vector-store-text_amd/$v/libvsg.so timeout -k 10 300 python bench.py --rows 10000000 --dim 128 --metric l2sq --quant f16 --data sift --config 3 --no-cpu --config-ef 0 --rerank-leg 0 --upper-ef 0 --gt-queries 500 --steps 5 > gpurun_out/shape16_$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && echo "$v rc=$rc" && exit $rc
  python -c "import json;d=json.loads(open('gpurun_out/shape16_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], d['config']['ef'], d['config']['recall_at_10'], d['roofline']['kernel_ms'], d['build_vectors_per_s'])"
done
