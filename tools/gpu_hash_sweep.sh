#!/bin/bash
# GPU: HNSW parity subset, then QPS vs visited-table factor for the default search kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "hnsw or edge or large_scale or batch_inv" -p no:cacheprovider > gpurun_out/pytest_probe.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_probe.log
[ $rc -ne 0 ] && exit $rc
fi
for ef in 192 512; do
timeout -k 10 300 python -u tools/hash_factor_probe.py 10000000 128 l2sq f16 sift $ef 2 3 4 6 8 > gpurun_out/hash_sift_$ef.jsonl 2>&1
rc=$?; echo "sift $ef rc=$rc"; grep '^{' gpurun_out/hash_sift_$ef.jsonl
[ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u tools/hash_factor_probe.py 1000000 768 cos f32 clustered 321 4 8 12 16 > gpurun_out/hash_c2_321.jsonl 2>&1
rc=$?; echo "c2 rc=$rc"; grep '^{' gpurun_out/hash_c2_321.jsonl
exit $rc
