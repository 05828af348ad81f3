#!/bin/bash
# GPU: cooperative-search parity tests, then QPS vs waves per query
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "cooperative or same_graph or forgetful" -p no:cacheprovider > gpurun_out/pytest_waves.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_waves.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/waves_probe.py 1000000 768 cos f32 clustered 36,128,321 1,2,4 > gpurun_out/waves_c2.jsonl 2>&1
rc=$?; echo "c2 rc=$rc"; cat gpurun_out/waves_c2.jsonl | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/waves_probe.py 10000000 128 l2sq f16 sift 64,192,512 1,2,4 > gpurun_out/waves_sift10m.jsonl 2>&1
rc=$?; echo "sift rc=$rc"; tail -12 gpurun_out/waves_sift10m.jsonl
exit $rc
