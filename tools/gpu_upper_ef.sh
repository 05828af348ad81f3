#!/bin/bash
# GPU: multi-entry descent probe -- small parity tests first, then C2 1M and C4 100M single graph
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "register or same_graph or full_size" > gpurun_out/pytest_ue.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ue.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/upper_ef_probe.py 1000000 768 cos f32 clustered 1 24,32,36,48 0,8,16,32 > gpurun_out/ue_c2.jsonl 2>&1
rc=$?; cat gpurun_out/ue_c2.jsonl | tail -17; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/upper_ef_probe.py 100000000 128 l2sq f16 sift 3 128,256,512,1024 0,16,64 > gpurun_out/ue_c4.jsonl 2>&1
rc=$?; cat gpurun_out/ue_c4.jsonl | tail -13
exit $rc
