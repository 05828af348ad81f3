#!/bin/bash
# GPU: HNSW parity subset, then search probe (QPS, phase clocks with the profiling build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "hnsw or edge or large_scale or batch_inv" -p no:cacheprovider > gpurun_out/pytest_probe.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_probe.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/waves_probe.py 1000000 768 cos f32 clustered ${EFS:-36,128,321} ${WAVES:-1,r} > gpurun_out/probe_c2.jsonl 2>&1
rc=$?; echo "c2 rc=$rc"; grep '^{' gpurun_out/probe_c2.jsonl
[ $rc -ne 0 ] && exit $rc
VSG_LIB_PATH=$PWD/vector-store-text_amd/lib_prof/libvsg.so timeout -k 10 300 python -u tools/waves_probe.py 1000000 768 cos f32 clustered ${EFS:-36,128,321} r > gpurun_out/probe_c2_prof.jsonl 2>&1
rc=$?; echo "c2 prof rc=$rc"; grep '^{' gpurun_out/probe_c2_prof.jsonl
[ $rc -ne 0 ] && exit $rc
if [ -n "$SIFT" ]; then
timeout -k 10 300 python -u tools/waves_probe.py 10000000 128 l2sq f16 sift 64,192,512 1,r > gpurun_out/probe_sift.jsonl 2>&1
rc=$?; echo "sift rc=$rc"; grep '^{' gpurun_out/probe_sift.jsonl
[ $rc -ne 0 ] && exit $rc
VSG_LIB_PATH=$PWD/vector-store-text_amd/lib_prof/libvsg.so timeout -k 10 300 python -u tools/waves_probe.py 10000000 128 l2sq f16 sift 64,192,512 r > gpurun_out/probe_sift_prof.jsonl 2>&1
rc=$?; echo "sift prof rc=$rc"; grep '^{' gpurun_out/probe_sift_prof.jsonl
fi
exit $rc
