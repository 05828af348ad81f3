#!/bin/bash
# GPU: level-ordered insertion vs random order: 100M sift-like (recall ceiling) and C2 1M
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VSG_BUILD_LEVEL_ORDER=1 timeout -k 10 500 python -u tools/tie_recall_probe.py 100000000 128 l2sq f16 sift 3 128,256,512,1024 0x5EED > gpurun_out/lo_c4.jsonl 2>&1
rc=$?; tail -5 gpurun_out/lo_c4.jsonl; [ $rc -ne 0 ] && exit $rc
for lo in 0 1; do
VSG_BUILD_LEVEL_ORDER=$lo timeout -k 10 300 python -u tools/tie_recall_probe.py 1000000 768 cos f32 clustered 2 24,32,36,48 0x5EED > gpurun_out/lo_c2_$lo.jsonl 2>&1
rc=$?; tail -5 gpurun_out/lo_c2_$lo.jsonl; [ $rc -ne 0 ] && exit $rc
done
exit 0
