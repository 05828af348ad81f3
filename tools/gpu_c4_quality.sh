#!/bin/bash
# GPU: 100M sift-like graph quality vs level seed and insertion batch size
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/tie_recall_probe.py 100000000 128 l2sq f16 sift 3 256,512,1024 0x5EED > gpurun_out/c4q_a.jsonl 2>&1
rc=$?; tail -4 gpurun_out/c4q_a.jsonl; [ $rc -ne 0 ] && exit $rc
VSG_BUILD_BATCH_MAX=8192 timeout -k 10 600 python -u tools/tie_recall_probe.py 100000000 128 l2sq f16 sift 3 256,512,1024 0x5EED > gpurun_out/c4q_b.jsonl 2>&1
rc=$?; tail -4 gpurun_out/c4q_b.jsonl
exit $rc
