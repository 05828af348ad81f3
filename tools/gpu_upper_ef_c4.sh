#!/bin/bash
# GPU: C4 100M single graph, wider level-1 beams
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/upper_ef_probe.py 100000000 128 l2sq f16 sift 3 256,512,1024 256,1024 > gpurun_out/ue_c4_wide.jsonl 2>&1
rc=$?; cat gpurun_out/ue_c4_wide.jsonl | tail -7
exit $rc
