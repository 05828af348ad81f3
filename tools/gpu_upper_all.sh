#!/bin/bash
# GPU: multi-entry variant with beams on every upper level (probe build lib_all)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export VSG_LIB_PATH=vector-store-text_amd/lib_all/libvsg.so
timeout -k 10 300 python -u tools/upper_ef_probe.py 1000000 768 cos f32 clustered 1 24,29,32 8,16 > gpurun_out/ue_all_c2.jsonl 2>&1
rc=$?; tail -6 gpurun_out/ue_all_c2.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/upper_ef_probe.py 100000000 128 l2sq f16 sift 3 256,512,1024 64,256 > gpurun_out/ue_all_c4.jsonl 2>&1
rc=$?; tail -6 gpurun_out/ue_all_c4.jsonl
exit $rc
