#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/probe.log
p() { timeout -k 10 300 python tools/scale_probe.py "$@" >> gpurun_out/probe.log 2> gpurun_out/probe_err.log; rc=$?; tail -1 gpurun_out/probe.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/probe_err.log; exit $rc; }; }
p 1000000 128 l2sq f16 sift 0 32 64
p 1000000 128 l2sq f32 sift 0 32 64
p 4000000 128 l2sq f16 sift 0 32 64
p 20000000 128 l2sq f16 sift 0 32 64
p 20000000 128 l2sq f32 sift 0 32 64
p 2000000 128 l2sq f32 clustered 0 32 64
p 4000000 768 cos f32 clustered 0 64 128
p 4000000 768 cos f32 clustered 4096 64 128
