#!/bin/bash
# GPU: selected test files / node ids (args) or all gpu tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest ${@:-tests} -m gpu -q --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "Error|assert|FAIL|passed|failed" gpurun_out/pytest_gpu.log | tail -30; exit $rc
