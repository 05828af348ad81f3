cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 ./tools/actor_load 200000 768 2 64 625 10 36 > gpurun_out/dbg0.log 2>&1
echo "rc=$?"; grep -v mismatch gpurun_out/dbg0.log
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 300 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
