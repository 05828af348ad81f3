#!/bin/bash
# Round 5: (1) searches beside a large add with the add's phase clock, persistent
# search grid on / off; (2) reverse-kernel variants (lib_<v>/libvsg.so from `make -C
# vector-store-text_amd variant VAR=<v> VFLAGS=...`; "base" = lib/) on the C2 1M build.
# gpurun_out/r05_conc_probe.{jsonl,log}, gpurun_out/r05_rev_probe.{jsonl,log}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 1 0; do
  VSG_SEARCH_PERSIST=$p VSG_DEBUG_TIMING=1 timeout -k 10 200 python3 -u tools/concurrency_probe.py \
    >> gpurun_out/r05_conc_probe.jsonl 2>> gpurun_out/r05_conc_probe.log || exit 1
done
for v in ${VARIANTS:-base}; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  echo "== variant $v" >> gpurun_out/r05_rev_probe.log
  VSG_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/build_probe.py --rows 1000000 --reps 2 --queries 2000 \
    --efs 16,32 --out gpurun_out/r05_rev_probe_$v.jsonl >> gpurun_out/r05_rev_probe.log 2>&1 || exit 1
done
echo done
