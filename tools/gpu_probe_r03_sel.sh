#!/bin/bash
# Round 3: selection pass-depth / block variants (lib_<var>/libvsg.so built by
# `make -C vector-store-text_amd variant`), C2 1M and a 125k shard; gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r03_sel_probe.jsonl
for v in ${VARIANTS:-"" n4u2 n3u2 n2u2}; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  echo "== variant ${v:-base}" >> gpurun_out/r03_sel_probe.log
  VSG_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/build_probe.py --rows 1000000 --reps 2 --queries 2000 --efs 16,32 --settings "${1:-base}" --out $out >> gpurun_out/r03_sel_probe.log 2>&1 || exit 1
done
