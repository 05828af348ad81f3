#!/bin/bash
# Round 3: selection variants (lib_<var>/libvsg.so built by `make -C vector-store-text_amd
# variant VAR=<var> VFLAGS=...`; "base" = lib/) on the C2 1M build, then the small-shard
# batch schedule on a 125k shard; gpurun_out/r03_sel_probe.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r03_sel_probe.jsonl
for v in ${VARIANTS:-base}; do
  lib=vector-store-text_amd/lib/libvsg.so
  [ "$v" != base ] && lib=vector-store-text_amd/lib_$v/libvsg.so
  echo "== variant $v" >> gpurun_out/r03_sel_probe.log
  VSG_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/build_probe.py --rows 1000000 --reps 2 --queries 2000 --efs 16,32 --settings "${1:-base}" --out $out >> gpurun_out/r03_sel_probe.log 2>&1 || exit 1
done
if [ -n "$SHARD_SETTINGS" ]; then
  timeout -k 10 300 python3 -u tools/build_probe.py --rows 125000 --reps 3 --queries 2000 --efs 10,16,24 --settings "$SHARD_SETTINGS" --out $out >> gpurun_out/r03_sel_probe.log 2>&1 || exit 1
fi
echo done
