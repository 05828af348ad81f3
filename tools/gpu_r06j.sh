#!/bin/bash
# Round 6: host-buffer search (vsg_index_search, PCIe both ways) at C2, 10k queries,
# ef 36: one piece vs 4 pieces each on its own stream (VSG_HOST_SEARCH_PIECES).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 1 2 4; do
  VSG_HOST_SEARCH_PIECES=$p timeout -k 10 200 python3 -u tools/host_search_probe.py 1000000 10000 36 10 \
    | sed "s/^{/{\"pieces\": $p, /" >> gpurun_out/r06j_host.jsonl || exit 2
done
cat gpurun_out/r06j_host.jsonl
