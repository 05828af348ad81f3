#!/bin/bash
# GPU: measurement chain only (bench, rocprof, PMC, rerank trace, gloo rehearsal)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_measure.sh
