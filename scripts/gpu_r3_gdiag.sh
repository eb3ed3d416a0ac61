#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/graph_diag.py > gpurun_out/r3_graph_diag.log 2>&1; rc=$?
cat gpurun_out/r3_graph_diag.log | grep -v amdgpu.ids; exit $rc
