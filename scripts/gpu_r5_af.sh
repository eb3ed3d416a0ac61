#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DL4J_AMD_TUNE_DB=off timeout -k 10 300 python3 tools/gemm_layout_probe.py > gpurun_out/r5af_layout.txt 2>&1 || { tail -10 gpurun_out/r5af_layout.txt; exit 1; }
cat gpurun_out/r5af_layout.txt
