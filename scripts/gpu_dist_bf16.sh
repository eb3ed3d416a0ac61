#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dist_bf16.log 2>&1 || { tail -40 gpurun_out/dist_bf16.log; exit 1; }
tail -5 gpurun_out/dist_bf16.log
