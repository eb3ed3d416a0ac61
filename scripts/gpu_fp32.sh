#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fallback.py tests/test_gpu_conv.py tests/test_gpu_dist.py > gpurun_out/fp32_tests.log 2>&1; rc=$?
tail -3 gpurun_out/fp32_tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/fp32_tests.log | head -20; exit $rc; }
