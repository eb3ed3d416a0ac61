#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_conv_benchscale.py > gpurun_out/benchscale.log 2>&1; rc=$?
grep -E "PASS|FAIL|SKIP|Error|assert" gpurun_out/benchscale.log | head -60; exit $rc
