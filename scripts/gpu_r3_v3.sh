#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/grad_diag.py 64 > gpurun_out/r3_graddiag.log 2>&1; echo "diag rc=$?"; cat gpurun_out/r3_graddiag.log | tail -12
DL4J_AMD_CONV_V3=0 timeout -k 10 120 python3 tools/grad_diag.py 64 > gpurun_out/r3_graddiag_v2.log 2>&1; tail -8 gpurun_out/r3_graddiag_v2.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv_v3.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_tests_v3.log 2>&1; rc=$?
tail -15 gpurun_out/r3_tests_v3.log; exit $rc
