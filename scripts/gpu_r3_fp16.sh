#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_conv_v3.py tests/test_gpu_nd4j_ops.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3_tests_fp16.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error |assert" gpurun_out/r3_tests_fp16.log | head -60; tail -3 gpurun_out/r3_tests_fp16.log; exit $rc
