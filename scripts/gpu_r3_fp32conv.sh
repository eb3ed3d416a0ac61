#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_nd4j_ops.py tests/test_gpu_fallback.py -x -v --timeout 300 --timeout-method thread -k "fp32 or lenet" > gpurun_out/r3_tests_fp32conv.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error |assert" gpurun_out/r3_tests_fp32conv.log | head -30; tail -3 gpurun_out/r3_tests_fp32conv.log; exit $rc
