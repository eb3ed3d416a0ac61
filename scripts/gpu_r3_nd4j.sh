#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_nd4j_ops.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_tests_nd4j.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r3_tests_nd4j.log | head -40; tail -3 gpurun_out/r3_tests_nd4j.log; exit $rc
