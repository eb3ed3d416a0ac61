#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_tests_rccl.log 2>&1; rc=$?
tail -25 gpurun_out/r3_tests_rccl.log; exit $rc
