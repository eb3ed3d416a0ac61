#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_updaters_gn.py tests/test_gpu_updaters_reference.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_tests_gn.log 2>&1; rc=$?
tail -15 gpurun_out/r3_tests_gn.log; exit $rc
