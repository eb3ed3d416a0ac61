#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_lstm_graph.py tests/test_gpu_lstm.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r3_tests_lstmg.log 2>&1; rc=$?
tail -30 gpurun_out/r3_tests_lstmg.log; exit $rc
