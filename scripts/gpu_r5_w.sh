#!/bin/bash
# r5: 1x1-conv GEMM configs (incl. new single-stage wide tiles 8/9) + GEMM GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gemm_conv1x1_bench.py > gpurun_out/r5w_conv1x1.txt 2> gpurun_out/r5w_conv1x1.err || { cat gpurun_out/r5w_conv1x1.txt; tail -5 gpurun_out/r5w_conv1x1.err; exit 1; }
cat gpurun_out/r5w_conv1x1.txt
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/r5w_tests.log 2>&1 || { tail -20 gpurun_out/r5w_tests.log; exit 1; }
tail -2 gpurun_out/r5w_tests.log
