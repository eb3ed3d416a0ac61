#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv_v3.py tests/test_gpu_conv_safety.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_tests_v3.log 2>&1 || { tail -30 gpurun_out/r3_tests_v3.log; exit 1; }
tail -3 gpurun_out/r3_tests_v3.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_v3.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r3_bench_v3.log; exit 1; }
tail -1 gpurun_out/r3_bench_v3.log
bash scripts/prof_resnet.sh r3_prof_v3
