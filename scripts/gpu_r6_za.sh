#!/bin/bash
# r6za: full GPU suite + ResNet-50 bench after the BatchNormalization regularisation fix and the config ports
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6za_gpu_suite.log 2>&1; rc=$?; tail -2 gpurun_out/r6za_gpu_suite.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r6za_gpu_suite.log | head -20; exit 1; }
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6za_bench.json 2> gpurun_out/r6za_bench.err || { tail -5 gpurun_out/r6za_bench.err; exit 1; }
cat gpurun_out/r6za_bench.json
