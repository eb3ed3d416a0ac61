#!/bin/bash
# r6t: full GPU suite after the fp32 / torch-op changes; host profile of the eager LeNet step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6t_gpu_suite.log 2>&1; rc=$?; tail -3 gpurun_out/r6t_gpu_suite.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r6t_gpu_suite.log | head -20; exit 1; }
timeout -k 10 300 python3 -m cProfile -s tottime tools/bench_lenet.py --device cuda --graph 0 --steps 300 --warmup 5 > gpurun_out/r6t_lenet_cprof.txt 2>&1 || { tail -5 gpurun_out/r6t_lenet_cprof.txt; exit 1; }
head -45 gpurun_out/r6t_lenet_cprof.txt
