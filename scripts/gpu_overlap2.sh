#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "overlap or graph" > gpurun_out/overlap_tests.log 2>&1 || { tail -30 gpurun_out/overlap_tests.log; exit 1; }
tail -2 gpurun_out/overlap_tests.log
DL4J_AMD_WRW_STREAM=0 timeout -k 10 300 python -u bench.py > gpurun_out/bench_nooverlap.log 2>&1 || { tail -20 gpurun_out/bench_nooverlap.log; exit 1; }
tail -1 gpurun_out/bench_nooverlap.log | cut -c1-200
timeout -k 10 300 python -u bench.py > gpurun_out/bench_overlap.log 2>&1 || { tail -20 gpurun_out/bench_overlap.log; exit 1; }
tail -1 gpurun_out/bench_overlap.log | cut -c1-200
bash scripts/prof_resnet.sh prof_resnet_overlap
