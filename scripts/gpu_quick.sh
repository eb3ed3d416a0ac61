#!/bin/bash
# Quick GPU iteration: GPU tests + bench (eager and HIP-graph), no profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --graph 0 > gpurun_out/bench_eager.log 2>&1 || { echo BENCH_EAGER_FAIL; tail -20 gpurun_out/bench_eager.log; exit 1; }
tail -1 gpurun_out/bench_eager.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --graph 1 > gpurun_out/bench_graph.log 2>&1 || { echo BENCH_GRAPH_FAIL; tail -20 gpurun_out/bench_graph.log; exit 1; }
tail -3 gpurun_out/bench_graph.log
