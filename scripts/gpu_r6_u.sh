#!/bin/bash
# r6u: host profile of the eager LeNet fp32 step (no test run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -m cProfile -s tottime tools/bench_lenet.py --device cuda --graph 0 --steps 300 --warmup 5 > gpurun_out/r6u_lenet_cprof.txt 2>&1 || { tail -5 gpurun_out/r6u_lenet_cprof.txt; exit 1; }
head -60 gpurun_out/r6u_lenet_cprof.txt | cut -c1-150
