#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/grad_diag.py 64 > gpurun_out/r3_graddiag.log 2>&1; echo "diag rc=$?"; tail -12 gpurun_out/r3_graddiag.log
DL4J_AMD_CONV_V3=0 timeout -k 10 120 python3 tools/grad_diag.py 64 > gpurun_out/r3_graddiag_v2.log 2>&1; tail -8 gpurun_out/r3_graddiag_v2.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_v3.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r3_bench_v3.log; exit 1; }
tail -1 gpurun_out/r3_bench_v3.log
timeout -k 10 300 python3 tools/conv_bench.py --batch 512 --reps 10 > gpurun_out/r3_conv_bench_v3.log 2>&1; tail -26 gpurun_out/r3_conv_bench_v3.log
bash scripts/prof_resnet.sh r3_prof_v3
