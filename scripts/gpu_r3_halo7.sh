#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv_v3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_tests_halo.log 2>&1 || { tail -40 gpurun_out/r3_tests_halo.log; exit 1; }
tail -2 gpurun_out/r3_tests_halo.log
timeout -k 10 400 python3 tools/wrw_halo_bench.py --batch 512 --reps 10 > gpurun_out/r3_wrw_halo_bench.log 2>&1 || { tail -20 gpurun_out/r3_wrw_halo_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_wrw_halo_bench.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_halo.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r3_bench_halo.log; exit 1; }
tail -1 gpurun_out/r3_bench_halo.log
