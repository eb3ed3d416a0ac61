#!/bin/bash
# BN-backward epilogue: numerics tests, then the ResNet-50 bench with and without it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bn_bwd_epilogue.py tests/test_gpu_kernels.py -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/r3c_bnb_tests.log 2>&1 || { tail -40 gpurun_out/r3c_bnb_tests.log; exit 1; }
tail -3 gpurun_out/r3c_bnb_tests.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3c_bench_bnb.log 2>&1 || { tail -20 gpurun_out/r3c_bench_bnb.log; exit 1; }
tail -1 gpurun_out/r3c_bench_bnb.log
DL4J_AMD_BN_BWD_EPILOGUE=0 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3c_bench_nobnb.log 2>&1 || { tail -20 gpurun_out/r3c_bench_nobnb.log; exit 1; }
tail -1 gpurun_out/r3c_bench_nobnb.log
