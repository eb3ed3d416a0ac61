#!/bin/bash
# Fold-path tests (conv tile statistics -> BN), BN kernel tests, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv_v3.py tests/test_gpu_kernels.py tests/test_gpu_bnpool.py tests/test_gpu_bn_bwd_epilogue.py -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/r3c_fold_tests.log 2>&1 || { tail -40 gpurun_out/r3c_fold_tests.log; exit 1; }
tail -1 gpurun_out/r3c_fold_tests.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3c_bench_fold.log 2>&1 || { tail -20 gpurun_out/r3c_bench_fold.log; exit 1; }
tail -1 gpurun_out/r3c_bench_fold.log | cut -c1-200
