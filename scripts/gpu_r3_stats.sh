#!/bin/bash
# Wave-parallel BN-statistics epilogue: GEMM/conv stats tests, skinny probe, ResNet-50 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv.py tests/test_gpu_kernels.py -x -q -rs --timeout 120 --timeout-method thread -k "tile_config or stats or phase or batchnorm" > gpurun_out/r3_tests_stats.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3_tests_stats.log | head -30; tail -5 gpurun_out/r3_tests_stats.log; exit 1; }
tail -3 gpurun_out/r3_tests_stats.log
timeout -k 10 300 python3 -u tools/skinny_probe.py > gpurun_out/r3_skinny_probe2.log 2>&1 || { tail -20 gpurun_out/r3_skinny_probe2.log; exit 1; }
grep -v "^W20\|^E20\|amdgpu.ids" gpurun_out/r3_skinny_probe2.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_stats.log 2>&1 || { tail -20 gpurun_out/r3_bench_stats.log; exit 1; }
tail -1 gpurun_out/r3_bench_stats.log
