#!/bin/bash
# Skinny-GEMM probe (1x1-conv shapes of the zoo ResNet-50): every tile config vs hipBLASLt; GEMM config tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv.py -x -q -rs --timeout 120 --timeout-method thread -k "tile_config or bn_stats_epilogue or phase" > gpurun_out/r3_tests_skinny.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3_tests_skinny.log | head -30; tail -5 gpurun_out/r3_tests_skinny.log; exit 1; }
tail -8 gpurun_out/r3_tests_skinny.log
timeout -k 10 300 python3 -u tools/skinny_probe.py > gpurun_out/r3_skinny_probe.log 2>&1 || { tail -20 gpurun_out/r3_skinny_probe.log; exit 1; }
grep -v "^W20\|^E20\|amdgpu.ids" gpurun_out/r3_skinny_probe.log
