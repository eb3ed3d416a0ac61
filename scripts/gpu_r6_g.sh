#!/bin/bash
# r6g: halo-staged 3x3 conv kernel: numerics, BN consuming chunk statistics, per-shape bench vs the tile variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_halo.py > gpurun_out/r6g_halo_tests.log 2>&1; rc=$?; echo "halo tests rc=$rc"; tail -15 gpurun_out/r6g_halo_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 tools/conv_stream_bench.py > gpurun_out/r6g_conv.log 2>&1 || { tail -20 gpurun_out/r6g_conv.log; exit 1; }
cat gpurun_out/r6g_conv.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_v3.py tests/test_gpu_res_bn_fusion.py tests/test_gpu_resnet_numerics.py > gpurun_out/r6g_conv_tests.log 2>&1; echo "conv/bn tests rc=$?"; tail -3 gpurun_out/r6g_conv_tests.log
