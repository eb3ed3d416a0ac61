#!/bin/bash
# r5: fast LDS epilogue sweep — GEMM / conv / transformer tests, phase stamps, probe, gemm table, ResNet bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv.py tests/test_gpu_conv_v3.py tests/test_gpu_transformer.py tests/test_gpu_bn_bwd_epilogue.py tests/test_gpu_kernels.py tests/test_gpu_coop_guard.py tests/test_gpu_graph_workspace.py tests/test_gpu_abi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1 || { tail -40 gpurun_out/r5d_tests.log; exit 1; }
tail -2 gpurun_out/r5d_tests.log
for s in "4096 2304 64" "4096 2304 768" "4096 4096 4096" "4096 768 3072"; do
  timeout -k 5 60 ./tools/native/gemm_stamps $s 4 >> gpurun_out/r5d_stamps.log 2>&1 || exit 1
done
cat gpurun_out/r5d_stamps.log
timeout -k 10 300 python3 -u tools/gemm_bench.py --rounds 3 > gpurun_out/r5d_gemm.log 2>&1 || { tail -20 gpurun_out/r5d_gemm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5d_gemm.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5d_bench.log 2>&1 || { tail -20 gpurun_out/r5d_bench.log; exit 1; }
tail -1 gpurun_out/r5d_bench.log
