#!/bin/bash
# r6: streaming 1x1-conv GEMM: numerics, per-shape bench, ResNet-50 with the gemm table re-tuned (and recorded)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_stream.py > gpurun_out/r6b_stream_tests.log 2>&1 || { tail -30 gpurun_out/r6b_stream_tests.log; exit 1; }
tail -1 gpurun_out/r6b_stream_tests.log
timeout -k 10 300 python3 tools/gemm_conv1x1_bench.py --cfgs 5,8,10 > gpurun_out/r6b_1x1.log 2>&1 || { tail -20 gpurun_out/r6b_1x1.log; exit 1; }
cat gpurun_out/r6b_1x1.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/r6b_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r6b_gemm_tests.log; exit 1; }
tail -1 gpurun_out/r6b_gemm_tests.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_res_bn_fusion.py > gpurun_out/r6b_rbn_tests.log 2>&1 || { tail -30 gpurun_out/r6b_rbn_tests.log; exit 1; }
tail -1 gpurun_out/r6b_rbn_tests.log
timeout -k 10 300 python3 -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_step_kernels.py > gpurun_out/r6b_step_kernels.log 2>&1; echo "step-kernels rc=$?"; grep -E "torch:|kernels,|passed|failed" gpurun_out/r6b_step_kernels.log | head -30
DL4J_AMD_TUNE_DB_SKIP=gemm DL4J_AMD_TUNE_RECORD=$R/gpurun_out/r6b_tune_zoo.json DL4J_AMD_TUNE_REPS=6 timeout -k 10 300 python3 -u bench.py > gpurun_out/r6b_bench_retune.log 2>&1 || { tail -20 gpurun_out/r6b_bench_retune.log; exit 1; }
tail -1 gpurun_out/r6b_bench_retune.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py > gpurun_out/r6b_bench_db.log 2>&1 || { tail -20 gpurun_out/r6b_bench_db.log; exit 1; }
tail -1 gpurun_out/r6b_bench_db.log | cut -c1-200
