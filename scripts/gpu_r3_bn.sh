#!/bin/bash
# BN relu bitmask + fused fold/finalize: numerics, then bench + last-step kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_conv.py tests/test_gpu_bnpool.py -x -v --timeout 300 --timeout-method thread -k "batchnorm or bn or resnet" > gpurun_out/r3_tests_bn.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3_tests_bn.log | head -30; tail -5 gpurun_out/r3_tests_bn.log; exit 1; }
tail -2 gpurun_out/r3_tests_bn.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_bn.log 2>&1 || { tail -20 gpurun_out/r3_bench_bn.log; exit 1; }
tail -1 gpurun_out/r3_bench_bn.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_bn" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_bn.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_bn.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_bn/run_results.db --top 45 > gpurun_out/r3_prof_bn_step.txt && rm -f gpurun_out/r3_prof_bn/run_results.db && head -30 gpurun_out/r3_prof_bn_step.txt
