#!/bin/bash
# BN backward partial (pipelined, packed loads, balanced grid) + LN backward fold. Tests, benches, profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_conv.py tests/test_gpu_bnpool.py tests/test_gpu_transformer.py tests/test_gpu_fallback.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread -k "batchnorm or bn or resnet or layernorm or bert or fp16 or engine or alloc or dlpack or graph or stream or device" > gpurun_out/r3_tests_bn4.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3_tests_bn4.log | head -30; tail -5 gpurun_out/r3_tests_bn4.log; exit 1; }
tail -1 gpurun_out/r3_tests_bn4.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_bn4.log 2>&1 || { tail -20 gpurun_out/r3_bench_bn4.log; exit 1; }
tail -1 gpurun_out/r3_bench_bn4.log
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r3_bench_bert4.log 2>&1 || { tail -20 gpurun_out/r3_bench_bert4.log; exit 1; }
tail -1 gpurun_out/r3_bench_bert4.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_bn4" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_bn4.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_bn4.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_bn4/run_results.db --top 45 > gpurun_out/r3_prof_bn4_step.txt && rm -f gpurun_out/r3_prof_bn4/run_results.db && grep -E "bn_|one step" gpurun_out/r3_prof_bn4_step.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_bert4" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_bert4.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_bert4.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_bert4/run_results.db --top 40 > gpurun_out/r3_prof_bert4_step.txt && rm -f gpurun_out/r3_prof_bert4/run_results.db && head -16 gpurun_out/r3_prof_bert4_step.txt
